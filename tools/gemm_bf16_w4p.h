// gemm_bf16_w4p.h -- development probe (not part of the library; included by
// tools/gemm_w4i_probe.hip): the bf16 chained GEMM on PACKED operands.
//
// Why: the flow probe (profiles/r05_mfma_flow.log) holds 2.0 GHz with 16
// ds_read_b128 per step (B as B^T) against 1.72 GHz with the library's
// 8 b128 + 16 ds_read_b64_tr_b16, and the library's stamps put ~5 cycles per
// MFMA in issuing fills that miss L2 from 256 scattered 128-B row lines per
// tile; B^T staged from the chunks as stored lost more to its own scattered
// lines than the reads gained (tools/gemm_bf16_w4t.h).  Here both operands
// are first packed (one pass each) into the LDS image itself: per 256-row
// panel of A (256-column panel of B^T) and 64-deep k tile, 32 KiB with row r
// at r * 128 and 16-B slot s holding k chunk s ^ ((r >> 1) & 7), the chain's
// K segments concatenated and every pad zero.  A staging piece is then 1 KiB
// of consecutive bytes, B fragments are ds_read_b128, and the K loop has no
// segment logic at all.  Requires k segments of the same width, a multiple of
// 8 (config 5: 5000); the library would pack per matmul.
#pragma once

struct PackGeom {
  int64_t nI, nK, nJ;   // chunk grid: A is nI x nK chunks, B nK x nJ
  int64_t cm, ck, cn;   // chunk extents (regular grid)
  int64_t K;            // total K
  int64_t TM, TN, KTL;  // tiles per chunk row / column, 64-k tiles over K
};

// A chunk (I, s) at A + (I * nK + s) * slot, row pitch ck; packed block
// (I, mt, kt) at PA + ((I * TM + mt) * KTL + kt) * 32 KiB
__global__ void k_packA(const char* __restrict__ A, int64_t slot, PackGeom g, char* __restrict__ PA) {
  const int64_t nblk = g.nI * g.TM * g.KTL;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t kt = blk % g.KTL, mt = (blk / g.KTL) % g.TM, I = blk / (g.KTL * g.TM);
    char* dst = PA + blk * 32768;
    for (int u = threadIdx.x; u < 2048; u += blockDim.x) {
      const int r = u >> 3, sl = u & 7, c = sl ^ ((r >> 1) & 7);
      const int64_t gm = mt * 256 + r, k = kt * 64 + c * 8;
      uint4 v = {0, 0, 0, 0};
      if (gm < g.cm && k < g.K) {
        const int64_t s = k / g.ck, kk = k - s * g.ck;
        v = *(const uint4*)(A + (I * g.nK + s) * slot + (gm * g.ck + kk) * 2);
      }
      *(uint4*)(dst + r * 128 + sl * 16) = v;
    }
  }
}

// B chunk (s, J) at B + (s * nJ + J) * slot, row pitch cn; packed B^T block
// (J, nt, kt) at PB + ((J * TN + nt) * KTL + kt) * 32 KiB: row = column n
__global__ void k_packBT(const char* __restrict__ B, int64_t slot, PackGeom g, char* __restrict__ PB) {
  __shared__ uint16_t t[64][258];
  const int64_t nblk = g.nJ * g.TN * g.KTL;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t kt = blk % g.KTL, nt = (blk / g.KTL) % g.TN, J = blk / (g.KTL * g.TN);
    for (int u = threadIdx.x; u < 64 * 256; u += blockDim.x) {
      const int kr = u >> 8, n = u & 255;
      const int64_t k = kt * 64 + kr, gn = nt * 256 + n;
      uint16_t v = 0;
      if (k < g.K && gn < g.cn) {
        const int64_t s = k / g.ck, kk = k - s * g.ck;
        v = *(const uint16_t*)(B + (s * g.nJ + J) * slot + (kk * g.cn + gn) * 2);
      }
      t[kr][n] = v;
    }
    __syncthreads();
    char* dst = PB + blk * 32768;
    for (int u = threadIdx.x; u < 2048; u += blockDim.x) {
      const int r = u >> 3, sl = u & 7, c = sl ^ ((r >> 1) & 7);
      uint16_t e[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) e[i] = t[c * 8 + i][r];
      *(uint4*)(dst + r * 128 + sl * 16) = *(const uint4*)e;
    }
    __syncthreads();
  }
}

// the same B^T blocks by an 8 x 8 register transpose per thread: thread t
// takes k chunk c = t & 7 and columns 8 (t >> 3) .. +7, reads 8 rows of 16 B
// and writes 8 rows' slot; 8 consecutive threads fill one 128-B row line.
// Needs cn % 8 == 0 (whole 16-B column groups) and 16-B aligned rows.
__global__ void k_packBT8(const char* __restrict__ B, int64_t slot, PackGeom g, char* __restrict__ PB) {
  const int64_t nblk = g.nJ * g.TN * g.KTL;
  const int c = threadIdx.x & 7, n8 = threadIdx.x >> 3;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t kt = blk % g.KTL, nt = (blk / g.KTL) % g.TN, J = blk / (g.KTL * g.TN);
    const int64_t gn = nt * 256 + n8 * 8, k0 = kt * 64 + c * 8;
    uint16_t in[8][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      uint4 v = {0, 0, 0, 0};
      const int64_t k = k0 + e;
      if (k < g.K && gn < g.cn) {
        const int64_t s = k / g.ck, kk = k - s * g.ck;
        v = *(const uint4*)(B + (s * g.nJ + J) * slot + (kk * g.cn + gn) * 2);
      }
      *(uint4*)in[e] = v;
    }
    char* dst = PB + blk * 32768;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = n8 * 8 + j, sl = c ^ ((r >> 1) & 7);
      uint16_t o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = in[e][j];
      *(uint4*)(dst + r * 128 + sl * 16) = *(const uint4*)o;
    }
  }
}

// SYNC: soft lockstep between tiles that share a panel (probe): per-tile
// progress words (zeroed before the launch), published every 8 steps by lane
// 0 of wave 0 with vector stores; a tile whose partner (next tile down the
// same column = same B^T panel, next tile along the row = same A panel, both
// in this XCD's run) has started and trails it by 9..64 steps waits for it
// (bounded spin: s_sleep, at most 4000 polls), so the group reads each block
// while it is still in the XCD's L2.
__device__ int* g_w4p_progress;

// ABL (ablation, results wrong when nonzero): 1 = A sources stay on tiles
// 0 / 1 (L2-resident fills), 2 = the same for B^T
template <bool OUT_BF16, bool STAMP = false, int ABL = 0, bool SYNC = false, int SI = 8, int SL = 8, int SW = 64, int GMT = 4>
__global__ __launch_bounds__(256, 1) void k_w4p_probe(const cubed_gemm_chain_t* __restrict__ tasks,
                                                       const char* __restrict__ PA, const char* __restrict__ PB,
                                                       PackGeom pg, int64_t tiles_m, int64_t tiles_n,
                                                       unsigned long long* __restrict__ stamp_out) {
  __shared__ __attribute__((aligned(1024))) char lds_[(WT_NA + WT_NB) * WL_ATILE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  CUBED_L char* ldsA = lds;
  CUBED_L char* ldsB = lds + WT_NA * WL_ATILE;
  int64_t t, m0, n0;
  const int64_t gt = xcd_remap(blockIdx.x, gridDim.x);
  tile_of<HB_BM, HB_BN, GMT>(gt, tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n;
  // partners (SYNC): -1 where none
  int64_t partB = -1, partA = -1;
  if constexpr (SYNC) {
    const int64_t nblk = gridDim.x, xcd = blockIdx.x & 7, q8 = nblk >> 3, r8 = nblk & 7;
    const int64_t run_end = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + q8 + (xcd < r8 ? 1 : 0);
    const int64_t tpt = tiles_m * tiles_n, tile = gt - t * tpt, per_group = 4 * tiles_n;
    const int64_t grp = tile / per_group, first_m = grp * 4;
    const int64_t gsz = (tiles_m - first_m) < 4 ? (tiles_m - first_m) : 4;
    const int64_t in_g = tile - grp * per_group;
    if (in_g % gsz < gsz - 1 && gt + 1 < run_end) partB = gt + 1;
    if (in_g + gsz < gsz * tiles_n && gt + gsz < run_end) partA = gt + gsz;
  }
  if (m0 >= M || n0 >= N) {
    if constexpr (SYNC)  // (a padded tile: let its partners see it as finished)
      if (threadIdx.x == 0) __hip_atomic_store(g_w4p_progress + gt, 1 << 30, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const int64_t I = t / pg.nJ, J = t % pg.nJ;
  const int64_t KTL = pg.KTL, ntile = KTL, nst = 2 * KTL;
  // this tile's two streams of 32 KiB blocks
  const char* sA = PA + ((I * pg.TM + m0 / 256) * KTL) * 32768;
  const char* sB = PB + ((J * pg.TN + n0 / 256) * KTL) * 32768;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const uint32_t loff = (uint32_t)((64 * w) * 128 + lane * 16);  // piece i adds i KiB

  const char* const sAl = sA + loff;
  const char* const sBl = sB + loff;
  CUBED_L char* const dA = ldsA + (64 * w) * 128;
  CUBED_L char* const dB = ldsB + (64 * w) * 128;
#define W4P_PIECE_A(i, tile) \
  glds16(sAl + ((ABL & 1) ? ((tile) & 1) : (tile)) * 32768 + (i) * 1024, dA + ((tile) % WT_NA) * WL_ATILE + (i) * 1024)
#define W4P_PIECE_B(i, tile) \
  glds16(sBl + ((ABL & 2) ? ((tile) & 1) : (tile)) * 32768 + (i) * 1024, dB + ((tile) % WT_NB) * WL_ATILE + (i) * 1024)

  const int ra = wr * 128 + (lane & 31), rb = wc * 128 + (lane & 31);
  // fragment offsets of the two 32-k halves of a 64-k tile: h selects by
  // arithmetic (a select of array elements becomes a scratch address)
  uint32_t oA0[2], oA1[2], oB0[2], oB1[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    oA0[kh] = ra * 128 + 16 * ((2 * kh + (lane >> 5)) ^ ((ra >> 1) & 7));
    oA1[kh] = ra * 128 + 16 * ((4 + 2 * kh + (lane >> 5)) ^ ((ra >> 1) & 7));
    oB0[kh] = rb * 128 + 16 * ((2 * kh + (lane >> 5)) ^ ((rb >> 1) & 7));
    oB1[kh] = rb * 128 + 16 * ((4 + 2 * kh + (lane >> 5)) ^ ((rb >> 1) & 7));
  }
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  struct Frags {
    bf16x8 a[4][2], b[4][2];
  };
  struct Bases {
    uint32_t a[2], b[2];
  } lb;
  auto set_bases = [&](int64_t p) __attribute__((always_inline)) {
    const uint32_t ba = (uint32_t)(uintptr_t)(ldsA + ((p >> 1) % WT_NA) * WL_ATILE);
    const uint32_t bb = (uint32_t)(uintptr_t)(ldsB + ((p >> 1) % WT_NB) * WL_ATILE);
    const uint32_t hm = 0u - (uint32_t)(p & 1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      lb.a[kh] = ba + ((oA1[kh] & hm) | (oA0[kh] & ~hm));
      lb.b[kh] = bb + ((oB1[kh] & hm) | (oB0[kh] & ~hm));
    }
  };
  auto read_a = [](auto Q, Frags& f, const Bases& bs) __attribute__((always_inline)) {
    constexpr int q = decltype(Q)::value;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.a[q & 3][q >> 2]) : "v"(bs.a[q >> 2]), "i"((q & 3) * 4096));
  };
  auto read_b = [](auto Q, Frags& f, const Bases& bs) __attribute__((always_inline)) {
    constexpr int q = decltype(Q)::value;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.b[q & 3][q >> 2]) : "v"(bs.b[q >> 2]), "i"((q & 3) * 4096));
  };
  auto read_all = [&](Frags& f) __attribute__((always_inline)) {
    wl_seq<8>([&](auto Q) __attribute__((always_inline)) { read_b(Q, f, lb); });
    wl_seq<8>([&](auto Q) __attribute__((always_inline)) { read_a(Q, f, lb); });
  };
  auto mfma = [](auto G, const Frags& f, f32x16 (&ac)[4][4]) __attribute__((always_inline)) {
    constexpr int g = decltype(G)::value, kh = g >> 4, mb = (g >> 2) & 3, nb = g & 3;
    ac[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[mb][kh], f.b[nb][kh], ac[mb][nb], 0, 0, 0);
  };

  // steady state: at odd p the 8 pieces of B^T tile (p+3)>>1, at even p those
  // of A tile (p>>1)+2, one per 4 MFMA gaps (w4t's balanced scheme)
  auto full_step = [&](int64_t p, const Frags& X, Frags& Y, auto Q) __attribute__((always_inline)) {
    constexpr int q = decltype(Q)::value;
    if constexpr (q == 0)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    set_bases(p + 1);
    const int64_t tx = q == 0 ? (p + 3) >> 1 : (p >> 1) + 2;
    __builtin_amdgcn_sched_barrier(0);
    wl_seq<32>([&](auto G) __attribute__((always_inline)) {
      constexpr int g = decltype(G)::value, j = g >> 2;
      mfma(G, X, acc);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((g & 3) == 0) {
        read_a(std::integral_constant<int, j>{}, Y, lb);
      } else if constexpr ((g & 3) == 2) {
        read_b(std::integral_constant<int, j>{}, Y, lb);
      } else if constexpr ((g & 3) == 1) {
        if constexpr (q == 0)
          W4P_PIECE_B(j, tx);
        else
          W4P_PIECE_A(j, tx);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto plain_step = [&](int64_t p, const Frags& X, Frags& Y) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (p & 1) {
      const int64_t tb = (p + 3) >> 1;
      if (tb < ntile)
        for (int i = 0; i < 8; ++i) W4P_PIECE_B(i, tb);
    } else {
      const int64_t ta = (p >> 1) + 2;
      if (ta < ntile)
        for (int i = 0; i < 8; ++i) W4P_PIECE_A(i, ta);
    }
    if (p + 1 < nst) {
      set_bases(p + 1);
      read_all(Y);
    }
    wl_seq<32>([&](auto G) __attribute__((always_inline)) { mfma(G, X, acc); });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  for (int64_t ta = 0; ta < WT_NA && ta < ntile; ++ta)
    for (int i = 0; i < 8; ++i) W4P_PIECE_A(i, ta);
  for (int64_t tb = 0; tb < WT_NB && tb < ntile; ++tb)
    for (int i = 0; i < 8; ++i) W4P_PIECE_B(i, tb);
  Frags f0, f1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  set_bases(0);
  read_all(f0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  {
    if (nst > 1) {
      set_bases(1);
      read_all(f1);
    }
    wl_seq<32>([&](auto G) __attribute__((always_inline)) { mfma(G, f0, acc); });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  int64_t p = 1;
  unsigned long long t0 = 0, t1 = 0;
  if constexpr (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (; p + 2 < nst && ((p + 5) >> 1) < ntile; p += 2) {
    if constexpr (SYNC) {
      if ((p & (SI - 1)) == 1 && w == 0) {
        if (lane == 0) {
          int* prog = g_w4p_progress;
          __hip_atomic_store(prog + gt, (int)p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          for (int k = 0; k < 2; ++k) {
            const int64_t pt = k ? partA : partB;
            if (pt < 0) continue;
            for (int it = 0; it < 4000; ++it) {
              const int v = __hip_atomic_load(prog + pt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const int d = (int)p + 1 - v;
              if (v == 0 || d <= SL || d > SW) break;
              __builtin_amdgcn_s_sleep(2);
            }
          }
        }
      }
    }
    full_step(p, f1, f0, std::integral_constant<int, 0>{});
    full_step(p + 1, f0, f1, std::integral_constant<int, 1>{});
  }
  if constexpr (SYNC)
    if (threadIdx.x == 0) __hip_atomic_store(g_w4p_progress + gt, 1 << 30, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (lane == 0) {
      stamp_out[(blockIdx.x * 4 + w) * 2] = t1 - t0;
      stamp_out[(blockIdx.x * 4 + w) * 2 + 1] = (unsigned long long)(p - 1);
    }
  }
  for (; p < nst; ++p) {
    plain_step(p, f1, f0);
    f1 = f0;
  }

  const bool accum = T->accumulate != 0;
  char* C = (char*)(uintptr_t)T->c;
  const int64_t ldc = T->ldc;
  const int64_t gn0 = n0 + wc * 128 + (lane & 31);
  const int64_t gm0 = m0 + wr * 128 + 4 * (lane >> 5);
  wl_seq<16>([&](auto MN) __attribute__((always_inline)) {
    constexpr int mb = decltype(MN)::value >> 2, nb = decltype(MN)::value & 3;
    const int64_t gn = gn0 + nb * 32;
    if (gn < N) {
      wl_seq<16>([&](auto R) __attribute__((always_inline)) {
        constexpr int r = decltype(R)::value;
        const int64_t gm = gm0 + mb * 32 + (r & 3) + 8 * (r >> 2);
        if (gm < M) {
          float v = acc[mb][nb][r];
          if constexpr (OUT_BF16) {
            CUBED_G uint16_t* c = (CUBED_G uint16_t*)(uintptr_t)(C + (gm * ldc + gn) * 2);
            if (accum) v += bf16_to_f32(*c);
            *c = f32_to_bf16(v);
          } else {
            CUBED_G float* c = (CUBED_G float*)(uintptr_t)(C + (gm * ldc + gn) * 4);
            if (accum) v += *c;
            *c = v;
          }
        }
      });
    }
  });
}
#undef W4P_PIECE_A
#undef W4P_PIECE_B
