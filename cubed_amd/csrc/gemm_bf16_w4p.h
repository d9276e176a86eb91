// gemm_bf16_w4p.h -- the library's bf16 chained GEMM on PACKED operands
// (round 5; included by gemm_chain.hip, launched by cubed_gemm_chain_packed).
//
// The one-wave kernel of gemm_bf16_w4l.h stages A from the chunks as stored:
// every 64-k tile is 256 scattered 128-B row lines, and B is read with
// ds_read_b64_tr_b16.  tools/mfma_gap_probe.hip (profiles/r05_mfma_flow.log)
// holds 2.0 GHz with 16 ds_read_b128 per step against 1.72 GHz for w4l's
// read mix, and w4l's stamps put ~5 cycles per MFMA into fills that miss L2.
// Here both operands are first rewritten, in one HBM pass each, into the LDS
// image itself: per 256-row panel of A (256-column panel of B^T) and 64-deep k
// tile one 32 KiB block, row r at r * 128 and 16-B slot s holding k chunk
// s ^ ((r >> 1) & 7) (the w4l A swizzle), the chain's K segments concatenated,
// every pad (rows past M, columns past N, k past K) zero.  The GEMM then
// stages each piece as 1 KiB of consecutive bytes from one uniform base, reads
// A and B fragments alike with ds_read_b128, and its K loop has no segment or
// edge logic -- which also makes 256 x 256 tiles over the WHOLE output (157^2
// instead of 8^2 x 20^2 padded per chunk on config 5) free: chunk boundaries
// matter only in the epilogue.
//
// Config 5 (tools/gemm_w4i_probe.hip, profiles/r05_gemm_bf16_w4p.log): GEMM
// 1330 TF vs 1214 for w4l on one box, bit-identical; pack A 1.37 ms + B^T
// 1.26 ms (~5 TB/s each, 3.3 GB written per operand).
//
// Same results contract as k_gemm_bf16_w4l: every element one f32 chain over K
// in the same 32x32x16 order (zero pads add exact zeros; the K loop stops at
// ceil(K / 32) steps like w4l's).
#pragma once

// geometry of one packed chain set (host-validated, see cubed_gemm_pack_bytes)
struct PackPlan {
  int64_t ti, tj, cm, cn, M, N, K;
  int64_t TM, TN, KTL;  // 256-row / 256-column panels over M / N, k blocks over K
  int64_t pstride;      // bytes from one panel's first block to the next panel's (B / B^T)
  // the A image: block (mt, kt) at mt * apstride + kt * akstride (one GPU:
  // panel-major, apstride = pstride; the multi-GPU image is k-major so every
  // k chunk's tile range is one contiguous run, cubed_gemm_dist_*)
  int64_t apstride, akstride;
  int64_t kt0, kt1;     // k blocks [kt0, kt1) the A pack writes
};

// segment containing k (start ks), walking from (s, ks): every task has the
// same k segmentation (cubed_gemm_grid_check), read from task 0's list
__device__ __forceinline__ void seg_at(const cubed_gemm_seg_t* __restrict__ sg, int64_t k, int64_t& s, int64_t& ks) {
  int64_t ke = ks + sg[s].k;
  while (k >= ke) {
    ks = ke;
    ++s;
    ke += sg[s].k;
  }
}

// A -> PA: block (mt, kt) = rows 256 mt .. +255 of the whole A, k 64 kt .. +63
__global__ __launch_bounds__(256) void k_pack_a(const cubed_gemm_chain_t* __restrict__ tasks,
                                                const cubed_gemm_seg_t* __restrict__ segs, PackPlan pp,
                                                char* __restrict__ PA) {
  const int64_t nkt = pp.kt1 - pp.kt0, nblk = pp.TM * nkt;
  const cubed_gemm_seg_t* __restrict__ sg0 = segs + tasks[0].seg0;
  const int sl = threadIdx.x & 7;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t mt = blk / nkt, kt = pp.kt0 + (blk - mt * nkt);
    // the panel's first chunk row (rows of a panel lie in at most two: cm >= 256)
    const int64_t I0 = (mt * 256) / pp.cm, mb = (I0 + 1) * pp.cm;
    int64_t s0 = 0, ks0 = 0;
    if (kt * 64 < pp.K) seg_at(sg0, kt * 64, s0, ks0);
    char* dst = PA + mt * pp.apstride + kt * pp.akstride;
#pragma unroll 2
    for (int j = 0; j < 8; ++j) {
      const int r = (threadIdx.x >> 3) + 32 * j, c = sl ^ ((r >> 1) & 7);
      const int64_t gm = mt * 256 + r, k = kt * 64 + c * 8;
      uint4 v = {0, 0, 0, 0};
      if (gm < pp.M && k < pp.K) {
        int64_t s = s0, ks = ks0;
        seg_at(sg0, k, s, ks);
        const bool hi = gm >= mb;
        const int64_t I = hi ? I0 + 1 : I0, lm = gm - I * pp.cm;
        const cubed_gemm_seg_t& S = segs[tasks[I * pp.tj].seg0 + s];
        v = *(const uint4*)((const char*)(uintptr_t)S.a + (lm * S.lda + (k - ks)) * 2);
      }
      *(uint4*)(dst + r * 128 + sl * 16) = v;
    }
  }
}

// B -> PB as B^T: block (nt, kt) = columns 256 nt .. +255 as rows.  Thread t
// takes k chunk c = t & 7 and columns 8 (t >> 3) .. +7: eight 16-B row reads,
// an 8 x 8 transpose in registers, eight 16-B writes (8 consecutive threads
// fill one 128-B row of the block).  cn % 8 == 0: a column group never
// straddles chunk columns; k_s % 8 == 0: a k chunk never straddles segments.
__global__ __launch_bounds__(256) void k_pack_bt(const cubed_gemm_chain_t* __restrict__ tasks,
                                                 const cubed_gemm_seg_t* __restrict__ segs, PackPlan pp,
                                                 char* __restrict__ PB) {
  const int64_t nblk = pp.TN * pp.KTL;
  const cubed_gemm_seg_t* __restrict__ sg0 = segs + tasks[0].seg0;
  const int c = threadIdx.x & 7, n8 = threadIdx.x >> 3;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t nt = blk / pp.KTL, kt = blk - nt * pp.KTL;
    const int64_t J0 = (nt * 256) / pp.cn, nb = (J0 + 1) * pp.cn;
    const int64_t gn = nt * 256 + n8 * 8, k0 = kt * 64 + c * 8;
    uint4 in[8];
    if (gn < pp.N && k0 < pp.K) {
      int64_t s = 0, ks = 0;
      seg_at(sg0, k0, s, ks);
      const bool hi = gn >= nb;
      const int64_t J = hi ? J0 + 1 : J0, ln = gn - J * pp.cn;
      const cubed_gemm_seg_t& S = segs[tasks[J].seg0 + s];
      const char* src = (const char*)(uintptr_t)S.b + ((k0 - ks) * S.ldb + ln) * 2;
#pragma unroll
      for (int e = 0; e < 8; ++e) in[e] = k0 + e < pp.K ? *(const uint4*)(src + e * S.ldb * 2) : uint4{0, 0, 0, 0};
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) in[e] = uint4{0, 0, 0, 0};
    }
    char* dst = PB + nt * pp.pstride + kt * 32768;
    const uint16_t(*w)[8] = (const uint16_t(*)[8])in;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = n8 * 8 + j, sl = c ^ ((r >> 1) & 7);
      uint16_t o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = w[e][j];
      *(uint4*)(dst + r * 128 + sl * 16) = *(const uint4*)o;
    }
  }
}

constexpr int WP_NA = 3, WP_NB = 2;  // ring depths (tiles of 32 KiB): 160 KiB

// One wave per SIMD, 128 x 128 per wave, 256 x 256 tiles over the whole
// output (tile_of over TM x TN panels).  Step p (32 k) reads half p & 1 of
// A tile p >> 1 (slot % 3) and of B^T tile p >> 1 (slot % 2).  Odd p stages
// the 8 pieces per wave of B^T tile (p + 3) >> 1, even p those of A tile
// (p >> 1) + 2, one piece per four MFMA gaps.  Waits: the fragments of step
// p + 1 were issued by step p - 1 at the latest (B^T) / p - 2 (A), so odd p
// waits vmcnt(8) (only step p - 1's pieces may still fly) and even p
// vmcnt(16).  B^T tile t's pieces go out at step 2t - 3, after every wave's
// reads of tile t - 2 (steps 2t - 4, 2t - 3's barrier); A tile t's at step
// 2t - 4, after tile t - 3's last reads (step 2t - 5).
// STAMP: lane 0 of each wave stores the main loop's cycles (s_memtime) and
// step count to stamp_out[(block * 4 + wave) * 2] (probe builds only).
template <bool OUT_BF16, bool STAMP = false>
__global__ __launch_bounds__(256, 1) void k_gemm_bf16_w4p(const cubed_gemm_chain_t* __restrict__ tasks,
                                                       const char* __restrict__ PA, const char* __restrict__ PB,
                                                       PackPlan pp, GemmGrid gg,
                                                       unsigned long long* __restrict__ stamp_out) {
  __shared__ __attribute__((aligned(1024))) char lds_[(WP_NA + WP_NB) * WL_ATILE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  CUBED_L char* ldsA = lds;
  CUBED_L char* ldsB = lds + WP_NA * WL_ATILE;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, 4>(xcd_remap(blockIdx.x, gridDim.x), pp.TM, pp.TN, t, m0, n0);
  const int64_t M = pp.M, N = pp.N;
  if (t != 0 || m0 >= M || n0 >= N) return;
  const int64_t ntile = pp.KTL, nst = (pp.K + HB_BK - 1) / HB_BK;
  // this tile's two streams of 32 KiB blocks
  const char* sA = PA + (m0 / 256) * pp.apstride;
  const int64_t aks = pp.akstride;
  const char* sB = PB + (n0 / 256) * pp.pstride;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  // piece i of wave w: block rows 64w + 8i .. +7 = bytes (64w + 8i) * 128 +
  // lane * 16 of both the block and the LDS slot.  (Plain expressions, not
  // lambdas: a lambda's captures here ended up in scratch memory.)
  const char* const sAl = sA + (64 * w) * 128 + lane * 16;
  const char* const sBl = sB + (64 * w) * 128 + lane * 16;
  CUBED_L char* const dA = ldsA + (64 * w) * 128;
  CUBED_L char* const dB = ldsB + (64 * w) * 128;
#define W4P_PIECE_A(i, tile) glds16(sAl + (tile) * aks + (i) * 1024, dA + ((tile) % WP_NA) * WL_ATILE + (i) * 1024)
#define W4P_PIECE_B(i, tile) glds16(sBl + (tile) * 32768 + (i) * 1024, dB + ((tile) % WP_NB) * WL_ATILE + (i) * 1024)

  // fragment (mb|nb, kh) of half h: row ra (rb) + 32 mb, k chunk
  // 4h + 2kh + (lane >> 5) at its swizzled slot; h selected by arithmetic (a
  // select between array elements became a scratch address)
  const int ra = wr * 128 + (lane & 31), rb = wc * 128 + (lane & 31);
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
    const uint32_t ba = (uint32_t)(uintptr_t)(ldsA + ((p >> 1) % WP_NA) * WL_ATILE);
    const uint32_t bb = (uint32_t)(uintptr_t)(ldsB + ((p >> 1) % WP_NB) * WL_ATILE);
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

  // steady state (every piece exists): MFMAs on X, in gap g one filler of
  // [A read, staging piece, B read, -] x 8 -- step p+1's fragments into Y
  auto full_step = [&](int64_t p, const Frags& X, Frags& Y, auto Q) __attribute__((always_inline)) {
    constexpr int q = decltype(Q)::value;  // p & 1 ^ 1: 0 = odd p (stage B^T), 1 = even p (stage A)
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
  // prologue / tail steps: whatever exists, issued plainly; waits drain fully
  auto plain_step = [&](int64_t p, const Frags& X, Frags& Y) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (p & 1) {
      const int64_t tb = (p + 3) >> 1;
      if (tb < ntile)
#pragma unroll
        for (int i = 0; i < 8; ++i) W4P_PIECE_B(i, tb);
    } else {
      const int64_t ta = (p >> 1) + 2;
      if (ta < ntile)
#pragma unroll
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

  // prologue: A tiles 0..2, B^T tiles 0..1; step 0 (even) would stage A tile
  // 2 again, so it only reads and multiplies
  for (int64_t ta = 0; ta < WP_NA && ta < ntile; ++ta)
#pragma unroll
    for (int i = 0; i < 8; ++i) W4P_PIECE_A(i, ta);
  for (int64_t tb = 0; tb < WP_NB && tb < ntile; ++tb)
#pragma unroll
    for (int i = 0; i < 8; ++i) W4P_PIECE_B(i, tb);
  Frags f0, f1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  set_bases(0);
  read_all(f0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (nst > 1) {
    set_bases(1);
    read_all(f1);
  }
  wl_seq<32>([&](auto G) __attribute__((always_inline)) { mfma(G, f0, acc); });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  int64_t p = 1;
  unsigned long long t0 = 0, t1 = 0;
  if constexpr (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (; p + 2 < nst && ((p + 5) >> 1) < ntile; p += 2) {
    full_step(p, f1, f0, std::integral_constant<int, 0>{});
    full_step(p + 1, f0, f1, std::integral_constant<int, 1>{});
  }
  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (lane == 0) {
      stamp_out[(blockIdx.x * 4 + w) * 2] = t1 - t0;
      stamp_out[(blockIdx.x * 4 + w) * 2 + 1] = (unsigned long long)(p - 1);
    }
  }
  // tail: f1 holds step p's fragments
  for (; p < nst; ++p) {
    plain_step(p, f1, f0);
    f1 = f0;
  }
#undef W4P_PIECE_A
#undef W4P_PIECE_B

  // epilogue (as w4l's GRID form): each element's chunk and offset inside it
  const GridTile gt = grid_tile(tasks, gg, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = gt.T;
  const bool accum = T->accumulate != 0;
  const int64_t gn0 = n0 + wc * 128 + (lane & 31);
  const int64_t gm0 = m0 + wr * 128 + 4 * (lane >> 5);
  uint64_t cbase[2][2];
  int64_t cld[2][2];
  const cubed_gemm_chain_t* TQ[2][2] = {{T, gt.TJ1}, {gt.TI1, gt.TI1 + (gt.TJ1 - T)}};
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      cbase[a][b] = (uint64_t)(uintptr_t)TQ[a][b]->c;
      cld[a][b] = TQ[a][b]->ldc;
    }
  wl_seq<16>([&](auto MN) __attribute__((always_inline)) {
    constexpr int mb = decltype(MN)::value >> 2, nb = decltype(MN)::value & 3;
    const int64_t gn = gn0 + nb * 32;
    if (gn < N) {
      const bool hn = gn >= gt.nb;
      const int64_t ln = gn - (hn ? gt.nb : gt.J0 * gg.cn);
      const uint64_t c0 = hn ? cbase[0][1] : cbase[0][0];
      const uint64_t c1 = hn ? cbase[1][1] : cbase[1][0];
      const int64_t l0 = hn ? cld[0][1] : cld[0][0];
      const int64_t l1 = hn ? cld[1][1] : cld[1][0];
      if constexpr (OUT_BF16) {
        // lanes 2i, 2i+1 hold columns 2i, 2i+1 of the same rows: per register
        // pair (r0, r0 + 1) one lane exchange gives the even lane row r0 and
        // the odd lane row r0 + 1 as two adjacent columns -- one 4-byte store
        // per two elements (columns never straddle a chunk: cn % 8 == 0)
        const bool odd = lane & 1;
        const int64_t le = ln - (odd ? 1 : 0);
        wl_seq<8>([&](auto P) __attribute__((always_inline)) {
          constexpr int r0 = 2 * decltype(P)::value, r1 = r0 + 1;
          const float x0 = acc[mb][nb][r0], x1 = acc[mb][nb][r1];
          const float y = __shfl_xor(odd ? x0 : x1, 1);
          float lo = odd ? y : x0, hi = odd ? x1 : y;
          const int64_t gm = gm0 + mb * 32 + (r0 & 3) + 8 * (r0 >> 2) + (odd ? 1 : 0);
          if (gm < M) {
            const bool hm = gm >= gt.mb;
            const int64_t lm = gm - (hm ? gt.mb : gt.I0 * gg.cm);
            const uint64_t C = hm ? c1 : c0;
            const int64_t ldc = hm ? l1 : l0;
            CUBED_G uint32_t* c = (CUBED_G uint32_t*)(uintptr_t)(C + (uint64_t)(lm * ldc + le) * 2);
            if (accum) {
              const uint32_t o = *c;
              lo += bf16_to_f32((uint16_t)(o & 0xffffu));
              hi += bf16_to_f32((uint16_t)(o >> 16));
            }
            *c = (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
          }
        });
      } else {
        wl_seq<16>([&](auto R) __attribute__((always_inline)) {
          constexpr int r = decltype(R)::value;
          const int64_t gm = gm0 + mb * 32 + (r & 3) + 8 * (r >> 2);
          if (gm < M) {
            const bool hm = gm >= gt.mb;
            const int64_t lm = gm - (hm ? gt.mb : gt.I0 * gg.cm);
            const uint64_t C = hm ? c1 : c0;
            const int64_t ldc = hm ? l1 : l0;
            float v = acc[mb][nb][r];
            CUBED_G float* c = (CUBED_G float*)(uintptr_t)(C + (uint64_t)(lm * ldc + ln) * 4);
            if (accum) v += *c;
            *c = v;
          }
        });
      }
    }
  });
}
