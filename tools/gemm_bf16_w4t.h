// gemm_bf16_w4t.h -- development probe (not part of the library; included by
// tools/gemm_w4i_probe.hip): the bf16 chained GEMM with B supplied TRANSPOSED.
// Measured SLOWER than the library's w4l (profiles/r05_gemm_bf16_w4t.log):
// 1034-1126 TF vs 1256, bit-identical -- staging B^T's 256 scattered 128-B
// row lines per tile costs more (~8 cycles per MFMA per operand against
// L2-resident ablations) than the transposed reads it removes.  The w4l schedule
// (one wave per SIMD, 128 x 128 per wave on v_mfma_f32_32x32x16_bf16, one
// filler per MFMA gap) with B staged exactly like A: the segments' b point at
// B^T chunks ([n][k], k contiguous, row pitch ldb elements), so B tiles are
// [256 n-rows][64 k] in full 128-B lines and B fragments are ONE
// ds_read_b128 each instead of two ds_read_b64_tr_b16.
//
// Why: with the real data flow (tools/mfma_gap_probe.hip k_flow,
// profiles/r05_mfma_flow.log) the fragment reads hide in the MFMA gaps but
// cost clock: the w4l step's 8 b128 + 16 tr_b16 reads hold 1.72 GHz, 8 + 8
// b128 reads 2.0 GHz -- the synthetic step runs 1.52 vs 1.82 PF.
//
// Rings (160 KiB): A 3 tiles of 64 k (as w4l), B^T 2 tiles of 64 k.  Step p
// (32 k) computes tile p >> 1, half p & 1, and reads step p + 1's fragments.
// Staged at step p, 8 pieces per wave, one per 4 MFMA gaps: at odd p all of
// B^T tile (p + 3) >> 1, at even p all of A tile (p >> 1) + 2.  Tile u's
// fragments are first read at step 2u - 1; its B^T went out at step 2u - 3
// and its A at step 2u - 4, so an odd step waits vmcnt(8) (only step p - 1's
// pieces may still be in flight), an even step needs nothing new
// (vmcnt(16)).  Slots: B^T tile u + 2 and A tile u + 3 overwrite tile u,
// whose last reads are in step 2u.
// Bit-identical to w4l / the ping-pong kernel: the same MFMA sequence over the
// same k order (a B^T fragment holds the bytes the two transposed reads
// assemble).  Requires every segment's k >= 64, like w4l.
#pragma once

constexpr int WT_NA = 3, WT_NB = 2;
constexpr int WT_LDS = (WT_NA + WT_NB) * WL_ATILE;  // 160 KiB

// ABL (tools/gemm_w4i_probe.hip ablations only, 0 in the library; results
// wrong when nonzero): 1 no K-loop barrier, 2 no vmcnt wait in the K loop,
// 16 A sources stay at their segment's start, 32 the same for B^T.
template <bool OUT_BF16, int GM = 4, bool STAMP = false, int ABL = 0>
__global__ __launch_bounds__(256, 1) void k_gemm_bf16_w4t(const cubed_gemm_chain_t* __restrict__ tasks,
                                                       const cubed_gemm_seg_t* __restrict__ segs,
                                                       int64_t tiles_m, int64_t tiles_n,
                                                       const char* __restrict__ zero, GemmGrid,
                                                       unsigned long long* __restrict__ stamp_out) {
  __shared__ __attribute__((aligned(1024))) char lds_[WT_LDS];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  CUBED_L char* ldsA = lds;
  CUBED_L char* ldsB = lds + WT_NA * WL_ATILE;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n;
  const int32_t KT = (int32_t)T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;

  // ---- staging geometry (A and B^T alike): piece i (0..7) of wave w = tile
  // row 64w + 8i + (lane >> 3); lane fetches k chunk (lane & 7) ^ ((row >> 1) & 7)
  const int c0 = (lane & 7) ^ ((lane >> 4) & 7), c1 = (lane & 7) ^ ((4 + (lane >> 4)) & 7);
  auto rowA = [&](int i) __attribute__((always_inline)) {
    const int64_t r = m0 + 64 * w + 8 * i + (lane >> 3);
    return r < M ? r : M - 1;
  };
  auto rowB = [&](int i) __attribute__((always_inline)) {
    const int64_t n = n0 + 64 * w + 8 * i + (lane >> 3);
    return n < N ? n : N - 1;
  };

  // per operand: the walk over the chain's K segments, 8 per-lane 32-bit
  // offsets (row * pitch + chunk * 16 inside the current segment's chunk;
  // the host checks every chunk spans < 4 GiB) and a wave-uniform base (the
  // segment's chunk + the tile's k offset).  A tile inside one segment: piece
  // i reads base + off[i] (no per-lane 64-bit state: 64-bit source arrays
  // for both operands spilled to scratch, and a scratch reload waits on
  // every LDS-DMA in flight).  A tile crossing its segment's end (or the
  // chain's): per-lane addresses computed at issue, all 8 pieces at once.
  struct Opnd {
    uint32_t off[8];
    uint64_t base;
    int64_t s;
    int32_t ks, ke, k0;
    Seg cur;
    bool fresh, edge;
  };
  Opnd oa, ob;
  oa.s = seg0;
  oa.ks = 0;
  oa.ke = (int32_t)segs[seg0].k;
  oa.cur = load_seg(segs, seg0);
  oa.fresh = true;
  oa.edge = false;
  oa.k0 = 0;
  oa.base = 0;
  ob = oa;
  const uint64_t z = (uint64_t)(uintptr_t)zero;
  using FA = std::integral_constant<bool, false>;
  using FB = std::integral_constant<bool, true>;
  auto setup = [&](auto IsB, Opnd& O, int32_t k0) __attribute__((always_inline)) {
    constexpr bool B = decltype(IsB)::value;
    if (O.fresh) {
      const int64_t ld = B ? O.cur.ldb2 : O.cur.lda2;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int64_t r = B ? rowB(i) : rowA(i);
        O.off[i] = (uint32_t)(r * ld + ((i & 1) ? c1 : c0) * 16);
      }
      O.fresh = false;
    }
    O.base = (uint64_t)(uintptr_t)(B ? O.cur.b : O.cur.a) + (uint64_t)(k0 - O.ks) * 2;
    O.edge = k0 + 64 > O.ke;
    O.k0 = k0;
  };
  auto advance = [&](Opnd& O) __attribute__((always_inline)) {
    if (O.k0 + 64 >= O.ke && O.s + 1 < segN) {
      O.ks = O.ke;
      ++O.s;
      O.cur = load_seg(segs, O.s);
      O.ke = O.ks + (int32_t)segs[O.s].k;
      O.fresh = true;
    }
  };
  auto dstA = [&](int i, int64_t tile) __attribute__((always_inline)) {
    return ldsA + (tile % WT_NA) * WL_ATILE + (64 * w + 8 * i) * 128;
  };
  auto dstB = [&](int i, int64_t tile) __attribute__((always_inline)) {
    return ldsB + (tile % WT_NB) * WL_ATILE + (64 * w + 8 * i) * 128;
  };
  // piece i of the operand's current tile (inside one segment)
  auto piece = [&](auto IsB, const Opnd& O, int i, int64_t tile) __attribute__((always_inline)) {
    constexpr bool B = decltype(IsB)::value;
    glds16((const char*)(uintptr_t)(O.base + O.off[i]), B ? dstB(i, tile) : dstA(i, tile));
  };
  // all 8 pieces of a tile that crosses its segment's end
  auto edge_pieces = [&](auto IsB, const Opnd& O, int64_t tile) __attribute__((always_inline)) {
    constexpr bool B = decltype(IsB)::value;
    const bool has_next = O.s + 1 < segN;
    const Seg nxt = load_seg(segs, has_next ? O.s + 1 : O.s);
    const uint64_t nbase = (uint64_t)(uintptr_t)(B ? nxt.b : nxt.a);
    const int64_t nld = B ? nxt.ldb2 : nxt.lda2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t r = B ? rowB(i) : rowA(i);
      const int32_t kk = O.k0 + 8 * ((i & 1) ? c1 : c0);
      const uint64_t na = nbase + (uint64_t)(r * nld + (int64_t)(kk - O.ke) * 2);
      const uint64_t a = kk < O.ke ? O.base + O.off[i] : ((has_next && kk < KT) ? na : z);
      glds16((const char*)(uintptr_t)a, B ? dstB(i, tile) : dstA(i, tile));
    }
  };
  // a whole tile, plainly (prologue / tail)
  auto tile_plain = [&](auto IsB, Opnd& O, int64_t tile) __attribute__((always_inline)) {
    setup(IsB, O, (int32_t)(tile * 64));
    if (O.edge) {
      edge_pieces(IsB, O, tile);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) piece(IsB, O, i, tile);
    }
    advance(O);
  };

  // ---- fragment read offsets: A row ra / B^T row rb of the tile, k chunk
  // c = 4h + 2kh + (lane >> 5) at slot c ^ ((row >> 1) & 7); mb / nb: +4096 B
  const int ra = wr * 128 + (lane & 31), rb = wc * 128 + (lane & 31);
  int offA[2][2], offB[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      offA[h][kh] = ra * 128 + 16 * ((4 * h + 2 * kh + (lane >> 5)) ^ ((ra >> 1) & 7));
      offB[h][kh] = rb * 128 + 16 * ((4 * h + 2 * kh + (lane >> 5)) ^ ((rb >> 1) & 7));
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
    const int h = (int)(p & 1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      lb.a[kh] = ba + (h ? offA[1][kh] : offA[0][kh]);
      lb.b[kh] = bb + (h ? offB[1][kh] : offB[0][kh]);
    }
  };
  // read q (0..7): fragment (q & 3, q >> 2) of A / B^T
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

  const int64_t nst = (KT + HB_BK - 1) / HB_BK;
  const int64_t ntile = (KT + 63) / 64;
  // a steady-state pair member: MFMAs on X; the gaps carry the reads of step
  // p+1 (even gaps: A at g % 4 == 0, B^T at g % 4 == 2) and, at gaps
  // g % 4 == 1, the 8 pieces of ONE tile -- B^T tile (p+3)>>1 at odd p, A tile
  // (p>>1)+2 at even p (sources advanced before the gaps): 8 pieces every
  // step, evenly spread (a step carrying 12 -- B^T + half an A tile -- and the
  // next 4 ran 57.6 cycles per MFMA, 12 of them at the barrier)
  auto full_step = [&](int64_t p, const Frags& X, Frags& Y, auto Q) __attribute__((always_inline)) {
    constexpr int q = decltype(Q)::value;  // (p + 1) & 1: 0 = odd p (B^T staged), 1 = even p (A)
    if constexpr (ABL & 2) {
    } else if constexpr (q == 0) {
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!(ABL & 1)) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    set_bases(p + 1);
    const int64_t tx = q == 0 ? (p + 3) >> 1 : (p >> 1) + 2;
    Opnd& O = q == 0 ? ob : oa;
    if constexpr (q == 0)
      setup(FB{}, ob, (int32_t)(tx * 64));
    else
      setup(FA{}, oa, (int32_t)(tx * 64));
    if constexpr (((q == 0) ? (ABL & 32) : (ABL & 16)) != 0)  // ablation: sources at the segment's start
      O.base = (uint64_t)(uintptr_t)(q == 0 ? O.cur.b : O.cur.a);
    const bool edge = O.edge;
    if (edge) {
      if constexpr (q == 0)
        edge_pieces(FB{}, ob, tx);
      else
        edge_pieces(FA{}, oa, tx);
    }
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
        if (!edge) {
          if constexpr (q == 0)
            piece(FB{}, ob, j, tx);
          else
            piece(FA{}, oa, j, tx);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    advance(O);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  // prologue / tail steps: whatever exists, issued plainly; waits drain fully
  auto plain_step = [&](int64_t p, const Frags& X, Frags& Y) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (p & 1) {
      const int64_t tb = (p + 3) >> 1;
      if (tb < ntile) tile_plain(FB{}, ob, tb);
    } else {
      const int64_t ta = (p >> 1) + 2;
      if (ta < ntile) tile_plain(FA{}, oa, ta);
    }
    if (p + 1 < nst) {
      set_bases(p + 1);
      read_all(Y);
    }
    wl_seq<32>([&](auto G) __attribute__((always_inline)) { mfma(G, X, acc); });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- prologue: A tiles 0, 1, 2 and B^T tiles 0, 1
  for (int64_t ta = 0; ta < WT_NA && ta < ntile; ++ta) tile_plain(FA{}, oa, ta);
  for (int64_t tb = 0; tb < WT_NB && tb < ntile; ++tb) tile_plain(FB{}, ob, tb);
  Frags f0, f1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  set_bases(0);
  read_all(f0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // step 0: its A tile (2) is in from the prologue
  {
    if (nst > 1) {
      set_bases(1);
      read_all(f1);
    }
    wl_seq<32>([&](auto G) __attribute__((always_inline)) { mfma(G, f0, acc); });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  // steady state from step 1: odd p stages B^T tile (p+3)>>1, even p A tile
  // (p>>1)+2
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
  for (; p < nst; ++p) {
    plain_step(p, f1, f0);
    f1 = f0;
  }

  // ---- epilogue: 32x32 C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
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
