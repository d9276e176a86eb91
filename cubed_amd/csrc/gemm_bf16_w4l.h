// gemm_bf16_w4l.h -- the library's bf16 chained GEMM (round 5; included by
// gemm_chain.hip): one wave per SIMD, 128 x 128 per wave on
// v_mfma_f32_32x32x16_bf16, the K step hand-scheduled one filler per MFMA gap
// (tools/gemm_bf16_w4i.h, tools/mfma_gap_probe.hip), A staged in FULL
// 128-byte lines.  Config 5 (40000^2 bf16, 64 chunk chains x 8 segments):
// 1256-1258 TF vs 1108-1111 for the round-2..4 ping-pong kernel on the same
// box, bit-identical results (profiles/r05_gemm_bf16_w4l.log).
//
// tools/gemm_w4i_probe.hip ablations (profiles/r05_gemm_bf16_w4i_ab.log):
// the one-wave kernel with A staged 32 k deep runs 61-63 cycles per MFMA; holding A's staging
// addresses still (B real) gives 42, holding B's (A real) 61 -- A's staging
// is the cost.  A was staged 32 k at a time: every row a 64-B HALF line,
// each global_load_lds piece 16 rows x 64 B (cdna_hip_programming.md:
// fragment-shaped staging of the re-read operand costs TA time at equal
// L2 traffic).  Here A is staged 64 k at a time, [256 rows][128 B] per
// tile, each piece 8 rows x one full 128-B line, with the row swizzle chunk
// slot s of row r = k chunk s ^ ((r >> 1) & 7) on the source addresses (the
// LDS side of global_load_lds is lane-linear), which also keeps the 32x32x16
// fragment reads (16 lanes = 16 consecutive rows, one chunk) conflict-free.
//
// Rings: A 3 tiles of 64 k (96 KiB), B 4 steps of 32 k (64 KiB) = 160 KiB.
// Step p (32 k) reads tile p >> 1, half p & 1.  Staged at step p: B for step
// p + 4 (slot p % 4, 4 pieces per wave) and part (p + 1) & 1 of A tile
// (p + 5) >> 1 (slot t % 3, 4 of the tile's 8 pieces per wave).  Step p+1's
// pieces were all issued by step p - 3, so the wait is vmcnt(16) (steps p-2
// and p-1 in flight).  Tile t's first pieces go out at step 2t - 5, after
// every wave's reads of tile t - 3 (steps 2t - 7 and 2t - 6) and the barrier
// that opens step 2t - 5.
#pragma once
#include <utility>

constexpr int WL_NA = 3, WL_NB = 4;
constexpr int WL_ATILE = HB_BM * 128;        // 32 KiB: 256 rows x 64 k
constexpr int WL_BSTEP = HB_BK * HB_BN * 2;  // 16 KiB: 32 k-rows x 256 n
constexpr int WL_LDS = WL_NA * WL_ATILE + WL_NB * WL_BSTEP;  // 160 KiB

template <typename F, int... I>
__device__ __forceinline__ void wl_seq_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void wl_seq(F&& f) {
  wl_seq_(f, std::make_integer_sequence<int, N>{});
}

// STAMP: lane 0 of each wave stores the main loop's cycles (s_memtime) and
// step count to stamp_out[(block * 4 + wave) * 2]
// Requires every segment's k >= 64 (a 64-k A tile spans at most two
// segments; cubed_gemm_chain checks) besides the MFMA path's rules.
// ABL (tools/gemm_w4i_probe.hip ablations only, 0 in the library; results
// wrong when nonzero): 1 no K-loop barrier, 2 no vmcnt wait in the K loop, 4 no fragment reads, 16 A
// sources never advance, 32 B sources never advance.  STAMP: probe builds
// store per-wave main-loop cycles to stamp_out (nullptr in the library).
// GRID (cubed_gemm_chain_grid): 256 x 256 tiles over the WHOLE output of a
// regular chunk grid, as k_gemm_bf16_chain<.., GRID>: a lane's A row / B
// column / C element lies in chunk row I0 or I0+1 / column J0 or J0+1
// (selected per lane where the sources are computed and in the epilogue),
// so 5000-wide chunks are not each padded to 5120 (4.9 % of the MFMAs).
template <bool OUT_BF16, int GM = 4, bool STAMP = false, int ABL = 0, bool GRID = false>
__global__ __launch_bounds__(256, 1) void k_gemm_bf16_w4l(const cubed_gemm_chain_t* __restrict__ tasks,
                                                       const cubed_gemm_seg_t* __restrict__ segs,
                                                       int64_t tiles_m, int64_t tiles_n,
                                                       const char* __restrict__ zero, GemmGrid gg,
                                                       unsigned long long* __restrict__ stamp_out) {
  __shared__ __attribute__((aligned(1024))) char lds_[WL_LDS];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  CUBED_L char* ldsA = lds;
  CUBED_L char* ldsB = lds + WL_NA * WL_ATILE;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  GridTile gt{0, 0, 0, 0, tasks + t, tasks + t, tasks + t};
  if constexpr (GRID) gt = grid_tile(tasks, gg, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = gt.T;
  const int64_t M = GRID ? gg.M : T->m, N = GRID ? gg.N : T->n;
  const int32_t KT = (int32_t)T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;
  // GRID: segment s of chunk row I0+1 / column J0+1 is s + dsI / s + dsJ
  const int64_t dsI = gt.TI1->seg0 - T->seg0, dsJ = gt.TJ1->seg0 - T->seg0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;

  // ---- A staging geometry: piece i (0..7) of wave w = tile rows 64w + 8i +
  // (lane >> 3); lane fetches k chunk cA(row) = (lane & 7) ^ ((row >> 1) & 7)
  // = (lane & 7) ^ ((4 (i & 1) + (lane >> 4)) & 7).  Computed where needed
  // (segment edges only): registers go to the fragments
  const int cA0 = (lane & 7) ^ ((lane >> 4) & 7), cA1 = (lane & 7) ^ ((4 + (lane >> 4)) & 7);
  // the row inside its chunk, and (GRID) whether that chunk is row I0 + 1
  auto rowA = [&](int i, bool& hi) __attribute__((always_inline)) {
    int64_t r = m0 + 64 * w + 8 * i + (lane >> 3);
    r = r < M ? r : M - 1;
    hi = GRID && r >= gt.mb;
    return GRID ? r - (hi ? gt.mb : gt.I0 * gg.cm) : r;
  };
  // ---- B staging geometry (as w4i): piece i (0..3) = k-rows 2(4w+i) + (lane>>5)
  auto rowB = [&](int i) __attribute__((always_inline)) { return 2 * (4 * w + i) + (lane >> 5); };
  auto colB = [&](int i, bool& hi) __attribute__((always_inline)) {
    const int r = rowB(i);
    int64_t n = n0 + 8 * ((lane & 31) ^ (4 * (r & 3)));
    n = n + 8 <= N ? n : N - 8;
    hi = GRID && n >= gt.nb;
    return GRID ? n - (hi ? gt.nb : gt.J0 * gg.cn) : n;
  };

  // ---- two independent segment walks: A in 64-k tiles, B in 32-k steps
  // GRID: whether B piece i's columns (this lane) lie in chunk column J0+1,
  // whose row pitch may differ (the last chunk column is narrower)
  bool hB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) colB(i, hB[i]);
  // (hi: GRID only, the same segment of chunk row I0+1 for A / column J0+1 for B)
  struct Walk {
    int64_t s;
    int32_t ks, ke;
    Seg cur, hi;
    bool inc_ok;
  };
  Walk wa{seg0, 0, (int32_t)segs[seg0].k, load_seg(segs, seg0), load_seg(segs, seg0 + dsI), false};
  Walk wb{seg0, 0, (int32_t)segs[seg0].k, load_seg(segs, seg0), load_seg(segs, seg0 + dsJ), false};
  auto advance = [&](Walk& W, int32_t k0, int32_t len, int64_t dh) __attribute__((always_inline)) {
    if (k0 + len >= W.ke && W.s + 1 < segN) {
      W.ks = W.ke;
      ++W.s;
      W.cur = load_seg(segs, W.s);
      if constexpr (GRID) W.hi = load_seg(segs, W.s + dh);
      W.ke = W.ks + (int32_t)segs[W.s].k;
      W.inc_ok = false;
    }
  };
  const uint64_t z = (uint64_t)(uintptr_t)zero;
  // A tile starting at k0: the 8 sources (per-lane selects where the tile
  // crosses a segment edge or the chain's end)
  uint64_t stA[8], stB[4];
  auto stageA_full = [&](int32_t k0) __attribute__((always_inline)) {
    wa.inc_ok = k0 + 64 <= wa.ke;
    const int64_t dk = (int64_t)(k0 - wa.ks) * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // (fields selected one by one: a per-lane select of a struct reference
      // puts the walks in scratch memory)
      bool hi;
      const int64_t r = rowA(i, hi);
      const uint64_t base = hi ? (uint64_t)(uintptr_t)wa.hi.a : (uint64_t)(uintptr_t)wa.cur.a;
      const int64_t ld = hi ? wa.hi.lda2 : wa.cur.lda2;
      stA[i] = base + (uint64_t)(dk + r * ld + ((i & 1) ? cA1 : cA0) * 16);
    }
    if (k0 + 64 > wa.ke) {
      const bool has_next = wa.s + 1 < segN;
      const int64_t sn = has_next ? wa.s + 1 : wa.s;
      const Seg nxt = load_seg(segs, sn);
      const Seg nxtI = GRID ? load_seg(segs, sn + dsI) : nxt;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        bool hi;
        const int64_t r = rowA(i, hi);
        const uint64_t nbase = hi ? (uint64_t)(uintptr_t)nxtI.a : (uint64_t)(uintptr_t)nxt.a;
        const int64_t nld = hi ? nxtI.lda2 : nxt.lda2;
        const int32_t ka = k0 + 8 * ((i & 1) ? cA1 : cA0);
        const uint64_t na = nbase + (uint64_t)(r * nld + (int64_t)(ka - wa.ke) * 2);
        const uint64_t alt = (has_next && ka < KT) ? na : z;
        stA[i] = ka < wa.ke ? stA[i] : alt;
      }
    }
  };
  auto stageB_full = [&](int32_t k0) __attribute__((always_inline)) {
    wb.inc_ok = k0 + HB_BK <= wb.ke;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool hi;
      const int64_t c = colB(i, hi);
      const uint64_t base = hi ? (uint64_t)(uintptr_t)wb.hi.b : (uint64_t)(uintptr_t)wb.cur.b;
      const int64_t ld = hi ? wb.hi.ldb2 : wb.cur.ldb2;
      stB[i] = base + (uint64_t)((int64_t)(k0 - wb.ks + rowB(i)) * ld + c * 2);
    }
    if (k0 + HB_BK > wb.ke) {
      const bool has_next = wb.s + 1 < segN;
      const int64_t sn = has_next ? wb.s + 1 : wb.s;
      const Seg nxt = load_seg(segs, sn);
      const Seg nxtJ = GRID ? load_seg(segs, sn + dsJ) : nxt;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bool hi;
        const int64_t c = colB(i, hi);
        const uint64_t nbase = hi ? (uint64_t)(uintptr_t)nxtJ.b : (uint64_t)(uintptr_t)nxt.b;
        const int64_t nld = hi ? nxtJ.ldb2 : nxt.ldb2;
        const int32_t kb = k0 + rowB(i);
        const uint64_t nbp = nbase + (uint64_t)((int64_t)(kb - wb.ke) * nld + c * 2);
        const uint64_t alt = (has_next && kb < KT) ? nbp : z;
        stB[i] = kb < wb.ke ? stB[i] : alt;
      }
    }
  };
  auto pieceA = [&](int i, int tile) __attribute__((always_inline)) {
    glds16((const char*)(uintptr_t)stA[i], ldsA + (tile % WL_NA) * WL_ATILE + (64 * w + 8 * i) * 128);
  };
  auto pieceB = [&](int i, int64_t step) __attribute__((always_inline)) {
    glds16((const char*)(uintptr_t)stB[i], ldsB + (step % WL_NB) * WL_BSTEP + (4 * w + i) * 1024);
  };

  // ---- fragment read offsets
  // A (mb, kh) of step p (half h = p & 1): row ra + 32 mb of the tile, k chunk
  // c = 4h + 2kh + (lane >> 5), at slot (c ^ ((ra >> 1) & 7)) -- mb: +4096 B
  const int ra = wr * 128 + (lane & 31);
  const int fA = (ra >> 1) & 7;
  int offA[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) offA[h][kh] = ra * 128 + 16 * ((4 * h + 2 * kh + (lane >> 5)) ^ fA);
  const int bq = lane >> 4;
  const int krow = (bq >> 1) * 8 + ((lane & 15) >> 2);
  int offB[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    offB[nb] = krow * 512 + 16 * ((wc * 16 + nb * 4 + (bq & 1) * 2 + ((lane & 3) >> 1)) ^ (4 * (krow & 3))) +
               8 * (lane & 1);

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  struct Frags {
    bf16x8 a[4][2];
    s16x4 bl[4][2], bh[4][2];
  };
  struct Bases {
    uint32_t a[2], b[4];
  } lb;
  // bases of step p's fragments: A tile p >> 1, half p & 1; B step slot p % 4
  auto set_bases = [&](int64_t p) __attribute__((always_inline)) {
    const uint32_t ba = (uint32_t)(uintptr_t)(ldsA + ((p >> 1) % WL_NA) * WL_ATILE);
    const uint32_t bb = (uint32_t)(uintptr_t)(ldsB + (p % WL_NB) * WL_BSTEP);
    const int h = (int)(p & 1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) lb.a[kh] = ba + (h ? offA[1][kh] : offA[0][kh]);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) lb.b[nb] = bb + offB[nb];
  };
  auto read_a = [](auto Q, Frags& f, const Bases& bs) __attribute__((always_inline)) {
    constexpr int q = decltype(Q)::value;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.a[q & 3][q >> 2]) : "v"(bs.a[q >> 2]), "i"((q & 3) * 4096));
  };
  auto read_b = [](auto J, Frags& f, const Bases& bs) __attribute__((always_inline)) {
    constexpr int j = decltype(J)::value, nb = (j >> 1) & 3, kh = j >> 3;
    const uint32_t vb = bs.b[nb];
    if constexpr (j & 1)
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(f.bh[nb][kh]) : "v"(vb), "i"(kh * 8192 + 2048));
    else
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(f.bl[nb][kh]) : "v"(vb), "i"(kh * 8192));
  };
  auto read_all = [&](Frags& f) __attribute__((always_inline)) {
    wl_seq<16>([&](auto J) __attribute__((always_inline)) { read_b(J, f, lb); });
    wl_seq<8>([&](auto Q) __attribute__((always_inline)) { read_a(Q, f, lb); });
  };
  auto mfma = [](auto G, const Frags& f, f32x16 (&ac)[4][4]) __attribute__((always_inline)) {
    constexpr int g = decltype(G)::value, kh = g >> 4, mb = (g >> 2) & 3, nb = g & 3;
    const bf16x8 b = __builtin_bit_cast(bf16x8, __builtin_shufflevector(f.bl[nb][kh], f.bh[nb][kh], 0, 1, 2, 3,
                                                                        4, 5, 6, 7));
    ac[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[mb][kh], b, ac[mb][nb], 0, 0, 0);
  };

  const int64_t nst = (KT + HB_BK - 1) / HB_BK;
  const int64_t ntile = (KT + 63) / 64;
  // what step p stages: A part (p + 1) & 1 of tile (p + 5) >> 1 (if it exists),
  // B for step p + 4 (if it exists).  The source updates: a tile's sources are
  // set up when its part 0 goes out (full recompute at segment edges, else +128 B)
  auto prep_stage = [&](int64_t p) __attribute__((always_inline)) {
    const int64_t ta = (p + 5) >> 1;
    if (((p + 1) & 1) == 0 && ta < ntile) {
      const int32_t k0 = (int32_t)(ta * 64);
      if (wa.inc_ok && k0 + 64 <= wa.ke) {
        if constexpr (!(ABL & 16)) {
#pragma unroll
          for (int i = 0; i < 8; ++i) stA[i] += 128;
        }
      } else if (!(ABL & 16) || k0 == 0) {
        stageA_full(k0);
      }
      advance(wa, k0, 64, dsI);
    }
    if (p + 4 < nst) {
      const int32_t k0 = (int32_t)((p + 4) * HB_BK);
      if (wb.inc_ok && k0 + HB_BK <= wb.ke) {
        const uint64_t dB = (uint64_t)(HB_BK * wb.cur.ldb2), dBh = (uint64_t)(HB_BK * wb.hi.ldb2);
        if constexpr (!(ABL & 32)) {
#pragma unroll
          for (int i = 0; i < 4; ++i) stB[i] += hB[i] ? dBh : dB;
        }
      } else if (!(ABL & 32) || k0 == 0) {
        stageB_full(k0);
      }
      advance(wb, k0, HB_BK, dsJ);
    }
  };

  // a steady-state step (every piece exists): MFMAs on X; in gap g one
  // filler of [A read, B read, staging piece, B read] x 8 -- step p+1's
  // fragments into Y; pieces 0-3: A part q of tile (p+5)>>1, 4-7: B of step p+4
  auto full_step = [&](int64_t p, const Frags& X, Frags& Y, auto Q) __attribute__((always_inline)) {
    constexpr int q = decltype(Q)::value;  // (p + 1) & 1, static in the unrolled loop
    if constexpr (!(ABL & 2)) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!(ABL & 1)) __builtin_amdgcn_s_barrier();  // every wave: step p+1 landed, step p's slots read
    __builtin_amdgcn_sched_barrier(0);
    set_bases(p + 1);
    const int ta = (int)((p + 5) >> 1);
    // sources: in the steady state each advances by one tile / step inside
    // the MFMA gaps (two adds beside a B read); at a segment edge they are
    // recomputed here first (scalar tests: K positions are 32-bit)
    const int32_t kA = ta * 64, kB = (int32_t)((p + 4) * HB_BK);
    bool incA = false;
    if constexpr (q == 0) {
      incA = wa.inc_ok && kA + 64 <= wa.ke;
      if (!incA && (!(ABL & 16) || kA == 0)) stageA_full(kA);
    }
    const bool incB = wb.inc_ok && kB + HB_BK <= wb.ke;
    if (!incB && (!(ABL & 32) || kB == 0)) stageB_full(kB);
    const uint64_t dB = (uint64_t)(HB_BK * wb.cur.ldb2), dBh = (uint64_t)(HB_BK * wb.hi.ldb2);
    __builtin_amdgcn_sched_barrier(0);
    wl_seq<32>([&](auto G) __attribute__((always_inline)) {
      constexpr int g = decltype(G)::value, r = g & 3, i = g >> 2;
      mfma(G, X, acc);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (r == 0) { if constexpr (!(ABL & 4)) read_a(std::integral_constant<int, i>{}, Y, lb); }
      else if constexpr (r == 1) {
        if constexpr (!(ABL & 4)) read_b(std::integral_constant<int, 2 * i>{}, Y, lb);
        if constexpr (i < 4) {
          if constexpr (q == 0 && !(ABL & 16)) if (incA) { stA[i] += 128; stA[i + 4] += 128; }
        } else {
          if constexpr (!(ABL & 32)) if (incB) stB[i - 4] += hB[i - 4] ? dBh : dB;
        }
      }
      else if constexpr (r == 2) {
        if constexpr (i < 4) pieceA(4 * q + i, ta);
        else pieceB(i - 4, p + 4);
      } else { if constexpr (!(ABL & 4)) read_b(std::integral_constant<int, 2 * i + 1>{}, Y, lb); }
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (q == 0) advance(wa, kA, 64, dsI);
    advance(wb, kB, HB_BK, dsJ);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  // prologue / tail steps: whatever exists, issued plainly; waits drain fully
  auto plain_step = [&](int64_t p, const Frags& X, Frags& Y) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    prep_stage(p);
    const int64_t ta = (p + 5) >> 1;
    // (static piece indices: a runtime index into stA puts it in scratch)
    if (ta < ntile) {
      if ((p + 1) & 1) {
#pragma unroll
        for (int i = 4; i < 8; ++i) pieceA(i, (int)ta);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) pieceA(i, (int)ta);
      }
    }
    if (p + 4 < nst) {
#pragma unroll
      for (int i = 0; i < 4; ++i) pieceB(i, p + 4);
    }
    if (p + 1 < nst) {
      set_bases(p + 1);
      read_all(Y);
    }
    wl_seq<32>([&](auto G) __attribute__((always_inline)) { mfma(G, X, acc); });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- prologue: A tiles 0, 1, 2 (parts as steps -5 .. 0 would have issued
  // them) and B steps 0 .. 3
  for (int64_t ta = 0; ta < WL_NA && ta < ntile; ++ta) {
    const int32_t k0 = (int32_t)(ta * 64);
    if (wa.inc_ok && k0 + 64 <= wa.ke) {
#pragma unroll
      for (int i = 0; i < 8; ++i) stA[i] += 128;
    } else {
      stageA_full(k0);
    }
    advance(wa, k0, 64, dsI);
#pragma unroll
    for (int i = 0; i < 8; ++i) pieceA(i, (int)ta);
  }
  for (int64_t pb = 0; pb < WL_NB && pb < nst; ++pb) {
    const int32_t k0 = (int32_t)(pb * HB_BK);
    if (wb.inc_ok && k0 + HB_BK <= wb.ke) {
      const uint64_t dB = (uint64_t)(HB_BK * wb.cur.ldb2), dBh = (uint64_t)(HB_BK * wb.hi.ldb2);
#pragma unroll
      for (int i = 0; i < 4; ++i) stB[i] += hB[i] ? dBh : dB;
    } else {
      stageB_full(k0);
    }
    advance(wb, k0, HB_BK, dsJ);
#pragma unroll
    for (int i = 0; i < 4; ++i) pieceB(i, pb);
  }
  // tile 2 is fully staged: step 0 stages part 1 of tile (0 + 5) >> 1 = 2
  // again -- skip it by starting the steady state at step 1 (part 0 of tile 3)
  Frags f0, f1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  set_bases(0);
  read_all(f0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // step 0: nothing new to stage for A (tile 2 is in), B step 4
  {
    const int64_t p = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (p + 4 < nst) {
      const int32_t k0 = (int32_t)((p + 4) * HB_BK);
      if (wb.inc_ok && k0 + HB_BK <= wb.ke) {
        const uint64_t dB = (uint64_t)(HB_BK * wb.cur.ldb2), dBh = (uint64_t)(HB_BK * wb.hi.ldb2);
#pragma unroll
        for (int i = 0; i < 4; ++i) stB[i] += hB[i] ? dBh : dB;
      } else {
        stageB_full(k0);
      }
      advance(wb, k0, HB_BK, dsJ);
#pragma unroll
      for (int i = 0; i < 4; ++i) pieceB(i, p + 4);
    }
    if (nst > 1) {
      set_bases(1);
      read_all(f1);
    }
    wl_seq<32>([&](auto G) __attribute__((always_inline)) { mfma(G, f0, acc); });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  // steady state from step 1: odd p stages part 0 (q = (p+1)&1 = 0), even p part 1
  int64_t p = 1;
  unsigned long long t0 = 0, t1 = 0;
  if constexpr (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (; p + 2 < nst && ((p + 6) >> 1) < ntile && p + 5 < nst; p += 2) {
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
  // tail: f1 holds step p's fragments (p odd here)
  for (; p < nst; ++p) {
    plain_step(p, f1, f0);
    f1 = f0;
  }

  // ---- epilogue: 32x32 C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  // (GRID: each element's chunk and its offset inside it)
  const bool accum = T->accumulate != 0;
  const int64_t gn0 = n0 + wc * 128 + (lane & 31);
  const int64_t gm0 = m0 + wr * 128 + 4 * (lane >> 5);
  // (static indices throughout: an accumulator indexed at run time would put
  // all of acc in scratch memory, main loop included).  GRID: the four
  // chunks' (C, ldc) are read once; per element only two selects
  uint64_t cbase[2][2];
  int64_t cld[2][2];
  const cubed_gemm_chain_t* TQ[2][2] = {{T, gt.TJ1}, {gt.TI1, gt.TI1 + (gt.TJ1 - T)}};
#pragma unroll
  for (int a = 0; a < (GRID ? 2 : 1); ++a)
#pragma unroll
    for (int b = 0; b < (GRID ? 2 : 1); ++b) {
      cbase[a][b] = (uint64_t)(uintptr_t)TQ[a][b]->c;
      cld[a][b] = TQ[a][b]->ldc;
    }
  wl_seq<16>([&](auto MN) __attribute__((always_inline)) {
    constexpr int mb = decltype(MN)::value >> 2, nb = decltype(MN)::value & 3;
    const int64_t gn = gn0 + nb * 32;
    if (gn < N) {
      const bool hn = GRID && gn >= gt.nb;
      const int64_t ln = GRID ? gn - (hn ? gt.nb : gt.J0 * gg.cn) : gn;
      const uint64_t c0 = GRID && hn ? cbase[0][1] : cbase[0][0];
      const uint64_t c1 = GRID && hn ? cbase[1][1] : cbase[1][0];
      const int64_t l0 = GRID && hn ? cld[0][1] : cld[0][0];
      const int64_t l1 = GRID && hn ? cld[1][1] : cld[1][0];
      wl_seq<16>([&](auto R) __attribute__((always_inline)) {
        constexpr int r = decltype(R)::value;
        const int64_t gm = gm0 + mb * 32 + (r & 3) + 8 * (r >> 2);
        if (gm < M) {
          const bool hm = GRID && gm >= gt.mb;
          const int64_t lm = GRID ? gm - (hm ? gt.mb : gt.I0 * gg.cm) : gm;
          const uint64_t C = hm ? c1 : c0;
          const int64_t ldc = hm ? l1 : l0;
          float v = acc[mb][nb][r];
          if constexpr (OUT_BF16) {
            CUBED_G uint16_t* c = (CUBED_G uint16_t*)(uintptr_t)(C + (uint64_t)(lm * ldc + ln) * 2);
            if (accum) v += bf16_to_f32(*c);
            *c = f32_to_bf16(v);
          } else {
            CUBED_G float* c = (CUBED_G float*)(uintptr_t)(C + (uint64_t)(lm * ldc + ln) * 4);
            if (accum) v += *c;
            *c = v;
          }
        }
      });
    }
  });
}
