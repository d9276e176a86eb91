// gemm_f32_w4p.h -- the library's f32 chained GEMM on PACKED operands
// (round 5; included by gemm_chain.hip after gemm_bf16_w4p.h, launched by
// cubed_gemm_chain_packed for f32 inputs).
//
// tools/gemm_f32_w4.h put one wave per SIMD on k_gemm_f32_chain's LDS image
// and measured parity, not more: its main loop ran 70.5-72.7 cycles per
// v_mfma_f32_32x32x2_f32 against 65.5 for the same instruction stream without
// the per-step bookkeeping (segment walk, per-lane piece addresses;
// profiles/r05_mfma_flow.log k_flow32, profiles/r05_gemm_f32_w4.log).  Packing
// removes that bookkeeping as it does for bf16 (gemm_bf16_w4p.h): A is
// rewritten per 256-row panel and 16-deep k step into the 16 KiB A half of the
// LDS stage (row r at r * 64, 16-B slot s holding k chunk s ^ ((r >> 2) & 3)),
// B per 256-column panel and step into the 16 KiB B half (k-row major, 1 KiB
// per k-row: B as stored, cut into panels), the K segments concatenated, pads
// zero.  A wave's 8 pieces per step are then 1 KiB runs at fixed offsets from
// two uniform bases that advance 16 KiB per step.
//
// Same schedule and fragment permutations as tools/gemm_f32_w4.h (itself
// k_gemm_f32_chain's): per output element the same f32 chain over K --
// bit-identical to cubed_gemm_chain / cubed_gemm_chain_grid.
#pragma once

constexpr int WPF_BK = 16, WPF_NS = 4;
constexpr int WPF_SA = HF_BM * WPF_BK * 4, WPF_SB = WPF_BK * HF_BN * 4, WPF_STAGE = WPF_SA + WPF_SB;  // 16 + 16 KiB

// A -> PA: block (mt, ks) = rows 256 mt .. +255, k 16 ks .. +15 (16 KiB)
__global__ __launch_bounds__(256) void k_pack_a_f32(const cubed_gemm_chain_t* __restrict__ tasks,
                                                    const cubed_gemm_seg_t* __restrict__ segs, PackPlan pp,
                                                    char* __restrict__ PA) {
  const int64_t nkt = pp.kt1 - pp.kt0, nblk = pp.TM * nkt;
  const cubed_gemm_seg_t* __restrict__ sg0 = segs + tasks[0].seg0;
  const int sl = threadIdx.x & 3;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t mt = blk / nkt, kt = pp.kt0 + (blk - mt * nkt);
    const int64_t I0 = (mt * 256) / pp.cm, mb = (I0 + 1) * pp.cm;
    int64_t s0 = 0, ks0 = 0;
    if (kt * 16 < pp.K) seg_at(sg0, kt * 16, s0, ks0);
    char* dst = PA + mt * pp.apstride + kt * pp.akstride;
#pragma unroll 2
    for (int j = 0; j < 4; ++j) {
      const int r = (threadIdx.x >> 2) + 64 * j, c = sl ^ ((r >> 2) & 3);
      const int64_t gm = mt * 256 + r, k = kt * 16 + c * 4;
      uint4 v = {0, 0, 0, 0};
      if (gm < pp.M && k < pp.K) {
        int64_t s = s0, ks = ks0;
        seg_at(sg0, k, s, ks);
        const bool hi = gm >= mb;
        const int64_t I = hi ? I0 + 1 : I0, lm = gm - I * pp.cm;
        const cubed_gemm_seg_t& S = segs[tasks[I * pp.tj].seg0 + s];
        v = *(const uint4*)((const char*)(uintptr_t)S.a + (lm * S.lda + (k - ks)) * 4);
      }
      *(uint4*)(dst + r * 64 + sl * 16) = v;
    }
  }
}

// B -> PB: block (nt, ks) = k-rows 16 ks .. +15 of columns 256 nt .. +255
// (16 KiB, 1 KiB per k-row); cn % 4 == 0: a 16-B column group never
// straddles chunk columns
__global__ __launch_bounds__(256) void k_pack_b_f32(const cubed_gemm_chain_t* __restrict__ tasks,
                                                    const cubed_gemm_seg_t* __restrict__ segs, PackPlan pp,
                                                    char* __restrict__ PB) {
  const int64_t nblk = pp.TN * pp.KTL;
  const cubed_gemm_seg_t* __restrict__ sg0 = segs + tasks[0].seg0;
  const int c4 = threadIdx.x & 63;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t nt = blk / pp.KTL, kt = blk - nt * pp.KTL;
    const int64_t J0 = (nt * 256) / pp.cn, nb = (J0 + 1) * pp.cn;
    const int64_t gn = nt * 256 + 4 * c4;
    const bool hi = gn >= nb;
    const int64_t J = hi ? J0 + 1 : J0, ln = gn - J * pp.cn;
    int64_t s = 0, ks = 0;
    if (kt * 16 < pp.K) seg_at(sg0, kt * 16, s, ks);
    char* dst = PB + nt * pp.pstride + kt * WPF_SB;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kr = (threadIdx.x >> 6) + 4 * j;
      const int64_t k = kt * 16 + kr;
      uint4 v = {0, 0, 0, 0};
      if (gn < pp.N && k < pp.K) {
        int64_t s1 = s, ks1 = ks;
        seg_at(sg0, k, s1, ks1);
        const cubed_gemm_seg_t& S = segs[tasks[J].seg0 + s1];
        v = *(const uint4*)((const char*)(uintptr_t)S.b + ((k - ks1) * S.ldb + ln) * 4);
      }
      *(uint4*)(dst + kr * 1024 + c4 * 16) = v;
    }
  }
}

// One wave per SIMD, 128 x 128 per wave, 256 x 256 tiles over the whole
// output.  Ring of 4 stages (A 16 KiB + B 16 KiB): step p computes stage
// p % 4 with fragments read during step p - 1, reads step p + 1's fragments
// and stages step p + 4 into stage p % 4 (free once every wave passed step p's
// barrier).  The wait before step p's barrier leaves steps p + 2 and p + 3's
// 16 pieces in flight.  STAMP: per-wave main-loop cycles (probe builds only).
// LOCK: tile order xcd_lockstep (probe: false = xcd_remap's contiguous ranges).
// SYNC (probe): round_wait / round_done around the K loop, counters at stamp_out.
template <bool STAMP = false, bool LOCK = true, bool SYNC = false>
__global__ __launch_bounds__(256, 1) void k_gemm_f32_w4p(const cubed_gemm_chain_t* __restrict__ tasks,
                                                      const char* __restrict__ PA, const char* __restrict__ PB,
                                                      PackPlan pp, GemmGrid gg,
                                                      unsigned long long* __restrict__ stamp_out) {
  constexpr int G = 2, LPS = 8;
  __shared__ __attribute__((aligned(1024))) char lds_[WPF_NS * WPF_STAGE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t, m0, n0;
  const int64_t lt = LOCK ? xcd_lockstep(blockIdx.x, gridDim.x, 4 * pp.TN, pp.TM / 4) : xcd_remap(blockIdx.x, gridDim.x);
  tile_of<HF_BM, HF_BN, 4>(lt, pp.TM, pp.TN, t, m0, n0);
  const int64_t M = pp.M, N = pp.N;
  unsigned* const rctr = SYNC ? (unsigned*)stamp_out : nullptr;
  if (t != 0 || m0 >= M || n0 >= N) {
    if constexpr (SYNC) round_done(rctr, blockIdx.x);
    return;
  }
  if constexpr (SYNC) round_wait(rctr, blockIdx.x, 32);
  const int64_t nst = pp.KTL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (w >> 1) * 128, wn = (w & 1) * 128;
  // pieces 0..3: A rows 64 w + 16 i .. +15 = block bytes (4 w + i) KiB; 4..7:
  // B k-row 4 w + i - 4 = block bytes (4 w + i - 4) KiB; lane-linear 16 B each
  const char* const sA = PA + (m0 / 256) * pp.apstride + (4 * w) * 1024 + lane * 16;
  const int64_t aks = pp.akstride;
  const char* const sB = PB + (n0 / 256) * pp.pstride + (4 * w) * 1024 + lane * 16;
#define WPF_PIECE(i, p, buf)                                                                    \
  do {                                                                                          \
    if constexpr ((i) < 4)                                                                      \
      glds16(sA + (p) * aks + (i) * 1024, (buf) + (4 * w + (i)) * 1024);                        \
    else                                                                                        \
      glds16(sB + (p) * WPF_SB + ((i) - 4) * 1024, (buf) + WPF_SA + (4 * w + (i) - 4) * 1024); \
  } while (0)

  // fragment read offsets (within a stage): A (rb, g): row wm + 32 rb + r32,
  // logical chunk 2g + h; B (g, j): k-row 8g + 4h + j, columns wn + 4 r32
  const int h = lane >> 5, r32 = lane & 31;
  int offA[4][G];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int g = 0; g < G; ++g)
      offA[rb][g] = (wm + 32 * rb + r32) * (WPF_BK * 4) + 16 * ((2 * g + h) ^ ((r32 >> 2) & 3));
  const int offB = WPF_SA + 4 * h * 1024 + (wn + 4 * r32) * 4;

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][q][r] = 0.f;

  struct Frags {
    f32x4 a[G][4], b[G][4];  // a[g][rb], b[g][j]
  };
  // read e (0..15) of a step: A (rb = e & 3, g = e >> 2) for e < 8, else B (j = e & 3, g = (e >> 2) & 1)
  auto read = [&](int e, Frags& f, const CUBED_L char* buf) __attribute__((always_inline)) {
    if (e < 8)
      f.a[e >> 2][e & 3] = *(const CUBED_L f32x4*)(buf + offA[e & 3][e >> 2]);
    else
      f.b[(e >> 2) & 1][e & 3] = *(const CUBED_L f32x4*)(buf + offB + (8 * ((e >> 2) & 1) + (e & 3)) * 1024);
  };
  auto slot = [&](int64_t p) { return lds + (p % WPF_NS) * WPF_STAGE; };
  // this wave's loads of step q landed (steps q+1, q+2 may be in flight)
  auto wait_step = [&](int64_t q) __attribute__((always_inline)) {
    int64_t younger = nst - 1 - q;
    if (younger > 2) younger = 2;
    if (younger >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPS) : "memory");
    else if (younger == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  // prologue: steps 0..3 staged, step 0's fragments read
  for (int64_t p = 0; p < WPF_NS && p < nst; ++p) {
    CUBED_L char* buf = slot(p);
    wl_seq<LPS>([&](auto I) __attribute__((always_inline)) { WPF_PIECE(decltype(I)::value, p, buf); });
  }
  Frags f0, f1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int e = 0; e < 16; ++e) read(e, f0, slot(0));

  // step p: MFMAs on X, reads of step p + 1 into Y (one per 4 MFMAs in the
  // first half), step p + 4's 8 pieces (one per 8 MFMAs in the second half)
  auto step = [&](int64_t p, const Frags& X, Frags& Y, auto Full) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(Full)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (FULL)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPS) : "memory");
    else if (p + 1 < nst)
      wait_step(p + 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // step p+1 landed everywhere; stage p % 4 read out
    __builtin_amdgcn_sched_barrier(0);
    const CUBED_L char* rbuf = slot(p + 1);
    CUBED_L char* sbuf = slot(p);
    const int64_t ps = p + WPF_NS;
    if constexpr (FULL) {
      wl_seq<128>([&](auto Gi) __attribute__((always_inline)) {
        constexpr int gi = decltype(Gi)::value;
        constexpr int g = gi >> 6, j = (gi >> 4) & 3, rb = (gi >> 2) & 3, q = gi & 3;
        acc[rb][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(X.a[g][rb][j], X.b[g][j][q], acc[rb][q], 0, 0, 0);
        if constexpr (gi < 64 && (gi & 3) == 0) {
          __builtin_amdgcn_sched_barrier(0);
          read(gi >> 2, Y, rbuf);
          __builtin_amdgcn_sched_barrier(0);
        } else if constexpr (gi >= 64 && (gi & 7) == 4) {
          __builtin_amdgcn_sched_barrier(0);
          WPF_PIECE((gi - 64) >> 3, ps, sbuf);
          __builtin_amdgcn_sched_barrier(0);
        }
      });
    } else {
      wl_seq<128>([&](auto Gi) __attribute__((always_inline)) {
        constexpr int gi = decltype(Gi)::value;
        constexpr int g = gi >> 6, j = (gi >> 4) & 3, rb = (gi >> 2) & 3, q = gi & 3;
        acc[rb][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(X.a[g][rb][j], X.b[g][j][q], acc[rb][q], 0, 0, 0);
      });
      if (ps < nst) wl_seq<LPS>([&](auto I) __attribute__((always_inline)) { WPF_PIECE(decltype(I)::value, ps, sbuf); });
      if (p + 1 < nst) {
#pragma unroll
        for (int e = 0; e < 16; ++e) read(e, Y, rbuf);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  using Full = std::integral_constant<bool, true>;
  using Tail = std::integral_constant<bool, false>;
  int64_t p = 0;
  unsigned long long t0 = 0, t1 = 0;
  if constexpr (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (; p + 1 + WPF_NS < nst; p += 2) {
    step(p, f0, f1, Full{});
    step(p + 1, f1, f0, Full{});
  }
  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (lane == 0) {
      stamp_out[(blockIdx.x * 4 + w) * 2] = t1 - t0;
      stamp_out[(blockIdx.x * 4 + w) * 2 + 1] = (unsigned long long)p;
    }
  }
  // tail (at most 5 steps, staging the last ones): step p's fragments are in f0
  for (; p < nst; ++p) {
    step(p, f0, f1, Tail{});
    f0 = f1;
  }
#undef WPF_PIECE
  if constexpr (SYNC) round_done(rctr, blockIdx.x);

  // epilogue: accumulator (rb, q) register r = row wm + 32 rb + (r&3) +
  // 8 (r>>2) + 4h, column wn + 4 r32 + q: one float4 per (rb, r)
  const GridTile gt = grid_tile(tasks, gg, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = gt.T;
  const bool accum = T->accumulate != 0;
  const int64_t gn = n0 + wn + 4 * r32;
  if (gn < N) {
    const bool hn = gn >= gt.nb;
    const cubed_gemm_chain_t* __restrict__ TC0 = hn ? gt.TJ1 : T;
    const cubed_gemm_chain_t* __restrict__ TC1 = TC0 + (gt.TI1 - T);
    const int64_t ln = gn - (hn ? gt.nb : gt.J0 * gg.cn);
    char* C0 = (char*)(uintptr_t)TC0->c;
    char* C1 = (char*)(uintptr_t)TC1->c;
    const int64_t ldc0 = TC0->ldc, ldc1 = TC1->ldc;
    wl_seq<64>([&](auto RR) __attribute__((always_inline)) {
      constexpr int rb = decltype(RR)::value >> 4, r = decltype(RR)::value & 15;
      const int64_t gm = m0 + wm + 32 * rb + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (gm < M) {
        const bool hm = gm >= gt.mb;
        const int64_t lm = gm - (hm ? gt.mb : gt.I0 * gg.cm);
        CUBED_G f32x4* c = (CUBED_G f32x4*)(uintptr_t)((hm ? C1 : C0) + (lm * (hm ? ldc1 : ldc0) + ln) * 4);
        f32x4 v = {acc[rb][0][r], acc[rb][1][r], acc[rb][2][r], acc[rb][3][r]};
        if (accum) v += *c;
        *c = v;
      }
    });
  }
}
