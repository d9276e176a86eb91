// gemm_f32_8p.h -- f32 chained GEMM on the PACKED operands of gemm_f32_w4p.h
// with TWO waves per SIMD (round 6; included by gemm_chain.hip after
// gemm_f32_w4p.h).  The structure of gemm_bf16_8p.h on the f32 image:
//
// * 8 waves, two groups of 4 (one wave of each group per SIMD), each wave
//   128 x 64 of the 256 x 256 tile on v_mfma_f32_32x32x2_f32 (4 x 2
//   accumulators of 32 x 32); a 16-deep k step = four phases, one 64 x 64
//   quadrant pair (16 MFMAs) each, every phase a READ interval and an MFMA
//   interval between raw s_barriers, group 1 one barrier behind group 0.
// * LDS: a ring of 20 half-step slots of 8 KiB (160 KiB).  Half-step u = 4 t
//   + h of k step t is A rows 128 h .. +127 (h = 0, 1) or B k-rows 8 (h - 2)
//   .. +7 (h = 2, 3) -- 8 KiB of consecutive bytes of the packed blocks -- in
//   slot u mod 20; phase s stages half-step s + 9 (one piece per thread), the
//   wait of phase 4t + 3 (vmcnt(4)) completes step t + 1.
// * Fragments: the f32 w4p kernel's permutations (a lane's 16-B A read holds
//   4 consecutive k of its row; the MFMA of index j of k group g pairs k = 8g
//   + j with 8g + 4 + j), with B read as 8-byte pairs of adjacent columns
//   (accumulator q covers columns 2 (lane & 31) + q of the wave's 64): every
//   accumulator walks the same (g, j) sequence per step as w4p's, so each
//   element is the same f32 fma chain over K -- bit-identical.
// Phase reads per wave and step: A rows 0-63 (4 x b128) + all of B (8 x b64),
// none, A rows 64-127 (4 x b128), none.
#pragma once

constexpr int F8_NSLOT = 20, F8_HALF = 8192, F8_LEAD = 9;
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int VAR = 0>
__global__ __launch_bounds__(512, 1) void k_gemm_f32_8p(const cubed_gemm_chain_t* __restrict__ tasks,
                                                     const char* __restrict__ PA, const char* __restrict__ PB,
                                                     PackPlan pp, GemmGrid gg,
                                                     unsigned long long* __restrict__ stamp_out) {
  __shared__ __attribute__((aligned(1024))) char lds_[F8_NSLOT * F8_HALF];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t0, m0, n0;
  tile_of<HF_BM, HF_BN, 4>(xcd_remap(blockIdx.x, gridDim.x), pp.TM, pp.TN, t0, m0, n0);
  const int64_t M = pp.M, N = pp.N;
  if (t0 != 0 || m0 >= M || n0 >= N) return;
  const int nst = (int)pp.KTL, nph = 4 * nst;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2, wc = w & 3, h = lane >> 5, r32 = lane & 31;
  // staging: this wave's 1 KiB piece of every half-step (8 pieces per 8 KiB)
  const char* const sA = PA + (m0 / 256) * pp.apstride + w * 1024 + lane * 16;
  const char* const sB = PB + (n0 / 256) * pp.pstride + w * 1024 + lane * 16;
  const int64_t aks = pp.akstride;
  CUBED_L char* const dw = lds + w * 1024;
  auto stage = [&](int u) __attribute__((always_inline)) {
    const int kt = u >> 2, hh = u & 3;
    const char* src = hh < 2 ? sA + kt * aks + hh * F8_HALF : sB + (int64_t)kt * WPF_SB + (hh - 2) * F8_HALF;
    glds16(src, dw + (u % F8_NSLOT) * F8_HALF);
  };
  // A fragment (rb, kg): row 32 rb + r32 of the wave's half, 16-B chunk 2 kg + h
  // at its swizzled slot (the pack's s ^ ((r >> 2) & 3)); B pair (kg, j): k-row
  // 4 h + j of half kg, columns 64 wc + 2 r32 .. +1
  int loA[2];
#pragma unroll
  for (int kg = 0; kg < 2; ++kg) loA[kg] = r32 * 64 + 16 * ((2 * kg + h) ^ ((r32 >> 2) & 3));
  const int loB = (4 * h) * 1024 + (wc * 64 + 2 * r32) * 4;

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][q][r] = 0.f;
  f32x4 a[2][2] = {};  // [rb within the pair][kg]: k 8 kg + 4 h + 0..3
  f32x2 b[2][4] = {};  // [kg][j]: columns (2 r32, 2 r32 + 1)

  auto read_a = [&](int t, int rbh) __attribute__((always_inline)) {
    CUBED_L const char* base = lds + ((4 * t + g) % F8_NSLOT) * F8_HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int kg = 0; kg < 2; ++kg) a[i][kg] = *(const CUBED_L f32x4*)(base + loA[kg] + (2 * rbh + i) * 32 * 64);
  };
  f32x4 a2[2][2] = {};  // rows 64-127 (two-phase form only)
  auto read_a2 = [&](int t) __attribute__((always_inline)) {
    CUBED_L const char* base = lds + ((4 * t + g) % F8_NSLOT) * F8_HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int kg = 0; kg < 2; ++kg) a2[i][kg] = *(const CUBED_L f32x4*)(base + loA[kg] + (2 + i) * 32 * 64);
  };
  auto read_b = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int kg = 0; kg < 2; ++kg) {
      CUBED_L const char* base = lds + ((4 * t + 2 + kg) % F8_NSLOT) * F8_HALF + loB;
#pragma unroll
      for (int j = 0; j < 4; ++j) b[kg][j] = *(const CUBED_L f32x2*)(base + j * 1024);
    }
  };
  // accumulators (2 rbh + i, q), the (kg, j) sequence of w4p's step
  auto quad = [&](int rbh, int q) __attribute__((always_inline)) {
#pragma unroll
    for (int kg = 0; kg < 2; ++kg)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[2 * rbh + i][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][kg][j], b[kg][j][q], acc[2 * rbh + i][q], 0, 0, 0);
  };
  auto quad2 = [&](int q) __attribute__((always_inline)) {
#pragma unroll
    for (int kg = 0; kg < 2; ++kg)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[2 + i][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[i][kg][j], b[kg][j][q], acc[2 + i][q], 0, 0, 0);
  };
  auto barrier = []() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma_begin = []() __attribute__((always_inline)) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };

  unsigned long long c0 = 0, c1 = 0;
  if constexpr ((VAR & 2) != 0) {
    // two phases per step (32 MFMAs each: q = 0, then q = 1), two pieces per
    // phase; phase p stages half-steps 2p + 8, 2p + 9
    for (int u = 0; u < 8 && u < nph; ++u) stage(u);
    switch ((nph < 8 ? nph : 8) - 4) {
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
    barrier();
    if (g == 1) barrier();
    if constexpr ((VAR & 1) != 0) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0)::"memory");
    for (int t = 0; t < nst; ++t) {
      const int p = 2 * t;
      read_a(t, 0);
      read_a2(t);
      read_b(t);
      if (2 * p + 8 < nph) stage(2 * p + 8);
      if (2 * p + 9 < nph) stage(2 * p + 9);
      barrier();
      mfma_begin();
      quad(0, 0);
      quad2(0);
      barrier();
      if (t + 2 < nst)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (2 * p + 10 < nph) stage(2 * p + 10);
      if (2 * p + 11 < nph) stage(2 * p + 11);
      barrier();
      mfma_begin();
      quad(0, 1);
      quad2(1);
      barrier();
    }
  } else {
  // prologue: half-steps 0 .. 8 staged, step 0 (halves 0 .. 3) waited
    for (int u = 0; u < F8_LEAD && u < nph; ++u) stage(u);
    switch ((nph < F8_LEAD ? nph : F8_LEAD) - 4) {
      case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
      case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
    barrier();
    if (g == 1) barrier();  // group 1 runs one interval behind group 0
  
    if constexpr ((VAR & 1) != 0) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0)::"memory");
    for (int t = 0; t < nst; ++t) {
      const int s = 4 * t;
      // phase 0: A rows 0-63 + B, accumulators (0-1, 0)
      read_a(t, 0);
      read_b(t);
      if (s + F8_LEAD < nph) stage(s + F8_LEAD);
      barrier();
      mfma_begin();
      quad(0, 0);
      barrier();
      // phase 1: accumulators (0-1, 1)
      if (s + 1 + F8_LEAD < nph) stage(s + 1 + F8_LEAD);
      barrier();
      mfma_begin();
      quad(0, 1);
      barrier();
      // phase 2: A rows 64-127, accumulators (2-3, 1)
      read_a(t, 1);
      if (s + 2 + F8_LEAD < nph) stage(s + 2 + F8_LEAD);
      barrier();
      mfma_begin();
      quad(1, 1);
      barrier();
      // phase 3: step t + 1 complete (every wave before the barrier its first
      // readers pass), accumulators (2-3, 0)
      if (t + 2 < nst)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // phases 4t - 1 .. 4t + 2 may fly
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (s + 3 + F8_LEAD < nph) stage(s + 3 + F8_LEAD);
      barrier();
      mfma_begin();
      quad(1, 0);
      barrier();
    }
  }
  if (g == 0) barrier();  // the same barrier count in both groups
  if constexpr ((VAR & 1) != 0) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1)::"memory");
    if (lane == 0) {
      stamp_out[(blockIdx.x * 8 + w) * 2] = c1 - c0;
      stamp_out[(blockIdx.x * 8 + w) * 2 + 1] = (unsigned long long)nph;
    }
  }

  // epilogue: accumulator (rb, q) register r = row 128 g + 32 rb + (r & 3) +
  // 8 (r >> 2) + 4 h, column 64 wc + 2 r32 + q: one float2 per (rb, r)
  const GridTile gt = grid_tile(tasks, gg, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = gt.T;
  const bool accum = T->accumulate != 0;
  const int64_t gn = n0 + wc * 64 + 2 * r32;
  if (gn < N) {
    const bool hn = gn >= gt.nb;  // cn % 4 == 0: a column pair never straddles chunks
    const cubed_gemm_chain_t* __restrict__ TC0 = hn ? gt.TJ1 : T;
    const cubed_gemm_chain_t* __restrict__ TC1 = TC0 + (gt.TI1 - T);
    const int64_t ln = gn - (hn ? gt.nb : gt.J0 * gg.cn);
    char* C0 = (char*)(uintptr_t)TC0->c;
    char* C1 = (char*)(uintptr_t)TC1->c;
    const int64_t ldc0 = TC0->ldc, ldc1 = TC1->ldc;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + g * 128 + 32 * rb + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gm < M) {
          const bool hm = gm >= gt.mb;
          const int64_t lm = gm - (hm ? gt.mb : gt.I0 * gg.cm);
          CUBED_G f32x2* c = (CUBED_G f32x2*)(uintptr_t)((hm ? C1 : C0) + (lm * (hm ? ldc1 : ldc0) + ln) * 4);
          f32x2 v = {acc[rb][0][r], acc[rb][1][r]};
          if (accum) v += *c;
          *c = v;
        }
      }
  }
}
