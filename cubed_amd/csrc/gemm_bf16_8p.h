// gemm_bf16_8p.h -- bf16 chained GEMM on the PACKED operands of
// gemm_bf16_w4p.h with TWO waves per SIMD (round 6; included by
// gemm_chain.hip after gemm_bf16_w4p.h).
//
// w4p runs one wave per SIMD: that wave issues its own LDS fragment reads and
// LDS-DMA staging between its MFMAs, 40 cycles per 32-cycle MFMA in its main
// loop.  Here the 256 x 256 tile has 8 waves in two groups of 4 (one wave of
// each group per SIMD), each wave owning 128 x 64 of the tile on
// v_mfma_f32_16x16x32_bf16 (32 accumulators of 16 x 16).  A wave's K tile (64
// k) is four phases, one 64 x 32 quadrant each (16 MFMAs), and every phase is
// a READ interval (this phase's fragments by ds_read_b128, one staging piece
// pair) and an MFMA interval, separated by raw s_barriers; group 1 starts one
// barrier late, so in every interval one wave of each SIMD multiplies while
// the other reads and stages (cdna_hip_programming.md, the 256^2 8-phase
// template's structure).
//
// LDS: a ring of 10 half-tile slots of 16 KiB (160 KiB).  Half-tile u = 4 t + h
// of K tile t is A rows 128 h .. +127 (h = 0, 1) or B^T rows 128 (h - 2) .. +127
// (h = 2, 3) -- 16 KiB of consecutive bytes of the packed block, already the
// LDS image (w4p's slot swizzle is bank-conflict free for the 16-row
// fragment reads too) -- in slot u mod 10.  Phase s stages half-tile s + 7:
// the slot it overwrites held half-tile s - 3, whose last read was issued two
// or more intervals earlier (A half 0: group 0's phase 4t + 2; B halves:
// group 1's phase 4t + 1) and retired by that reader's lgkmcnt(0) before the
// barrier.  The wait of phase 4t + 3 (before its own staging) retires every
// piece but the two newer phases' (vmcnt(4)): K tile t + 1 is complete before
// the barrier its first readers pass.
//
// Reads per wave and K tile: phase 0 A sub-tile 0 (8 x b128) + B sub-tile 0
// (4), phase 1 B sub-tile 1 (4), phase 2 A sub-tile 1 (8), phase 3 none (B
// sub-tile 0 kept in registers).  Per output element: one f32 chain over K in
// k order, 32 k per MFMA -- the same products and order as w4p / w4l
// (bit-identical results are checked by the tests).
#pragma once

constexpr int E8_NSLOT = 10, E8_HALF = 16384, E8_LEAD = 7;
constexpr int E8_ROUNDS = 512;  // VAR bit: round_wait / round_done around the K loop (counters at stamp_out)

// Measured on config 5 (tools/gemm_8p_probe.hip, profiles/r06_gemm_bf16_8p*.log,
// every arm bit-identical to w4p): the library form -- each phase's two
// staging pieces issued AFTER its fragment reads, no s_setprio -- 89.9-90.8
// ms (1410-1424 TF) against w4p's 97.6-98.4 in the same process.  VAR (probe
// arms only): 1 = staging pieces before the reads (the first form, 94.5-97.0
// ms), 2 = s_setprio(1) / (0) around every MFMA cluster (91.0-91.8), 4 =
// group 1 at priority 1 for the whole loop (91.1).  Also measured and
// dropped: phase 0 reading B before A (equal), the wait for K tile t + 1 in
// phase 2 with its B sub-tile 0 read in phase 3 (reads 8 / 4 / 8 / 4; 95.1-99.3
// ms: the shorter lead of the last half-tile), phase 0's pieces split around
// its B reads (99.6), tile groups of 2 / 8 / 16 rows (95.4 / 90.7 / 97.8).
// Ablations (probe only, WRONG results): 8 = no staging in the K loop, 16 =
// every half-tile staged from K tile 0's addresses (L2-resident fills), 32 =
// no fragment reads in the K loop.  64 = the round-5 tile order (xcd_remap:
// each XCD a contiguous range of the grouped order) instead of xcd_lockstep;
// 128 = xcd_lockstep without the round-robin tail; E8_ROUNDS (512, the
// 1-GPU library form) = round_wait / round_done around the K loop (probe:
// + 1024 / 2048 = a round may start with 4 / 8 of the last one unfinished): 84.3-84.5
// ms against 85.0-85.2 (profiles/r06_gemm_round_sync.log).  (A 4 x 2 arrangement of
// the XCDs, 16 A + 16 B^T panels per round, ran 88.5-88.8 ms against 87.7-88.1:
// commit "Probe: 4 x 2 XCD tile arrangement", profiles/r06_gemm_tile_order.log.)
template <bool OUT_BF16, bool STAMP = false, int VAR = 0, int GM = 4>
__global__ __launch_bounds__(512, 1) void k_gemm_bf16_8p(const cubed_gemm_chain_t* __restrict__ tasks,
                                                      const char* __restrict__ PA, const char* __restrict__ PB,
                                                      PackPlan pp, GemmGrid gg,
                                                      unsigned long long* __restrict__ stamp_out) {
  __shared__ __attribute__((aligned(1024))) char lds_[E8_NSLOT * E8_HALF];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t0, m0, n0;
  const int64_t lt = (VAR & 64)    ? xcd_remap(blockIdx.x, gridDim.x)
                     : (VAR & 128) ? xcd_lockstep<false>(blockIdx.x, gridDim.x, GM * pp.TN, pp.TM / GM)
                                   : xcd_lockstep(blockIdx.x, gridDim.x, GM * pp.TN, pp.TM / GM);
  tile_of<HB_BM, HB_BN, GM>(lt, pp.TM, pp.TN, t0, m0, n0);
  const int64_t M = pp.M, N = pp.N;
  unsigned* const rctr = (VAR & E8_ROUNDS) ? (unsigned*)stamp_out : nullptr;
  if (t0 != 0 || m0 >= M || n0 >= N) {
    if constexpr ((VAR & E8_ROUNDS) != 0) round_done(rctr, blockIdx.x);
    return;
  }
  if constexpr ((VAR & E8_ROUNDS) != 0) round_wait(rctr, blockIdx.x, 32, (VAR & 1024) ? 4 : (VAR & 2048) ? 8 : 0);
  const int ktl = (int)pp.KTL, nph = 4 * ktl;
  // the last K tile holds <= 32 live k: its second 32-k half is not
  // multiplied (w4p's K loop stops at ceil(K / 32) steps too)
  const bool half_last = (pp.K & 63) != 0 && (pp.K & 63) <= 32;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2, wc = w & 3, hb = wc >> 1;
  // staging: this wave's two 1 KiB pieces of every half-tile
  const char* const sA = PA + (m0 / 256) * pp.apstride + (2 * w) * 1024 + lane * 16;
  const char* const sB = PB + (n0 / 256) * pp.pstride + (2 * w) * 1024 + lane * 16;
  const int64_t aks = pp.akstride;
  CUBED_L char* const dw = lds + (2 * w) * 1024;
  auto stage = [&](int u) __attribute__((always_inline)) {
    if constexpr ((VAR & 8) != 0) return;
    const int kt = (VAR & 16) ? 0 : u >> 2, h = u & 3;
    const char* src = h < 2 ? sA + kt * aks + h * E8_HALF : sB + (int64_t)kt * 32768 + (h - 2) * E8_HALF;
    CUBED_L char* d = dw + (u % E8_NSLOT) * E8_HALF;
    glds16(src, d);
    glds16(src + 1024, d + 1024);
  };

  // fragment offsets inside a half-tile slot: row rl = sub-tile rows + (lane
  // & 15), 16-B chunk (4 kq + (lane >> 4)) at its swizzled slot; only the
  // lane part varies at run time (the sub-tile part is a ds_read offset)
  int lo[2];
#pragma unroll
  for (int kq = 0; kq < 2; ++kq) lo[kq] = (lane & 15) * 128 + 16 * ((4 * kq + (lane >> 4)) ^ ((lane >> 1) & 7));
  const int bcol = (wc & 1) * 64 * 128;  // this wave's 64 B^T rows inside its half

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4][2] = {}, b0[2][2] = {}, b1[2][2] = {};

  auto rd = [&](CUBED_L const char* base, int off) __attribute__((always_inline)) {
    return *(const CUBED_L bf16x8*)(base + off);
  };
  auto read_a = [&](int t, int qm) __attribute__((always_inline)) {
    if constexpr ((VAR & 32) != 0) return;
    CUBED_L const char* base = lds + ((4 * t + g) % E8_NSLOT) * E8_HALF;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int kq = 0; kq < 2; ++kq) a[mt][kq] = rd(base, lo[kq] + (qm * 64 + mt * 16) * 128);
  };
  auto read_b = [&](int t, int qn, bf16x8 (&b)[2][2]) __attribute__((always_inline)) {
    if constexpr ((VAR & 32) != 0) return;
    CUBED_L const char* base = lds + ((4 * t + 2 + hb) % E8_NSLOT) * E8_HALF + bcol;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int kq = 0; kq < 2; ++kq) b[nt][kq] = rd(base, lo[kq] + (qn * 32 + nt * 16) * 128);
  };
  // one quadrant: acc rows 4 qm .. +3, columns 2 qn .. +1, K = 64 (or 32)
  auto quad = [&](int qm, int qn, const bf16x8 (&b)[2][2], bool half) __attribute__((always_inline)) {
#pragma unroll
    for (int kq = 0; kq < 2; ++kq) {
      if (kq == 1 && half) break;  // (compile-time)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[4 * qm + mt][2 * qn + nt] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][kq], b[nt][kq], acc[4 * qm + mt][2 * qn + nt], 0, 0, 0);
    }
  };
  auto barrier = []() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma_begin = []() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr ((VAR & 2) != 0) __builtin_amdgcn_s_setprio(1);
  };
  auto mfma_end = []() __attribute__((always_inline)) {
    if constexpr ((VAR & 2) != 0) __builtin_amdgcn_s_setprio(0);
  };

  // prologue: half-tiles 0 .. 6 staged, K tile 0 (halves 0 .. 3) waited
  for (int u = 0; u < E8_LEAD && u < nph; ++u) stage(u);
  switch (nph < E8_LEAD ? nph - 4 : E8_LEAD - 4) {
    case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
  barrier();
  if (g == 1) barrier();  // group 1 runs one interval behind group 0
  if constexpr ((VAR & 4) != 0) {
    if (g == 1) __builtin_amdgcn_s_setprio(1);
  }

  unsigned long long c0 = 0, c1 = 0;
  if constexpr (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0)::"memory");
  // one K tile: four phases (the last K tile may multiply 32 k only)
  auto ktile = [&](int t, auto Half) __attribute__((always_inline)) {
    constexpr bool half = decltype(Half)::value;
    const int s = 4 * t;
    // phase 0: A sub-tile 0 + B sub-tile 0, quadrant (0, 0)
    if ((VAR & 1) && s + E8_LEAD < nph) stage(s + E8_LEAD);
    read_a(t, 0);
    read_b(t, 0, b0);
    if (!(VAR & 1) && s + E8_LEAD < nph) stage(s + E8_LEAD);
    barrier();
    mfma_begin();
    quad(0, 0, b0, half);
    mfma_end();
    barrier();
    // phase 1: B sub-tile 1, quadrant (0, 1)
    if ((VAR & 1) && s + 1 + E8_LEAD < nph) stage(s + 1 + E8_LEAD);
    read_b(t, 1, b1);
    if (!(VAR & 1) && s + 1 + E8_LEAD < nph) stage(s + 1 + E8_LEAD);
    barrier();
    mfma_begin();
    quad(0, 1, b1, half);
    mfma_end();
    barrier();
    // phase 2: A sub-tile 1, quadrant (1, 1)
    if ((VAR & 1) && s + 2 + E8_LEAD < nph) stage(s + 2 + E8_LEAD);
    read_a(t, 1);
    if (!(VAR & 1) && s + 2 + E8_LEAD < nph) stage(s + 2 + E8_LEAD);
    barrier();
    mfma_begin();
    quad(1, 1, b1, half);
    mfma_end();
    barrier();
    // phase 3: K tile t + 1 complete (this wave's pieces; every wave waits
    // before the barrier K tile t + 1's first readers pass), quadrant (1, 0)
    if (t + 2 < ktl)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (s + 3 + E8_LEAD < nph) stage(s + 3 + E8_LEAD);
    barrier();
    mfma_begin();
    quad(1, 0, b0, half);
    mfma_end();
    barrier();
  };
  for (int t = 0; t + 1 < ktl; ++t) ktile(t, std::false_type{});
  if (half_last)
    ktile(ktl - 1, std::true_type{});
  else
    ktile(ktl - 1, std::false_type{});
  if (g == 0) barrier();  // the same barrier count in both groups
  if constexpr ((VAR & E8_ROUNDS) != 0) round_done(rctr, blockIdx.x);
  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1)::"memory");
    if (lane == 0) {
      stamp_out[(blockIdx.x * 8 + w) * 2] = c1 - c0;
      stamp_out[(blockIdx.x * 8 + w) * 2 + 1] = (unsigned long long)nph;
    }
  }

  // epilogue: accumulator (mi, ni) register i = row 128 g + 16 mi + 4 (lane >>
  // 4) + i, column 64 wc + 16 ni + (lane & 15); chunk selects as w4p's
  const GridTile gt = grid_tile(tasks, gg, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = gt.T;
  const bool accum = T->accumulate != 0;
  uint64_t cbase[2][2];
  int64_t cld[2][2];
  const cubed_gemm_chain_t* TQ[2][2] = {{T, gt.TJ1}, {gt.TI1, gt.TI1 + (gt.TJ1 - T)}};
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      cbase[x][y] = (uint64_t)(uintptr_t)TQ[x][y]->c;
      cld[x][y] = TQ[x][y]->ldc;
    }
  const int64_t gm0 = m0 + g * 128 + 4 * (lane >> 4);
  const int64_t gn0 = n0 + wc * 64 + (lane & 15);
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int64_t gn = gn0 + ni * 16;
    if (gn >= N) continue;
    const bool hn = gn >= gt.nb;
    const int64_t ln = gn - (hn ? gt.nb : gt.J0 * gg.cn);
    const uint64_t cc0 = hn ? cbase[0][1] : cbase[0][0];
    const uint64_t cc1 = hn ? cbase[1][1] : cbase[1][0];
    const int64_t l0 = hn ? cld[0][1] : cld[0][0];
    const int64_t l1 = hn ? cld[1][1] : cld[1][0];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      if constexpr (OUT_BF16) {
        // lanes 2i, 2i + 1 hold columns 2i, 2i + 1 of the same rows: per
        // register pair (r, r + 1) one exchange gives the even lane row r and
        // the odd lane row r + 1 as two adjacent columns (cn % 8 == 0: a pair
        // never straddles a chunk column)
        const bool odd = lane & 1;
        const int64_t le = ln - (odd ? 1 : 0);
#pragma unroll
        for (int r0 = 0; r0 < 4; r0 += 2) {
          const float x0 = acc[mi][ni][r0], x1 = acc[mi][ni][r0 + 1];
          const float y = __shfl_xor(odd ? x0 : x1, 1);
          float vlo = odd ? y : x0, vhi = odd ? x1 : y;
          const int64_t gm = gm0 + mi * 16 + r0 + (odd ? 1 : 0);
          if (gm < M) {
            const bool hm = gm >= gt.mb;
            const int64_t lm = gm - (hm ? gt.mb : gt.I0 * gg.cm);
            const uint64_t C = hm ? cc1 : cc0;
            const int64_t ldc = hm ? l1 : l0;
            CUBED_G uint32_t* c = (CUBED_G uint32_t*)(uintptr_t)(C + (uint64_t)(lm * ldc + le) * 2);
            if (accum) {
              const uint32_t o = *c;
              vlo += bf16_to_f32((uint16_t)(o & 0xffffu));
              vhi += bf16_to_f32((uint16_t)(o >> 16));
            }
            *c = (uint32_t)f32_to_bf16(vlo) | ((uint32_t)f32_to_bf16(vhi) << 16);
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = gm0 + mi * 16 + r;
          if (gm < M) {
            const bool hm = gm >= gt.mb;
            const int64_t lm = gm - (hm ? gt.mb : gt.I0 * gg.cm);
            const uint64_t C = hm ? cc1 : cc0;
            const int64_t ldc = hm ? l1 : l0;
            float v = acc[mi][ni][r];
            CUBED_G float* c = (CUBED_G float*)(uintptr_t)(C + (uint64_t)(lm * ldc + ln) * 4);
            if (accum) v += *c;
            *c = v;
          }
        }
      }
    }
  }
}
