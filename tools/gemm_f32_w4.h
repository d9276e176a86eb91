// gemm_f32_w4.h -- development probe (not part of the library; included by
// tools/gemm_f32_probe.hip after gemm_chain.hip): the f32 chained GEMM with
// ONE wave per SIMD, keeping k_gemm_f32_chain's LDS image, staging geometry
// and value-preserving fragment permutations.  Bit-identical; measured at
// parity with the library (per chunk 132.9-133.9 TF vs 129.8, grid 133.0-133.4
// vs 132.9-133.5: profiles/r05_gemm_f32_w4.log), so not adopted.  256 x 256 tile per 256-thread workgroup, 128 x 128 per wave: 4 row
// blocks x 4 column-interleaved accumulators of v_mfma_f32_32x32x2_f32 = 256
// AGPRs.  Per 16-deep K step a wave issues 128 MFMAs (64 cycles each), and in
// their gaps the 16 ds_read_b128 of the NEXT step's fragments (a second
// register set) and the 8 LDS-DMA pieces of step p + 4: the 8-wave kernel
// (2 waves per SIMD, 64 MFMAs per wave per step) read each step's first
// fragments after the step's barrier, with both waves of a SIMD waiting on
// them at once (MFMA pipe busy 0.86, profiles/r04_gemm_f32_grid_pmc.log).
//
// Ring: 4 slots of one step (A [256][16] + B [16][256] f32 = 32 KiB).  Step
// p computes slot p % 4 with fragments read during step p - 1, reads step
// p + 1's fragments from slot (p + 1) % 4 and stages step p + 4 into slot
// p % 4 -- free once every wave passed step p's barrier (its last reads were
// step p - 1's).  Step p + 1's loads went out at step p - 3: the wait before
// step p's barrier allows the loads of steps p + 2 and p + 3 in flight.
// Per output element the same f32 chain as k_gemm_f32_chain (steps, then k
// group g, then j; each MFMA pairs k = 8g + j with 8g + 4 + j): bit-identical.
#pragma once

constexpr int WF_BK = 16, WF_NS = 4;
constexpr int WF_SA = HF_BM * WF_BK * 4, WF_SB = WF_BK * HF_BN * 4, WF_STAGE = WF_SA + WF_SB;

// ABL (tools/gemm_f32_probe.hip only; results wrong when nonzero): 1 no
// K-loop barrier, 2 no K-loop vmcnt wait, 16 every staged step reads step 0's
// sources (L2-resident fills).
template <bool GRID = false, bool STAMP = false, int ABL = 0>
__global__ __launch_bounds__(256, 1) void k_gemm_f32_w4(const cubed_gemm_chain_t* __restrict__ tasks,
                                                     const cubed_gemm_seg_t* __restrict__ segs,
                                                     int64_t tiles_m, int64_t tiles_n,
                                                     const char* __restrict__ zero, GemmGrid gg,
                                                     unsigned long long* __restrict__ stamp_out) {
  constexpr int CPR = 4, RPI = 16, NA = 4, NB = 4, SWS = 2, G = 2, LPS = NA + NB;
  __shared__ __attribute__((aligned(1024))) char lds_[WF_NS * WF_STAGE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t, m0, n0;
  tile_of<HF_BM, HF_BN, 4>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  int64_t I0 = 0, J0 = 0, mb = 0, nb = 0;
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const cubed_gemm_chain_t* __restrict__ TI1 = T;
  const cubed_gemm_chain_t* __restrict__ TJ1 = T;
  if constexpr (GRID) {
    I0 = m0 / gg.cm;
    J0 = n0 / gg.cn;
    mb = (I0 + 1) * gg.cm;
    nb = (J0 + 1) * gg.cn;
    T = tasks + I0 * gg.tj + J0;
    TI1 = (I0 + 1 < gg.ti) ? T + gg.tj : T;
    TJ1 = (J0 + 1 < gg.tj) ? T + 1 : T;
  }
  const int64_t M = GRID ? gg.M : T->m, N = GRID ? gg.N : T->n, KT = T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;
  const int64_t dsI = TI1->seg0 - T->seg0, dsJ = TJ1->seg0 - T->seg0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (w >> 1) * 128, wn = (w & 1) * 128;

  // ---- staging geometry (k_gemm_f32_chain's, 4 waves): A instruction i of
  // wave w stages rows RPI*(NA*w + i) + lane/CPR; B instruction i k-row NB*w + i
  int64_t gmA[NA];
  int kA[NA];
  bool hiA[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int r = RPI * (NA * w + i) + lane / CPR;
    const int64_t g = (m0 + r < M ? m0 + r : M - 1);
    hiA[i] = GRID && g >= mb;
    gmA[i] = GRID ? g - (hiA[i] ? mb : I0 * gg.cm) : g;
    kA[i] = 4 * ((lane % CPR) ^ ((r >> SWS) & (CPR - 1)));
  }
  const int rB0 = NB * w;
  int64_t gnB = (n0 + 4 * lane + 4 <= N ? n0 + 4 * lane : N - 4);
  const bool hiB = GRID && gnB >= nb;
  if constexpr (GRID) gnB -= hiB ? nb : J0 * gg.cn;
  const int64_t gnB4 = gnB * 4;
  // per-lane A source offsets inside the staged step's segment (row * pitch +
  // chunk): recomputed when that segment changes; a piece adds one uniform
  // base (A rows I0 / I0+1 of a segment share the pitch)
  int64_t soffA[NA];
  int64_t soffA_seg = -1;

  int64_t s = seg0, ks = 0;
  auto ptr = [&](int64_t i) { return (const char*)(uintptr_t)segs[i].a; };
  auto ptrb = [&](int64_t i) { return (const char*)(uintptr_t)segs[i].b; };
  const char* a_cur = ptr(s);
  const char* a_hi = ptr(s + dsI);
  const char* b_cur = ptrb(s);
  const char* b_hi = ptrb(s + dsJ);
  int64_t lda4 = segs[s].lda * 4, ldb4 = segs[s].ldb * 4, ldb4h = segs[s + dsJ].ldb * 4;
  int64_t ke = segs[s].k;

  // the step being staged: its k0 and the walk's state for it (wave-uniform,
  // scalar registers); each piece computes its source when it is issued (per
  // -lane 64-bit source arrays held over the 128-MFMA gap loop spilled)
  struct Src {
    int64_t k0, ks, ke, lda4, ldb4, ldb4h, nlda4, nldb4;
    const char *a_cur, *a_hi, *b_cur, *b_hi, *nal, *nah, *nbp;
    const char *abase, *abase_hi;  // a_cur / a_hi + (k0 - ks) * 4
    const char *brow, *brow_hi;    // B k-row rB0 of the step: b_cur / b_hi + (k0 - ks + rB0) * pitch
    bool edge, has_next;
  } src;
  auto sources = [&](int64_t k0) __attribute__((always_inline)) {
    if (soffA_seg != s) {  // uniform: a new segment for the staged steps
#pragma unroll
      for (int i = 0; i < NA; ++i) soffA[i] = gmA[i] * lda4 + kA[i] * 4;
      soffA_seg = s;
    }
    src.abase = a_cur + (k0 - ks) * 4;
    src.abase_hi = a_hi + (k0 - ks) * 4;
    src.brow = b_cur + (k0 - ks + rB0) * ldb4;
    if constexpr (GRID) src.brow_hi = b_hi + (k0 - ks + rB0) * ldb4h;
    src.k0 = k0;
    src.ks = ks;
    src.ke = ke;
    src.lda4 = lda4;
    src.ldb4 = ldb4;
    src.ldb4h = ldb4h;
    src.a_cur = a_cur;
    src.a_hi = a_hi;
    src.b_cur = b_cur;
    src.b_hi = b_hi;
    src.edge = k0 + WF_BK > ke;
    src.has_next = s + 1 < segN;
    if (src.edge) {
      const int64_t sn = src.has_next ? s + 1 : s;
      src.nal = ptr(sn);
      src.nah = ptr(sn + dsI);
      src.nbp = hiB ? ptrb(sn + dsJ) : ptrb(sn);
      src.nlda4 = segs[sn].lda * 4;
      src.nldb4 = (hiB ? segs[sn + dsJ].ldb : segs[sn].ldb) * 4;
    }
    if (k0 + WF_BK >= ke && s + 1 < segN) {
      ks = ke;
      ++s;
      a_cur = ptr(s);
      a_hi = ptr(s + dsI);
      b_cur = ptrb(s);
      b_hi = ptrb(s + dsJ);
      lda4 = segs[s].lda * 4;
      ldb4 = segs[s].ldb * 4;
      ldb4h = segs[s + dsJ].ldb * 4;
      ke = ks + segs[s].k;
    }
  };
  // piece i (0..7) of the staged step into slot buffer buf: inside one
  // segment (simple: one 64-bit add per A piece, a uniform B row) ...
  auto piece = [&](auto I, CUBED_L char* buf) __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
    if constexpr (i < NA) {
      const char* base = GRID ? (hiA[i] ? src.abase_hi : src.abase) : src.abase;
      glds16(base + soffA[i], buf + (NA * w + i) * 1024);
    } else {
      constexpr int b = i - NA;
      const char* row = GRID ? (hiB ? src.brow_hi + b * src.ldb4h : src.brow + b * src.ldb4) : src.brow + b * src.ldb4;
      glds16(row + gnB4, buf + WF_SA + (rB0 + b) * 1024);
    }
  };
  // ... or crossing the segment's end / the chain's end (per-lane selects;
  // issued all at once where the step's sources are set)
  auto piece_edge = [&](auto I, CUBED_L char* buf) __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
    if constexpr (i < NA) {
      const int64_t ka = src.k0 + kA[i];
      const char* pa = (hiA[i] ? src.a_hi : src.a_cur) + gmA[i] * src.lda4 + (ka - src.ks) * 4;
      const char* na = (hiA[i] ? src.nah : src.nal) + gmA[i] * src.nlda4 + (ka - src.ke) * 4;
      const char* alt = (src.has_next && ka < KT) ? na : zero;
      glds16(ka >= src.ke ? alt : pa, buf + (NA * w + i) * 1024);
    } else {
      constexpr int b = i - NA;
      const int64_t kb = src.k0 + rB0 + b;
      const char* pb = (hiB ? src.b_hi : src.b_cur) + (kb - src.ks) * (hiB ? src.ldb4h : src.ldb4) + gnB4;
      const char* nbq = src.nbp + (kb - src.ke) * src.nldb4 + gnB4;
      const char* alt = (src.has_next && kb < KT) ? nbq : zero;
      glds16(kb >= src.ke ? alt : pb, buf + WF_SA + (rB0 + b) * 1024);
    }
  };
  auto all_pieces = [&](CUBED_L char* buf) __attribute__((always_inline)) {
    if (src.edge)
      wl_seq<LPS>([&](auto I) __attribute__((always_inline)) { piece_edge(I, buf); });
    else
      wl_seq<LPS>([&](auto I) __attribute__((always_inline)) { piece(I, buf); });
  };

  // ---- fragment read offsets (within a slot): A (rb, g): row wm + 32 rb +
  // r32, logical chunk 2g + h; B (g, j): k-row 8g + 4h + j, columns wn + 4 r32
  const int h = lane >> 5, r32 = lane & 31;
  int offA[4][G];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int g = 0; g < G; ++g)
      offA[rb][g] = (wm + 32 * rb + r32) * (WF_BK * 4) + 16 * ((2 * g + h) ^ ((r32 >> SWS) & (CPR - 1)));
  const int offB = WF_SA + 4 * h * 1024 + (wn + 4 * r32) * 4;

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

  const int64_t nst = (KT + WF_BK - 1) / WF_BK;
  auto slot = [&](int64_t p) { return lds + (p % WF_NS) * WF_STAGE; };
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
  for (int64_t p = 0; p < WF_NS && p < nst; ++p) {
    sources(p * WF_BK);
    all_pieces(slot(p));
  }
  Frags f0, f1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int e = 0; e < 16; ++e) read(e, f0, slot(0));

  // step p: MFMAs on X (step p's fragments), reads of step p + 1 into Y, and
  // step p + 4's pieces.  FULL: the steady state (both exist; no branch in
  // the MFMA stream -- uniform branches there split it into blocks across
  // which the register allocator copied all 256 accumulator registers per
  // step); otherwise the tail: the MFMAs, then whatever reads remain.
  auto step = [&](int64_t p, const Frags& X, Frags& Y, auto Full) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(Full)::value;
    // this wave's reads of step p's fragments (issued in step p - 1) are in
    // registers before any wave restages slot p % 4 after the barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(ABL & 2)) {
      if constexpr (FULL)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPS) : "memory");
      else if (p + 1 < nst)
        wait_step(p + 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!(ABL & 1)) __builtin_amdgcn_s_barrier();  // step p+1 landed everywhere; slot p % 4 read out
    __builtin_amdgcn_sched_barrier(0);
    const CUBED_L char* rbuf = slot(p + 1);
    CUBED_L char* sbuf = slot(p);
    if constexpr (FULL) {
      // first half: the 16 reads of step p + 1 (one per 4 MFMAs); at MFMA 64
      // the staged step's sources (scalar loads of the segment table: their
      // wait also waits for the reads, long landed by then); second half:
      // its 8 pieces (one per 8 MFMAs)
      wl_seq<128>([&](auto Gi) __attribute__((always_inline)) {
        constexpr int gi = decltype(Gi)::value;
        constexpr int g = gi >> 6, j = (gi >> 4) & 3, rb = (gi >> 2) & 3, q = gi & 3;
        acc[rb][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(X.a[g][rb][j], X.b[g][j][q], acc[rb][q], 0, 0, 0);
        if constexpr (gi < 64 && (gi & 3) == 0) {
          __builtin_amdgcn_sched_barrier(0);
          read(gi >> 2, Y, rbuf);
          __builtin_amdgcn_sched_barrier(0);
        } else if constexpr (gi == 64) {
          __builtin_amdgcn_sched_barrier(0);
          sources((ABL & 16) ? 0 : (p + WF_NS) * WF_BK);
          if (src.edge)  // uniform, ~1 step in 300: all 8 pieces here
            wl_seq<LPS>([&](auto I) __attribute__((always_inline)) { piece_edge(I, sbuf); });
          __builtin_amdgcn_sched_barrier(0);
        } else if constexpr (gi > 64 && (gi & 7) == 4) {
          __builtin_amdgcn_sched_barrier(0);
          if (!src.edge) piece(std::integral_constant<int, ((gi - 64) >> 3)>{}, sbuf);
          __builtin_amdgcn_sched_barrier(0);
        }
      });
    } else {
      wl_seq<128>([&](auto Gi) __attribute__((always_inline)) {
        constexpr int gi = decltype(Gi)::value;
        constexpr int g = gi >> 6, j = (gi >> 4) & 3, rb = (gi >> 2) & 3, q = gi & 3;
        acc[rb][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(X.a[g][rb][j], X.b[g][j][q], acc[rb][q], 0, 0, 0);
      });
      if (p + WF_NS < nst) {
        sources((p + WF_NS) * WF_BK);
        all_pieces(sbuf);
      }
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
  for (; p + 1 + WF_NS < nst; p += 2) {
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

  // ---- epilogue: accumulator (rb, q) register r = row wm + 32 rb + (r&3) +
  // 8 (r>>2) + 4h, column wn + 4 r32 + q: one float4 per (rb, r)
  const bool accum = T->accumulate != 0;
  const int64_t gn = n0 + wn + 4 * r32;
  if (gn < N) {
    const bool hn = GRID && gn >= nb;
    const cubed_gemm_chain_t* __restrict__ TC0 = hn ? TJ1 : T;
    const cubed_gemm_chain_t* __restrict__ TC1 = TC0 + (TI1 - T);
    const int64_t ln = GRID ? gn - (hn ? nb : J0 * gg.cn) : gn;
    char* C0 = (char*)(uintptr_t)TC0->c;
    char* C1 = (char*)(uintptr_t)TC1->c;
    const int64_t ldc0 = TC0->ldc, ldc1 = TC1->ldc;
    wl_seq<64>([&](auto RR) __attribute__((always_inline)) {
      constexpr int rb = decltype(RR)::value >> 4, r = decltype(RR)::value & 15;
      const int64_t gm = m0 + wm + 32 * rb + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (gm < M) {
        const bool hm = GRID && gm >= mb;
        const int64_t lm = GRID ? gm - (hm ? mb : I0 * gg.cm) : gm;
        CUBED_G f32x4* c = (CUBED_G f32x4*)(uintptr_t)((hm ? C1 : C0) + (lm * (hm ? ldc1 : ldc0) + ln) * 4);
        f32x4 v = {acc[rb][0][r], acc[rb][1][r], acc[rb][2][r], acc[rb][3][r]};
        if (accum) v += *c;
        *c = v;
      }
    });
  }
}
