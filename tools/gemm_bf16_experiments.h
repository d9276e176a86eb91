// gemm_bf16_experiments.h -- two bf16 chained-GEMM schedules measured against
// the library's ping-pong kernel and NOT adopted (tools/gemm_bf16_probe.hip
// includes this after csrc/gemm_chain.hip; profiles/r02_gemm_bf16_q4_w4.log).
// Both are bit-identical to the library kernel on config 5 and slower:
//   k_gemm_bf16_q4  4 phases of 16 MFMAs per 64-deep K tile   820 vs 1028 TF
//   k_gemm_bf16_w4  one wave per SIMD, 128 x 128 per wave      791 vs 1066 TF

// ------------------------------------------------- bf16 MFMA, 4-phase K tiles
// Same 256x256 tile, 8 waves (2 M x 4 N, 128 x 64 each), but K tiles 64 deep
// in two LDS buffers (tile t in buffer t&1), each tile split into four
// 16 KiB HALF-TILES by C quadrant:
//   A0 / A1 = the tile rows with ((row >> 6) & 1) == 0 / 1   [128 rows x 128 B]
//   B0 / B1 = the tile cols with ((col >> 5) & 1) == 0 / 1   [64 k-rows x 256 B]
// A wave's 128 x 64 output is four 64 x 32 quadrants (qm, qn); a tile is
// four PHASES, one quadrant each (16 MFMAs = 4 mb x 2 nb x 2 k-halves), in
// the order (0,0) (0,1) (1,1) (1,0), so each phase reads at most one new A
// half and one new B half from LDS:
//   P1 reads A0 + B0, P2 reads B1, P3 reads A1, P4 reads nothing (B0 kept).
// A half-tile is restaged (global_load_lds, 2 per thread) for tile t+2 two
// phases after its last read: A0 + B0 in P3, B1 in P4, A1 in P1 of t+1, so
// every half-tile has six phases to land.
// Phase = {LDS reads; staging loads} barrier {lgkmcnt(0); 16 MFMAs;
// vmcnt(8)} barrier.  The two wave rows run one barrier apart (row 1 enters
// one barrier later), so on each SIMD one wave's MFMAs overlap the other's
// LDS reads (cdna_hip_programming.md §5 "256² 8-phase template").
//   RAW: loads issued in phase X are retired by every wave at the end of
//   phase X+4 (vmcnt(8) = the 8 loads of the four youngest phases) and read
//   in X+6; the stagger needs only X+4.
//   WAR: a half last read in phase r (reads retired by the lgkmcnt(0) after
//   the phase's first barrier) is restaged in r+2, after both rows' retire.
// LDS images (lane-linear global_load_lds destinations, swizzle on the
// SOURCE): A half row i (128 B) holds 16-B chunk slot s = c ^ ((i >> 1) & 7)
// of k-chunk c -- conflict-free ds_read_b128; B half k-row r (256 B) holds
// slot s = c ^ 2*((r & 3) | ((r >> 3) & 1) << 2) of col chunk c (c >> 2 =
// wave column, c & 3 = 8 cols of its quadrant) -- conflict-free
// ds_read_b64_tr_b16.
// Why slower: P1 reads 8 b128 + 8 tr_b64 per wave against the other row's 16
// MFMAs (256 cycles), so the phases are unbalanced; the ping-pong slot hides
// the same reads behind 32 MFMAs.
constexpr int HQ_BK = 64;
constexpr int HQ_HALF = 16384;
constexpr int HQ_BUF = 4 * HQ_HALF;  // A0 A1 B0 B1

template <bool OUT_BF16, int GM = 4>
__global__ __launch_bounds__(512, 2) void k_gemm_bf16_q4(const cubed_gemm_chain_t* __restrict__ tasks,
                                                      const cubed_gemm_seg_t* __restrict__ segs,
                                                      int64_t tiles_m, int64_t tiles_n,
                                                      const char* __restrict__ zero) {
  __shared__ __attribute__((aligned(1024))) char lds_[2 * HQ_BUF];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n, KT = T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- staging geometry: load j (0, 1) of wave w fills 1 KiB of a half
  // A half qm, LDS row i = 8*(2w+j) + (lane>>3), slot lane&7
  int64_t gmA[2][2];
  int kA[2];  // k offset (elements) inside the tile of this lane's chunk, per j
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = 8 * (2 * w + j) + (lane >> 3);
    kA[j] = 8 * ((lane & 7) ^ ((i >> 1) & 7));
#pragma unroll
    for (int qm = 0; qm < 2; ++qm) {
      const int64_t r = m0 + (i >> 6) * 128 + qm * 64 + (i & 63);
      gmA[qm][j] = r < M ? r : M - 1;
    }
  }
  // B half qn, k-row r = 4*(2w+j) + (lane>>4), slot lane&15
  int rB[2];
  int64_t gnB[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 4 * (2 * w + j) + (lane >> 4);
    rB[j] = r;
    const int c = (lane & 15) ^ (2 * ((r & 3) | (((r >> 3) & 1) << 2)));
#pragma unroll
    for (int qn = 0; qn < 2; ++qn) {
      const int64_t n = n0 + (c >> 2) * 64 + qn * 32 + (c & 3) * 8;
      gnB[qn][j] = n + 8 <= N ? n : N - 8;
    }
  }

  // ---- wave-uniform segment state of the tile being staged
  int64_t s = seg0, ks = 0;
  Seg cur = load_seg(segs, s);
  int64_t ke = segs[s].k;

  // issue the 2 loads of one half (h: 0 = A0, 1 = A1, 2 = B0, 3 = B1) of the
  // tile starting at k0 into buffer buf
  auto stage = [&](int64_t k0, int h, CUBED_L char* buf) {
    const bool edge = k0 + HQ_BK > ke;  // uniform: a segment boundary / the end inside this tile
    const bool has_next = s + 1 < segN;
    Seg nxt = cur;
    if (edge) nxt = load_seg(segs, has_next ? s + 1 : s);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const char* src;
      if (h < 2) {
        const int64_t gm = gmA[h][j], k = k0 + kA[j];
        src = cur.a + gm * cur.lda2 + (k - ks) * 2;
        if (edge && k >= ke) src = (has_next && k < KT) ? nxt.a + gm * nxt.lda2 + (k - ke) * 2 : zero;
      } else {
        const int64_t gn = gnB[h - 2][j], k = k0 + rB[j];
        src = cur.b + (k - ks) * cur.ldb2 + gn * 2;
        if (edge && k >= ke) src = (has_next && k < KT) ? nxt.b + (k - ke) * nxt.ldb2 + gn * 2 : zero;
      }
      glds16(src, buf + h * HQ_HALF + (2 * w + j) * 1024);
    }
  };
  // after the last half of a tile: move on if the next tile starts in the next segment
  auto advance = [&](int64_t k0) {
    if (k0 + HQ_BK >= ke && s + 1 < segN) {
      ks = ke;
      ++s;
      cur = load_seg(segs, s);
      ke = ks + segs[s].k;
    }
  };

  // ---- LDS read offsets (inside a buffer): A half qm, LDS row
  // wr*64 + mb*16 + (lane&15) = tile row wr*128 + qm*64 + mb*16 + (lane&15),
  // k chunk kh*4 + (lane>>4)
  const int ra = wr * 64 + (lane & 15);
  int offA[2];  // per k-half
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) offA[kh] = ra * 128 + 16 * ((kh * 4 + (lane >> 4)) ^ ((ra >> 1) & 7));
  // (mb adds 16 rows = 2048 B and leaves (row >> 1) & 7 unchanged)
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int hq = 2 * (q | ((g & 1) << 2));
  int offB[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) offB[nb] = 2 * HQ_HALF + (8 * g + q) * 256 + 16 * ((wc * 4 + nb * 2 + (pp >> 1)) ^ hq) + 8 * (pp & 1);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2];     // [mb in quadrant][k half]
  bf16x8 bfr[2][2][2]; // [qn][nb][k half]

  auto read_a = [&](const CUBED_L char* buf, int qm) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) af[mb][kh] = *(const CUBED_L bf16x8*)(buf + qm * HQ_HALF + offA[kh] + mb * 2048);
  };
  auto read_b = [&](const CUBED_L char* buf, int qn) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const uint32_t pb = (uint32_t)(uintptr_t)(buf + qn * HQ_HALF + offB[nb] + kh * 8192);
        s16x4 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(pb));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:1024" : "=v"(hi) : "v"(pb));
        bfr[qn][nb][kh] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
  };
  auto mfma_q = [&](int qm, int qn) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[qm * 4 + mb][qn * 2 + nb] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb][kh], bfr[qn][nb][kh], acc[qm * 4 + mb][qn * 2 + nb], 0, 0, 0);
  };
  // vmcnt(n) for the loads of the four youngest phases (0, 2, 4, 6 or 8)
  auto wait_vm = [&](int n) {
    if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  const int64_t nt = (KT + HQ_BK - 1) / HQ_BK;
  // prologue: tile 0 whole, tile 1's A0, B0, B1 (the steady state at P1(0))
  if (nt > 0) {
    stage(0, 0, lds); stage(0, 2, lds); stage(0, 3, lds); stage(0, 1, lds);
    advance(0);
  }
  int l1 = 0, l2 = 0, l3 = 0;  // loads issued in the 3 previous phases
  if (nt > 1) {
    stage(HQ_BK, 0, lds + HQ_BUF); stage(HQ_BK, 2, lds + HQ_BUF); stage(HQ_BK, 3, lds + HQ_BUF);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    l2 = 4; l1 = 2;  // "P3(-1)" and "P4(-1)" (l3 = 0: P2(-1) issued nothing)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  auto phase_end = [&](int issued) {
    wait_vm(l3 + l2 + l1 + issued);
    l3 = l2; l2 = l1; l1 = issued;
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mid = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
  };
  auto post = [&]() {
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  for (int64_t tt = 0; tt < nt; ++tt) {
    CUBED_L char* bc = lds + (tt & 1) * HQ_BUF;
    const int64_t k1 = (tt + 1) * HQ_BK, k2 = (tt + 2) * HQ_BK;
    // ---- P1: quadrant (0,0); restage A1 of tile t+1 (read in P3 of t-1)
    read_b(bc, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(bc, 0);
    int is = 0;
    if (tt + 1 < nt) { stage(k1, 1, lds + ((tt + 1) & 1) * HQ_BUF); advance(k1); is = 2; }
    mid();
    mfma_q(0, 0);
    post();
    phase_end(is);
    // ---- P2: quadrant (0,1)
    read_b(bc, 1);
    mid();
    mfma_q(0, 1);
    post();
    phase_end(0);
    // ---- P3: quadrant (1,1); restage A0 + B0 of tile t+2 (read in P1)
    read_a(bc, 1);
    is = 0;
    if (tt + 2 < nt) { stage(k2, 0, bc); stage(k2, 2, bc); is = 4; }
    mid();
    mfma_q(1, 1);
    post();
    phase_end(is);
    // ---- P4: quadrant (1,0); restage B1 of tile t+2 (read in P2)
    is = 0;
    if (tt + 2 < nt) { stage(k2, 3, bc); is = 2; }
    mid();
    mfma_q(1, 0);
    post();
    phase_end(is);
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // same barrier count in both rows

  // ---- epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r
  char* C = (char*)(uintptr_t)T->c;
  const int64_t ldc = T->ldc;
  const bool accum = T->accumulate != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int nbq = 0; nbq < 4; ++nbq)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // acc[qm*4 + mb][qn*2 + nb]: tile row wr*128 + qm*64 + mb*16, tile col wc*64 + qn*32 + nb*16
        const int64_t gm = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + (lane >> 4) * 4 + r;
        const int64_t gn = n0 + wc * 64 + (nbq >> 1) * 32 + (nbq & 1) * 16 + (lane & 15);
        if (gm < M && gn < N) {
          float v = acc[i][nbq][r];
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
      }
}

// ------------------------------------- bf16 MFMA, one wave per SIMD, 128x128
// Hypothesis: the 8-wave kernels are LDS-bandwidth bound -- per 32-deep K
// step a CU reads 96 KiB of fragments and writes 32 KiB of staging into the
// same 256 B/clk array against 1024 MFMA cycles (ablation: no staging
// 1.8 PF, L2-resident staging 1.25 PF, base 1.09 PF).  Here the 256 x 256
// tile is split over 4 waves (2 x 2, one per SIMD, 512 registers each), each
// a 128 x 128 sub-tile of 4 x 4 v_mfma_f32_32x32x16_bf16 accumulators (256
// AGPRs): fragment reads drop to 64 KiB per step.  Step p+1's fragments are
// read into a second register set while step p's MFMAs run, one barrier per
// step, K steps staged four ahead in a 4-slot ring (slot p%4 is free once
// step p's fragments are in registers).
//   A slot image: [256 rows][64 B], 16-B chunk slot s of row r holds k-chunk
//   s ^ ((r >> 2) & 3): conflict-free ds_read_b128 (rows 32 per fragment).
//   B slot image: [32 k-rows][512 B] as in HBM, chunk slot s of k-row r holds
//   col chunk s ^ 4*(r & 3): conflict-free ds_read_b64_tr_b16.
// Measured 791 vs 1066 TF: one wave per SIMD cannot issue its LDS reads and
// staging loads while its own MFMA queue is full, so the 2-wave ping-pong's
// overlap is lost.  Launch with 256 threads.
constexpr int HW_NS = 4;

template <bool OUT_BF16, int GM = 4>
__global__ __launch_bounds__(256, 1) void k_gemm_bf16_w4(const cubed_gemm_chain_t* __restrict__ tasks,
                                                      const cubed_gemm_seg_t* __restrict__ segs,
                                                      int64_t tiles_m, int64_t tiles_n,
                                                      const char* __restrict__ zero) {
  __shared__ __attribute__((aligned(1024))) char lds_[HW_NS * HB_STAGE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n, KT = T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;

  // ---- staging geometry: load i (0..3) of wave w fills 1 KiB of a slot
  // A rows 16*(4w+i) + (lane>>2), slot lane&3 <- k chunk (lane&3) ^ ((lane>>4)&3)
  int64_t gmA[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t r = m0 + 16 * (4 * w + i) + (lane >> 2);
    gmA[i] = r < M ? r : M - 1;
  }
  const int dA = 8 * ((lane & 3) ^ ((lane >> 4) & 3));
  // B k-rows 2*(4w+i) + (lane>>5), slot lane&31 <- col chunk (lane&31) ^ 4*(row&3)
  int rB[4];
  int64_t gnB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 2 * (4 * w + i) + (lane >> 5);
    rB[i] = r;
    const int64_t n = n0 + 8 * ((lane & 31) ^ (4 * (r & 3)));
    gnB[i] = n + 8 <= N ? n : N - 8;
  }

  int64_t s = seg0, ks = 0;
  Seg cur = load_seg(segs, s);
  int64_t ke = segs[s].k;
  int64_t offSA[4], offSB[4];
  auto seg_offsets = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      offSA[i] = gmA[i] * cur.lda2 + dA * 2;
      offSB[i] = rB[i] * cur.ldb2 + gnB[i] * 2;
    }
  };
  seg_offsets();
  auto stage = [&](int64_t k0, CUBED_L char* buf) {
    const char* a0 = cur.a + (k0 - ks) * 2;
    const char* b0 = cur.b + (k0 - ks) * cur.ldb2;
    const char* sa[4];
    const char* sb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sa[i] = a0 + offSA[i];
      sb[i] = b0 + offSB[i];
    }
    if (k0 + HB_BK > ke) {  // uniform: a segment boundary (or the chain's end) inside this step
      const bool has_next = s + 1 < segN;
      const Seg nxt = load_seg(segs, has_next ? s + 1 : s);
      const int64_t ka = k0 + dA;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const char* na = nxt.a + gmA[i] * nxt.lda2 + (ka - ke) * 2;
        sa[i] = ka < ke ? sa[i] : ((has_next && ka < KT) ? na : zero);
        const int64_t kb = k0 + rB[i];
        const char* nbp = nxt.b + (kb - ke) * nxt.ldb2 + gnB[i] * 2;
        sb[i] = kb < ke ? sb[i] : ((has_next && kb < KT) ? nbp : zero);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(sa[i], buf + (4 * w + i) * 1024);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(sb[i], buf + HB_A + (4 * w + i) * 1024);
    if (k0 + HB_BK >= ke && s + 1 < segN) {
      ks = ke;
      ++s;
      cur = load_seg(segs, s);
      ke = ks + segs[s].k;
      seg_offsets();
    }
  };

  // ---- fragment read offsets inside a slot
  // A (mb, kh): row wr*128 + mb*32 + (lane&31), k chunk kh*2 + (lane>>5)
  const int ra = wr * 128 + (lane & 31);
  int offA[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) offA[kh] = ra * 64 + 16 * ((kh * 2 + (lane >> 5)) ^ ((ra >> 2) & 3));
  // B (nb, kh): 16-lane block b = lane>>4 reads k-rows kh*16 + (b>>1)*8 + ((lane&15)>>2)
  // (+4: hi half) x cols wc*128 + nb*32 + (b&1)*16 + 4*(lane&3)
  const int bq = lane >> 4;
  const int krow = (bq >> 1) * 8 + ((lane & 15) >> 2);
  int offB[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    offB[nb] = HB_A + krow * 512 + 16 * ((wc * 16 + nb * 4 + (bq & 1) * 2 + ((lane & 3) >> 1)) ^ (4 * (krow & 3))) +
               8 * (lane & 1);

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto read_frags = [&](const CUBED_L char* buf, bf16x8 (&fa)[4][2], bf16x8 (&fb)[4][2]) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const uint32_t pb = (uint32_t)(uintptr_t)(buf + offB[nb] + kh * 8192);
        s16x4 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(pb));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(hi) : "v"(pb));
        fb[nb][kh] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const uint32_t pa = (uint32_t)(uintptr_t)(buf + offA[kh] + mb * 2048);
        bf16x8 v;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(pa));
        fa[mb][kh] = v;
      }
  };
  auto mfmas = [&](const bf16x8 (&fa)[4][2], const bf16x8 (&fb)[4][2]) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mb][kh], fb[nb][kh], acc[mb][nb], 0, 0, 0);
  };
  // retire this wave's loads of step q (8 per step) while younger ones stay in flight
  const int64_t nst = (KT + HB_BK - 1) / HB_BK;
  auto wait_step = [&](int64_t q, int64_t issued_to) {  // steps <= issued_to have been issued
    int64_t younger = issued_to - q;
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  bf16x8 fa0[4][2], fb0[4][2], fa1[4][2], fb1[4][2];
  for (int64_t p = 0; p < HW_NS && p < nst; ++p) stage(p * HB_BK, lds + p * HB_STAGE);
  int64_t issued = (nst < HW_NS ? nst : HW_NS) - 1;
  if (nst > 0) {
    wait_step(0, issued);
    __builtin_amdgcn_s_barrier();
    read_frags(lds, fa0, fb0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  // K loop: (fa0, fb0) hold step p's fragments; step p+1's are read into
  // (fa1, fb1) while step p's MFMAs run, then moved down
  for (int64_t p = 0; p < nst; ++p) {
    if (p + 1 < nst) wait_step(p + 1, issued);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // every wave: step p+1 landed, step p's slot read
    __builtin_amdgcn_sched_barrier(0);
    if (p + HW_NS < nst) {
      stage((p + HW_NS) * HB_BK, lds + (p % HW_NS) * HB_STAGE);
      issued = p + HW_NS;
    }
    const bool more = p + 1 < nst;
    if (more) read_frags(lds + ((p + 1) % HW_NS) * HB_STAGE, fa1, fb1);
    mfmas(fa0, fb0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        fa0[i][kh] = fa1[i][kh];
        fb0[i][kh] = fb1[i][kh];
      }
  }

  // ---- epilogue: 32x32 C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  char* C = (char*)(uintptr_t)T->c;
  const int64_t ldc = T->ldc;
  const bool accum = T->accumulate != 0;
  const int64_t gn0 = n0 + wc * 128 + (lane & 31);
  const int64_t gm0 = m0 + wr * 128 + 4 * (lane >> 5);
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int64_t gn = gn0 + nb * 32;
      if (gn >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
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
      }
    }
}
