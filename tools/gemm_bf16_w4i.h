// gemm_bf16_w4i.h -- bf16 chained GEMM, ONE wave per SIMD, 128 x 128 per wave,
// with the K step hand-scheduled one filler per MFMA gap (round 5).
//
// tools/mfma_gap_probe.hip (profiles/r05_mfma_gap.log) measured what a
// filler costs beside v_mfma_f32_32x32x16_bf16 when one wave owns its SIMD:
// a conflict-free ds_read_b128 +16 cycles of its gap, a ds_read_b64_tr_b16
// +12, a global_load_lds piece +19, additive; the 32-MFMA step of a 128 x 128
// wave tile with its 24 fragment reads and 8 staging pieces one per gap runs
// 47 cycles per MFMA (1.37 PF at the probe's clocks) against the current
// ping-pong kernel's 1.09 PF.  The round-3 one-wave kernel (791 TF,
// tools/gemm_bf16_experiments.h k_gemm_bf16_w4) issued the same work in
// blocks: 8 staging pieces, then 24 reads, then 32 MFMAs.
//
// Layout (as k_gemm_bf16_w4): 256 x 256 tile per 256-thread workgroup, waves
// 2 (M) x 2 (N), each 4 x 4 accumulators of 32 x 32 (256 AGPRs); K staged 32
// deep by global_load_lds into a 4-slot ring (8 pieces of 1 KiB per wave per
// step); A slot image [256 rows][64 B] with chunk slot s of row r = k chunk
// s ^ ((r >> 2) & 3), B [32 k-rows][512 B] with chunk slot s of k-row r = col
// chunk s ^ 4 (r & 3): both fragment reads conflict-free.
//
// Step p (fragments of step p already in register set X):
//   wait this wave's loads of step p+1, barrier (every wave: step p+1
//   landed, step p's slot no longer read), compute step p+4's staging
//   addresses, then 32 MFMAs on set X with, in gap g, filler g of the
//   pattern [A read, B read, staging piece, B read] x 8 -- step p+1's 8 A and
//   16 B fragment reads into set Y, step p+4's 8 pieces into slot p % 4 --
//   and lgkmcnt(0).  The loop is unrolled by two so X / Y swap without moves.
#pragma once
#include <utility>

constexpr int W4_NS = 4;

// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>): a
// compile-time unrolled sequence (immediate LDS offsets need constants)
template <typename F, int... I>
__device__ __forceinline__ void seq_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void seq(F&& f) {
  seq_(f, std::make_integer_sequence<int, N>{});
}

// STAMP: diagnostic build -- lane 0 of each wave stores the K loop's cycles
// (s_memtime) and its step count to stamp_out[(block * 4 + wave) * 2]
// ABL (probe ablations, results wrong when nonzero): 1 no K-loop barrier,
// 2 no staging pieces in the stream, 4 no fragment reads in the stream,
// 8 no staging-address update, 16 A staging addresses never advance (B's do),
// 32 B staging addresses never advance (A's do)
template <bool OUT_BF16, int GM = 4, bool STAMP = false, int ABL = 0, int NS = W4_NS>
__global__ __launch_bounds__(256, 1) void k_gemm_bf16_w4i(const cubed_gemm_chain_t* __restrict__ tasks,
                                                        const cubed_gemm_seg_t* __restrict__ segs,
                                                        int64_t tiles_m, int64_t tiles_n,
                                                        const char* __restrict__ zero, GemmGrid,
                                                        unsigned long long* __restrict__ stamp_out) {
  static_assert(NS >= 3 && NS * HB_STAGE <= 160 * 1024, "ring of 3..5 32-KiB slots");
  __shared__ __attribute__((aligned(1024))) char lds_[NS * HB_STAGE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n;
  const int32_t KT = (int32_t)T->ktot;  // K positions fit 32 bits: compares stay on the scalar unit
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;

  // ---- staging geometry: piece i (0..3) of wave w fills 1 KiB of a slot
  int64_t gmA[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t r = m0 + 16 * (4 * w + i) + (lane >> 2);
    gmA[i] = r < M ? r : M - 1;
  }
  const int dA = 8 * ((lane & 3) ^ ((lane >> 4) & 3));
  int rB[4];
  int64_t gnB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 2 * (4 * w + i) + (lane >> 5);
    rB[i] = r;
    const int64_t n = n0 + 8 * ((lane & 31) ^ (4 * (r & 3)));
    gnB[i] = n + 8 <= N ? n : N - 8;
  }

  int64_t s = seg0;
  int32_t ks = 0;
  Seg cur = load_seg(segs, s);
  int32_t ke = (int32_t)segs[s].k;
  int64_t offSA[4], offSB[4];
  auto seg_offsets = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      offSA[i] = gmA[i] * cur.lda2 + dA * 2;
      offSB[i] = rB[i] * cur.ldb2 + gnB[i] * 2;
    }
  };
  seg_offsets();
  // the 8 staging sources of the step starting at k0 (A pieces 0-3, B 4-7),
  // as integers: pointer selects through a private array spilled to scratch
  uint64_t st[8];
  bool inc_ok = false;  // st[] holds the previous step of the same segment: advance by one step
  // the step's sources from scratch, with the per-lane selects of a step that
  // crosses a segment boundary (or the chain's end: a zero page)
  auto stage_full = [&](int32_t k0) __attribute__((always_inline)) {
    inc_ok = k0 + HB_BK <= ke;
    const uint64_t a0 = (uint64_t)(uintptr_t)cur.a + (uint64_t)((int64_t)(k0 - ks) * 2);
    const uint64_t b0 = (uint64_t)(uintptr_t)cur.b + (uint64_t)((int64_t)(k0 - ks) * cur.ldb2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st[i] = a0 + (uint64_t)offSA[i];
      st[4 + i] = b0 + (uint64_t)offSB[i];
    }
    if (k0 + HB_BK > ke) {  // uniform: a segment boundary (or the chain's end) in this step
      const bool has_next = s + 1 < segN;
      const Seg nxt = load_seg(segs, has_next ? s + 1 : s);
      const uint64_t z = (uint64_t)(uintptr_t)zero;
      const int32_t ka = k0 + dA;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint64_t na = (uint64_t)(uintptr_t)nxt.a + (uint64_t)(gmA[i] * nxt.lda2 + (int64_t)(ka - ke) * 2);
        const uint64_t alt_a = (has_next && ka < KT) ? na : z;
        st[i] = ka < ke ? st[i] : alt_a;
        const int32_t kb = k0 + rB[i];
        const uint64_t nbp = (uint64_t)(uintptr_t)nxt.b + (uint64_t)((int64_t)(kb - ke) * nxt.ldb2 + gnB[i] * 2);
        const uint64_t alt_b = (has_next && kb < KT) ? nbp : z;
        st[4 + i] = kb < ke ? st[4 + i] : alt_b;
      }
    }
  };
  // after the step starting at k0 was staged: move to the next segment when
  // the next step starts in it
  auto seg_advance = [&](int32_t k0) __attribute__((always_inline)) {
    if (k0 + HB_BK >= ke && s + 1 < segN) {
      ks = ke;
      ++s;
      cur = load_seg(segs, s);
      ke = ks + (int32_t)segs[s].k;
      seg_offsets();
      inc_ok = false;
    }
  };
  auto stage_addrs = [&](int32_t k0) __attribute__((always_inline)) {
    if (inc_ok && k0 + HB_BK <= ke) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st[i] += 2 * HB_BK;
        st[4 + i] += (uint64_t)(HB_BK * cur.ldb2);
      }
    } else {
      stage_full(k0);
    }
    seg_advance(k0);
  };
  auto piece = [&](int i, CUBED_L char* buf) __attribute__((always_inline)) {
    glds16((const char*)(uintptr_t)st[i], buf + (i < 4 ? (4 * w + i) * 1024 : HB_A + (4 * w + i - 4) * 1024));
  };

  // ---- fragment read offsets inside a slot
  const int ra = wr * 128 + (lane & 31);
  int offA[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) offA[kh] = ra * 64 + 16 * ((kh * 2 + (lane >> 5)) ^ ((ra >> 2) & 3));
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

  struct Frags {
    bf16x8 a[4][2];
    s16x4 bl[4][2], bh[4][2];
  };
  // A read q (0..7): (mb, kh) = (q & 3, q >> 2), at base A[kh] + mb * 2048 (an
  // immediate offset); B read j (0..15): nb = (j >> 1) & 3, kh = j >> 3, half
  // = j & 1, at base B[nb] + kh * 8192 (+ 2048 for the high half)
  struct Bases {
    uint32_t a[2], b[4];
  } lb;
  auto set_bases = [&](const CUBED_L char* buf) __attribute__((always_inline)) {
    const uint32_t b = (uint32_t)(uintptr_t)buf;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) lb.a[kh] = b + offA[kh];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) lb.b[nb] = b + offB[nb];
  };
  auto read_a = [](auto Q, Frags& f, const Bases& bs) __attribute__((always_inline)) {
    constexpr int q = decltype(Q)::value;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.a[q & 3][q >> 2]) : "v"(bs.a[q >> 2]), "i"((q & 3) * 2048));
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
    seq<16>([&](auto J) __attribute__((always_inline)) { read_b(J, f, lb); });
    seq<8>([&](auto Q) __attribute__((always_inline)) { read_a(Q, f, lb); });
  };
  // MFMA g (0..31): kh = g >> 4, mb = (g >> 2) & 3, nb = g & 3
  auto mfma = [](auto G, const Frags& f, f32x16 (&ac)[4][4]) __attribute__((always_inline)) {
    constexpr int g = decltype(G)::value, kh = g >> 4, mb = (g >> 2) & 3, nb = g & 3;
    const bf16x8 b = __builtin_bit_cast(bf16x8, __builtin_shufflevector(f.bl[nb][kh], f.bh[nb][kh], 0, 1, 2, 3,
                                                                        4, 5, 6, 7));
    ac[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[mb][kh], b, ac[mb][nb], 0, 0, 0);
  };

  const int64_t nst = (KT + HB_BK - 1) / HB_BK;
  auto wait_step = [&](int64_t q, int64_t issued_to) __attribute__((always_inline)) {  // steps <= issued_to issued
    const int64_t younger = issued_to - q;
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  int64_t issued = -1;
  // a steady-state K step (p + 4 < nst): MFMAs on X; in gap g one filler of
  // [A read, B read, staging piece, B read] x 8 -- step p+1's fragments into
  // Y, step p+4's pieces into slot p % 4
  auto full_step = [&](int64_t p, const Frags& X, Frags& Y) __attribute__((always_inline)) {
    // steps p+1 .. p+NS-1 in flight (the last staged by the previous step):
    // step p+1's 8 pieces have landed once at most 8 (NS - 2) are outstanding
    if constexpr (!(ABL & 2)) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(8 * (NS - 2)) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!(ABL & 1)) __builtin_amdgcn_s_barrier();  // every wave: step p+1 landed, step p's slot read
    __builtin_amdgcn_sched_barrier(0);
    CUBED_L char* wslot = lds + (p % NS) * HB_STAGE;
    set_bases(lds + ((p + 1) % NS) * HB_STAGE);
    const int32_t k0 = (int32_t)((p + NS) * HB_BK);
    // steady state: each source advances by one step, in the gap before its
    // piece; otherwise (a segment edge) recompute them first
    const bool inc = (ABL & 8) || (inc_ok && k0 + HB_BK <= ke);
    if (!inc) stage_full(k0);
    const uint64_t dB = (uint64_t)(HB_BK * cur.ldb2);
    issued = p + NS;
    __builtin_amdgcn_sched_barrier(0);
    seq<32>([&](auto G) __attribute__((always_inline)) {
      constexpr int g = decltype(G)::value, r = g & 3, i = g >> 2;
      mfma(G, X, acc);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (r == 0) { if constexpr (!(ABL & 4)) read_a(std::integral_constant<int, i>{}, Y, lb); }
      else if constexpr (r == 1) {
        if constexpr (!(ABL & 4)) read_b(std::integral_constant<int, 2 * i>{}, Y, lb);
        if constexpr (!(ABL & 8) && !((ABL & 16) && i < 4) && !((ABL & 32) && i >= 4))
          if (inc) st[i] += i < 4 ? (uint64_t)(2 * HB_BK) : dB;
      }
      else if constexpr (r == 2) { if constexpr (!(ABL & 2)) piece(i, wslot); }
      else { if constexpr (!(ABL & 4)) read_b(std::integral_constant<int, 2 * i + 1>{}, Y, lb); }
      __builtin_amdgcn_sched_barrier(0);
    });
    seg_advance(k0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  // the last steps: whatever remains to stage / read, issued plainly
  auto tail_step = [&](int64_t p, const Frags& X, Frags& Y) __attribute__((always_inline)) {
    if (p + 1 < nst) wait_step(p + 1, issued);
    __builtin_amdgcn_s_barrier();
    if (p + NS < nst) {
      stage_addrs((int32_t)((p + NS) * HB_BK));
#pragma unroll
      for (int i = 0; i < 8; ++i) piece(i, lds + (p % NS) * HB_STAGE);
      issued = p + NS;
    }
    if (p + 1 < nst) {
      set_bases(lds + ((p + 1) % NS) * HB_STAGE);
      read_all(Y);
    }
    seq<32>([&](auto G) __attribute__((always_inline)) { mfma(G, X, acc); });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  Frags f0, f1;
  for (int64_t p = 0; p < NS && p < nst; ++p) {
    stage_addrs((int32_t)(p * HB_BK));
#pragma unroll
    for (int i = 0; i < 8; ++i) piece(i, lds + p * HB_STAGE);
    issued = p;
  }
  if (nst > 0) {
    wait_step(0, issued);
    __builtin_amdgcn_s_barrier();
    set_bases(lds);
    read_all(f0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  int64_t p = 0;
  unsigned long long t0 = 0, t1 = 0;
  if constexpr (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (; p + 1 + NS < nst; p += 2) {
    full_step(p, f0, f1);
    full_step(p + 1, f1, f0);
  }
  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (lane == 0) {
      stamp_out[(blockIdx.x * 4 + w) * 2] = t1 - t0;
      stamp_out[(blockIdx.x * 4 + w) * 2 + 1] = (unsigned long long)p;
    }
  }
  for (; p < nst; ++p) {
    tail_step(p, f0, f1);
    f0 = f1;
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
