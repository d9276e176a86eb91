// gemm_bf16_stamp.h -- DIAGNOSTIC build of the library's ping-pong bf16
// kernel (generated copy of k_gemm_bf16_chain's PP = 1 branch) with
// s_memtime stamps around each part of a K step: M = fragment reads (0-1),
// staging issue (1-2), lgkmcnt + vmcnt waits (2-3), barrier into C (3-4),
// MFMA issue (4-5), barrier out of C (5-0).  Each wave sums the segment
// lengths in scalar registers and lane 0 stores them once (vector store)
// into dbg[(block * 8 + wave) * 8 + seg].  Timing of this build is not the
// kernel's: read the shares.
#define STAMP(i) do { \
    unsigned long long t_; \
    __builtin_amdgcn_sched_barrier(0); \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_) :: "memory"); \
    __builtin_amdgcn_sched_barrier(0); \
    if (i != 0 || have_) sums_[(i + 5) % 6] += t_ - last_; \
    last_ = t_; have_ = true; } while (0)
template <bool OUT_BF16, int ABL = 0, int PP = 1, int NS = HB_NS, int GM = 4>
__global__ __launch_bounds__(512, 2) void k_gemm_bf16_stamp(unsigned long long* __restrict__ dbg, const cubed_gemm_chain_t* __restrict__ tasks,
                                                         const cubed_gemm_seg_t* __restrict__ segs,
                                                         int64_t tiles_m, int64_t tiles_n,
                                                         const char* __restrict__ zero) {
  __shared__ __attribute__((aligned(1024))) char lds_[NS * HB_STAGE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  unsigned long long sums_[6] = {0, 0, 0, 0, 0, 0}, last_ = 0;
  bool have_ = false;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n, KT = T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- per-lane staging geometry (constant over the K loop)
  // A: wave w stages rows 16*(2w+i) + lane>>2 (i = 0, 1); 16-B chunk lane&3 of
  // the 64-B LDS row holds global chunk (lane&3) ^ 2*((row>>3)&1)
  // [(row>>3)&1 = (lane>>5)&1], which makes the fragment reads conflict-free.
  int64_t gmA[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t r = 16 * (2 * w + i) + (lane >> 2);
    gmA[i] = (m0 + r < M ? m0 + r : M - 1);
  }
  const int dA = 8 * ((lane & 3) ^ (2 * ((lane >> 5) & 1)));
  // B: wave w stages k-rows 2*(2w+i) + lane>>5; 16-B chunk c = lane&31 of the
  // LDS row holds global chunk c ^ swz(row), swz(r) = 2*((r&3) | ((r>>3)&1)<<2).
  int rB[2];
  int64_t gnB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 2 * (2 * w + i) + (lane >> 5);
    rB[i] = r;
    const int swz = 2 * ((r & 3) | (((r >> 3) & 1) << 2));
    int64_t n = n0 + 8 * ((lane & 31) ^ swz);
    gnB[i] = (n + 8 <= N ? n : N - 8);
  }

  // ---- wave-uniform segment state (the segment containing the next step to stage)
  int64_t s = seg0, ks = 0;
  Seg cur = load_seg(segs, s);
  int64_t ke = segs[s].k;

  // per-lane byte offsets of this lane's 4 pieces inside the current segment
  // (recomputed only when the segment changes)
  int64_t offSA[2], offSB[2];
  auto seg_offsets = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      offSA[i] = gmA[i] * cur.lda2 + dA * 2;
      offSB[i] = rB[i] * cur.ldb2 + gnB[i] * 2;
    }
  };
  seg_offsets();

  // the 4 global->LDS loads of the K step starting at k0 into slot buf:
  // sources / destinations (stage_addrs) and their issue
  const char* st_src[4];
  CUBED_L char* st_dst[4];
  auto stage_addrs = [&](int64_t k0, CUBED_L char* buf) {
    const char* a0 = cur.a + (k0 - ks) * 2;        // uniform
    const char* b0 = cur.b + (k0 - ks) * cur.ldb2;  // uniform
    const char* sa[2];
    const char* sb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sa[i] = a0 + offSA[i];
      sb[i] = b0 + offSB[i];
    }
    if (k0 + HB_BK > ke) {  // uniform: a segment boundary (or the chain's end) inside this step
      const bool has_next = s + 1 < segN;
      const Seg nxt = load_seg(segs, has_next ? s + 1 : s);
      const int64_t ka = k0 + dA;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const char* na = nxt.a + gmA[i] * nxt.lda2 + (ka - ke) * 2;
        sa[i] = ka < ke ? sa[i] : ((has_next && ka < KT) ? na : zero);
        const int64_t kb = k0 + rB[i];
        const char* nbp = nxt.b + (kb - ke) * nxt.ldb2 + gnB[i] * 2;
        sb[i] = kb < ke ? sb[i] : ((has_next && kb < KT) ? nbp : zero);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      st_src[i] = sa[i];
      st_dst[i] = buf + (2 * w + i) * 1024;
      st_src[2 + i] = sb[i];
      st_dst[2 + i] = buf + HB_A + (2 * w + i) * 1024;
    }
    // the next step to stage starts at k0 + HB_BK: move on if it is in the next segment
    if (k0 + HB_BK >= ke && s + 1 < segN) {
      ks = ke;
      ++s;
      cur = load_seg(segs, s);
      ke = ks + segs[s].k;
      seg_offsets();
    }
  };
  auto stage = [&](int64_t k0, CUBED_L char* buf) {
    stage_addrs(k0, buf);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(st_src[i], st_dst[i]);
  };

  // ---- per-lane LDS read offsets (within a slot)
  // A fragment mb: row wr*128 + mb*16 + (lane&15), chunk (lane>>4) ^ 2*((lane>>3)&1)
  const int offA = wr * 8192 + (lane & 15) * 64 + 16 * ((lane >> 4) ^ (2 * ((lane >> 3) & 1)));
  // B fragment (nb, half): row 8g + 4*half + q, chunk (8wc + 2nb + (p>>1)) ^ swz
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int swzq = 2 * (q | ((g & 1) << 2));
  int offB[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    offB[nb] = HB_A + (8 * g + q) * 512 + 16 * ((8 * wc + 2 * nb + (pp >> 1)) ^ swzq) + 8 * (pp & 1);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 bf[4];

  const int64_t nst = (KT + HB_BK - 1) / HB_BK;
  constexpr int D = NS - 1;  // steps staged ahead
  // prologue: steps 0 .. D-1 in flight (LDS-DMA schedules)
  if constexpr (PP != 2)
    for (int64_t p = 0; p < D && p < nst; ++p) stage(p * HB_BK, lds + p * HB_STAGE);
  // retire this wave's loads of step q (4 per step; steps up to q + D - 1 issued)
  auto wait_step = [&](int64_t q) {
    int64_t younger = nst - 1 - q;
    if (younger > D - 1) younger = D - 1;
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  int rd = 0, wr_slot = D % NS;  // ring slots of steps p and p + D
  {
    // Ping-pong: the two wave rows (wr = 0, 1: one wave of each per SIMD)
    // run one barrier-delimited slot apart, alternating a memory slot M(p)
    // -- step p's fragments into registers, step p+3's global->LDS loads --
    // and a compute slot C(p) of 32 MFMAs, so each SIMD's matrix core is fed
    // by one wave while the other reads LDS.  Global slot 2p: row 0 in M(p),
    // row 1 in C(p-1); slot 2p+1: row 0 in C(p), row 1 in M(p).
    // RAW: every wave retires its step p+1 loads at the end of M(p) (slot 2p
    //   or 2p+1), before the barrier ending slot 2p+1; step p+1 is read in
    //   slot 2p+2 at the earliest.
    // WAR: M(p) restages slot (p+3)%4 = step p-1's, whose last reader (row 1,
    //   M(p-1), slot 2p-1) retired its reads (lgkmcnt(0)) before the barrier
    //   ending slot 2p-1.
    if (nst > 0) wait_step(0);
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 af[8];
    for (int64_t p = 0; p < nst; ++p) {
      // ---- M(p)
      STAMP(0);
      const CUBED_L char* bufc = lds + rd * HB_STAGE;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const uint32_t pb = (uint32_t)(uintptr_t)(bufc + offB[nb]);
        s16x4 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(pb));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(hi) : "v"(pb));
        bf[nb] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) af[mb] = *(const CUBED_L bf16x8*)(bufc + offA + mb * 1024);
      STAMP(1);
      if (!(ABL & 1) && p + D < nst) stage((ABL & 32) ? 0 : (p + D) * HB_BK, lds + wr_slot * HB_STAGE);
      rd = rd + 1 == NS ? 0 : rd + 1;
      wr_slot = wr_slot + 1 == NS ? 0 : wr_slot + 1;
      STAMP(2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (!(ABL & 16) && p + 1 < nst) wait_step(p + 1);
      STAMP(3);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- C(p)
      STAMP(4);
#pragma unroll
      for (int mb = 0; mb < 8; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb], bf[nb], acc[mb][nb], 0, 0, 0);
      STAMP(5);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    STAMP(0);
    if (wr == 0) __builtin_amdgcn_s_barrier();  // same barrier count in both rows
  }

  if (lane == 0) {
    unsigned long long* o = dbg + ((int64_t)blockIdx.x * 8 + w) * 8;
#pragma unroll
    for (int i = 0; i < 6; ++i) o[i] = sums_[i];
  }
  // ---- epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r
  char* C = (char*)(uintptr_t)T->c;
  const int64_t ldc = T->ldc;
  const bool accum = T->accumulate != 0;
#pragma unroll
  for (int mb = 0; mb < 8; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + wr * 128 + mb * 16 + (lane >> 4) * 4 + r;
        const int64_t gn = n0 + wc * 64 + nb * 16 + (lane & 15);
        if (gm < M && gn < N) {
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


// the same with step p+3's loads issued between the MFMAs of C(p)
template <bool OUT_BF16, int ABL = 0, int PP = 1, int NS = HB_NS, int GM = 4>
__global__ __launch_bounds__(512, 2) void k_gemm_bf16_stamp_cs(unsigned long long* __restrict__ dbg, const cubed_gemm_chain_t* __restrict__ tasks,
                                                         const cubed_gemm_seg_t* __restrict__ segs,
                                                         int64_t tiles_m, int64_t tiles_n,
                                                         const char* __restrict__ zero) {
  __shared__ __attribute__((aligned(1024))) char lds_[NS * HB_STAGE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  unsigned long long sums_[6] = {0, 0, 0, 0, 0, 0}, last_ = 0;
  bool have_ = false;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n, KT = T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- per-lane staging geometry (constant over the K loop)
  // A: wave w stages rows 16*(2w+i) + lane>>2 (i = 0, 1); 16-B chunk lane&3 of
  // the 64-B LDS row holds global chunk (lane&3) ^ 2*((row>>3)&1)
  // [(row>>3)&1 = (lane>>5)&1], which makes the fragment reads conflict-free.
  int64_t gmA[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t r = 16 * (2 * w + i) + (lane >> 2);
    gmA[i] = (m0 + r < M ? m0 + r : M - 1);
  }
  const int dA = 8 * ((lane & 3) ^ (2 * ((lane >> 5) & 1)));
  // B: wave w stages k-rows 2*(2w+i) + lane>>5; 16-B chunk c = lane&31 of the
  // LDS row holds global chunk c ^ swz(row), swz(r) = 2*((r&3) | ((r>>3)&1)<<2).
  int rB[2];
  int64_t gnB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 2 * (2 * w + i) + (lane >> 5);
    rB[i] = r;
    const int swz = 2 * ((r & 3) | (((r >> 3) & 1) << 2));
    int64_t n = n0 + 8 * ((lane & 31) ^ swz);
    gnB[i] = (n + 8 <= N ? n : N - 8);
  }

  // ---- wave-uniform segment state (the segment containing the next step to stage)
  int64_t s = seg0, ks = 0;
  Seg cur = load_seg(segs, s);
  int64_t ke = segs[s].k;

  // per-lane byte offsets of this lane's 4 pieces inside the current segment
  // (recomputed only when the segment changes)
  int64_t offSA[2], offSB[2];
  auto seg_offsets = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      offSA[i] = gmA[i] * cur.lda2 + dA * 2;
      offSB[i] = rB[i] * cur.ldb2 + gnB[i] * 2;
    }
  };
  seg_offsets();

  // the 4 global->LDS loads of the K step starting at k0 into slot buf:
  // sources / destinations (stage_addrs) and their issue
  const char* st_src[4];
  CUBED_L char* st_dst[4];
  auto stage_addrs = [&](int64_t k0, CUBED_L char* buf) {
    const char* a0 = cur.a + (k0 - ks) * 2;        // uniform
    const char* b0 = cur.b + (k0 - ks) * cur.ldb2;  // uniform
    const char* sa[2];
    const char* sb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sa[i] = a0 + offSA[i];
      sb[i] = b0 + offSB[i];
    }
    if (k0 + HB_BK > ke) {  // uniform: a segment boundary (or the chain's end) inside this step
      const bool has_next = s + 1 < segN;
      const Seg nxt = load_seg(segs, has_next ? s + 1 : s);
      const int64_t ka = k0 + dA;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const char* na = nxt.a + gmA[i] * nxt.lda2 + (ka - ke) * 2;
        sa[i] = ka < ke ? sa[i] : ((has_next && ka < KT) ? na : zero);
        const int64_t kb = k0 + rB[i];
        const char* nbp = nxt.b + (kb - ke) * nxt.ldb2 + gnB[i] * 2;
        sb[i] = kb < ke ? sb[i] : ((has_next && kb < KT) ? nbp : zero);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      st_src[i] = sa[i];
      st_dst[i] = buf + (2 * w + i) * 1024;
      st_src[2 + i] = sb[i];
      st_dst[2 + i] = buf + HB_A + (2 * w + i) * 1024;
    }
    // the next step to stage starts at k0 + HB_BK: move on if it is in the next segment
    if (k0 + HB_BK >= ke && s + 1 < segN) {
      ks = ke;
      ++s;
      cur = load_seg(segs, s);
      ke = ks + segs[s].k;
      seg_offsets();
    }
  };
  auto stage = [&](int64_t k0, CUBED_L char* buf) {
    stage_addrs(k0, buf);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(st_src[i], st_dst[i]);
  };

  // ---- per-lane LDS read offsets (within a slot)
  // A fragment mb: row wr*128 + mb*16 + (lane&15), chunk (lane>>4) ^ 2*((lane>>3)&1)
  const int offA = wr * 8192 + (lane & 15) * 64 + 16 * ((lane >> 4) ^ (2 * ((lane >> 3) & 1)));
  // B fragment (nb, half): row 8g + 4*half + q, chunk (8wc + 2nb + (p>>1)) ^ swz
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int swzq = 2 * (q | ((g & 1) << 2));
  int offB[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    offB[nb] = HB_A + (8 * g + q) * 512 + 16 * ((8 * wc + 2 * nb + (pp >> 1)) ^ swzq) + 8 * (pp & 1);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 bf[4];

  const int64_t nst = (KT + HB_BK - 1) / HB_BK;
  constexpr int D = NS - 1;  // steps staged ahead
  // prologue: steps 0 .. D-1 in flight (LDS-DMA schedules)
  if constexpr (PP != 2)
    for (int64_t p = 0; p < D && p < nst; ++p) stage(p * HB_BK, lds + p * HB_STAGE);
  // retire this wave's loads of step q (4 per step; steps up to q + D - 1 issued)
  auto wait_step = [&](int64_t q) {
    int64_t younger = nst - 1 - q;
    if (younger > D - 1) younger = D - 1;
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  int rd = 0, wr_slot = D % NS;  // ring slots of steps p and p + D
  {
    // Ping-pong: the two wave rows (wr = 0, 1: one wave of each per SIMD)
    // run one barrier-delimited slot apart, alternating a memory slot M(p)
    // -- step p's fragments into registers, step p+3's global->LDS loads --
    // and a compute slot C(p) of 32 MFMAs, so each SIMD's matrix core is fed
    // by one wave while the other reads LDS.  Global slot 2p: row 0 in M(p),
    // row 1 in C(p-1); slot 2p+1: row 0 in C(p), row 1 in M(p).
    // RAW: every wave retires its step p+1 loads at the end of M(p) (slot 2p
    //   or 2p+1), before the barrier ending slot 2p+1; step p+1 is read in
    //   slot 2p+2 at the earliest.
    // WAR: M(p) restages slot (p+3)%4 = step p-1's, whose last reader (row 1,
    //   M(p-1), slot 2p-1) retired its reads (lgkmcnt(0)) before the barrier
    //   ending slot 2p-1.
    if (nst > 0) wait_step(0);
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 af[8];
    for (int64_t p = 0; p < nst; ++p) {
      // ---- M(p)
      STAMP(0);
      const CUBED_L char* bufc = lds + rd * HB_STAGE;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const uint32_t pb = (uint32_t)(uintptr_t)(bufc + offB[nb]);
        s16x4 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(pb));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(hi) : "v"(pb));
        bf[nb] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) af[mb] = *(const CUBED_L bf16x8*)(bufc + offA + mb * 1024);
      STAMP(1);
      const bool st = p + D < nst;
      if (st) stage_addrs((p + D) * HB_BK, lds + wr_slot * HB_STAGE);
      rd = rd + 1 == NS ? 0 : rd + 1;
      wr_slot = wr_slot + 1 == NS ? 0 : wr_slot + 1;
      STAMP(2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (p + 1 < nst) {
        if (p + 2 < nst) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      STAMP(3);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- C(p)
      STAMP(4);
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb], bf[nb], acc[mb][nb], 0, 0, 0);
        if (mb & 1) {
          __builtin_amdgcn_sched_barrier(0);
          if (st) glds16(st_src[mb >> 1], st_dst[mb >> 1]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      STAMP(5);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    STAMP(0);
    if (wr == 0) __builtin_amdgcn_s_barrier();  // same barrier count in both rows
  }

  if (lane == 0) {
    unsigned long long* o = dbg + ((int64_t)blockIdx.x * 8 + w) * 8;
#pragma unroll
    for (int i = 0; i < 6; ++i) o[i] = sums_[i];
  }
  // ---- epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r
  char* C = (char*)(uintptr_t)T->c;
  const int64_t ldc = T->ldc;
  const bool accum = T->accumulate != 0;
#pragma unroll
  for (int mb = 0; mb < 8; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + wr * 128 + mb * 16 + (lane >> 4) * 4 + r;
        const int64_t gn = n0 + wc * 64 + nb * 16 + (lane & 15);
        if (gm < M && gn < N) {
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

