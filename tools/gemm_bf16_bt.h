// gemm_bf16_bt.h -- bf16 chained GEMM on a TRANSPOSED B image (probe; the
// segments' b point at B^T chunks, n x k row-major, ldb = the B^T row pitch).
// Same 256x256 tile, 8 waves, 4-slot global_load_lds ring and ping-pong
// schedule as the library's k_gemm_bf16_chain, but B^T is staged exactly
// like A ([n][32 k] 64-B rows, XOR-swizzled 16-B chunks) and its fragments
// are read with ds_read_b128 instead of ds_read_b64_tr_b16.  Every MFMA sees
// the same (row, col, 32-k slice) operands in the same K order, so the
// results are bit-identical to the library kernel's.
template <bool OUT_BF16, int GM = 4>
__global__ __launch_bounds__(512, 2) void k_gemm_bf16_bt(const cubed_gemm_chain_t* __restrict__ tasks,
                                                      const cubed_gemm_seg_t* __restrict__ segs,
                                                      int64_t tiles_m, int64_t tiles_n,
                                                      const char* __restrict__ zero) {
  constexpr int NS = HB_NS;
  __shared__ __attribute__((aligned(1024))) char lds_[NS * HB_STAGE];
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

  // staging: wave w stages rows 16*(2w+i) + lane>>2 of A and of B^T (i = 0,
  // 1); chunk lane&3 of the 64-B LDS row holds global chunk
  // (lane&3) ^ 2*((row>>3)&1)
  int64_t gmA[2], gnB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t r = 16 * (2 * w + i) + (lane >> 2);
    gmA[i] = (m0 + r < M ? m0 + r : M - 1);
    gnB[i] = (n0 + r < N ? n0 + r : N - 1);
  }
  const int dK = 8 * ((lane & 3) ^ (2 * ((lane >> 5) & 1)));

  int64_t s = seg0, ks = 0;
  Seg cur = load_seg(segs, s);
  int64_t ke = segs[s].k;
  int64_t offSA[2], offSB[2];
  auto seg_offsets = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      offSA[i] = gmA[i] * cur.lda2 + dK * 2;
      offSB[i] = gnB[i] * cur.ldb2 + dK * 2;
    }
  };
  seg_offsets();

  auto stage = [&](int64_t k0, CUBED_L char* buf) {
    const char* a0 = cur.a + (k0 - ks) * 2;
    const char* b0 = cur.b + (k0 - ks) * 2;
    const char* sa[2];
    const char* sb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sa[i] = a0 + offSA[i];
      sb[i] = b0 + offSB[i];
    }
    if (k0 + HB_BK > ke) {
      const bool has_next = s + 1 < segN;
      const Seg nxt = load_seg(segs, has_next ? s + 1 : s);
      const int64_t kk = k0 + dK;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const char* na = nxt.a + gmA[i] * nxt.lda2 + (kk - ke) * 2;
        const char* nb = nxt.b + gnB[i] * nxt.ldb2 + (kk - ke) * 2;
        const bool in_next = has_next && kk < KT;
        sa[i] = kk < ke ? sa[i] : (in_next ? na : zero);
        sb[i] = kk < ke ? sb[i] : (in_next ? nb : zero);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(sa[i], buf + (2 * w + i) * 1024);
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(sb[i], buf + HB_A + (2 * w + i) * 1024);
    if (k0 + HB_BK >= ke && s + 1 < segN) {
      ks = ke;
      ++s;
      cur = load_seg(segs, s);
      ke = ks + segs[s].k;
      seg_offsets();
    }
  };

  // fragment reads: row (A) / column (B^T) r, chunk (lane>>4) ^ 2*((lane>>3)&1)
  const int frag = (lane & 15) * 64 + 16 * ((lane >> 4) ^ (2 * ((lane >> 3) & 1)));
  const int offA = wr * 8192 + frag;
  const int offB = HB_A + wc * 4096 + frag;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t nst = (KT + HB_BK - 1) / HB_BK;
  constexpr int D = NS - 1;
  for (int64_t p = 0; p < D && p < nst; ++p) stage(p * HB_BK, lds + p * HB_STAGE);
  auto wait_step = [&](int64_t q) {
    int64_t younger = nst - 1 - q;
    if (younger > D - 1) younger = D - 1;
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  int rd = 0, wr_slot = D % NS;
  if (nst > 0) wait_step(0);
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  bf16x8 af[8], bf[4];
  for (int64_t p = 0; p < nst; ++p) {
    // ---- M(p)
    const CUBED_L char* bufc = lds + rd * HB_STAGE;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) bf[nb] = *(const CUBED_L bf16x8*)(bufc + offB + nb * 1024);
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) af[mb] = *(const CUBED_L bf16x8*)(bufc + offA + mb * 1024);
    if (p + D < nst) stage((p + D) * HB_BK, lds + wr_slot * HB_STAGE);
    rd = rd + 1 == NS ? 0 : rd + 1;
    wr_slot = wr_slot + 1 == NS ? 0 : wr_slot + 1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (p + 1 < nst) wait_step(p + 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- C(p)
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb], bf[nb], acc[mb][nb], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();

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

// B (k x n, row-major, pitch ld) -> B^T (n x k, pitch k) for every chunk:
// 64 x 64 tiles through LDS (probe only; the library uses cubed_copy_boxes'
// tile path)
__global__ __launch_bounds__(256) void k_transpose_bf16(const uint16_t* __restrict__ src,
                                                        uint16_t* __restrict__ dst, int64_t K,
                                                        int64_t Nn, int64_t slot, int64_t nchunks) {
  __shared__ uint16_t tile[64][65];
  const int64_t tk = (K + 63) / 64, tn = (Nn + 63) / 64;
  const int64_t per = tk * tn;
  const int64_t c = blockIdx.x / per, tt = blockIdx.x % per;
  if (c >= nchunks) return;
  const int64_t k0 = (tt / tn) * 64, n0 = (tt % tn) * 64;
  const uint16_t* s = src + c * (slot / 2);
  uint16_t* d = dst + c * (slot / 2);
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i / 64, q = i % 64;
    if (k0 + r < K && n0 + q < Nn) tile[r][q] = s[(k0 + r) * Nn + n0 + q];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i / 64, q = i % 64;  // r: n, q: k
    if (n0 + r < Nn && k0 + q < K) d[(n0 + r) * K + k0 + q] = tile[q][r];
  }
}

// ---------------------------------------------------------------------------
// k_gemm_bf16_a64: the library's ping-pong kernel (BK = 32 compute steps,
// B through a 4-slot ring of [32 k][256 n] images read by ds_read_b64_tr_b16)
// with A staged 64 k at a time in FULL 128-B lines: a 2-slot A ring of
// [256 rows][64 k] images (A tile a = steps 2a, 2a+1), staged at M(2a-2)
// for the next pair of steps.  A's global loads then fetch 8 rows x 128 B
// per wave instruction instead of 16 rows x 64 B (half lines).  Same MFMA
// operands in the same order: bit-identical results.
// A image: row r (128 B) holds 16-B chunk c at position c ^ ((r >> 1) & 7).
// Needs every segment's k >= 64 (one boundary per A tile at most).
template <bool OUT_BF16, int GM = 4>
__global__ __launch_bounds__(512, 2) void k_gemm_bf16_a64(const cubed_gemm_chain_t* __restrict__ tasks,
                                                       const cubed_gemm_seg_t* __restrict__ segs,
                                                       int64_t tiles_m, int64_t tiles_n,
                                                       const char* __restrict__ zero) {
  constexpr int NSB = 4;                     // B ring slots (32 k each)
  constexpr int SLOT_A = HB_BM * 64 * 2;     // 32 KiB
  constexpr int SLOT_B = HB_B;               // 16 KiB
  __shared__ __attribute__((aligned(1024))) char lds_[2 * SLOT_A + NSB * SLOT_B];
  CUBED_L char* ldsA = (CUBED_L char*)lds_;
  CUBED_L char* ldsB = ldsA + 2 * SLOT_A;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n, KT = T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- A staging: wave w instruction i (0..3) covers rows 8*(4w+i) + lane>>3,
  // LDS position lane&7 holds chunk (lane&7) ^ ((row>>1)&7)
  int64_t gmA[4];
  int kA[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 8 * (4 * w + i) + (lane >> 3);
    gmA[i] = (m0 + r < M ? m0 + r : M - 1);
    kA[i] = 8 * ((lane & 7) ^ ((r >> 1) & 7));
  }
  // ---- B staging (as the library kernel)
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

  // separate segment cursors for the A tiles (64 k) and the B steps (32 k)
  int64_t sA = seg0, ksA = 0, keA = segs[seg0].k;
  Seg curA = load_seg(segs, sA);
  int64_t sB = seg0, ksB = 0, keB = segs[seg0].k;
  Seg curB = load_seg(segs, sB);

  auto stageA = [&](int64_t k0, CUBED_L char* buf) {
    const char* sa[4];
    const bool cross = k0 + 64 > keA;  // uniform
    const bool has_next = sA + 1 < segN;
    const Seg nxt = load_seg(segs, (cross && has_next) ? sA + 1 : sA);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t ka = k0 + kA[i];
      const char* pc = curA.a + gmA[i] * curA.lda2 + (ka - ksA) * 2;
      const char* pn = nxt.a + gmA[i] * nxt.lda2 + (ka - keA) * 2;
      sa[i] = (!cross || ka < keA) ? pc : ((has_next && ka < KT) ? pn : zero);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(sa[i], buf + (4 * w + i) * 1024);
    if (k0 + 64 >= keA && sA + 1 < segN) {
      ksA = keA;
      ++sA;
      curA = load_seg(segs, sA);
      keA = ksA + segs[sA].k;
    }
  };
  auto stageB = [&](int64_t k0, CUBED_L char* buf) {
    const char* sb[2];
    const char* b0 = curB.b + (k0 - ksB) * curB.ldb2;
#pragma unroll
    for (int i = 0; i < 2; ++i) sb[i] = b0 + rB[i] * curB.ldb2 + gnB[i] * 2;
    if (k0 + HB_BK > keB) {
      const bool has_next = sB + 1 < segN;
      const Seg nxt = load_seg(segs, has_next ? sB + 1 : sB);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int64_t kb = k0 + rB[i];
        const char* nbp = nxt.b + (kb - keB) * nxt.ldb2 + gnB[i] * 2;
        sb[i] = kb < keB ? sb[i] : ((has_next && kb < KT) ? nbp : zero);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(sb[i], buf + (2 * w + i) * 1024);
    if (k0 + HB_BK >= keB && sB + 1 < segN) {
      ksB = keB;
      ++sB;
      curB = load_seg(segs, sB);
      keB = ksB + segs[sB].k;
    }
  };

  // ---- fragment offsets
  // A: row wr*128 + mb*16 + (lane&15), chunk 4*(p&1) + (lane>>4), row stride 128 B
  const int ra = wr * 128 + (lane & 15);
  const int swa = (ra >> 1) & 7;  // mb*16 keeps (row>>1)&7
  const int offA0 = ra * 128 + 16 * ((lane >> 4) ^ swa);
  const int offA1 = ra * 128 + 16 * ((4 + (lane >> 4)) ^ swa);
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int swzq = 2 * (q | ((g & 1) << 2));
  int offB[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    offB[nb] = (8 * g + q) * 512 + 16 * ((8 * wc + 2 * nb + (pp >> 1)) ^ swzq) + 8 * (pp & 1);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 bf[4], af[8];

  const int64_t nst = (KT + HB_BK - 1) / HB_BK;
  const int64_t nat = (KT + 63) / 64;
  // prologue: A tile 0, B steps 0..2
  stageA(0, ldsA);
  for (int64_t p = 0; p < 3 && p < nst; ++p) stageB(p * HB_BK, ldsB + p * SLOT_B);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  for (int64_t p = 0; p < nst; ++p) {
    // ---- M(p): step p's fragments; stage A tile p/2+1 (p even) and B step p+3
    const CUBED_L char* bufA = ldsA + ((p >> 1) & 1) * SLOT_A;
    const CUBED_L char* bufB = ldsB + (p & 3) * SLOT_B;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const uint32_t pb = (uint32_t)(uintptr_t)(bufB + offB[nb]);
      s16x4 lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(pb));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(hi) : "v"(pb));
      bf[nb] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
    const int offA = (p & 1) ? offA1 : offA0;
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) af[mb] = *(const CUBED_L bf16x8*)(bufA + offA + mb * 2048);
    const bool sa = !(p & 1) && (p >> 1) + 1 < nat;
    if (sa) stageA(((p >> 1) + 1) * 64, ldsA + (((p >> 1) + 1) & 1) * SLOT_A);
    if (p + 3 < nst) stageB((p + 3) * HB_BK, ldsB + ((p + 3) & 3) * SLOT_B);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // retire what step p+1 reads: steady state leaves B(p+2), B(p+3) [+ A]
    if (p + 1 < nst) {
      if (p + 4 < nst && (p & 1)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (p + 4 < nst && (p >> 1) + 1 < nat) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- C(p)
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb], bf[nb], acc[mb][nb], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();

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
