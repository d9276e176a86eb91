// gemm_bf16_8ph.h -- bf16 chained GEMM, the guide's 256^2 8-phase schedule on
// a TRANSPOSED B image (probe; segments' b point at B^T chunks, n x k
// row-major, ldb = the B^T row pitch).
//
// Tile 256 x 256, K tiles 64 deep, 8 waves 2 (M) x 4 (N), each 128 x 64 =
// 8 x 4 accumulators of 16 x 16 (v_mfma_f32_16x16x32_bf16).  LDS: two K-tile
// buffers of 64 KiB, each an A image [256 rows][64 k] and a B^T image
// [256 n][64 k] in full 128-B rows (16-B chunk c of row r at position
// c ^ ((r >> 1) & 7): conflict-free ds_read_b128 fragments), filled by
// global_load_lds in half-tiles (128 rows of one operand = 2 loads per
// thread).  A K tile is consumed in four phases, one accumulator quadrant
// (4 row blocks x 2 column blocks x 2 k halves = 16 MFMAs) each:
//   q0: read A(rows 0-63 of the wave), B(cols 0-31)       MFMA (qm0, qn0)
//   q1: read B(cols 32-63); stage A1(t+1)                 MFMA (qm0, qn1)
//   q2: read A(rows 64-127); stage B0(t+2)                MFMA (qm1, qn1)
//   q3: no reads; stage B1(t+2), A0(t+2); wait tile t+1   MFMA (qm1, qn0)
// Each phase is {ds_reads + stage; lgkmcnt(0); s_barrier; MFMAs; s_barrier}
// and the two wave rows run one barrier apart, so on every SIMD one wave's
// MFMAs overlap the other's reads and staging.
// RAW: tile t+1's last half (A1, staged in q1 of tile t) is retired by each
//   wave's vmcnt(6) in q3 of tile t (6 younger loads: B0, B1, A0 of t+2),
//   before the barrier both rows pass ahead of tile t+1's first reads.
// WAR: B halves of tile t are last read in q1 (B(qn0) is kept in registers
//   for q3) and restaged (tile t+2) from q2; A halves last read in q2,
//   restaged from q3; every read is retired (lgkmcnt(0)) before the barrier
//   that ends its phase, so the restaging wave issues after it.
// Same MFMA operands in the same order per accumulator as the library
// kernel: bit-identical results.
template <bool OUT_BF16, int GM = 4, bool PRIO = true>
__global__ __launch_bounds__(512, 2) void k_gemm_bf16_8ph(const cubed_gemm_chain_t* __restrict__ tasks,
                                                       const cubed_gemm_seg_t* __restrict__ segs,
                                                       int64_t tiles_m, int64_t tiles_n,
                                                       const char* __restrict__ zero) {
  constexpr int BUF = 65536, BOFF = 32768, HALF = 16384;
  __shared__ __attribute__((aligned(1024))) char lds_[2 * BUF];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t, m0, n0;
  tile_of<256, 256, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n, KT = T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- staging cursors: `lead` serves B0/B1/A0 of a tile, `lag` its A1 one
  // K tile later (segment containing the tile's first k; a boundary inside a
  // tile is a per-lane select into the next segment)
  struct Cur {
    int64_t s, ks, ke;
    Seg cur;
  };
  Cur lead;
  lead.s = seg0;
  lead.ks = 0;
  lead.ke = segs[seg0].k;
  lead.cur = load_seg(segs, seg0);
  Cur lag = lead;
  auto advance = [&](Cur& c, int64_t k_end) {
    if (k_end >= c.ke && c.s + 1 < segN) {
      c.ks = c.ke;
      ++c.s;
      c.cur = load_seg(segs, c.s);
      c.ke = c.ks + segs[c.s].k;
    }
  };
  // half h (0 = B0, 1 = B1, 2 = A0, 3 = A1) of K tile tt into buffer buf
  auto stage_half = [&](const Cur& c, int h, int64_t tt, CUBED_L char* buf) {
    const bool isA = h >= 2;
    const int hh = h & 1;
    const int64_t k0 = tt * 64;
    const int64_t lim = isA ? M : N;
    const int64_t rbase = (isA ? m0 : n0) + hh * 128 + 16 * w + (lane >> 3);
    const char* op = isA ? c.cur.a : c.cur.b;
    const int64_t ld2 = isA ? c.cur.lda2 : c.cur.ldb2;
    CUBED_L char* dst = buf + (isA ? 0 : BOFF) + hh * HALF + (2 * w) * 1024;
    if (k0 + 64 <= c.ke) {  // uniform: the whole tile inside the segment
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        int64_t r = rbase + 8 * i;
        r = r < lim ? r : lim - 1;
        const int kc = 8 * ((lane & 7) ^ (4 * i + (lane >> 4)));
        glds16(op + r * ld2 + (k0 + kc - c.ks) * 2, dst + i * 1024);
      }
    } else {
      const bool has_next = c.s + 1 < segN;
      const Seg nx = load_seg(segs, has_next ? c.s + 1 : c.s);
      const char* opn = isA ? nx.a : nx.b;
      const int64_t ldn = isA ? nx.lda2 : nx.ldb2;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        int64_t r = rbase + 8 * i;
        r = r < lim ? r : lim - 1;
        const int64_t kl = k0 + 8 * ((lane & 7) ^ (4 * i + (lane >> 4)));
        const char* p = kl < c.ke ? op + r * ld2 + (kl - c.ks) * 2
                                  : ((has_next && kl < KT) ? opn + r * ldn + (kl - c.ke) * 2 : zero);
        glds16(p, dst + i * 1024);
      }
    }
  };

  // ---- fragment offsets (within a buffer)
  const int fsw = (lane & 15) >> 1;
  int offA[2], offB[2];  // [k half s]
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int ch = 16 * ((4 * s + (lane >> 4)) ^ fsw);
    offA[s] = (wr * 128 + (lane & 15)) * 128 + ch;
    offB[s] = BOFF + (wc * 64 + (lane & 15)) * 128 + ch;
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][4], bq0[2][2], bq1[2][2];  // [s][block]

  const int64_t nt = (KT + 63) / 64;
  // prologue: tile 0 whole, tile 1's B0, B1, A0
  for (int h = 0; h < 4; ++h) stage_half(lead, h, 0, lds);
  lag = lead;
  advance(lead, 64);
  if (nt > 1) {
    for (int h = 0; h < 3; ++h) stage_half(lead, h, 1, lds + BUF);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // lag: tile 0's cursor until its A1 is staged (already done): move to tile 1
  lag = lead;
  if (nt > 1) advance(lead, 128);
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  auto mfma_quadrant = [&](int qm, int qn, const bf16x8 (&a)[2][4], const bf16x8 (&b)[2][2]) {
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * qm + i][2 * qn + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][i], b[s][j], acc[4 * qm + i][2 * qn + j], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  auto sync_in = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  for (int64_t kt = 0; kt < nt; ++kt) {
    const CUBED_L char* buf = lds + (kt & 1) * BUF;
    CUBED_L char* nbuf = lds + ((kt + 1) & 1) * BUF;  // tile kt+1's buffer
    CUBED_L char* obuf = lds + (kt & 1) * BUF;        // tile kt+2's buffer
    // ---- q0: A rows 0-63, B cols 0-31
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int j = 0; j < 2; ++j) bq0[s][j] = *(const CUBED_L bf16x8*)(buf + offB[s] + j * 2048);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[s][i] = *(const CUBED_L bf16x8*)(buf + offA[s] + i * 2048);
    }
    sync_in();
    mfma_quadrant(0, 0, af, bq0);
    sync_out();
    // ---- q1: B cols 32-63; stage A1 of tile kt+1
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j) bq1[s][j] = *(const CUBED_L bf16x8*)(buf + offB[s] + (2 + j) * 2048);
    if (kt + 1 < nt) stage_half(lag, 3, kt + 1, nbuf);
    sync_in();
    mfma_quadrant(0, 1, af, bq1);
    sync_out();
    // ---- q2: A rows 64-127; stage B0 of tile kt+2
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[s][i] = *(const CUBED_L bf16x8*)(buf + offA[s] + (4 + i) * 2048);
    if (kt + 2 < nt) stage_half(lead, 0, kt + 2, obuf);
    sync_in();
    mfma_quadrant(1, 1, af, bq1);
    sync_out();
    // ---- q3: no reads; stage B1, A0 of tile kt+2; retire tile kt+1
    if (kt + 2 < nt) {
      stage_half(lead, 1, kt + 2, obuf);
      stage_half(lead, 2, kt + 2, obuf);
      lag = lead;
      advance(lead, (kt + 3) * 64);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sync_in();
    mfma_quadrant(1, 0, af, bq0);
    sync_out();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // same barrier count in both rows

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
