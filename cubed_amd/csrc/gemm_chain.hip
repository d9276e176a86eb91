// gemm_chain.hip -- blockwise matmul / tensordot as chained chunk GEMMs.
//
// The reference computes matmul(A, B) in (i, k, j) tasks, each one numpy BLAS
// call on a chunk pair, writing a (m, 1, n) partial product that a sum
// reduction over the k axis then reads back
// (cubed/array_api/linear_algebra_functions.py:13-78, _matmul :62-64,
// _sum_wo_cat :67-78).  Here one task is one OUTPUT chunk C_ij, and its
// contraction walks the k chunks in order: C_ij = sum_k A_ik @ B_kj, each
// (A_ik, B_kj) pair a "segment" of one continuous K loop.  The partial
// products never exist in HBM (at 40000^2 in 5000^2 chunks they would be
// 2 x 51.2 GB of f32 written and re-read), and a per-chunk product is simply
// a chain of one segment.
//
// Kernels:
//   k_gemm_bf16_chain  bf16 x bf16 -> f32 accumulate (-> f32 / bf16 out) on
//                      v_mfma_f32_16x16x32_bf16.  256 x 256 output tile per
//                      512-thread workgroup (8 waves, 2 (M) x 4 (N), each
//                      128 x 64 = 8 x 4 accumulators), K staged 32 deep
//                      straight from HBM into LDS with global_load_lds
//                      (16 B per lane) through a 4-slot ring: three K steps
//                      in flight while the fourth feeds the MFMAs.  The two
//                      wave rows run "ping-pong", one barrier apart: on each
//                      SIMD one wave issues its 32 MFMAs while the other
//                      reads the next step's fragments and issues the
//                      staging loads.
//                      A is staged k-contiguous [m][64] (XOR-swizzled 16-B
//                      chunks, conflict-free ds_read_b128 fragments); B is
//                      staged as it lies in HBM, [k][256] rows, and read
//                      transposed by ds_read_b64_tr_b16 (no transpose pass).
//                      A segment boundary inside a K tile is a per-lane
//                      pointer select; rows/cols past the chunk edge are
//                      clamped (results discarded), k past the chain's end
//                      reads a zero page.
//   k_gemm_f32_chain   f32 on v_mfma_f32_32x32x2_f32 (exact f32 products, f32
//                      accumulate): the bf16 kernel's 256 x 256 tile and
//                      global_load_lds ring, K 16 deep per step, ds_read_b128
//                      fragments for both operands (k and column
//                      permutations, see the kernel).
//   k_gemm_any_chain   any dtype (f64 / int64 / ragged bf16 or f32 shapes):
//                      64 x 64 tiles of scalar FMAs, every element bounds-
//                      checked.  Correctness path, not a fast path.
#include "common.h"
#include <stdio.h>
#include <stdlib.h>

namespace cubed {
extern thread_local char g_err[512];
}
using namespace cubed;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define CUBED_L __attribute__((address_space(3)))

namespace {

// XCD-aware block order: blocks b and b+8 share an XCD (round-robin
// dispatch), so map each XCD's blocks onto one contiguous run of tiles
// (bijective for any grid size; cdna_hip_programming.md T1).
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nblk) {
  if (nblk < 8) return b;
  const int64_t xcd = b & 7, q = nblk >> 3, r = nblk & 7, i = b >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + i;
}

// (probe) the 8 XCDs on different row groups of GM tile rows (per_group
// tiles each) but at the same columns: XCD x's i-th workgroup takes group x + 8
// (i / per_group) while every XCD has whole groups left, then a contiguous
// share of the rest (as xcd_remap) -- B column panels read by all eight XCDs
// at about the same time, for the memory-side cache to serve.
// The rest (rr_tail): runs of 32 tiles of the grouped order (GM x 8 of one
// group) dealt round robin, so the eight XCDs work on neighbouring columns of
// one row group (its A panels read by all eight together); the last < 256
// tiles as contiguous shares.
template <bool RR_TAIL = true>
__device__ __forceinline__ int64_t xcd_tail(int64_t x, int64_t j, int64_t S, int64_t base) {
  if constexpr (RR_TAIL) {
    const int64_t runs = (S >> 8) << 8 >> 5;  // whole rounds of 8 runs of 32
    if (j < runs * 4) return base + ((j >> 5) * 8 + x) * 32 + (j & 31);
    base += runs * 32;
    S -= runs * 32;
    j -= runs * 4;
  }
  const int64_t q = S >> 3, r = S & 7;
  return base + (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
}

template <bool RR_TAIL = true>
__device__ __forceinline__ int64_t xcd_lockstep(int64_t b, int64_t nblk, int64_t per_group, int64_t full_groups) {
  const int64_t main = (full_groups >> 3) * per_group;
  const int64_t x = b & 7, i = b >> 3;
  if (nblk < 8 || main == 0) return xcd_remap(b, nblk);
  if (i < main) return (x + 8 * (i / per_group)) * per_group + i % per_group;
  return xcd_tail<RR_TAIL>(x, i - main, nblk - 8 * main, 8 * main);
}

// Tile-round alignment (the 1-GPU packed bf16 GEMM): the i-th workgroup on an XCD (b & 7, local
// index b >> 3) waits -- one lane polling, bounded -- until the XCD's tiles
// of earlier rounds of R (one per CU) have left their K loops, so a round's
// tiles start their K walks together and share panel lines in L2; a timeout
// only costs the alignment.  ctr: one uint32 per XCD, 128 B apart, zeroed
// before the launch.
__device__ __forceinline__ void round_wait(unsigned* ctr, int64_t b, int64_t R, int64_t slack = 0) {
  const int64_t i = b >> 3;
  if (i >= R) {
    if (threadIdx.x == 0) {
      const unsigned need = (unsigned)((i / R) * R - slack);
      // ~1.5 us per poll: a few ms at most (a round's spread is tens of us)
      for (int it = 0; it < 2000; ++it) {
        if (__hip_atomic_load(ctr + (b & 7) * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need) break;
        __builtin_amdgcn_s_sleep(4);
      }
    }
    __syncthreads();
  }
}
__device__ __forceinline__ void round_done(unsigned* ctr, int64_t b) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr + (b & 7) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int64_t PACK_CTR_BYTES = 8 * 128;  // round_wait counters: one per XCD, 128 B apart

// tile -> (task, m0, n0): tasks outermost, then groups of GM tile rows walked
// column by column, so the workgroups resident on one XCD share A row panels
// and B column panels in its L2.
template <int BM, int BN, int GM>
__device__ __forceinline__ bool tile_of(int64_t g, int64_t tiles_m, int64_t tiles_n, int64_t& t,
                                        int64_t& m0, int64_t& n0) {
  const int64_t tpt = tiles_m * tiles_n;
  t = g / tpt;
  const int64_t tile = g - t * tpt;
  const int64_t per_group = GM * tiles_n;
  const int64_t grp = tile / per_group, first_m = grp * GM;
  const int64_t gsz = (tiles_m - first_m) < GM ? (tiles_m - first_m) : GM;
  const int64_t in_g = tile - grp * per_group;
  m0 = (first_m + in_g % gsz) * BM;
  n0 = (in_g / gsz) * BN;
  return true;
}

// GRID: the output is one (M, N) matrix of ti x tj chunks (task I*tj + J =
// chunk (I, J), every chunk cm x cn except the last row / column, the same
// k segmentation in every task) and 256 x 256 tiles cover the WHOLE matrix:
// a tile that straddles a chunk boundary takes each row's A from its chunk
// row I0 or I0 + 1 and each column's B / C from chunk column J0 or J0 + 1
// (cm, cn >= 256, so never more than two).  Per-chunk tiling pads every
// 5000-wide chunk to 20 x 256 = 5120 (4.9 % of the MFMAs discarded); the grid
// pads 40000 to 157 x 256 = 40192 (1 %).
struct GemmGrid {
  int64_t ti, tj, cm, cn, M, N;
};

// The tile's chunk rows / columns (GRID): T = chunk (I0, J0), TI1 = (I0+1, J0),
// TJ1 = (I0, J0+1) (T itself past the last row / column); mb / nb = first row
// / column of chunk row I0+1 / column J0+1.
struct GridTile {
  int64_t I0, J0, mb, nb;
  const cubed_gemm_chain_t* T;
  const cubed_gemm_chain_t* TI1;
  const cubed_gemm_chain_t* TJ1;
};

__device__ __forceinline__ GridTile grid_tile(const cubed_gemm_chain_t* tasks, const GemmGrid& gg, int64_t m0,
                                              int64_t n0) {
  GridTile g;
  g.I0 = m0 / gg.cm;
  g.J0 = n0 / gg.cn;
  g.mb = (g.I0 + 1) * gg.cm;
  g.nb = (g.J0 + 1) * gg.cn;
  g.T = tasks + g.I0 * gg.tj + g.J0;
  g.TI1 = (g.I0 + 1 < gg.ti) ? g.T + gg.tj : g.T;
  g.TJ1 = (g.J0 + 1 < gg.tj) ? g.T + 1 : g.T;
  return g;
}

// ------------------------------------------------------------------ bf16 MFMA
// LDS is a ring of HB_NS slots, each one 32-deep K step of the 256x256 tile:
// A [256 rows][32 k] (64-B rows) + B [32 k-rows][256 n] (512-B rows).  The
// loads of step p+3 are issued right after the barrier of step p, so three
// steps (96 KiB per CU) are always in flight; the wait for a step is a
// counted vmcnt (4 global_load_lds per wave per step), never vmcnt(0) in the
// steady state, and the barrier is a raw s_barrier (a __syncthreads() would
// drain every LDS-DMA in flight).
constexpr int HB_BM = 256, HB_BN = 256, HB_BK = 32, HB_NS = 4;
constexpr int HB_A = HB_BM * HB_BK * 2;   // 16 KiB
constexpr int HB_B = HB_BK * HB_BN * 2;   // 16 KiB
constexpr int HB_STAGE = HB_A + HB_B;

struct Seg {  // wave-uniform view of one segment
  const char* a;
  const char* b;
  int64_t lda2, ldb2;  // row pitches in bytes
};

__device__ __forceinline__ Seg load_seg(const cubed_gemm_seg_t* __restrict__ segs, int64_t i) {
  Seg s;
  s.a = (const char*)(uintptr_t)segs[i].a;
  s.b = (const char*)(uintptr_t)segs[i].b;
  s.lda2 = segs[i].lda * 2;
  s.ldb2 = segs[i].ldb * 2;
  return s;
}

__device__ __forceinline__ void glds16(const char* src, CUBED_L char* dst) {
  __builtin_amdgcn_global_load_lds((const CUBED_G void*)(uintptr_t)src, (CUBED_L void*)dst, 16, 0, 0);
}

// ABL: ablation bits for tools/gemm_bf16_probe.hip only (0 in the library):
// 1 = no K-loop staging, 2 = no B fragment reads, 4 = no A fragment reads,
// 8 = no K-loop barrier; ping-pong only: 16 = no vmcnt wait in the K loop,
// 32 = every K step staged from step 0's addresses (L2-resident), 1 = no
// K-loop staging.  Any nonzero value computes wrong results.
// PP: 0 = one barrier per step, 1 = ping-pong (the library's), 2 = ping-pong
// with register staging (see the K loop).
// NS: ring slots (each step p+NS-1 is staged while step p is consumed);
// GM: tile rows per XCD tile group.
template <bool OUT_BF16, int ABL = 0, int PP = 0, int NS = HB_NS, int GM = 4, bool GRID = false>
__global__ __launch_bounds__(512, 2) void k_gemm_bf16_chain(const cubed_gemm_chain_t* __restrict__ tasks,
                                                         const cubed_gemm_seg_t* __restrict__ segs,
                                                         int64_t tiles_m, int64_t tiles_n,
                                                         const char* __restrict__ zero, GemmGrid gg) {
  __shared__ __attribute__((aligned(1024))) char lds_[(PP == 2 ? 2 : NS) * HB_STAGE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t, m0, n0;
  tile_of<HB_BM, HB_BN, GM>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  GridTile gt{0, 0, 0, 0, tasks + t, tasks + t, tasks + t};
  if constexpr (GRID) gt = grid_tile(tasks, gg, m0, n0);
  const cubed_gemm_chain_t* __restrict__ T = gt.T;
  const int64_t M = GRID ? gg.M : T->m, N = GRID ? gg.N : T->n, KT = T->ktot;
  if (m0 >= M || n0 >= N) return;
  const int64_t seg0 = T->seg0, segN = T->seg0 + T->nseg;
  const int64_t dsI = gt.TI1->seg0 - T->seg0, dsJ = gt.TJ1->seg0 - T->seg0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- per-lane staging geometry (constant over the K loop)
  // A: wave w stages rows 16*(2w+i) + lane>>2 (i = 0, 1); 16-B chunk lane&3 of
  // the 64-B LDS row holds global chunk (lane&3) ^ 2*((row>>3)&1)
  // [(row>>3)&1 = (lane>>5)&1], which makes the fragment reads conflict-free.
  // (GRID: rows / columns local to their chunk; hiA / hiB select chunk row
  // I0 + 1 / column J0 + 1)
  int64_t gmA[2];
  bool hiA[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t r = 16 * (2 * w + i) + (lane >> 2);
    const int64_t g = (m0 + r < M ? m0 + r : M - 1);
    hiA[i] = GRID && g >= gt.mb;
    gmA[i] = GRID ? g - (hiA[i] ? gt.mb : gt.I0 * gg.cm) : g;
  }
  const int dA = 8 * ((lane & 3) ^ (2 * ((lane >> 5) & 1)));
  // B: wave w stages k-rows 2*(2w+i) + lane>>5; 16-B chunk c = lane&31 of the
  // LDS row holds global chunk c ^ swz(row), swz(r) = 2*((r&3) | ((r>>3)&1)<<2).
  int rB[2];
  int64_t gnB[2];
  bool hiB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 2 * (2 * w + i) + (lane >> 5);
    rB[i] = r;
    const int swz = 2 * ((r & 3) | (((r >> 3) & 1) << 2));
    int64_t n = n0 + 8 * ((lane & 31) ^ swz);
    n = (n + 8 <= N ? n : N - 8);
    hiB[i] = GRID && n >= gt.nb;
    gnB[i] = GRID ? n - (hiB[i] ? gt.nb : gt.J0 * gg.cn) : n;
  }

  // ---- wave-uniform segment state (the segment containing the next step to stage)
  int64_t s = seg0, ks = 0;
  Seg cur = load_seg(segs, s);
  Seg curI = load_seg(segs, s + dsI), curJ = load_seg(segs, s + dsJ);  // GRID: chunk row I0+1 / column J0+1
  int64_t ke = segs[s].k;

  // per-lane byte offsets of this lane's 4 pieces inside the current segment
  // (recomputed only when the segment changes)
  int64_t offSA[2], offSB[2];
  auto seg_offsets = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      offSA[i] = gmA[i] * cur.lda2 + dA * 2;
      offSB[i] = rB[i] * (hiB[i] ? curJ.ldb2 : cur.ldb2) + gnB[i] * 2;
    }
  };
  seg_offsets();

  // the 4 global->LDS loads of the K step starting at k0 into slot buf:
  // sources / destinations (stage_addrs) and their issue
  const char* st_src[4];
  CUBED_L char* st_dst[4];
  auto stage_addrs = [&](int64_t k0, CUBED_L char* buf) {
    const char* sa[2];
    const char* sb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sa[i] = (hiA[i] ? curI.a : cur.a) + (k0 - ks) * 2 + offSA[i];
      sb[i] = hiB[i] ? curJ.b + (k0 - ks) * curJ.ldb2 + offSB[i] : cur.b + (k0 - ks) * cur.ldb2 + offSB[i];
    }
    if (k0 + HB_BK > ke) {  // uniform: a segment boundary (or the chain's end) inside this step
      const bool has_next = s + 1 < segN;
      const int64_t sn = has_next ? s + 1 : s;
      const Seg nxt = load_seg(segs, sn);
      const Seg nxtI = load_seg(segs, sn + dsI), nxtJ = load_seg(segs, sn + dsJ);
      const int64_t ka = k0 + dA;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const char* na = (hiA[i] ? nxtI.a : nxt.a) + gmA[i] * nxt.lda2 + (ka - ke) * 2;
        sa[i] = ka < ke ? sa[i] : ((has_next && ka < KT) ? na : zero);
        const int64_t kb = k0 + rB[i];
        const char* nbp = hiB[i] ? nxtJ.b + (kb - ke) * nxtJ.ldb2 + gnB[i] * 2
                                 : nxt.b + (kb - ke) * nxt.ldb2 + gnB[i] * 2;
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
      curI = load_seg(segs, s + dsI);
      curJ = load_seg(segs, s + dsJ);
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
  static_assert(PP == 2 ? (NS >= 2 && NS <= 4) : (NS >= 3 && NS <= 5), "ring of 3..5 slots (PP 2: 2..4 register sets)");
  int rd = 0, wr_slot = D % NS;  // ring slots of steps p and p + D
  if constexpr (PP == 2) {
    // Ping-pong with REGISTER staging: global_load_dwordx4 into VGPRs, then
    // ds_write_b128, instead of LDS-DMA (an LDS-DMA instruction costs its
    // wave 60-185 issue cycles, MI355X_MICROARCH.md per-instruction
    // constants).  LDS holds two slots: M(p) reads step p from slot p&1,
    // writes step p+1 (loaded NS-1 memory slots earlier) into slot (p+1)&1
    // and issues step p+NS's loads into the register set step p vacated.
    // RAW: M(p)'s ds_writes retire (lgkmcnt(0)) before the barrier ending its
    //   slot; step p+1 is read in M(p+1), which in both rows starts after
    //   both rows' M(p) ended.
    // WAR: slot (p+1)&1 last held step p-1, read in M(p-1), which ended in
    //   both rows before either row's M(p) started.
    constexpr int RD = NS;  // register sets: loads of RD steps in flight
    u32x4 rs[RD][4];
    int wdst[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      wdst[i] = (2 * w + i) * 1024 + lane * 16;
      wdst[2 + i] = HB_A + (2 * w + i) * 1024 + lane * 16;
    }
    auto gload = [&](int64_t k0, u32x4 (&dst)[4]) {
      stage_addrs(k0, lds);
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[i] = *(const CUBED_G u32x4*)(uintptr_t)st_src[i];
    };
    auto swrite = [&](CUBED_L char* buf, const u32x4 (&src)[4]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) *(CUBED_L u32x4*)(buf + wdst[i]) = src[i];
    };
#pragma unroll
    for (int r = 0; r < RD; ++r)
      if (r < nst) gload(r * HB_BK, rs[r]);
    if (nst > 0) swrite(lds, rs[0]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 af[8];
    for (int64_t p0 = 0; p0 < nst; p0 += RD) {
#pragma unroll
      for (int r = 0; r < RD; ++r) {
        const int64_t p = p0 + r;
        if (p >= nst) break;
        // ---- M(p)
        const CUBED_L char* bufc = lds + (p & 1) * HB_STAGE;
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
        if (p + 1 < nst) swrite(lds + ((p + 1) & 1) * HB_STAGE, rs[(r + 1) % RD]);
        if (p + RD < nst) gload((p + RD) * HB_BK, rs[r]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
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
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // same barrier count in both rows
  } else if constexpr (PP == 1) {
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
      if (!(ABL & 1) && p + D < nst) stage((ABL & 32) ? 0 : (p + D) * HB_BK, lds + wr_slot * HB_STAGE);
      rd = rd + 1 == NS ? 0 : rd + 1;
      wr_slot = wr_slot + 1 == NS ? 0 : wr_slot + 1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (!(ABL & 16) && p + 1 < nst) wait_step(p + 1);
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
    if (wr == 0) __builtin_amdgcn_s_barrier();  // same barrier count in both rows
  } else
  for (int64_t p = 0; p < nst; ++p) {
    // this wave's loads of step p have landed once at most the younger
    // steps' loads (4 per step) are outstanding
    if (ABL & 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else wait_step(p);
    // every wave's step p landed; every wave finished reading step p-1's slot
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(ABL & 8)) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (!(ABL & 1) && p + D < nst) stage((p + D) * HB_BK, lds + wr_slot * HB_STAGE);
    const CUBED_L char* bufc = lds + rd * HB_STAGE;
    rd = rd + 1 == NS ? 0 : rd + 1;
    wr_slot = wr_slot + 1 == NS ? 0 : wr_slot + 1;
    // B fragments by transposed reads.  Inline asm: the builtin has no memory
    // operand, so hipcc would put an s_waitcnt vmcnt(0) in front of it --
    // draining the three K steps in flight -- and the reads only touch slot
    // p, which the vmcnt + barrier above already made visible.
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      if ((ABL & 2) && p > 0) break;
      const uint32_t pb = (uint32_t)(uintptr_t)(bufc + offB[nb]);
      s16x4 lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(pb));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(hi) : "v"(pb));
      bf[nb] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // (s_setprio(1) around this MFMA cluster measured 1046 vs 1069 TF: not used)
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) {
      const bf16x8 af = (ABL & 4) ? bf[mb & 3] : *(const CUBED_L bf16x8*)(bufc + offA + mb * 1024);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[nb], acc[mb][nb], 0, 0, 0);
    }
  }

  // ---- epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r
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
          // the element's chunk (GRID) and its offset inside it
          const bool hm = GRID && gm >= gt.mb, hn = GRID && gn >= gt.nb;
          const cubed_gemm_chain_t* TC = hn ? gt.TJ1 : T;
          if (hm) TC += gt.TI1 - T;
          const int64_t lm = GRID ? gm - (hm ? gt.mb : gt.I0 * gg.cm) : gm;
          const int64_t ln = GRID ? gn - (hn ? gt.nb : gt.J0 * gg.cn) : gn;
          char* C = (char*)(uintptr_t)TC->c;
          const int64_t ldc = TC->ldc;
          float v = acc[mb][nb][r];
          if constexpr (OUT_BF16) {
            CUBED_G uint16_t* c = (CUBED_G uint16_t*)(uintptr_t)(C + (lm * ldc + ln) * 2);
            if (accum) v += bf16_to_f32(*c);
            *c = f32_to_bf16(v);
          } else {
            CUBED_G float* c = (CUBED_G float*)(uintptr_t)(C + (lm * ldc + ln) * 4);
            if (accum) v += *c;
            *c = v;
          }
        }
      }
}

#include "gemm_bf16_w4l.h"
#include "gemm_bf16_w4p.h"
#include "gemm_bf16_8p.h"

// ------------------------------------------------------------------ f32 MFMA
// v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate): lane l gives
// A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31].  256x256 output tile per
// 512-thread workgroup (8 waves, 4 (M) x 2 (N), each 64 x 128 = 2 x 4
// accumulators of 32x32), K staged 16 deep straight from HBM into LDS by
// global_load_lds (16 B per lane) through a 4-slot ring (three steps in
// flight), counted vmcnt + raw s_barrier, one barrier per step -- the bf16
// kernel's pipeline.  Both operands are read with ds_read_b128 by two
// permutations that change no value:
//  * K: a lane's 16-B A read holds 4 consecutive k of its row; in an 8-deep
//    k group g the MFMA of step j (0..3) pairs k = 8g+j (lanes 0-31) with
//    k = 8g+4+j (lanes 32-63), and B supplies the same k rows;
//  * N: a lane's 16-B B read holds 4 consecutive columns of one k row, one
//    per accumulator q: accumulator q covers columns wn + 4j + q (j = lane
//    column), so the epilogue stores the 4 accumulators of a row as one
//    float4.
// Each output element is one f32 fma chain over its K (the per-element
// order is (segment, k group, j, half), every product exact).
// LDS slot: A [256 rows][16 k] (64-B rows, 16-B chunk c of row r at
// position c ^ ((r >> 2) & 3): conflict-free b128 reads) + B [16 k][256 n]
// (1 KiB rows, as in HBM).
constexpr int HF_BM = 256, HF_BN = 256;

// BK: K depth of one ring slot (16 or 32); NS: ring slots.  A slot holds A
// [256 rows][BK k] (BK*4-byte rows, CPR = BK/4 16-B chunks, chunk c of row
// r at position c ^ swz(r): conflict-free b128 reads) + B [BK k][256 n]
// (1 KiB rows, as in HBM).
template <int BK, int NS, bool PP = false, bool GRID = false>
__global__ __launch_bounds__(512, 2) void k_gemm_f32_chain(const cubed_gemm_chain_t* __restrict__ tasks,
                                                        const cubed_gemm_seg_t* __restrict__ segs,
                                                        int64_t tiles_m, int64_t tiles_n,
                                                        const char* __restrict__ zero, GemmGrid gg) {
  static_assert(BK == 16 || BK == 32, "K step of 16 or 32");
  constexpr int SA = HF_BM * BK * 4, SB = BK * HF_BN * 4, STAGE = SA + SB;
  constexpr int CPR = BK / 4;            // 16-B chunks per A row
  constexpr int RPI = 1024 / (BK * 4);   // A rows per wave instruction (1 KiB)
  constexpr int NA = HF_BM / RPI / 8;    // A loads per wave per step
  constexpr int NB = BK / 8;             // B loads per wave per step
  constexpr int LPS = NA + NB;           // vmcnt per step
  constexpr int SWS = BK == 16 ? 2 : 1;  // swz(r) = (r >> SWS) & (CPR - 1)
  constexpr int G = BK / 8;              // 8-deep k groups per step
  static_assert(NS * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char lds_[NS * STAGE];
  CUBED_L char* lds = (CUBED_L char*)lds_;
  int64_t t, m0, n0;
  tile_of<HF_BM, HF_BN, 4>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  // GRID: (m0, n0) in the whole matrix; chunk rows I0 (, I0 + 1) and columns
  // J0 (, J0 + 1) of the tile; mb / nb: the first row / column of chunk I0+1 / J0+1
  int64_t I0 = 0, J0 = 0, mb = 0, nb = 0;
  const cubed_gemm_chain_t* __restrict__ T = tasks + t;
  const cubed_gemm_chain_t* __restrict__ TI1 = T;  // chunk (I0 + 1, J0): A rows
  const cubed_gemm_chain_t* __restrict__ TJ1 = T;  // chunk (I0, J0 + 1): B columns
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
  // segment s of chunk (I0 + 1, J0) / (I0, J0 + 1): same index offset
  const int64_t dsI = TI1->seg0 - T->seg0, dsJ = TJ1->seg0 - T->seg0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (w >> 1) * 64, wn = (w & 1) * 128;

  // ---- staging geometry (constant over the K loop)
  // A: wave w instruction i stages rows RPI*(NA*w + i) + lane/CPR; LDS
  // position lane%CPR of the row holds global chunk (lane%CPR) ^ swz(row)
  // (GRID: a lane's row / column is local to its chunk, hiA / hiB select
  // chunk row I0 + 1 / column J0 + 1)
  int64_t gmA[NA];
  int kA[NA];
  bool hiA[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int r = RPI * (NA * w + i) + lane / CPR;
    int64_t g = (m0 + r < M ? m0 + r : M - 1);
    hiA[i] = GRID && g >= mb;
    gmA[i] = GRID ? g - (hiA[i] ? mb : I0 * gg.cm) : g;
    kA[i] = 4 * ((lane % CPR) ^ ((r >> SWS) & (CPR - 1)));
  }
  // B: wave w instruction i stages k-row NB*w + i, columns n0 + 4*lane .. +3
  const int rB0 = NB * w;
  int64_t gnB = (n0 + 4 * lane + 4 <= N ? n0 + 4 * lane : N - 4);
  const bool hiB = GRID && gnB >= nb;
  if constexpr (GRID) gnB -= hiB ? nb : J0 * gg.cn;

  int64_t s = seg0, ks = 0;
  // per segment: A of chunk rows I0 / I0+1, B (and its row pitch) of chunk
  // columns J0 / J0+1 -- wave-uniform; a lane selects with hiA / hiB
  auto ptr = [&](int64_t i) { return (const char*)(uintptr_t)segs[i].a; };
  auto ptrb = [&](int64_t i) { return (const char*)(uintptr_t)segs[i].b; };
  const char* a_cur = ptr(s);
  const char* a_hi = ptr(s + dsI);
  const char* b_cur = ptrb(s);
  const char* b_hi = ptrb(s + dsJ);
  int64_t lda4 = segs[s].lda * 4, ldb4 = segs[s].ldb * 4, ldb4h = segs[s + dsJ].ldb * 4;
  int64_t ke = segs[s].k;

  auto stage = [&](int64_t k0, CUBED_L char* buf) {
    const char* sa[NA];
    const char* sb[NB];
    const char* bb = hiB ? b_hi : b_cur;
    const int64_t lb = hiB ? ldb4h : ldb4;
#pragma unroll
    for (int i = 0; i < NA; ++i) sa[i] = (hiA[i] ? a_hi : a_cur) + gmA[i] * lda4 + (k0 - ks + kA[i]) * 4;
#pragma unroll
    for (int i = 0; i < NB; ++i) sb[i] = bb + (k0 - ks + rB0 + i) * lb + gnB * 4;
    if (k0 + BK > ke) {  // uniform: a segment boundary (or the chain's end) inside this step
      const bool has_next = s + 1 < segN;
      const int64_t sn = has_next ? s + 1 : s;
      const char* nal = ptr(sn);
      const char* nah = ptr(sn + dsI);
      const char* nbp = hiB ? ptrb(sn + dsJ) : ptrb(sn);
      const int64_t nlda4 = segs[sn].lda * 4, nldb4 = (hiB ? segs[sn + dsJ].ldb : segs[sn].ldb) * 4;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int64_t ka = k0 + kA[i];
        const char* pa = (hiA[i] ? nah : nal) + gmA[i] * nlda4 + (ka - ke) * 4;
        sa[i] = ka < ke ? sa[i] : ((has_next && ka < KT) ? pa : zero);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int64_t kb = k0 + rB0 + i;
        const char* pb = nbp + (kb - ke) * nldb4 + gnB * 4;
        sb[i] = kb < ke ? sb[i] : ((has_next && kb < KT) ? pb : zero);
      }
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) glds16(sa[i], buf + (NA * w + i) * 1024);
#pragma unroll
    for (int i = 0; i < NB; ++i) glds16(sb[i], buf + SA + (rB0 + i) * 1024);
    if (k0 + BK >= ke && s + 1 < segN) {  // the next step starts in the next segment
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

  // ---- fragment read offsets (within a slot)
  const int h = lane >> 5, r32 = lane & 31;
  // A, row block rb, k group g: row wm + 32 rb + r32, logical chunk 2g + h
  int offA[2][G];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int g = 0; g < G; ++g)
      offA[rb][g] = (wm + 32 * rb + r32) * (BK * 4) + 16 * ((2 * g + h) ^ ((r32 >> SWS) & (CPR - 1)));
  // B, k group g, step j: k-row 8g + 4h + j, columns wn + 4 r32 .. +3
  const int offB = SA + 4 * h * 1024 + (wn + 4 * r32) * 4;

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][q][r] = 0.f;

  const int64_t nst = (KT + BK - 1) / BK;
  constexpr int D = NS - 1;  // steps staged ahead
  for (int64_t p = 0; p < D && p < nst; ++p) stage(p * BK, lds + p * STAGE);
  // retire this wave's loads of step q (LPS per step; steps up to q + D - 1 issued)
  auto wait_step = [&](int64_t q) {
    int64_t younger = nst - 1 - q;
    if (younger > D - 1) younger = D - 1;
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * LPS) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(LPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  int rd = 0, wr_slot = D % NS;
  if constexpr (PP) {
    // Ping-pong (the bf16 kernel's schedule): wave rows 0-1 (w < 4) and 2-3
    // run one barrier apart, alternating a memory slot M(p) -- step p's 12
    // fragment reads into registers, step p+D's staging loads, the wait for
    // step p+1 -- and a compute slot C(p) of 64 MFMAs, so on every SIMD one
    // wave's MFMAs cover the other's LDS reads.  RAW / WAR as in
    // k_gemm_bf16_chain (same ring).
    const int half = w >> 2;
    if (nst > 0) wait_step(0);
    __builtin_amdgcn_s_barrier();
    if (half == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    f32x4 af[G][2], bq[G][4];
    for (int64_t p = 0; p < nst; ++p) {
      const CUBED_L char* bufc = lds + rd * STAGE;
#pragma unroll
      for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) af[g][rb] = *(const CUBED_L f32x4*)(bufc + offA[rb][g]);
#pragma unroll
        for (int j = 0; j < 4; ++j) bq[g][j] = *(const CUBED_L f32x4*)(bufc + offB + (8 * g + j) * 1024);
      }
      if (p + D < nst) stage((p + D) * BK, lds + wr_slot * STAGE);
      rd = rd + 1 == NS ? 0 : rd + 1;
      wr_slot = wr_slot + 1 == NS ? 0 : wr_slot + 1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (p + 1 < nst) wait_step(p + 1);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[rb][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[g][rb][j], bq[g][j][q], acc[rb][q], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (half == 0) __builtin_amdgcn_s_barrier();  // same barrier count in both halves
  } else
  for (int64_t p = 0; p < nst; ++p) {
    // this wave's step p landed; then every wave's (barrier), and every wave
    // finished reading step p-1's slot (restaged below)
    wait_step(p);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (p + D < nst) stage((p + D) * BK, lds + wr_slot * STAGE);
    const CUBED_L char* bufc = lds + rd * STAGE;
    rd = rd + 1 == NS ? 0 : rd + 1;
    wr_slot = wr_slot + 1 == NS ? 0 : wr_slot + 1;
    // fragments of group g+1 are read while group g's 32 MFMAs run
    f32x4 af[G][2], bq[G][4];
    auto read_group = [&](int g) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) af[g][rb] = *(const CUBED_L f32x4*)(bufc + offA[rb][g]);
#pragma unroll
      for (int j = 0; j < 4; ++j) bq[g][j] = *(const CUBED_L f32x4*)(bufc + offB + (8 * g + j) * 1024);
    };
    read_group(0);
    if constexpr (G > 1) read_group(1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[rb][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[g][rb][j], bq[g][j][q], acc[rb][q], 0, 0, 0);
      if (g + 2 < G) {
        __builtin_amdgcn_sched_barrier(0);
        read_group(g + 2);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }

  // ---- epilogue: accumulator (rb, q) register r = row wm + 32 rb + (r&3) +
  // 8 (r>>2) + 4h, column wn + 4 r32 + q: one float4 per (rb, r)
  const bool accum = T->accumulate != 0;
  const int64_t gn = n0 + wn + 4 * r32;
  if (gn < N) {
    // GRID: this lane's 4 columns lie in chunk column J0 or J0 + 1 (cn % 4 == 0);
    // each row in chunk row I0 or I0 + 1
    const bool hn = GRID && gn >= nb;
    const cubed_gemm_chain_t* __restrict__ TC0 = hn ? TJ1 : T;  // chunk (I0, J)
    const cubed_gemm_chain_t* __restrict__ TC1 = TC0 + (TI1 - T);  // chunk (I0 + 1, J)
    const int64_t ln = GRID ? gn - (hn ? nb : J0 * gg.cn) : gn;
    char* C0 = (char*)(uintptr_t)TC0->c;
    char* C1 = (char*)(uintptr_t)TC1->c;
    const int64_t ldc0 = TC0->ldc, ldc1 = TC1->ldc;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + wm + 32 * rb + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gm < M) {
          const bool hm = GRID && gm >= mb;
          const int64_t lm = GRID ? gm - (hm ? mb : I0 * gg.cm) : gm;
          CUBED_G f32x4* c = (CUBED_G f32x4*)(uintptr_t)((hm ? C1 : C0) + (lm * (hm ? ldc1 : ldc0) + ln) * 4);
          f32x4 v = {acc[rb][0][r], acc[rb][1][r], acc[rb][2][r], acc[rb][3][r]};
          if (accum) v += *c;
          *c = v;
        }
      }
  }
}

// ------------------------------------------------------------------ any dtype
// c + a*b: fused for floats (BLAS-style FMA accumulation), wrapping for int64
CUBED_DEV float mul_add(float a, float b, float c) { return fmaf(a, b, c); }
CUBED_DEV double mul_add(double a, double b, double c) { return fma(a, b, c); }
CUBED_DEV int64_t mul_add(int64_t a, int64_t b, int64_t c) {
  return (int64_t)((uint64_t)c + (uint64_t)a * (uint64_t)b);
}

static constexpr int TM = 64, TN = 64, TK = 16;

// IN: storage dtype of A and B (cubed_dtype); V: accumulator type
template <int IN, typename V>
__global__ __launch_bounds__(256) void k_gemm_any_chain(const cubed_gemm_chain_t* __restrict__ tasks,
                                                     const cubed_gemm_seg_t* __restrict__ segs,
                                                     int64_t tiles_m, int64_t tiles_n, int32_t out_dt) {
  __shared__ V As[TK][TM + 1];
  __shared__ V Bs[TK][TN + 1];
  int64_t t, m0, n0;
  tile_of<TM, TN, 8>(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, t, m0, n0);
  const cubed_gemm_chain_t* __restrict__ TT = tasks + t;
  const int64_t M = TT->m, N = TT->n;
  if (m0 >= M || n0 >= N) return;
  const int isz = dt_size(IN);
  const int tid = threadIdx.x;
  const int tr = (tid >> 4) * 4, tc = (tid & 15) * 4;  // 4x4 per thread
  V acc[4][4] = {};
  for (int64_t si = TT->seg0; si < TT->seg0 + TT->nseg; ++si) {
    const char* A = (const char*)(uintptr_t)segs[si].a;
    const char* B = (const char*)(uintptr_t)segs[si].b;
    const int64_t K = segs[si].k, lda = segs[si].lda, ldb = segs[si].ldb;
    for (int64_t k0 = 0; k0 < K; k0 += TK) {
      for (int i = tid; i < TM * TK; i += 256) {
        const int mm = i / TK, kk = i % TK;
        const int64_t gm = m0 + mm, gk = k0 + kk;
        As[kk][mm] = (gm < M && gk < K) ? ld1<V>(A + (gm * lda + gk) * isz, IN) : (V)0;
      }
      for (int i = tid; i < TN * TK; i += 256) {
        const int kk = i / TN, nn = i % TN;
        const int64_t gk = k0 + kk, gn = n0 + nn;
        Bs[kk][nn] = (gk < K && gn < N) ? ld1<V>(B + (gk * ldb + gn) * isz, IN) : (V)0;
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < TK; ++kk) {
        V a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { a[i] = As[kk][tr + i]; b[i] = Bs[kk][tc + i]; }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mul_add(a[i], b[j], acc[i][j]);
      }
      __syncthreads();
    }
  }
  const int osz = dt_size(out_dt);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gm = m0 + tr + i, gn = n0 + tc + j;
      if (gm < M && gn < N) {
        char* c = (char*)(uintptr_t)TT->c + (gm * TT->ldc + gn) * osz;
        V v = acc[i][j];
        if (TT->accumulate) v = v + ld1<V>(c, out_dt);
        st1<V>(c, out_dt, v);
      }
    }
}

#include "gemm_f32_w4p.h"

int fail(const char* m) {
  snprintf(g_err, sizeof(g_err), "cubed_gemm_chain: %s", m);
  return CUBED_E_ARG;
}

bool aligned16(int64_t x) { return (x & 15) == 0; }

}  // namespace

// Which kernel serves a chain set (host tables): the MFMA fast paths need
// every segment's k a multiple of 8 (bf16) / 4 (f32) and >= the K step
// (32), 16-B aligned operand rows, and (bf16) n a multiple of 8.
extern "C" int cubed_gemm_chain_path(const cubed_gemm_chain_t* tasks, int64_t ntasks,
                                     const cubed_gemm_seg_t* segs, int32_t in_dtype,
                                     int32_t out_dtype) {
  if (in_dtype == CUBED_BF16 && (out_dtype == CUBED_F32 || out_dtype == CUBED_BF16)) {
    for (int64_t t = 0; t < ntasks; ++t) {
      const cubed_gemm_chain_t& T = tasks[t];
      if (T.n < 8 || T.n % 8 || T.m < 1) return CUBED_GEMM_ANY;
      for (int64_t i = T.seg0; i < T.seg0 + T.nseg; ++i) {
        const cubed_gemm_seg_t& s = segs[i];
        if (s.k < 32 || s.k % 8 || s.lda % 8 || s.ldb % 8 || !aligned16(s.a) || !aligned16(s.b))
          return CUBED_GEMM_ANY;
      }
    }
    return CUBED_GEMM_MFMA;
  }
  if (in_dtype == CUBED_F32 && out_dtype == CUBED_F32) {
    for (int64_t t = 0; t < ntasks; ++t) {
      const cubed_gemm_chain_t& T = tasks[t];
      if (T.n % 4 || T.m < 1) return CUBED_GEMM_ANY;
      for (int64_t i = T.seg0; i < T.seg0 + T.nseg; ++i) {
        const cubed_gemm_seg_t& s = segs[i];
        if (s.k < 32 || s.k % 4 || s.lda % 4 || s.ldb % 4 || !aligned16(s.a) || !aligned16(s.b))
          return CUBED_GEMM_ANY;
      }
    }
    return CUBED_GEMM_MFMA;
  }
  return CUBED_GEMM_ANY;
}

extern "C" int cubed_gemm_chain(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks,
                                int64_t ntasks, const cubed_gemm_seg_t* segs,
                                const cubed_gemm_seg_t* d_segs, int64_t nsegs, int32_t in_dtype,
                                int32_t out_dtype, const void* d_zero, int32_t path, void* stream) {
  if (ntasks == 0) return 0;
  if (!tasks || !d_tasks || !segs || !d_segs || ntasks < 0 || nsegs <= 0) return fail("bad argument");
  int64_t max_m = 1, max_n = 1;
  for (int64_t t = 0; t < ntasks; ++t) {
    const cubed_gemm_chain_t& T = tasks[t];
    if (T.m < 0 || T.n < 0 || T.nseg < 1 || T.seg0 < 0 || T.seg0 + T.nseg > nsegs || T.c == 0)
      return fail("task out of range");
    int64_t kt = 0;
    for (int64_t i = T.seg0; i < T.seg0 + T.nseg; ++i) {
      if (segs[i].k < 0 || !segs[i].a || !segs[i].b) return fail("bad segment");
      kt += segs[i].k;
    }
    if (kt != T.ktot) return fail("ktot is not the sum of the task's segments");
    max_m = T.m > max_m ? T.m : max_m;
    max_n = T.n > max_n ? T.n : max_n;
  }
  const int auto_path = cubed_gemm_chain_path(tasks, ntasks, segs, in_dtype, out_dtype);
  if (path == CUBED_GEMM_AUTO) path = auto_path;
  if (path == CUBED_GEMM_MFMA && auto_path != CUBED_GEMM_MFMA) return fail("shapes do not fit the MFMA path");
  hipStream_t st = (hipStream_t)stream;
  if (path == CUBED_GEMM_MFMA && in_dtype == CUBED_BF16) {
    if (!d_zero) return fail("the bf16 path needs a zero page");
    const int64_t tm = (max_m + HB_BM - 1) / HB_BM, tn = (max_n + HB_BN - 1) / HB_BN;
    const int64_t blocks = ntasks * tm * tn;
    if (blocks > 0x7fffffff) return fail("grid too large");
    const dim3 grid((unsigned)blocks), blk(512);
    const char* z = (const char*)d_zero;
    // round 5: one wave per SIMD with A staged in full 128-B lines
    // (gemm_bf16_w4l.h: 1256-1258 TF on config 5) whenever every segment
    // spans a 64-k A tile; otherwise the round-2 ping-pong schedule
    // (1072-1098 TF, profiles/r02_gemm_bf16_variants.log)
    bool w4l = true;
    for (int64_t t = 0; t < ntasks && w4l; ++t)
      for (int64_t i = tasks[t].seg0; i < tasks[t].seg0 + tasks[t].nseg; ++i)
        if (segs[i].k < 64) { w4l = false; break; }
    if (w4l) {
      if (out_dtype == CUBED_BF16)
        hipLaunchKernelGGL((k_gemm_bf16_w4l<true>), grid, dim3(256), 0, st, d_tasks, d_segs, tm, tn, z, GemmGrid{},
                           nullptr);
      else
        hipLaunchKernelGGL((k_gemm_bf16_w4l<false>), grid, dim3(256), 0, st, d_tasks, d_segs, tm, tn, z, GemmGrid{},
                           nullptr);
    } else if (out_dtype == CUBED_BF16)
      hipLaunchKernelGGL((k_gemm_bf16_chain<true, 0, 1>), grid, blk, 0, st, d_tasks, d_segs, tm, tn, z, GemmGrid{});
    else
      hipLaunchKernelGGL((k_gemm_bf16_chain<false, 0, 1>), grid, blk, 0, st, d_tasks, d_segs, tm, tn, z, GemmGrid{});
  } else if (path == CUBED_GEMM_MFMA && in_dtype == CUBED_F32) {
    if (!d_zero) return fail("the f32 path needs a zero page");
    const int64_t tm = (max_m + HF_BM - 1) / HF_BM, tn = (max_n + HF_BN - 1) / HF_BN;
    const int64_t blocks = ntasks * tm * tn;
    if (blocks > 0x7fffffff) return fail("grid too large");
    hipLaunchKernelGGL((k_gemm_f32_chain<16, 4>), dim3((unsigned)blocks), dim3(512), 0, st, d_tasks, d_segs, tm,
                       tn, (const char*)d_zero, GemmGrid{});
  } else {
    const int64_t tm = (max_m + TM - 1) / TM, tn = (max_n + TN - 1) / TN;
    const int64_t blocks = ntasks * tm * tn;
    if (blocks > 0x7fffffff) return fail("grid too large");
    dim3 grid((unsigned)blocks), blk(256);
    switch (in_dtype) {
      case CUBED_BF16:
        hipLaunchKernelGGL((k_gemm_any_chain<CUBED_BF16, float>), grid, blk, 0, st, d_tasks, d_segs, tm, tn, out_dtype);
        break;
      case CUBED_F32:
        hipLaunchKernelGGL((k_gemm_any_chain<CUBED_F32, float>), grid, blk, 0, st, d_tasks, d_segs, tm, tn, out_dtype);
        break;
      case CUBED_F64:
        hipLaunchKernelGGL((k_gemm_any_chain<CUBED_F64, double>), grid, blk, 0, st, d_tasks, d_segs, tm, tn, out_dtype);
        break;
      case CUBED_I64:
        hipLaunchKernelGGL((k_gemm_any_chain<CUBED_I64, int64_t>), grid, blk, 0, st, d_tasks, d_segs, tm, tn, out_dtype);
        break;
      default:
        snprintf(g_err, sizeof(g_err), "cubed_gemm_chain: input dtype %d not supported", in_dtype);
        return CUBED_E_DTYPE;
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}

// ---- grid tiling (f32 MFMA): the chain set is a ti x tj chunk grid of one
// (M, N) output, task I*tj + J = chunk (I, J); see k_gemm_f32_chain<.., GRID>.
extern "C" int cubed_gemm_grid_check(const cubed_gemm_chain_t* tasks, int64_t ti, int64_t tj,
                                     const cubed_gemm_seg_t* segs, int64_t nsegs, int32_t in_dtype,
                                     int32_t out_dtype) {
  if (!tasks || !segs || ti < 1 || tj < 1) return fail("grid: bad argument");
  const bool bf = in_dtype == CUBED_BF16;
  if (!(in_dtype == CUBED_F32 && out_dtype == CUBED_F32) &&
      !(bf && (out_dtype == CUBED_F32 || out_dtype == CUBED_BF16))) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_chain_grid: f32 or bf16 inputs only");
    return CUBED_E_LAYOUT;
  }
  const int64_t n = ti * tj;
  if (cubed_gemm_chain_path(tasks, n, segs, in_dtype, out_dtype) != CUBED_GEMM_MFMA) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_chain_grid: shapes do not fit the MFMA path");
    return CUBED_E_LAYOUT;
  }
  const cubed_gemm_chain_t& T0 = tasks[0];
  const int64_t cm = T0.m, cn = T0.n;
  auto bad = [&](const char* why) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_chain_grid: %s", why);
    return CUBED_E_LAYOUT;
  };
  // a tile spans at most two chunks per dim; a lane's 16-B column group
  // (4 f32 / 8 bf16) never straddles a chunk column
  if ((ti > 1 && cm < HF_BM) || (tj > 1 && cn < HF_BN) || cn % (bf ? 8 : 4)) return bad("chunks narrower than a tile");
  for (int64_t I = 0; I < ti; ++I)
    for (int64_t J = 0; J < tj; ++J) {
      const cubed_gemm_chain_t& T = tasks[I * tj + J];
      if (T.seg0 < 0 || T.seg0 + T.nseg > nsegs) return fail("task out of range");
      if (T.nseg != T0.nseg || T.ktot != T0.ktot || T.accumulate != T0.accumulate) return bad("tasks differ in k");
      if ((I + 1 < ti && T.m != cm) || (J + 1 < tj && T.n != cn) || T.m > cm || T.n > cn || T.m < 1 || T.n < 1)
        return bad("not a regular chunk grid");
      if (T.m != tasks[I * tj].m || T.n != tasks[J].n) return bad("not a regular chunk grid");
      for (int64_t s = 0; s < T.nseg; ++s) {
        const cubed_gemm_seg_t &a = segs[T.seg0 + s], &b = segs[T0.seg0 + s];
        if (a.k != b.k || a.lda != segs[tasks[J].seg0 + s].lda) return bad("segments differ across the grid");
        if (a.ldb != segs[tasks[J].seg0 + s].ldb) return bad("B row pitches differ down a chunk column");
      }
    }
  return 0;
}

extern "C" int cubed_gemm_chain_grid(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks,
                                     int64_t ti, int64_t tj, const cubed_gemm_seg_t* segs,
                                     const cubed_gemm_seg_t* d_segs, int64_t nsegs, int32_t in_dtype,
                                     int32_t out_dtype, const void* d_zero, void* stream) {
  if (!d_tasks || !d_segs || !d_zero) return fail("grid: bad argument");
  if (int rc = cubed_gemm_grid_check(tasks, ti, tj, segs, nsegs, in_dtype, out_dtype)) return rc;
  GemmGrid gg;
  gg.ti = ti;
  gg.tj = tj;
  gg.cm = tasks[0].m;
  gg.cn = tasks[0].n;
  gg.M = (ti - 1) * gg.cm + tasks[(ti - 1) * tj].m;
  gg.N = (tj - 1) * gg.cn + tasks[tj - 1].n;
  const int64_t tm = (gg.M + HF_BM - 1) / HF_BM, tn = (gg.N + HF_BN - 1) / HF_BN;
  if (tm * tn > 0x7fffffff) return fail("grid too large");
  const dim3 grid((unsigned)(tm * tn)), blk(512);
  hipStream_t st = (hipStream_t)stream;
  const char* z = (const char*)d_zero;
  static_assert(HB_BM == HF_BM && HB_BN == HF_BN, "one tile size");
  // bf16: the one-wave full-line kernel (gemm_bf16_w4l.h) when every segment
  // spans a 64-k A tile, else the ping-pong kernel's grid form
  bool w4l = in_dtype == CUBED_BF16;
  for (int64_t i = 0; i < ti * tj && w4l; ++i)
    for (int64_t s = tasks[i].seg0; s < tasks[i].seg0 + tasks[i].nseg; ++s)
      if (segs[s].k < 64) { w4l = false; break; }
  if (w4l && out_dtype == CUBED_BF16)
    hipLaunchKernelGGL((k_gemm_bf16_w4l<true, 4, false, 0, true>), grid, dim3(256), 0, st, d_tasks, d_segs, tm, tn, z,
                       gg, nullptr);
  else if (w4l)
    hipLaunchKernelGGL((k_gemm_bf16_w4l<false, 4, false, 0, true>), grid, dim3(256), 0, st, d_tasks, d_segs, tm, tn, z,
                       gg, nullptr);
  else if (in_dtype == CUBED_BF16 && out_dtype == CUBED_BF16)
    hipLaunchKernelGGL((k_gemm_bf16_chain<true, 0, 1, HB_NS, 4, true>), grid, blk, 0, st, d_tasks, d_segs, tm, tn, z, gg);
  else if (in_dtype == CUBED_BF16)
    hipLaunchKernelGGL((k_gemm_bf16_chain<false, 0, 1, HB_NS, 4, true>), grid, blk, 0, st, d_tasks, d_segs, tm, tn, z, gg);
  else
    hipLaunchKernelGGL((k_gemm_f32_chain<16, 4, false, true>), grid, blk, 0, st, d_tasks, d_segs, tm, tn, z, gg);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}

// ---- packed operands (bf16: gemm_bf16_w4p.h, f32: gemm_f32_w4p.h): the chain set must be a
// regular chunk grid (cubed_gemm_grid_check) of ONE product -- segment s of
// every task in chunk row I reads the same A chunk, of every task in chunk
// column J the same B chunk.
namespace {
constexpr int64_t PACK_SKEW = 0;  // bytes added to every panel's span (L2 set spread)
int pack_plan(const cubed_gemm_chain_t* tasks, int64_t ti, int64_t tj, const cubed_gemm_seg_t* segs, int64_t nsegs,
              int32_t in_dtype, int32_t out_dtype, PackPlan& pp, GemmGrid& gg) {
  if (in_dtype != CUBED_BF16 && in_dtype != CUBED_F32) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_chain_packed: bf16 or f32 inputs only");
    return CUBED_E_LAYOUT;
  }
  if (int rc = cubed_gemm_grid_check(tasks, ti, tj, segs, nsegs, in_dtype, out_dtype)) return rc;
  const int64_t nseg = tasks[0].nseg;
  for (int64_t I = 0; I < ti; ++I)
    for (int64_t J = 0; J < tj; ++J)
      for (int64_t s = 0; s < nseg; ++s) {
        const cubed_gemm_seg_t &g = segs[tasks[I * tj + J].seg0 + s], &a = segs[tasks[I * tj].seg0 + s],
                               &b = segs[tasks[J].seg0 + s];
        if (g.a != a.a || g.lda != a.lda || g.b != b.b || g.ldb != b.ldb) {
          snprintf(g_err, sizeof(g_err), "cubed_gemm_chain_packed: the tasks are not one chunked product");
          return CUBED_E_LAYOUT;
        }
      }
  gg.ti = ti;
  gg.tj = tj;
  gg.cm = tasks[0].m;
  gg.cn = tasks[0].n;
  gg.M = (ti - 1) * gg.cm + tasks[(ti - 1) * tj].m;
  gg.N = (tj - 1) * gg.cn + tasks[tj - 1].n;
  pp.ti = ti;
  pp.tj = tj;
  pp.cm = gg.cm;
  pp.cn = gg.cn;
  pp.M = gg.M;
  pp.N = gg.N;
  pp.K = tasks[0].ktot;
  pp.TM = (pp.M + HB_BM - 1) / HB_BM;
  pp.TN = (pp.N + HB_BN - 1) / HB_BN;
  // k blocks: bf16 64-deep tiles (32 KiB per panel), f32 16-deep steps (16 KiB)
  pp.KTL = in_dtype == CUBED_BF16 ? (pp.K + 63) / 64 : (pp.K + WPF_BK - 1) / WPF_BK;
  if (pp.TM * pp.TN > 0x7fffffff) return fail("grid too large");
  pp.pstride = pp.KTL * (in_dtype == CUBED_BF16 ? WL_ATILE : WPF_SA) + PACK_SKEW;
  pp.apstride = pp.pstride;
  pp.akstride = in_dtype == CUBED_BF16 ? WL_ATILE : WPF_SA;
  pp.kt0 = 0;
  pp.kt1 = pp.KTL;
  return 0;
}

int64_t kblock_k(int32_t in_dtype) { return in_dtype == CUBED_BF16 ? 64 : WPF_BK; }
int64_t kblock_bytes(int32_t in_dtype) { return in_dtype == CUBED_BF16 ? WL_ATILE : WPF_SA; }

// the multi-GPU A image: k-major blocks of the whole A (K blocks x TM panels)
void dist_image(PackPlan& pp, int32_t in_dtype) {
  pp.apstride = kblock_bytes(in_dtype);
  pp.akstride = pp.TM * pp.apstride;
}

// A pack plan of the multi-GPU matmul: ti tasks = A's chunk rows (task I:
// m = rows of chunk row I, segments = the k chunks of that row, a = the
// chunk -- or, where this rank does not hold it, 0 or a halo buffer of the
// few columns its k blocks reach into), packing k blocks [kt0, kt1)
int dist_a_plan(const cubed_gemm_chain_t* at, int64_t ti, const cubed_gemm_seg_t* as, int64_t nsegs,
                int32_t in_dtype, int64_t kt0, int64_t kt1, PackPlan& pp) {
  auto bad = [&](const char* why) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_dist_pack_a: %s", why);
    return CUBED_E_LAYOUT;
  };
  if (in_dtype != CUBED_BF16 && in_dtype != CUBED_F32) return bad("bf16 or f32 inputs only");
  const int64_t isz = in_dtype == CUBED_BF16 ? 2 : 4, kq = 16 / isz;
  const cubed_gemm_chain_t& T0 = at[0];
  const int64_t nseg = T0.nseg, cm = T0.m;
  if (nseg < 1) return bad("no k chunks");
  int64_t M = 0;
  for (int64_t I = 0; I < ti; ++I) {
    const cubed_gemm_chain_t& T = at[I];
    if (T.seg0 < 0 || T.seg0 + T.nseg > nsegs || T.nseg != nseg) return bad("task out of range");
    if ((I + 1 < ti && T.m != cm) || T.m > cm || T.m < 1) return bad("not a regular chunk column");
    for (int64_t s = 0; s < nseg; ++s) {
      const cubed_gemm_seg_t &g = as[T.seg0 + s], &g0 = as[T0.seg0 + s];
      if (g.k != g0.k || g.k < 1 || g.k % kq) return bad("k chunks differ or are not 16-B multiples");
      if ((g.a & 15) || g.lda < 1 || (g.lda * isz) % 16) return bad("A rows not 16-B aligned");
    }
    M += T.m;
  }
  if (ti > 1 && cm < 256) return bad("chunk rows narrower than a panel");
  int64_t K = 0;
  for (int64_t s = 0; s < nseg; ++s) K += as[T0.seg0 + s].k;
  pp.ti = ti;
  pp.tj = 1;
  pp.cm = cm;
  pp.cn = 1;
  pp.M = M;
  pp.N = 1;
  pp.K = K;
  pp.TM = (M + 255) / 256;
  pp.TN = 1;
  const int64_t kb = kblock_k(in_dtype);
  pp.KTL = (K + kb - 1) / kb;
  pp.pstride = 0;
  dist_image(pp, in_dtype);
  if (kt0 < 0 || kt1 > pp.KTL || kt0 >= kt1) return bad("k block range outside the image");
  pp.kt0 = kt0;
  pp.kt1 = kt1;
  // every chunk the range reads must be present (a 0 address is a chunk this
  // rank neither holds nor received: reading it would fault)
  const int64_t k0 = kt0 * kb, k1 = kt1 * kb < K ? kt1 * kb : K;
  int64_t ks = 0;
  for (int64_t s = 0; s < nseg; ++s) {
    const int64_t ke = ks + as[T0.seg0 + s].k;
    if (ks < k1 && ke > k0)
      for (int64_t I = 0; I < ti; ++I)
        if (!as[at[I].seg0 + s].a) return bad("a k chunk the range reads is missing");
    ks = ke;
  }
  return 0;
}
}  // namespace

extern "C" int64_t cubed_gemm_dist_image_bytes(int64_t M, int64_t K, int32_t in_dtype) {
  if (M < 1 || K < 1 || (in_dtype != CUBED_BF16 && in_dtype != CUBED_F32)) return fail("dist image: bad argument");
  const int64_t kb = kblock_k(in_dtype);
  return ((M + 255) / 256) * ((K + kb - 1) / kb) * kblock_bytes(in_dtype);
}

extern "C" int cubed_gemm_dist_pack_a(const cubed_gemm_chain_t* a_tasks, const cubed_gemm_chain_t* d_a_tasks,
                                      int64_t ti, const cubed_gemm_seg_t* a_segs, const cubed_gemm_seg_t* d_a_segs,
                                      int64_t nsegs, int32_t in_dtype, int64_t kt0, int64_t kt1, void* d_image,
                                      int64_t image_bytes, void* stream) {
  if (!a_tasks || !d_a_tasks || !a_segs || !d_a_segs || ti < 1) return fail("dist pack: bad argument");
  PackPlan pp;
  if (int rc = dist_a_plan(a_tasks, ti, a_segs, nsegs, in_dtype, kt0, kt1, pp)) return rc;
  if (!d_image || image_bytes < pp.KTL * pp.akstride || ((uintptr_t)d_image & 255)) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_dist_pack_a: the image is missing, short or not 256-B aligned");
    return CUBED_E_WORKSPACE;
  }
  const int64_t na = pp.TM * (kt1 - kt0);
  const dim3 ga((unsigned)(na < 16384 ? na : 16384));
  hipStream_t st = (hipStream_t)stream;
  if (in_dtype == CUBED_F32)
    hipLaunchKernelGGL(k_pack_a_f32, ga, dim3(256), 0, st, d_a_tasks, d_a_segs, pp, (char*)d_image);
  else
    hipLaunchKernelGGL(k_pack_a, ga, dim3(256), 0, st, d_a_tasks, d_a_segs, pp, (char*)d_image);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}

// the rank's local product: its C chunks (ti x tj grid, columns it owns), B
// from its own chunks, A from the k-major image all ranks filled
static int dist_local_plan(const cubed_gemm_chain_t* tasks, int64_t ti, int64_t tj, const cubed_gemm_seg_t* segs,
                           int64_t nsegs, int32_t in_dtype, int32_t out_dtype, PackPlan& pp, GemmGrid& gg) {
  if (int rc = pack_plan(tasks, ti, tj, segs, nsegs, in_dtype, out_dtype, pp, gg)) return rc;
  dist_image(pp, in_dtype);
  return 0;
}

extern "C" int64_t cubed_gemm_dist_b_bytes(const cubed_gemm_chain_t* tasks, int64_t ti, int64_t tj,
                                           const cubed_gemm_seg_t* segs, int64_t nsegs, int32_t in_dtype,
                                           int32_t out_dtype) {
  if (!tasks || !segs || ti < 1 || tj < 1) return fail("dist: bad argument");
  PackPlan pp;
  GemmGrid gg;
  if (int rc = dist_local_plan(tasks, ti, tj, segs, nsegs, in_dtype, out_dtype, pp, gg)) return rc;
  return pp.TN * pp.pstride;
}

extern "C" int cubed_gemm_dist_pack_b(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks, int64_t ti,
                                      int64_t tj, const cubed_gemm_seg_t* segs, const cubed_gemm_seg_t* d_segs,
                                      int64_t nsegs, int32_t in_dtype, int32_t out_dtype, void* d_ws,
                                      int64_t ws_bytes, void* stream) {
  if (!tasks || !segs || !d_tasks || !d_segs || ti < 1 || tj < 1) return fail("dist: bad argument");
  PackPlan pp;
  GemmGrid gg;
  if (int rc = dist_local_plan(tasks, ti, tj, segs, nsegs, in_dtype, out_dtype, pp, gg)) return rc;
  if (!d_ws || ws_bytes < pp.TN * pp.pstride || ((uintptr_t)d_ws & 255)) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_dist_pack_b: the workspace is missing, short or not 256-B aligned");
    return CUBED_E_WORKSPACE;
  }
  const int64_t nb = pp.TN * pp.KTL;
  const dim3 gb((unsigned)(nb < 16384 ? nb : 16384));
  hipStream_t st = (hipStream_t)stream;
  if (in_dtype == CUBED_F32)
    hipLaunchKernelGGL(k_pack_b_f32, gb, dim3(256), 0, st, d_tasks, d_segs, pp, (char*)d_ws);
  else
    hipLaunchKernelGGL(k_pack_bt, gb, dim3(256), 0, st, d_tasks, d_segs, pp, (char*)d_ws);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}

extern "C" int cubed_gemm_dist_gemm(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks, int64_t ti,
                                    int64_t tj, const cubed_gemm_seg_t* segs, int64_t nsegs, int32_t in_dtype,
                                    int32_t out_dtype, const void* d_image, int64_t image_bytes, const void* d_ws,
                                    int64_t ws_bytes, void* stream) {
  if (!tasks || !segs || !d_tasks || ti < 1 || tj < 1) return fail("dist: bad argument");
  PackPlan pp;
  GemmGrid gg;
  if (int rc = dist_local_plan(tasks, ti, tj, segs, nsegs, in_dtype, out_dtype, pp, gg)) return rc;
  if (!d_image || image_bytes < pp.KTL * pp.akstride || ((uintptr_t)d_image & 255) || !d_ws ||
      ws_bytes < pp.TN * pp.pstride || ((uintptr_t)d_ws & 255)) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_dist_gemm: the A image or B workspace is missing, short or misaligned");
    return CUBED_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(pp.TM * pp.TN));
  const char* PA = (const char*)d_image;
  const char* PB = (const char*)d_ws;
  if (in_dtype == CUBED_F32)
    hipLaunchKernelGGL((k_gemm_f32_w4p<false>), grid, dim3(256), 0, st, d_tasks, PA, PB, pp, gg, nullptr);
  else if (out_dtype == CUBED_BF16)
    hipLaunchKernelGGL((k_gemm_bf16_8p<true>), grid, dim3(512), 0, st, d_tasks, PA, PB, pp, gg, nullptr);
  else
    hipLaunchKernelGGL((k_gemm_bf16_8p<false>), grid, dim3(512), 0, st, d_tasks, PA, PB, pp, gg, nullptr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}

extern "C" int64_t cubed_gemm_pack_bytes(const cubed_gemm_chain_t* tasks, int64_t ti, int64_t tj,
                                         const cubed_gemm_seg_t* segs, int64_t nsegs, int32_t in_dtype,
                                         int32_t out_dtype) {
  if (!tasks || !segs || ti < 1 || tj < 1) return fail("packed: bad argument");
  PackPlan pp;
  GemmGrid gg;
  if (int rc = pack_plan(tasks, ti, tj, segs, nsegs, in_dtype, out_dtype, pp, gg)) return rc;
  // the two images, then the bf16 GEMM's per-XCD round counters (round_wait)
  return (pp.TM + pp.TN) * pp.pstride + PACK_CTR_BYTES;
}

extern "C" int cubed_gemm_chain_packed(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks,
                                       int64_t ti, int64_t tj, const cubed_gemm_seg_t* segs,
                                       const cubed_gemm_seg_t* d_segs, int64_t nsegs, int32_t in_dtype,
                                       int32_t out_dtype, void* d_ws, int64_t ws_bytes, void* stream) {
  if (!tasks || !segs || !d_tasks || !d_segs || ti < 1 || tj < 1) return fail("packed: bad argument");
  PackPlan pp;
  GemmGrid gg;
  if (int rc = pack_plan(tasks, ti, tj, segs, nsegs, in_dtype, out_dtype, pp, gg)) return rc;
  const int64_t bytesA = pp.TM * pp.pstride, bytesB = pp.TN * pp.pstride;
  if (!d_ws || ws_bytes < bytesA + bytesB + PACK_CTR_BYTES || ((uintptr_t)d_ws & 255)) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_chain_packed: the workspace is missing, short or not 256-B aligned");
    return CUBED_E_WORKSPACE;
  }
  char* PA = (char*)d_ws;
  char* PB = PA + bytesA;
  hipStream_t st = (hipStream_t)stream;
  const int64_t na = pp.TM * pp.KTL, nb = pp.TN * pp.KTL;
  const dim3 ga((unsigned)(na < 16384 ? na : 16384)), gb((unsigned)(nb < 16384 ? nb : 16384));
  const dim3 grid((unsigned)(pp.TM * pp.TN));
  if (in_dtype == CUBED_F32) {
    hipLaunchKernelGGL(k_pack_a_f32, ga, dim3(256), 0, st, d_tasks, d_segs, pp, PA);
    hipLaunchKernelGGL(k_pack_b_f32, gb, dim3(256), 0, st, d_tasks, d_segs, pp, PB);
    hipLaunchKernelGGL((k_gemm_f32_w4p<false>), grid, dim3(256), 0, st, d_tasks, (const char*)PA, (const char*)PB, pp,
                       gg, nullptr);
  } else {
    hipLaunchKernelGGL(k_pack_a, ga, dim3(256), 0, st, d_tasks, d_segs, pp, PA);
    hipLaunchKernelGGL(k_pack_bt, gb, dim3(256), 0, st, d_tasks, d_segs, pp, PB);
    // two waves per SIMD on the packed image (gemm_bf16_8p.h; round 6:
    // 1410-1424 TF against the one-wave w4p kernel's 1301-1317, bit-identical),
    // each XCD's rounds of tiles aligned on counters zeroed here (E8_ROUNDS)
    unsigned long long* ctr = (unsigned long long*)(PB + bytesB);
    hipError_t me = hipMemsetAsync(ctr, 0, PACK_CTR_BYTES, st);
    if (me != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(me)); return (int)me; }
    if (out_dtype == CUBED_BF16)
      hipLaunchKernelGGL((k_gemm_bf16_8p<true, false, E8_ROUNDS>), grid, dim3(512), 0, st, d_tasks, (const char*)PA,
                         (const char*)PB, pp, gg, ctr);
    else
      hipLaunchKernelGGL((k_gemm_bf16_8p<false, false, E8_ROUNDS>), grid, dim3(512), 0, st, d_tasks, (const char*)PA,
                         (const char*)PB, pp, gg, ctr);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}
