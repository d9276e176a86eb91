// gemm.hip -- batched chunk GEMMs for blockwise matmul / tensordot.
//
// Replaces the per-task numpy BLAS call of _matmul
// (cubed/array_api/linear_algebra_functions.py:62-64): every (i, k, j) task of
// the blockwise contraction is one C_t = A_t @ B_t on a chunk pair.
// f32: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate), 128x128
// output tiles (below).  f64 / int64: 64x64 tiles of vector FMAs.
// f32 and f64 products run on rocBLAS by default (blas.hip: 125 TF vs this
// kernel's 102 TF on 8 x 5000^3, tools/gemm_probe.py); these kernels serve
// int64 and CUBED_AMD_GEMM=native.  A K-permuted variant reading b128 operand
// fragments (4 MFMAs per LDS read) measured 72 TF -- the transposed B staging
// stores conflict -- and was dropped.
#include "common.h"
#include <stdio.h>

namespace cubed {
extern thread_local char g_err[512];
}
using namespace cubed;

typedef float f32x16 __attribute__((ext_vector_type(16)));

static constexpr int TM = 64, TN = 64, TK = 16;  // scalar (f64 / int64) kernel tile

// ------------------------------------------------------------------ f32 on MFMA
// 128x128 output tile per 256-thread workgroup: 2x2 waves, each wave a 64x64
// sub-tile = 2x2 v_mfma_f32_32x32x2_f32 accumulators (64 acc VGPRs).  K is
// staged through LDS 32 deep, k-major (As[k][m], Bs[k][n]) so a half-wave
// reads 32 consecutive floats per operand; the next K tile's global loads
// (float4 where the rows allow it) are issued before the current tile's 64
// MFMAs per wave, so HBM/L2 latency hides behind the matrix cores.
// Blocks are remapped so that each XCD walks a contiguous run of tiles (the
// 8 XCDs have private L2s; consecutive tiles share an A row panel).
static constexpr int BM = 128, BN = 128, BK = 32;

struct F4 { float x, y, z, w; };

template <int KU, int MINW, int LDA_S, int LDB_S>
__global__ __launch_bounds__(256, MINW) void k_gemm_f32(const cubed_gemm_task_t* __restrict__ tasks,
                                                  int64_t ntasks, int64_t tiles_m, int64_t tiles_n) {
  __shared__ float As[BK][LDA_S];
  __shared__ float Bs[BK][LDB_S];
  const int64_t nblk = (int64_t)gridDim.x * gridDim.y;
  int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  if ((nblk & 7) == 0) g = (g & 7) * (nblk >> 3) + (g >> 3);  // XCD-contiguous tile runs
  const int64_t tpt = tiles_m * tiles_n;
  const int64_t t = g / tpt, tile = g % tpt;
  if (t >= ntasks) return;
  const cubed_gemm_task_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n, K = T->k;
  // group-M swizzle: tiles walk 8 tile-rows at a time, column by column, so
  // the blocks resident on one XCD share 8 A panels and 8 B panels in L2
  constexpr int64_t GM = 8;
  const int64_t per_group = GM * tiles_n;
  const int64_t grp = tile / per_group, first_m = grp * GM;
  const int64_t gsz = (tiles_m - first_m) < GM ? (tiles_m - first_m) : GM;
  const int64_t in_g = tile - grp * per_group;
  const int64_t m0 = (first_m + in_g % gsz) * BM, n0 = (in_g / gsz) * BN;
  if (m0 >= M || n0 >= N) return;
  const int64_t lda = T->lda, ldb = T->ldb;
  // float4 operand loads where every row of the operand is 16-B aligned
  const bool VA = (((uint64_t)T->a | (uint64_t)(lda * 4)) & 15) == 0;
  const bool VB = (((uint64_t)T->b | (uint64_t)(ldb * 4)) & 15) == 0;
  const CUBED_G float* __restrict__ A = (const CUBED_G float*)(uintptr_t)T->a;
  const CUBED_G float* __restrict__ B = (const CUBED_G float*)(uintptr_t)T->b;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  F4 ra[4], rb[4];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 256 * i;
      // A tile: 128 rows x 8 float4 along k
      const int row = f >> 3, kq = (f & 7) * 4;
      const int64_t gm = m0 + row, gk = k0 + kq;
      if (VA && gm < M && gk + 3 < K) {
        const f32x4 v = *(const CUBED_G f32x4*)(A + gm * lda + gk);
        ra[i] = F4{v.x, v.y, v.z, v.w};
      } else {
        float e[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) e[c] = (gm < M && gk + c < K) ? A[gm * lda + gk + c] : 0.f;
        ra[i] = F4{e[0], e[1], e[2], e[3]};
      }
      // B tile: 32 k-rows x 32 float4 along n
      const int kr = f >> 5, nq = (f & 31) * 4;
      const int64_t gk2 = k0 + kr, gn = n0 + nq;
      if (VB && gk2 < K && gn + 3 < N) {
        const f32x4 v = *(const CUBED_G f32x4*)(B + gk2 * ldb + gn);
        rb[i] = F4{v.x, v.y, v.z, v.w};
      } else {
        float e[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) e[c] = (gk2 < K && gn + c < N) ? B[gk2 * ldb + gn + c] : 0.f;
        rb[i] = F4{e[0], e[1], e[2], e[3]};
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 256 * i;
      const int row = f >> 3, kq = (f & 7) * 4;
      As[kq + 0][row] = ra[i].x;
      As[kq + 1][row] = ra[i].y;
      As[kq + 2][row] = ra[i].z;
      As[kq + 3][row] = ra[i].w;
      const int kr = f >> 5, nq = (f & 31) * 4;
      f32x4 v;
      v.x = rb[i].x; v.y = rb[i].y; v.z = rb[i].z; v.w = rb[i].w;
      *(f32x4*)&Bs[kr][nq] = v;
    }
  };

  load(0);
  store();
  __syncthreads();
  const int hi = lane >> 5, lo = lane & 31;
  for (int64_t k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more) load(k0 + BK);  // in flight during this tile's MFMAs
#pragma unroll KU
    for (int kk = 0; kk < BK; kk += 2) {
      const float a0 = As[kk + hi][wm + lo], a1 = As[kk + hi][wm + 32 + lo];
      const float b0 = Bs[kk + hi][wn + lo], b1 = Bs[kk + hi][wn + 32 + lo];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }
  // C/D map of a 32x32 accumulator: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  CUBED_G float* __restrict__ C = (CUBED_G float*)(uintptr_t)T->c;
  const bool accum = T->accumulate != 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * hi;
        const int64_t gm = m0 + wm + 32 * i + row, gn = n0 + wn + 32 * j + lo;
        if (gm < M && gn < N) {
          CUBED_G float* c = C + gm * T->ldc + gn;
          *c = accum ? (*c + acc[i][j][r]) : acc[i][j][r];
        }
      }
}

// c + a*b: fused for f64 (matches BLAS dgemm's FMA accumulation), wrapping for int64
CUBED_DEV double mul_add(double a, double b, double c) { return fma(a, b, c); }
CUBED_DEV int64_t mul_add(int64_t a, int64_t b, int64_t c) {
  return (int64_t)((uint64_t)c + (uint64_t)a * (uint64_t)b);
}

template <typename T>
__global__ __launch_bounds__(256) void k_gemm_scalar(const cubed_gemm_task_t* __restrict__ tasks,
                                                  int64_t ntasks, int64_t tiles_m, int64_t tiles_n) {
  __shared__ T As[TK][TM + 1];
  __shared__ T Bs[TK][TN + 1];
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int64_t tpt = tiles_m * tiles_n;
  const int64_t t = g / tpt, tile = g % tpt;
  if (t >= ntasks) return;
  const cubed_gemm_task_t* __restrict__ TT = tasks + t;
  const int64_t M = TT->m, N = TT->n, K = TT->k;
  const int64_t m0 = (tile / tiles_n) * TM, n0 = (tile % tiles_n) * TN;
  if (m0 >= M || n0 >= N) return;
  const T* __restrict__ A = (const T*)TT->a;
  const T* __restrict__ B = (const T*)TT->b;
  T* __restrict__ C = (T*)TT->c;
  const int tid = threadIdx.x;
  const int tr = (tid >> 4) * 4, tc = (tid & 15) * 4;  // 4x4 per thread
  T acc[4][4] = {};
  for (int64_t k0 = 0; k0 < K; k0 += TK) {
    for (int i = tid; i < TM * TK; i += 256) {
      const int mm = i / TK, kk = i % TK;
      const int64_t gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < M && gk < K) ? A[gm * TT->lda + gk] : (T)0;
    }
    for (int i = tid; i < TN * TK; i += 256) {
      const int kk = i / TN, nn = i % TN;
      const int64_t gk = k0 + kk, gn = n0 + nn;
      Bs[kk][nn] = (gk < K && gn < N) ? B[gk * TT->ldb + gn] : (T)0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; ++kk) {
      T a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = As[kk][tr + i]; b[i] = Bs[kk][tc + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mul_add(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gm = m0 + tr + i, gn = n0 + tc + j;
      if (gm < M && gn < N) {
        T* c = C + gm * TT->ldc + gn;
        *c = TT->accumulate ? (*c + acc[i][j]) : acc[i][j];
      }
    }
}

extern "C" int cubed_gemm_chunks(const cubed_gemm_task_t* d_tasks, int64_t ntasks, int32_t dtype,
                                 int64_t max_m, int64_t max_n, void* stream) {
  if (ntasks == 0) return 0;
  if (!d_tasks || max_m <= 0 || max_n <= 0) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_chunks: bad argument");
    return CUBED_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CUBED_F32) {
    const int64_t tm = (max_m + BM - 1) / BM, tn = (max_n + BN - 1) / BN;
    const int64_t blocks = ntasks * tm * tn;
    if (blocks > 0x7fffffff) { snprintf(g_err, sizeof(g_err), "cubed_gemm_chunks: grid too large"); return CUBED_E_ARG; }
    // KU=4 (k-steps unrolled), >= 2 workgroups per CU of registers (3 waves
    // per SIMD), B tile rows 160 floats apart (conflict-free half-wave reads):
    // 102 TF on 8 x 5000^3 vs 90 TF fully unrolled at 2 waves/SIMD
    // (tools/gemm_probe.py; LDS padding of A and unroll 2/8 within 2 %)
    hipLaunchKernelGGL((k_gemm_f32<4, 2, BM + 4, BN + 32>), dim3((unsigned)blocks, 1, 1), dim3(256), 0, st,
                       d_tasks, ntasks, tm, tn);
  } else if (dtype == CUBED_F64 || dtype == CUBED_I64) {
    const int64_t tm = (max_m + TM - 1) / TM, tn = (max_n + TN - 1) / TN;
    const int64_t blocks = ntasks * tm * tn;
    dim3 grid(blocks <= 0x7fffffff ? (unsigned)blocks : 0x7fffffffu,
              blocks <= 0x7fffffff ? 1u : (unsigned)((blocks + 0x7ffffffe) / 0x7fffffff));
    if (dtype == CUBED_F64)
      hipLaunchKernelGGL(k_gemm_scalar<double>, grid, dim3(256), 0, st, d_tasks, ntasks, tm, tn);
    else
      hipLaunchKernelGGL(k_gemm_scalar<int64_t>, grid, dim3(256), 0, st, d_tasks, ntasks, tm, tn);
  } else {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_chunks: dtype %d not supported", dtype);
    return CUBED_E_DTYPE;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}
