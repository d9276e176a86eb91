// gemm.hip -- batched chunk GEMMs for blockwise matmul / tensordot.
//
// Replaces the per-task numpy BLAS call of _matmul
// (cubed/array_api/linear_algebra_functions.py:62-64): every (i, k, j) task of
// the blockwise contraction is one C_t = A_t @ B_t on a chunk pair.
// f32: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate), a 64x64
// output tile per 256-thread workgroup (2x2 waves of 32x32), K staged through
// LDS 16 deep.  f64 uses the same tiling with vector FMAs.
#include "common.h"
#include <stdio.h>

namespace cubed {
extern thread_local char g_err[512];
}
using namespace cubed;

typedef float f32x16 __attribute__((ext_vector_type(16)));

static constexpr int TM = 64, TN = 64, TK = 16;

__global__ __launch_bounds__(256) void k_gemm_f32(const cubed_gemm_task_t* __restrict__ tasks,
                                                  int64_t ntasks, int64_t tiles_m, int64_t tiles_n) {
  __shared__ float As[TK][TM + 4];
  __shared__ float Bs[TK][TN + 4];
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int64_t tpt = tiles_m * tiles_n;
  const int64_t t = g / tpt, tile = g % tpt;
  if (t >= ntasks) return;
  const cubed_gemm_task_t* __restrict__ T = tasks + t;
  const int64_t M = T->m, N = T->n, K = T->k;
  const int64_t m0 = (tile / tiles_n) * TM, n0 = (tile % tiles_n) * TN;
  if (m0 >= M || n0 >= N) return;
  const float* __restrict__ A = (const float*)T->a;
  const float* __restrict__ B = (const float*)T->b;
  float* __restrict__ C = (float*)T->c;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int64_t k0 = 0; k0 < K; k0 += TK) {
    // stage A[m0:m0+64, k0:k0+16] transposed into As[k][m], B[k0:k0+16, n0:n0+64] into Bs[k][n]
    for (int i = tid; i < TM * TK; i += 256) {
      const int mm = i / TK, kk = i % TK;
      const int64_t gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < M && gk < K) ? A[gm * T->lda + gk] : 0.f;
    }
    for (int i = tid; i < TN * TK; i += 256) {
      const int kk = i / TN, nn = i % TN;
      const int64_t gk = k0 + kk, gn = n0 + nn;
      Bs[kk][nn] = (gk < K && gn < N) ? B[gk * T->ldb + gn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; kk += 2) {
      // lane l: A[i = l&31][k = l>>5], B[k = l>>5][j = l&31]
      const float a = As[kk + (lane >> 5)][wm + (lane & 31)];
      const float b = Bs[kk + (lane >> 5)][wn + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // C/D map: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int64_t gm = m0 + wm + row, gn = n0 + wn + (lane & 31);
    if (gm < M && gn < N) {
      float* c = C + gm * T->ldc + gn;
      *c = T->accumulate ? (*c + acc[r]) : acc[r];
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
  const int64_t tm = (max_m + TM - 1) / TM, tn = (max_n + TN - 1) / TN;
  const int64_t blocks = ntasks * tm * tn;
  dim3 grid(blocks <= 0x7fffffff ? (unsigned)blocks : 0x7fffffffu,
            blocks <= 0x7fffffff ? 1u : (unsigned)((blocks + 0x7ffffffe) / 0x7fffffff));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CUBED_F32) {
    hipLaunchKernelGGL(k_gemm_f32, grid, dim3(256), 0, st, d_tasks, ntasks, tm, tn);
  } else if (dtype == CUBED_F64) {
    hipLaunchKernelGGL(k_gemm_scalar<double>, grid, dim3(256), 0, st, d_tasks, ntasks, tm, tn);
  } else if (dtype == CUBED_I64) {
    hipLaunchKernelGGL(k_gemm_scalar<int64_t>, grid, dim3(256), 0, st, d_tasks, ntasks, tm, tn);
  } else {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_chunks: dtype %d not supported", dtype);
    return CUBED_E_DTYPE;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}
