// blas.hip -- chunk GEMMs through rocBLAS (plain library GEMMs).
//
// The per-task product of blockwise matmul / tensordot
// (cubed/array_api/linear_algebra_functions.py:62-64, numpy's BLAS call) is a
// plain GEMM with no fused prologue/epilogue, so it goes to the vendor BLAS:
// tasks of equal shape form one rocblas_{s,d}gemm_batched call (pointer
// arrays built by the host from the task table).  Row-major C = A @ B is the
// column-major product C^T = B^T A^T, so B and A swap places in the call.
// The hand-written MFMA kernel (gemm.hip) remains for int64 and as the
// CUBED_AMD_GEMM=native path.  One rocBLAS handle per device, created once.
#include "common.h"
#include <rocblas/rocblas.h>
#include <mutex>
#include <stdio.h>

namespace cubed {
extern thread_local char g_err[512];
}
using namespace cubed;

static std::mutex g_blas_mu;
static rocblas_handle g_handles[64];

static rocblas_handle handle_for_current_device(int* err) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) { *err = CUBED_E_ARG; return nullptr; }
  if (!g_handles[dev]) {
    rocblas_handle h;
    if (rocblas_create_handle(&h) != rocblas_status_success) { *err = CUBED_E_ARG; return nullptr; }
    g_handles[dev] = h;
  }
  return g_handles[dev];
}

extern "C" int cubed_gemm_batched(int32_t dtype, const void* d_a_ptrs, const void* d_b_ptrs,
                                  const void* d_c_ptrs, int64_t batch, int64_t m, int64_t n, int64_t k,
                                  int64_t lda, int64_t ldb, int64_t ldc, int32_t accumulate,
                                  void* stream) {
  if (batch == 0 || m == 0 || n == 0) return 0;
  if (!d_a_ptrs || !d_b_ptrs || !d_c_ptrs || batch < 0 || m < 0 || n < 0 || k < 0) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_batched: bad argument");
    return CUBED_E_ARG;
  }
  std::lock_guard<std::mutex> lock(g_blas_mu);
  int err = 0;
  rocblas_handle h = handle_for_current_device(&err);
  if (!h) {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_batched: rocblas_create_handle failed");
    return err;
  }
  rocblas_set_stream(h, (hipStream_t)stream);
  rocblas_status s;
  if (dtype == CUBED_F32) {
    const float alpha = 1.f, beta = accumulate ? 1.f : 0.f;
    s = rocblas_sgemm_batched_64(h, rocblas_operation_none, rocblas_operation_none, n, m, k, &alpha,
                                 (const float* const*)d_b_ptrs, ldb, (const float* const*)d_a_ptrs, lda,
                                 &beta, (float* const*)d_c_ptrs, ldc, batch);
  } else if (dtype == CUBED_F64) {
    const double alpha = 1.0, beta = accumulate ? 1.0 : 0.0;
    s = rocblas_dgemm_batched_64(h, rocblas_operation_none, rocblas_operation_none, n, m, k, &alpha,
                                 (const double* const*)d_b_ptrs, ldb, (const double* const*)d_a_ptrs, lda,
                                 &beta, (double* const*)d_c_ptrs, ldc, batch);
  } else {
    snprintf(g_err, sizeof(g_err), "cubed_gemm_batched: dtype %d has no BLAS path", dtype);
    return CUBED_E_DTYPE;
  }
  if (s != rocblas_status_success) {
    snprintf(g_err, sizeof(g_err), "rocBLAS gemm failed: %s", rocblas_status_to_string(s));
    return CUBED_E_ARG;
  }
  return 0;
}
