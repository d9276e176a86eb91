// gemm_f32_probe.hip -- development probe (not part of the library): times
// the chained f32 GEMM of BASELINE config 5 (40000^2 in 5000^2 chunks: 64
// output chunks x 8 k segments, chunk-contiguous slots) for kernel variants
// of csrc/gemm_chain.hip's k_gemm_f32_chain<BK, NS>, in one process; every
// variant's output is compared with the first's (max |diff|).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude \
//          -o tools/gemm_f32_probe tools/gemm_f32_probe.hip
// Run:   tools/gemm_f32_probe [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

namespace cubed {
thread_local char g_err[512];
}
#include "../cubed_amd/csrc/gemm_chain.hip"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_fill(float* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = (float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f;  // [-1, 1)
  }
}

__global__ void k_diff(const float* a, const float* b, int64_t n, float* out) {
  float m = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(a[i] - b[i]));
  atomicMax((int*)out, __float_as_int(m));
}

typedef void (*kfn)(const cubed_gemm_chain_t*, const cubed_gemm_seg_t*, int64_t, int64_t, const char*, GemmGrid);

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 1;
  const int64_t N = 40000, Cc = 5000, nb = N / Cc;
  const int64_t slot = (Cc * Cc * 4 + 255) / 256 * 256;
  char *A, *B, *C0, *C1, *Z;
  CHECK(hipMalloc(&A, slot * nb * nb));
  CHECK(hipMalloc(&B, slot * nb * nb));
  CHECK(hipMalloc(&C0, slot * nb * nb));
  CHECK(hipMalloc(&C1, slot * nb * nb));
  CHECK(hipMalloc(&Z, 4096));
  CHECK(hipMemset(Z, 0, 4096));
  k_fill<<<4096, 256>>>((float*)A, slot * nb * nb / 4, 12345u);
  k_fill<<<4096, 256>>>((float*)B, slot * nb * nb / 4, 777u);
  std::vector<cubed_gemm_chain_t> tasks(nb * nb);
  std::vector<cubed_gemm_seg_t> segs(nb * nb * nb);
  for (int64_t i = 0; i < nb; ++i)
    for (int64_t j = 0; j < nb; ++j) {
      const int64_t t = i * nb + j;
      tasks[t] = {0, Cc, Cc, Cc, t * nb, nb, N, 0};
      for (int64_t k = 0; k < nb; ++k)
        segs[t * nb + k] = {(int64_t)(uintptr_t)(A + (i * nb + k) * slot), (int64_t)(uintptr_t)(B + (k * nb + j) * slot),
                            Cc, Cc, Cc, 0};
    }
  cubed_gemm_chain_t *dt0, *dt1;
  cubed_gemm_seg_t* ds;
  CHECK(hipMalloc(&dt0, sizeof(cubed_gemm_chain_t) * tasks.size()));
  CHECK(hipMalloc(&dt1, sizeof(cubed_gemm_chain_t) * tasks.size()));
  CHECK(hipMalloc(&ds, sizeof(cubed_gemm_seg_t) * segs.size()));
  for (auto& t : tasks) t.c = (int64_t)(uintptr_t)(C0 + (&t - &tasks[0]) * slot);
  CHECK(hipMemcpy(dt0, tasks.data(), sizeof(cubed_gemm_chain_t) * tasks.size(), hipMemcpyHostToDevice));
  for (auto& t : tasks) t.c = (int64_t)(uintptr_t)(C1 + (&t - &tasks[0]) * slot);
  CHECK(hipMemcpy(dt1, tasks.data(), sizeof(cubed_gemm_chain_t) * tasks.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(ds, segs.data(), sizeof(cubed_gemm_seg_t) * segs.size(), hipMemcpyHostToDevice));
  const int64_t tm = (Cc + HF_BM - 1) / HF_BM, tn = (Cc + HF_BN - 1) / HF_BN;
  const dim3 grid((unsigned)(nb * nb * tm * tn)), blk(512);
  const double flop = 2.0 * N * N * N;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float* dmax;
  CHECK(hipMalloc(&dmax, 4));
  struct V { const char* name; kfn f; bool check; };
  V vs[] = {
      {"BK16 NS4 (library)", k_gemm_f32_chain<16, 4>, false},
      {"BK16 NS4 ping-pong", k_gemm_f32_chain<16, 4, true>, true},
      {"BK16 NS3 ping-pong", k_gemm_f32_chain<16, 3, true>, true},
      {"BK16 NS4 (again)", k_gemm_f32_chain<16, 4>, true},
      {"BK16 NS4 ping-pong (again)", k_gemm_f32_chain<16, 4, true>, true},
  };
  for (const V& v : vs) {
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(v.f, grid, blk, 0, 0, v.check ? dt1 : dt0, ds, tm, tn, (const char*)Z, GemmGrid{});
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    printf("%-28s %9.3f ms %7.1f TF\n", v.name, best, flop / best / 1e9);
    if (v.check) {
      CHECK(hipMemset(dmax, 0, 4));
      k_diff<<<4096, 256>>>((const float*)C0, (const float*)C1, slot * nb * nb / 4, dmax);
      float m;
      CHECK(hipMemcpy(&m, dmax, 4, hipMemcpyDeviceToHost));
      printf("   max |diff| vs first: %g\n", m);
    }
    fflush(stdout);
  }
  return 0;
}
