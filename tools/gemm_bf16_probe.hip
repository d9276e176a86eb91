// gemm_bf16_probe.hip -- development probe (not part of the library): times
// the chained bf16 GEMM of BASELINE config 5 (40000^2 in 5000^2 chunks: 64
// output chunks x 8 k segments, chunk-contiguous slots as the executor lays
// them out) for kernel variants and ablations, in one process.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude \
//          -o tools/gemm_bf16_probe tools/gemm_bf16_probe.hip
// Run:   tools/gemm_bf16_probe [reps]
// (Rounds 2-3.  The library kernels gained a GemmGrid argument in round 4;
// the experiment kernels here keep the 5-argument form, so this probe builds
// against gemm_chain.hip as of commit 1cdef52^ -- its logs are in profiles/.)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

namespace cubed {
thread_local char g_err[512];
}
#include "../cubed_amd/csrc/gemm_chain.hip"
#include "gemm_bf16_experiments.h"
#include "gemm_bf16_bt.h"
#include "gemm_bf16_8ph.h"
#include "gemm_bf16_stamp.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_fill(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float v = (float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f;  // [-1, 1)
    p[i] = (uint16_t)(__float_as_uint(v) >> 16);
  }
}

__global__ void k_diff(const float* a, const float* b, int64_t n, float* out) {
  float m = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(a[i] - b[i]));
  atomicMax((int*)out, __float_as_int(m));
}

typedef void (*kfn)(const cubed_gemm_chain_t*, const cubed_gemm_seg_t*, int64_t, int64_t, const char*);

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 2;
  const int64_t N = 40000, Cc = 5000, nb = N / Cc;
  const int64_t slot_in = (Cc * Cc * 2 + 255) / 256 * 256, slot_out = (Cc * Cc * 4 + 255) / 256 * 256;
  char *A, *B, *C0, *C1, *Z;
  CHECK(hipMalloc(&A, slot_in * nb * nb));
  CHECK(hipMalloc(&B, slot_in * nb * nb));
  CHECK(hipMalloc(&C0, slot_out * nb * nb));
  CHECK(hipMalloc(&C1, slot_out * nb * nb));
  CHECK(hipMalloc(&Z, 4096));
  CHECK(hipMemset(Z, 0, 4096));
  CHECK(hipMemset(C0, 0, slot_out * nb * nb));
  CHECK(hipMemset(C1, 0, slot_out * nb * nb));
  k_fill<<<4096, 256>>>((uint16_t*)A, slot_in * nb * nb / 2, 12345u);
  k_fill<<<4096, 256>>>((uint16_t*)B, slot_in * nb * nb / 2, 777u);
  std::vector<cubed_gemm_chain_t> tasks(nb * nb);
  std::vector<cubed_gemm_seg_t> segs(nb * nb * nb);
  for (int64_t i = 0; i < nb; ++i)
    for (int64_t j = 0; j < nb; ++j) {
      const int64_t t = i * nb + j;
      tasks[t] = {0, Cc, Cc, Cc, t * nb, nb, N, 0};
      for (int64_t k = 0; k < nb; ++k)
        segs[t * nb + k] = {(int64_t)(uintptr_t)(A + (i * nb + k) * slot_in),
                            (int64_t)(uintptr_t)(B + (k * nb + j) * slot_in), Cc, Cc, Cc, 0};
    }
  // B^T chunks (n x k, pitch k) for the transposed-B variants
  char* BT;
  CHECK(hipMalloc(&BT, slot_in * nb * nb));
  {
    const int64_t per = ((Cc + 63) / 64) * ((Cc + 63) / 64);
    k_transpose_bf16<<<(unsigned)(per * nb * nb), 256>>>((const uint16_t*)B, (uint16_t*)BT, Cc, Cc, slot_in,
                                                        nb * nb);
    CHECK(hipDeviceSynchronize());
  }
  std::vector<cubed_gemm_seg_t> segs_bt(segs);
  for (int64_t i = 0; i < nb; ++i)
    for (int64_t j = 0; j < nb; ++j)
      for (int64_t k = 0; k < nb; ++k)
        segs_bt[(i * nb + j) * nb + k].b = (int64_t)(uintptr_t)(BT + (k * nb + j) * slot_in);
  cubed_gemm_seg_t* dsbt;
  CHECK(hipMalloc(&dsbt, sizeof(cubed_gemm_seg_t) * segs.size()));
  CHECK(hipMemcpy(dsbt, segs_bt.data(), sizeof(cubed_gemm_seg_t) * segs.size(), hipMemcpyHostToDevice));
  cubed_gemm_chain_t *dt0, *dt1;
  cubed_gemm_seg_t* ds;
  CHECK(hipMalloc(&dt0, sizeof(cubed_gemm_chain_t) * tasks.size()));
  CHECK(hipMalloc(&dt1, sizeof(cubed_gemm_chain_t) * tasks.size()));
  CHECK(hipMalloc(&ds, sizeof(cubed_gemm_seg_t) * segs.size()));
  for (auto& t : tasks) t.c = (int64_t)(uintptr_t)(C0 + (&t - &tasks[0]) * slot_out);
  CHECK(hipMemcpy(dt0, tasks.data(), sizeof(cubed_gemm_chain_t) * tasks.size(), hipMemcpyHostToDevice));
  for (auto& t : tasks) t.c = (int64_t)(uintptr_t)(C1 + (&t - &tasks[0]) * slot_out);
  CHECK(hipMemcpy(dt1, tasks.data(), sizeof(cubed_gemm_chain_t) * tasks.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(ds, segs.data(), sizeof(cubed_gemm_seg_t) * segs.size(), hipMemcpyHostToDevice));
  const int64_t tm = (Cc + HB_BM - 1) / HB_BM, tn = (Cc + HB_BN - 1) / HB_BN;
  const dim3 grid((unsigned)(nb * nb * tm * tn)), blk(512);
  const double flop = 2.0 * N * N * N;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float* dmax;
  CHECK(hipMalloc(&dmax, 4));

  struct V { const char* name; kfn f; bool check; int threads = 0; bool bt = false; };
  V vs[] = {
      {"ping-pong NS4 (default)", k_gemm_bf16_chain<false, 0, 1>, false},
      {"8-phase, B^T", k_gemm_bf16_8ph<false, 4, true>, true, 0, true},
      {"8-phase, B^T, no setprio", k_gemm_bf16_8ph<false, 4, false>, true, 0, true},
      {"ping-pong NS4 (again)", k_gemm_bf16_chain<false, 0, 1>, true},
  };
  const int only = argc > 2 ? atoi(argv[2]) : -1;  // run one variant (PMC passes)
  if (only == 99 || only == 98) {  // stamped diagnostic builds: per-segment cycle shares
    unsigned long long* dbg;
    const size_t nd = (size_t)grid.x * 8 * 8;
    CHECK(hipMalloc(&dbg, nd * 8));
    std::vector<unsigned long long> h(nd);
    for (int r = 0; r < 3; ++r) {
      CHECK(hipMemset(dbg, 0, nd * 8));
      CHECK(hipEventRecord(e0));
      if (only == 99)
        hipLaunchKernelGGL((k_gemm_bf16_stamp<false>), grid, blk, 0, 0, dbg, dt1, ds, tm, tn, (const char*)Z);
      else
        hipLaunchKernelGGL((k_gemm_bf16_stamp_cs<false>), grid, blk, 0, 0, dbg, dt1, ds, tm, tn, (const char*)Z);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      CHECK(hipMemcpy(h.data(), dbg, nd * 8, hipMemcpyDeviceToHost));
      const char* names[6] = {"M: fragment reads (+lgkm wait)", only == 99 ? "M: staging issue" : "M: staging addresses", "M: vmcnt wait",
                              "barrier into C", "C: 32 MFMA issue", "barrier out of C + loop"};
      double tot[2][6] = {{0}}, cnt[2] = {0, 0};
      for (size_t b = 0; b < grid.x; ++b)
        for (int w = 0; w < 8; ++w) {
          const unsigned long long* o = &h[(b * 8 + w) * 8];
          unsigned long long s = 0;
          for (int i = 0; i < 6; ++i) s += o[i];
          if (!s) continue;
          for (int i = 0; i < 6; ++i) tot[w >> 2][i] += (double)o[i];
          cnt[w >> 2] += 1;
        }
      const double steps = (double)((N + 31) / 32);
      printf("stamped run %d: %.3f ms (%.1f TF, diagnostic build)\n", r, ms, flop / ms / 1e9);
      for (int i = 0; i < 6; ++i)
        printf("  %-34s row0 %8.1f  row1 %8.1f cyc/step\n", names[i], tot[0][i] / cnt[0] / steps,
               tot[1][i] / cnt[1] / steps);
    }
    return 0;
  }
  for (const V& v : vs) {
    if (only >= 0 && &v - vs != only) continue;
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(v.f, grid, v.threads ? dim3(v.threads) : blk, 0, 0, v.check ? dt1 : dt0, v.bt ? dsbt : ds,
                         tm, tn, (const char*)Z);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    printf("%-36s %9.3f ms %7.1f TF\n", v.name, best, flop / best / 1e9);
    if (v.check) {
      CHECK(hipMemset(dmax, 0, 4));
      k_diff<<<4096, 256>>>((const float*)C0, (const float*)C1, slot_out * nb * nb / 4, dmax);
      float m;
      CHECK(hipMemcpy(&m, dmax, 4, hipMemcpyDeviceToHost));
      printf("   max |diff| vs base: %g\n", m);
    }
    fflush(stdout);
  }
  return 0;
}
