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
#include "gemm_f32_w4.h"

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
typedef void (*kfn_s)(const cubed_gemm_chain_t*, const cubed_gemm_seg_t*, int64_t, int64_t, const char*, GemmGrid,
                      unsigned long long*);

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
  if (argc > 2 && argv[2][0] == 'p') {  // packed operands (csrc/gemm_f32_w4p.h) vs the library grid kernel
    GemmGrid gg{nb, nb, Cc, Cc, N, N};
    const int64_t gtm = (N + HF_BM - 1) / HF_BM;
    const int64_t wsb = cubed_gemm_pack_bytes(tasks.data(), nb, nb, segs.data(), segs.size(), CUBED_F32, CUBED_F32);
    if (wsb <= 0) { printf("pack_bytes: %s\n", g_err); return 1; }
    char* ws;
    CHECK(hipMalloc(&ws, wsb));
    PackPlan pp;
    if (pack_plan(tasks.data(), nb, nb, segs.data(), segs.size(), CUBED_F32, CUBED_F32, pp, gg)) return 1;
    unsigned long long* st;
    CHECK(hipMalloc(&st, (size_t)gtm * gtm * 8 * 8));
    if (argv[2][1] == 's') {  // panel-stride skews: pack + GEMM launched here, each skew twice
      char* ws2;
      const int64_t extra = 1 << 20;
      CHECK(hipMalloc(&ws2, wsb + (pp.TM + pp.TN) * extra));
      const int64_t base_stride = pp.KTL * WPF_SA;
      const int64_t skews[] = {0, 1024, 2048 + 128, 4096, 65536 + 1024, 0};
      for (int64_t sk : skews) {
        PackPlan q = pp;
        q.pstride = base_stride + sk;
        char* QA = ws2;
        char* QB = ws2 + q.TM * q.pstride;
        const int64_t na = q.TM * q.KTL, nbk = q.TN * q.KTL;
        hipLaunchKernelGGL(k_pack_a_f32, dim3((unsigned)(na < 16384 ? na : 16384)), dim3(256), 0, 0, dt1, ds, q, QA);
        hipLaunchKernelGGL(k_pack_b_f32, dim3((unsigned)(nbk < 16384 ? nbk : 16384)), dim3(256), 0, 0, dt1, ds, q, QB);
        for (int r = 0; r < 2; ++r) {
          float ms;
          CHECK(hipEventRecord(e0));
          hipLaunchKernelGGL((k_gemm_f32_w4p<false>), dim3((unsigned)(gtm * gtm)), dim3(256), 0, 0, dt1, (const char*)QA,
                             (const char*)QB, q, gg, (unsigned long long*)nullptr);
          CHECK(hipEventRecord(e1));
          CHECK(hipEventSynchronize(e1));
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          printf("skew %6lld: w4p GEMM %9.3f ms %7.1f TF\n", (long long)sk, ms, flop / ms / 1e9);
          fflush(stdout);
        }
      }
      return 0;
    }
    for (int r = 0; r < reps + 1; ++r) {
      float ms;
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL((k_gemm_f32_chain<16, 4, false, true>), dim3((unsigned)(gtm * gtm)), dim3(512), 0, 0, dt0, ds,
                         gtm, gtm, (const char*)Z, gg);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("library f32 GRID                       %9.3f ms %7.1f TF\n", ms, flop / ms / 1e9);
      CHECK(hipEventRecord(e0));
      if (cubed_gemm_chain_packed(tasks.data(), dt1, nb, nb, segs.data(), ds, segs.size(), CUBED_F32, CUBED_F32, ws, wsb,
                                  nullptr)) { printf("packed: %s\n", g_err); return 1; }
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("cubed_gemm_chain_packed (pack + GEMM)  %9.3f ms %7.1f TF\n", ms, flop / ms / 1e9);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL((k_gemm_f32_w4p<true>), dim3((unsigned)(gtm * gtm)), dim3(256), 0, 0, dt1, (const char*)ws,
                         (const char*)(ws + pp.TM * pp.pstride), pp, gg, st);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<unsigned long long> hs((size_t)gtm * gtm * 8);
      CHECK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
      double cyc = 0, steps = 0;
      for (size_t i = 0; i < hs.size(); i += 2) {
        cyc += (double)hs[i];
        steps += (double)hs[i + 1];
      }
      printf("w4p GEMM only, stamped                 %9.3f ms %7.1f TF  main loop %.2f cyc/MFMA  clock ~%.2f GHz\n", ms,
             flop / ms / 1e9, cyc / (steps * 128), (cyc / (hs.size() / 2)) * ((double)gtm * gtm / 256.0) / (ms * 1e-3) / 1e9);
      CHECK(hipMemset(dmax, 0, 4));
      k_diff<<<4096, 256>>>((const float*)C0, (const float*)C1, slot * nb * nb / 4, dmax);
      float m;
      CHECK(hipMemcpy(&m, dmax, 4, hipMemcpyDeviceToHost));
      printf("   max |diff| packed vs library GRID: %g\n", m);
      fflush(stdout);
    }
    return 0;
  }
  struct V { const char* name; kfn f; bool check; kfn_s fs; };
  V vs[] = {
      {"BK16 NS4 (library)", k_gemm_f32_chain<16, 4>, false, nullptr},
      {"w4: one wave per SIMD", nullptr, true, k_gemm_f32_w4<false>},
      {"BK16 NS4 (again)", k_gemm_f32_chain<16, 4>, true, nullptr},
      {"w4 (again)", nullptr, true, k_gemm_f32_w4<false>},
  };
  unsigned long long* dstamp;
  CHECK(hipMalloc(&dstamp, (size_t)(grid.x + 30000) * 8 * 8));
  for (const V& v : vs) {
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(e0));
      if (v.fs)
        hipLaunchKernelGGL(v.fs, grid, dim3(256), 0, 0, v.check ? dt1 : dt0, ds, tm, tn, (const char*)Z, GemmGrid{},
                           (unsigned long long*)nullptr);
      else
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
  auto stamped = [&](const char* name, kfn_s f) {  // main-loop cycles per MFMA (the floor is 64: 32x32x2 f32)
    CHECK(hipMemset(dstamp, 0, (size_t)grid.x * 8 * 8));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(f, grid, dim3(256), 0, 0, dt1, ds, tm, tn, (const char*)Z, GemmGrid{}, dstamp);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> hs((size_t)grid.x * 8);
    CHECK(hipMemcpy(hs.data(), dstamp, hs.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, steps = 0;
    for (size_t i = 0; i < hs.size(); i += 2) {
      cyc += (double)hs[i];
      steps += (double)hs[i + 1];
    }
    printf("%-28s %9.3f ms %7.1f TF  main loop %.2f cyc/MFMA  clock ~%.2f GHz\n", name, ms, flop / ms / 1e9,
           cyc / (steps * 128), (cyc / (hs.size() / 2)) * ((double)grid.x / 256.0) / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  stamped("w4 stamped", k_gemm_f32_w4<false, true>);
  stamped("  ABL no barrier", k_gemm_f32_w4<false, true, 1>);
  stamped("  ABL no vmcnt wait", k_gemm_f32_w4<false, true, 2>);
  stamped("  ABL fills from step 0", k_gemm_f32_w4<false, true, 16>);
  stamped("  ABL all three", k_gemm_f32_w4<false, true, 19>);
  {  // the grid form stamped (157 x 157 tiles)
    GemmGrid gg{nb, nb, Cc, Cc, N, N};
    const int64_t gtm = (N + HF_BM - 1) / HF_BM;
    CHECK(hipMemset(dstamp, 0, (size_t)grid.x * 8 * 8));
    hipLaunchKernelGGL((k_gemm_f32_w4<true, true>), dim3((unsigned)(gtm * gtm)), dim3(256), 0, 0, dt1, ds, gtm, gtm,
                       (const char*)Z, gg, dstamp);
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> hs((size_t)gtm * gtm * 8);
    CHECK(hipMemcpy(hs.data(), dstamp, hs.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, steps = 0;
    for (size_t i = 0; i < hs.size(); i += 2) {
      cyc += (double)hs[i];
      steps += (double)hs[i + 1];
    }
    printf("w4 GRID stamped: main loop %.2f cyc/MFMA\n", cyc / (steps * 128));
  }
  {  // the grid tiling: library f32 (grid) vs w4 grid
    GemmGrid gg{nb, nb, Cc, Cc, N, N};
    const int64_t gtm = (N + HF_BM - 1) / HF_BM;
    for (int r = 0; r < 2; ++r) {
      float ms;
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL((k_gemm_f32_chain<16, 4, false, true>), dim3((unsigned)(gtm * gtm)), blk, 0, 0, dt0, ds, gtm,
                         gtm, (const char*)Z, gg);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("library f32 GRID            %9.3f ms %7.1f TF\n", ms, flop / ms / 1e9);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL((k_gemm_f32_w4<true>), dim3((unsigned)(gtm * gtm)), dim3(256), 0, 0, dt1, ds, gtm, gtm,
                         (const char*)Z, gg, (unsigned long long*)nullptr);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("w4 GRID                     %9.3f ms %7.1f TF\n", ms, flop / ms / 1e9);
    }
    CHECK(hipMemset(dmax, 0, 4));
    k_diff<<<4096, 256>>>((const float*)C0, (const float*)C1, slot * nb * nb / 4, dmax);
    float m;
    CHECK(hipMemcpy(&m, dmax, 4, hipMemcpyDeviceToHost));
    printf("   max |diff| w4 GRID vs library GRID: %g\n", m);
  }
  return 0;
}
