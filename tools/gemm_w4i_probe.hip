// gemm_w4i_probe.hip -- development probe (not part of the library): the
// chained bf16 GEMM of BASELINE config 5 (40000^2 in 5000^2 chunks, 64 output
// chunks x 8 k segments, chunk-contiguous slots as the executor lays them out)
// on the library's ping-pong kernel and on the one-wave interleaved kernel
// (tools/gemm_bf16_w4i.h), in one process; max |diff| between the two (they
// sum each K=16/32 slice in a different MFMA shape: not bit-identical).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude \
//          -o tools/gemm_w4i_probe tools/gemm_w4i_probe.hip
// Run:   tools/gemm_w4i_probe [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

namespace cubed {
thread_local char g_err[512];
}
#include "../cubed_amd/csrc/gemm_chain.hip"
#include "gemm_bf16_w4i.h"
#include "gemm_bf16_w4t.h"
#include "gemm_bf16_w4p.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_fill(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float v = (float)(h >> 8) * (1.0f / 16777216.0f);  // U[0, 1) as config 5
    p[i] = (uint16_t)(__float_as_uint(v) >> 16);
  }
}

// B^T chunks for the w4t kernel: dst (n, k) = src (k, n) of one 5000^2 chunk
// per blockIdx.y (64 x 64 tiles through LDS)
__global__ void k_transpose(const uint16_t* src, uint16_t* dst, int64_t C, int64_t slot_elems) {
  __shared__ uint16_t tile[64][65];
  const uint16_t* s = src + blockIdx.y * slot_elems;
  uint16_t* d = dst + blockIdx.y * slot_elems;
  const int64_t tiles = (C + 63) / 64;
  for (int64_t tt = blockIdx.x; tt < tiles * tiles; tt += gridDim.x) {
    const int64_t r0 = (tt / tiles) * 64, c0 = (tt % tiles) * 64;
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) {
      const int64_t r = r0 + i / 64, c = c0 + i % 64;
      tile[i / 64][i % 64] = (r < C && c < C) ? s[r * C + c] : 0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) {
      const int64_t r = c0 + i / 64, c = r0 + i % 64;  // dst row = src column
      if (r < C && c < C) d[r * C + c] = tile[i % 64][i / 64];
    }
    __syncthreads();
  }
}

__global__ void k_diff(const float* a, const float* b, int64_t n, float* out) {
  float m = 0.f, r = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float d = fabsf(a[i] - b[i]);
    m = fmaxf(m, d);
    r = fmaxf(r, d / fmaxf(fabsf(a[i]), 1e-30f));
  }
  atomicMax((int*)out, __float_as_int(m));
  atomicMax((int*)out + 1, __float_as_int(r));
}

typedef void (*kfn)(const cubed_gemm_chain_t*, const cubed_gemm_seg_t*, int64_t, int64_t, const char*, GemmGrid);
typedef void (*kfn_s)(const cubed_gemm_chain_t*, const cubed_gemm_seg_t*, int64_t, int64_t, const char*, GemmGrid,
                      unsigned long long*);

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 2;
  const int64_t N = argc > 2 ? atoll(argv[2]) : 40000, Cc = 5000, nb = N / Cc;
  // chunk slot alignment: 256 B, or the executor's 32 B (storage.SLOT_ALIGN) with argv[4] = 32
  const int64_t al = argc > 4 ? atoll(argv[4]) : 256;
  const int64_t slot_in = (Cc * Cc * 2 + al - 1) / al * al, slot_out = (Cc * Cc * 4 + al - 1) / al * al;
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
  const dim3 grid((unsigned)(nb * nb * tm * tn));
  const double flop = 2.0 * N * N * N;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float* dmax;
  CHECK(hipMalloc(&dmax, 8));

  struct V { const char* name; kfn f; kfn_s fs; int threads; bool check; };
  V vs[] = {
      {"library ping-pong (16x16x32, 8 waves)", k_gemm_bf16_chain<false, 0, 1>, nullptr, 512, false},
      {"w4l: A staged in full 128-B lines", nullptr, k_gemm_bf16_w4l<false>, 256, true},
      {"library ping-pong (again)", k_gemm_bf16_chain<false, 0, 1>, nullptr, 512, false},
      {"w4l (again)", nullptr, k_gemm_bf16_w4l<false>, 256, true},
      {"w4l GM=2 (tile-row groups)", nullptr, k_gemm_bf16_w4l<false, 2>, 256, true},
      {"w4l GM=8", nullptr, k_gemm_bf16_w4l<false, 8>, 256, true},
      {"w4l GM=20 (a chunk's tile column)", nullptr, k_gemm_bf16_w4l<false, 20>, 256, true},
      {"w4l GM=4 (again)", nullptr, k_gemm_bf16_w4l<false>, 256, true},

  };
  // B^T chunks and a segment table pointing at them (w4t)
  char* BT;
  CHECK(hipMalloc(&BT, slot_in * nb * nb));
  k_transpose<<<dim3(1024, (unsigned)(nb * nb)), 256>>>((const uint16_t*)B, (uint16_t*)BT, Cc, slot_in / 2);
  CHECK(hipGetLastError());
  std::vector<cubed_gemm_seg_t> segsT(segs);
  for (auto& g : segsT) g.b = (int64_t)(uintptr_t)(BT + ((char*)(uintptr_t)g.b - B));
  cubed_gemm_seg_t* dsT;
  CHECK(hipMalloc(&dsT, sizeof(cubed_gemm_seg_t) * segsT.size()));
  CHECK(hipMemcpy(dsT, segsT.data(), sizeof(cubed_gemm_seg_t) * segsT.size(), hipMemcpyHostToDevice));
  CHECK(hipDeviceSynchronize());
  auto run_t = [&](const char* name, bool stamp, kfn_s fst = nullptr) {
    unsigned long long* st = nullptr;
    if (stamp) CHECK(hipMalloc(&st, (size_t)grid.x * 4 * 2 * 8));
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(e0));
      if (stamp)
        hipLaunchKernelGGL(fst ? fst : (kfn_s)(k_gemm_bf16_w4t<false, 4, true>), grid, dim3(256), 0, 0, dt1, dsT,
                           tm, tn, (const char*)Z, GemmGrid{}, st);
      else
        hipLaunchKernelGGL((k_gemm_bf16_w4t<false>), grid, dim3(256), 0, 0, dt1, dsT, tm, tn, (const char*)Z,
                           GemmGrid{}, (unsigned long long*)nullptr);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    printf("%-40s best %9.3f ms %7.1f TF\n", name, best, flop / best / 1e9);
    if (stamp) {
      std::vector<unsigned long long> h((size_t)grid.x * 8);
      CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
      double cyc = 0, steps = 0;
      for (size_t i = 0; i < h.size(); i += 2) {
        cyc += (double)h[i];
        steps += (double)h[i + 1];
      }
      printf("   main loop %6.2f cyc/MFMA  clock ~%.2f GHz\n", cyc / (steps * 32),
             (cyc / (h.size() / 2)) * ((double)grid.x / 256.0) / (best * 1e-3) / 1e9);
      CHECK(hipFree(st));
    }
    CHECK(hipMemset(dmax, 0, 8));
    k_diff<<<4096, 256>>>((const float*)C0, (const float*)C1, slot_out * nb * nb / 4, dmax);
    float m[2];
    CHECK(hipMemcpy(m, dmax, 8, hipMemcpyDeviceToHost));
    printf("   vs library ping-pong: max |diff| %g, max rel %g\n", m[0], m[1]);
    fflush(stdout);
  };
  unsigned long long* dstamp;
  CHECK(hipMalloc(&dstamp, (size_t)(grid.x + 4096) * 4 * 2 * 8));
  const int only = argc > 3 ? atoi(argv[3]) : -1;
  printf("# N %lld, chunk %lld, slot alignment %lld B\n", (long long)N, (long long)Cc, (long long)al);
  for (const V& v : vs) {
    if (only >= 0 && only != 99 && &v - vs != only) continue;
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(e0));
      if (v.f)
        hipLaunchKernelGGL(v.f, grid, dim3(v.threads), 0, 0, v.check ? dt1 : dt0, ds, tm, tn, (const char*)Z,
                           GemmGrid{});
      else
        hipLaunchKernelGGL(v.fs, grid, dim3(v.threads), 0, 0, v.check ? dt1 : dt0, ds, tm, tn, (const char*)Z,
                           GemmGrid{}, (unsigned long long*)nullptr);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) {
        sum += ms;
        if (ms < best) best = ms;
      }
    }
    printf("%-40s best %9.3f ms %7.1f TF   mean %9.3f ms\n", v.name, best, flop / best / 1e9, sum / reps);
    if (v.check) {
      CHECK(hipMemset(dmax, 0, 8));
      k_diff<<<4096, 256>>>((const float*)C0, (const float*)C1, slot_out * nb * nb / 4, dmax);
      float m[2];
      CHECK(hipMemcpy(m, dmax, 8, hipMemcpyDeviceToHost));
      printf("   vs library: max |diff| %g, max rel %g\n", m[0], m[1]);
    }
    fflush(stdout);
  }
  // stamped builds of w4i: K-loop cycles per MFMA (clock-independent) and the
  // clock, for the kernel and its ablations (results wrong for ABL != 0)
  auto stamped = [&](const char* name, kfn_s f) {
    CHECK(hipMemset(dstamp, 0, (size_t)grid.x * 4 * 2 * 8));
    hipLaunchKernelGGL(f, grid, dim3(256), 0, 0, dt1, ds, tm, tn, (const char*)Z, GemmGrid{}, dstamp);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(f, grid, dim3(256), 0, 0, dt1, ds, tm, tn, (const char*)Z, GemmGrid{}, dstamp);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h((size_t)grid.x * 8);
    CHECK(hipMemcpy(h.data(), dstamp, h.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, steps = 0;
    for (size_t i = 0; i < h.size(); i += 2) {
      cyc += (double)h[i];
      steps += (double)h[i + 1];
    }
    printf("%-44s %8.3f ms %7.1f TF  main loop %6.2f cyc/MFMA  clock ~%.2f GHz\n", name, ms, flop / ms / 1e9,
           cyc / (steps * 32), (cyc / (h.size() / 2)) * ((double)grid.x / 256.0) / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  if (only == 97) {  // packed operands (tools/gemm_bf16_w4p.h) vs the library w4l kernel
    PackGeom pg{nb, nb, nb, Cc, Cc, Cc, N, tm, tn, (N + 63) / 64};
    char *PA, *PB;
    const size_t pbytes = (size_t)nb * tm * pg.KTL * 32768;
    CHECK(hipMalloc(&PA, pbytes));
    CHECK(hipMalloc(&PB, pbytes));
    hipLaunchKernelGGL((k_gemm_bf16_w4l<false>), grid, dim3(256), 0, 0, dt0, ds, tm, tn, (const char*)Z, GemmGrid{},
                       (unsigned long long*)nullptr);  // C0: the library kernel's result
    CHECK(hipGetLastError());
    for (int r = 0; r < 3; ++r) {
      CHECK(hipEventRecord(e0));
      k_packA<<<8192, 256>>>(A, slot_in, pg, PA);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ma, mb;
      CHECK(hipEventElapsedTime(&ma, e0, e1));
      CHECK(hipEventRecord(e0));
      k_packBT<<<8192, 256>>>(B, slot_in, pg, PB);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipGetLastError());
      CHECK(hipEventElapsedTime(&mb, e0, e1));
      printf("pack A %.3f ms (%.0f GB/s)  pack B^T %.3f ms (%.0f GB/s)\n", ma, 2.0 * pbytes / ma / 1e6, mb,
             2.0 * pbytes / mb / 1e6);
    }
    {  // the register-transpose B^T pack must give the same blocks
      char* PB2;
      CHECK(hipMalloc(&PB2, pbytes));
      for (int r = 0; r < 3; ++r) {
        CHECK(hipEventRecord(e0));
        k_packBT8<<<8192, 256>>>(B, slot_in, pg, PB2);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipGetLastError());
        float mb;
        CHECK(hipEventElapsedTime(&mb, e0, e1));
        printf("pack B^T (8x8 register transpose) %.3f ms (%.0f GB/s)\n", mb, 2.0 * pbytes / mb / 1e6);
      }
      CHECK(hipMemset(dmax, 0, 8));
      k_diff<<<4096, 256>>>((const float*)PB, (const float*)PB2, pbytes / 4, dmax);
      float m[2];
      CHECK(hipMemcpy(m, dmax, 8, hipMemcpyDeviceToHost));
      printf("   vs LDS transpose: max |diff| %g (bit patterns as f32)\n", m[0]);
      CHECK(hipFree(PB2));
    }
    typedef void (*kfn_p)(const cubed_gemm_chain_t*, const char*, const char*, PackGeom, int64_t, int64_t,
                          unsigned long long*);
    int* prog_host = nullptr;  // SYNC progress words, zeroed before every launch
    auto run_p = [&](const char* name, bool stamp, kfn_p fst = nullptr) {
      unsigned long long* st = nullptr;
      if (stamp) CHECK(hipMalloc(&st, (size_t)grid.x * 4 * 2 * 8));
      float best = 1e30f;
      for (int r = 0; r < reps + 1; ++r) {
        if (prog_host) CHECK(hipMemset(prog_host, 0, (size_t)grid.x * 4));
        CHECK(hipMemset(C1, 0, slot_out * nb * nb));
        CHECK(hipEventRecord(e0));
        if (stamp)
          hipLaunchKernelGGL(fst ? fst : (kfn_p)(k_w4p_probe<false, true>), grid, dim3(256), 0, 0, dt1, (const char*)PA,
                             (const char*)PB, pg, tm, tn, st);
        else
          hipLaunchKernelGGL((k_w4p_probe<false, false>), grid, dim3(256), 0, 0, dt1, (const char*)PA,
                             (const char*)PB, pg, tm, tn, (unsigned long long*)nullptr);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
      }
      printf("%-40s best %9.3f ms %7.1f TF\n", name, best, flop / best / 1e9);
      if (stamp) {
        std::vector<unsigned long long> h((size_t)grid.x * 8);
        CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
        double cyc = 0, steps = 0;
        for (size_t i = 0; i < h.size(); i += 2) {
          cyc += (double)h[i];
          steps += (double)h[i + 1];
        }
        printf("   main loop %6.2f cyc/MFMA  clock ~%.2f GHz\n", cyc / (steps * 32),
               (cyc / (h.size() / 2)) * ((double)grid.x / 256.0) / (best * 1e-3) / 1e9);
        CHECK(hipFree(st));
      }
      CHECK(hipMemset(dmax, 0, 8));
      k_diff<<<4096, 256>>>((const float*)C0, (const float*)C1, slot_out * nb * nb / 4, dmax);
      float m[2];
      CHECK(hipMemcpy(m, dmax, 8, hipMemcpyDeviceToHost));
      printf("   vs library w4l: max |diff| %g, max rel %g\n", m[0], m[1]);
      fflush(stdout);
    };
    for (const V& v : vs) {  // the library kernel timed in the same process
      if (&v - vs != 1) continue;
      float best = 1e30f;
      for (int r = 0; r < reps + 1; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(v.fs, grid, dim3(256), 0, 0, dt0, ds, tm, tn, (const char*)Z, GemmGrid{},
                           (unsigned long long*)nullptr);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
      }
      printf("%-40s best %9.3f ms %7.1f TF\n", "library w4l", best, flop / best / 1e9);
    }
    run_p("w4p: packed A and B^T", false);
    run_p("w4p stamped", true);
    run_p("w4p (again)", false);
    run_p("  w4p ABL A sources L2-resident", true, k_w4p_probe<false, true, 1>);
    run_p("  w4p ABL B^T sources L2-resident", true, k_w4p_probe<false, true, 2>);
    run_p("  w4p ABL both L2-resident", true, k_w4p_probe<false, true, 3>);
    run_p("w4p stamped (again)", true);
    {
      CHECK(hipMalloc(&prog_host, (size_t)grid.x * 4));
      CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_w4p_progress), &prog_host, sizeof(prog_host)));
      if (argc > 5 && argv[5][0] == 'g') {  // tile-group rows (GM) of the packed kernel
        run_p("w4p GM=2", true, k_w4p_probe<false, true, 0, false, 8, 8, 64, 2>);
        run_p("w4p GM=4", true, k_w4p_probe<false, true, 0, false, 8, 8, 64, 4>);
        run_p("w4p GM=8", true, k_w4p_probe<false, true, 0, false, 8, 8, 64, 8>);
        run_p("w4p GM=16", true, k_w4p_probe<false, true, 0, false, 8, 8, 64, 16>);
        run_p("w4p GM=1", true, k_w4p_probe<false, true, 0, false, 8, 8, 64, 1>);
        run_p("w4p GM=4 (again)", true, k_w4p_probe<false, true, 0, false, 8, 8, 64, 4>);
        return 0;
      }
      run_p("w4p SYNC every 8 lag 8, stamped", true, k_w4p_probe<false, true, 0, true>);
      run_p("w4p SYNC every 32 lag 32 window 128", true, k_w4p_probe<false, true, 0, true, 32, 32, 128>);
      run_p("w4p SYNC every 16 lag 24 window 96", true, k_w4p_probe<false, true, 0, true, 16, 24, 96>);
      run_p("w4p SYNC every 64 lag 48 window 192", true, k_w4p_probe<false, true, 0, true, 64, 48, 192>);
      run_p("w4p SYNC every 32 lag 16 window 128", true, k_w4p_probe<false, true, 0, true, 32, 16, 128>);
      run_p("w4p (no sync, again)", true);
    }
    {  // the library form: packed over the WHOLE matrix (157 panels), whole-matrix tiles
      char* ws;
      const int64_t wsb = cubed_gemm_pack_bytes(tasks.data(), nb, nb, segs.data(), segs.size(), CUBED_BF16, CUBED_F32);
      if (wsb <= 0) { printf("pack_bytes: %s\n", g_err); return 1; }
      CHECK(hipMalloc(&ws, wsb));
      PackPlan pp;
      GemmGrid gg;
      if (pack_plan(tasks.data(), nb, nb, segs.data(), segs.size(), CUBED_BF16, CUBED_F32, pp, gg)) return 1;
      for (int r = 0; r < reps + 1; ++r) {
        CHECK(hipMemset(C1, 0, slot_out * nb * nb));
        CHECK(hipEventRecord(e0));
        if (cubed_gemm_chain_packed(tasks.data(), dt1, nb, nb, segs.data(), ds, segs.size(), CUBED_BF16, CUBED_F32, ws,
                                    wsb, nullptr)) { printf("packed: %s\n", g_err); return 1; }
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("library cubed_gemm_chain_packed (pack + GEMM) %9.3f ms %7.1f TF\n", ms, flop / ms / 1e9);
      }
      CHECK(hipMemset(dmax, 0, 8));
      k_diff<<<4096, 256>>>((const float*)C0, (const float*)C1, slot_out * nb * nb / 4, dmax);
      float m[2];
      CHECK(hipMemcpy(m, dmax, 8, hipMemcpyDeviceToHost));
      printf("   vs library w4l: max |diff| %g\n", m[0]);
      auto gemm_only = [&](const char* name, auto kern) {
        float best = 1e30f;
        for (int r = 0; r < reps + 1; ++r) {
          CHECK(hipEventRecord(e0));
          hipLaunchKernelGGL(kern, dim3((unsigned)(pp.TM * pp.TN)), dim3(256), 0, 0, dt1, (const char*)ws,
                             (const char*)(ws + pp.TM * pp.pstride), pp, gg, (unsigned long long*)nullptr);
          CHECK(hipEventRecord(e1));
          CHECK(hipEventSynchronize(e1));
          float ms;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          if (r > 0 && ms < best) best = ms;
        }
        printf("%-44s best %9.3f ms %7.1f TF\n", name, best, flop / best / 1e9);
        fflush(stdout);
      };
      gemm_only("library w4p GEMM only (f32 out)", k_gemm_bf16_w4p<false>);
      gemm_only("library w4p GEMM only (bf16 out)", k_gemm_bf16_w4p<true>);
      gemm_only("library w4p GEMM only (f32 out, again)", k_gemm_bf16_w4p<false>);
    }
    return 0;
  }
  if (only == 98 || only < 0) {
    {  // timing of the transpose (one-off per matmul)
      CHECK(hipEventRecord(e0));
      k_transpose<<<dim3(1024, (unsigned)(nb * nb)), 256>>>((const uint16_t*)B, (uint16_t*)BT, Cc, slot_in / 2);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("probe transpose of B (all chunks): %.3f ms\n", ms);
    }
    hipLaunchKernelGGL((k_gemm_bf16_chain<false, 0, 1>), grid, dim3(512), 0, 0, dt0, ds, tm, tn, (const char*)Z,
                       GemmGrid{});  // the library ping-pong result (C0) to compare with
    run_t("w4t: B^T staged like A, b128 B reads", false);
    run_t("w4t stamped", true);
    run_t("  w4t ABL no barrier", true, k_gemm_bf16_w4t<false, 4, true, 1>);
    run_t("  w4t ABL no vmcnt wait", true, k_gemm_bf16_w4t<false, 4, true, 2>);
    run_t("  w4t ABL A stale", true, k_gemm_bf16_w4t<false, 4, true, 16>);
    run_t("  w4t ABL B^T stale", true, k_gemm_bf16_w4t<false, 4, true, 32>);
    run_t("  w4t ABL both stale", true, k_gemm_bf16_w4t<false, 4, true, 48>);
    run_t("w4t (again)", false);
  }
  if (only == 98) return 0;
  {  // the grid tiling (cubed_gemm_chain_grid) of w4l: 157 x 157 tiles over the 40000^2 output
    GemmGrid gg{nb, nb, Cc, Cc, N, N};
    const int64_t gtm = (N + HB_BM - 1) / HB_BM;
    CHECK(hipMemset(dstamp, 0, (size_t)grid.x * 4 * 2 * 8));
    for (int r = 0; r < 2; ++r) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL((k_gemm_bf16_w4l<false, 4, true, 0, true>), dim3((unsigned)(gtm * gtm)), dim3(256), 0, 0,
                         dt1, ds, gtm, gtm, (const char*)Z, gg, dstamp);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<unsigned long long> h((size_t)gtm * gtm * 8);
      CHECK(hipMemcpy(h.data(), dstamp, h.size() * 8, hipMemcpyDeviceToHost));
      double cyc = 0, steps = 0;
      for (size_t i = 0; i < h.size(); i += 2) {
        cyc += (double)h[i];
        steps += (double)h[i + 1];
      }
      printf("w4l GRID stamped: %.3f ms %.1f TF, main-loop steps per wave %.1f, %.2f cyc/MFMA\n", ms, flop / ms / 1e9,
             steps / (h.size() / 2), cyc / (steps * 32));
    }
    CHECK(hipMemset(dmax, 0, 8));
    k_diff<<<4096, 256>>>((const float*)C0, (const float*)C1, slot_out * nb * nb / 4, dmax);
    float m[2];
    CHECK(hipMemcpy(m, dmax, 8, hipMemcpyDeviceToHost));
    printf("   vs library per-chunk: max |diff| %g, max rel %g\n", m[0], m[1]);
    fflush(stdout);
  }
  if (only == 99) {
    stamped("w4l stamped", k_gemm_bf16_w4l<false, 4, true>);
    stamped("  w4l ABL no barrier", k_gemm_bf16_w4l<false, 4, true, 1>);
    stamped("  w4l ABL no vmcnt wait", k_gemm_bf16_w4l<false, 4, true, 2>);
    stamped("  w4l ABL no barrier, no vmcnt wait", k_gemm_bf16_w4l<false, 4, true, 3>);
    stamped("  w4l ABL A stale", k_gemm_bf16_w4l<false, 4, true, 16>);
    stamped("  w4l ABL B stale", k_gemm_bf16_w4l<false, 4, true, 32>);
    stamped("  w4l ABL both stale", k_gemm_bf16_w4l<false, 4, true, 48>);
  }
  return 0;
}
