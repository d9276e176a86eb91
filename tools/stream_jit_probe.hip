// stream_jit_probe.hip -- development probe (not part of the library): the
// library's JIT streaming kernel for the elided rechunk + mean (BASELINE
// config 3 "rechunk+reduce": column means of x (50000, 50000) f32 read
// through 4000-B rows, one task per 1000-column output block, rows split 19
// ways) next to a minimal kernel with the same geometry, in one process.
// tools/stream_jit_elided.inc is the source libcubed_amd's JIT generated for
// that program (cubed_fused_source; mode set to the non-partials form), so
// the kernel below is the library's, compiled by hipcc instead of hipRTC.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//          -Icubed_amd/csrc -Iinclude -o tools/stream_jit_probe tools/stream_jit_probe.hip
// Run:   tools/stream_jit_probe [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "stream_jit_elided.inc"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define GA __attribute__((address_space(1)))
typedef float pf32x4 __attribute__((ext_vector_type(4)));

static constexpr long NR = 50000, NC = 50000, CB = 1000, NJ = NC / CB;

__global__ void k_fill(float* p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = (float)(h >> 8) * (1.0f / 16777216.0f);
  }
}

template <int U, int S>
__global__ __launch_bounds__(256) void k_minimal(const float* __restrict__ x, double* __restrict__ part, long stride) {
  const long g = blockIdx.x;
  const int s = (int)(g % S);
  const long j = g / S;
  const long r0 = NR * s / S, r1 = NR * (s + 1) / S;
  const int c4 = threadIdx.x;
  if (c4 * 4 >= CB) return;
  const long col = j * CB + c4 * 4;
  const float* p = x + r0 * stride + col;
  double acc[4] = {0, 0, 0, 0};
  long r = r0;
  for (; r + U <= r1; r += U) {
    pf32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load((const GA pf32x4*)(p + u * stride));
    p += U * stride;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc[0] += v[u].x; acc[1] += v[u].y; acc[2] += v[u].z; acc[3] += v[u].w;
    }
  }
  for (; r < r1; ++r, p += stride) {
    const pf32x4 v = __builtin_nontemporal_load((const GA pf32x4*)p);
    acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
  }
  for (int e = 0; e < 4; ++e) part[(long)s * NC + col + e] = acc[e];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  float* x;
  double* part;
  cubed::Acc* ws;
  cubed_task_t* dt;
  const int S = 19;
  CHECK(hipMalloc(&x, NR * NC * 4));
  CHECK(hipMalloc(&part, (long)S * NC * 8));
  CHECK(hipMalloc(&ws, (long)S * NJ * CB * 2 * sizeof(cubed::Acc)));
  CHECK(hipMalloc(&dt, NJ * sizeof(cubed_task_t)));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, x, NR * NC, 7u);
  std::vector<cubed_task_t> tasks(NJ);
  for (long j = 0; j < NJ; ++j) {
    cubed_task_t& T = tasks[j];
    memset(&T, 0, sizeof(T));
    T.extent[0] = NR;
    T.extent[1] = CB;
    T.leaf_base[0] = (int64_t)(uintptr_t)(x + j * CB);
    T.leaf_stride[0][0] = NC;
    T.leaf_stride[0][1] = 1;
  }
  CHECK(hipMemcpy(dt, tasks.data(), NJ * sizeof(cubed_task_t), hipMemcpyHostToDevice));
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) { best = ms < best ? ms : best; sum += ms; }
    }
    printf("%-40s best %.3f ms mean %.3f ms %6.0f GB/s\n", name, best, sum / reps, NR * NC * 4 / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  // hipRTC-built code objects of the same source (argv[2], argv[3], ...): the
  // library's own build path
  struct Mod { const char* path; hipFunction_t fn; };
  std::vector<Mod> mods;
  for (int a = 2; a < argc; ++a) {
    FILE* f = fopen(argv[a], "rb");
    if (!f) { printf("cannot open %s\n", argv[a]); return 1; }
    std::vector<char> buf;
    char tmp[65536];
    size_t n;
    while ((n = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    fclose(f);
    hipModule_t m;
    CHECK(hipModuleLoadData(&m, buf.data()));
    hipFunction_t fn;
    CHECK(hipModuleGetFunction(&fn, m, "jit_stream"));
    mods.push_back({argv[a], fn});
  }
  for (int rep = 0; rep < 2; ++rep) {
    for (auto& md : mods) {
      timeit(md.path, [&] {
        struct { const cubed_task_t* t; int64_t nt; int64_t bpt; int32_t ns; int32_t pad; cubed::Acc* ws; int64_t mk; } args;
        args.t = dt; args.nt = NJ; args.bpt = 1; args.ns = S; args.pad = 0; args.ws = ws; args.mk = CB;
        size_t sz = sizeof(args);
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
        CHECK(hipModuleLaunchKernel(md.fn, NJ * S, 1, 1, 256, 1, 1, 0, 0, nullptr, cfg));
      });
    }
    timeit("library JIT stream_body<f32,1,8,1>", [&] {
      hipLaunchKernelGGL(jit_stream, dim3(NJ * S), dim3(256), 0, 0, dt, (int64_t)NJ, (int64_t)1, (int32_t)S, ws,
                         (int64_t)CB);
    });
    timeit("minimal kernel, same geometry", [&] {
      hipLaunchKernelGGL((k_minimal<8, 19>), dim3(NJ * S), dim3(256), 0, 0, x, part, NC);
    });
  }
  // sums agree (split 0 of task 0, first 8 columns)
  std::vector<cubed::Acc> hw(16);
  std::vector<double> hp(8);
  CHECK(hipMemcpy(hw.data(), ws, 16 * sizeof(cubed::Acc), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hp.data(), part, 8 * 8, hipMemcpyDeviceToHost));
  printf("check: ws total[0] %.9g vs minimal %.9g\n", hw[1].f, hp[0]);
  return 0;
}
