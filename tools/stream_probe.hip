// stream_probe.hip -- development probe (not part of the library): the read
// pattern of BASELINE config 2's streaming reduction (sum over t of u*v,
// u, v (1000, 720*1440) f32, f64 accumulation) under different per-thread
// widths, rows in flight and time splits, next to a contiguous read-only
// stream of the same bytes.  Every variant checks its sums against the first.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/stream_probe tools/stream_probe.hip
// Run:   tools/stream_probe [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define G __attribute__((address_space(1)))
typedef float f32x4 __attribute__((ext_vector_type(4)));

static constexpr long T = 1000, P = 720L * 1440;

__global__ void k_fill(float* p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = (float)(h >> 8) * (1.0f / 16777216.0f);
  }
}

// W 16-byte loads per row per leaf per lane, lane-interleaved (load j of a
// wave reads 1 KiB contiguous at wave base + j KiB); U rows in flight.
template <int W, int U, bool NT>
__global__ __launch_bounds__(256) void k_qm(const float* __restrict__ u, const float* __restrict__ v,
                                            double* __restrict__ part, int nsplit) {
  const long bpt = (P + 1024L * W - 1) / (1024L * W);
  const long b = blockIdx.x % bpt;
  const int s = blockIdx.x / bpt;
  const long r0 = T * s / nsplit, r1 = T * (s + 1) / nsplit;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long base = b * 1024L * W + wave * 256L * W + lane * 4;  // floats
  double acc[W][4];
#pragma unroll
  for (int j = 0; j < W; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[j][e] = 0.0;
  bool ok[W];
#pragma unroll
  for (int j = 0; j < W; ++j) ok[j] = base + j * 256 + 4 <= P;
  const G f32x4* pu = (const G f32x4*)(u + r0 * P + base);
  const G f32x4* pv = (const G f32x4*)(v + r0 * P + base);
  const long rs = P / 4;
  long r = r0;
  for (; r + U <= r1; r += U) {
    f32x4 a[U][W], c[U][W];
#pragma unroll
    for (int q = 0; q < U; ++q)
#pragma unroll
      for (int j = 0; j < W; ++j) {
        if (ok[j]) {
          if (NT) {
            a[q][j] = __builtin_nontemporal_load(pu + q * rs + j * 64);
            c[q][j] = __builtin_nontemporal_load(pv + q * rs + j * 64);
          } else {
            a[q][j] = pu[q * rs + j * 64];
            c[q][j] = pv[q * rs + j * 64];
          }
        } else {
          a[q][j] = f32x4{0, 0, 0, 0};
          c[q][j] = f32x4{0, 0, 0, 0};
        }
      }
#pragma unroll
    for (int q = 0; q < U; ++q)
#pragma unroll
      for (int j = 0; j < W; ++j) {
        acc[j][0] += (double)(a[q][j].x * c[q][j].x);
        acc[j][1] += (double)(a[q][j].y * c[q][j].y);
        acc[j][2] += (double)(a[q][j].z * c[q][j].z);
        acc[j][3] += (double)(a[q][j].w * c[q][j].w);
      }
    pu += U * rs;
    pv += U * rs;
  }
  for (; r < r1; ++r) {
#pragma unroll
    for (int j = 0; j < W; ++j)
      if (ok[j]) {
        const f32x4 a = pu[j * 64], c = pv[j * 64];
        acc[j][0] += (double)(a.x * c.x);
        acc[j][1] += (double)(a.y * c.y);
        acc[j][2] += (double)(a.z * c.z);
        acc[j][3] += (double)(a.w * c.w);
      }
    pu += rs;
    pv += rs;
  }
#pragma unroll
  for (int j = 0; j < W; ++j)
    if (ok[j])
#pragma unroll
      for (int e = 0; e < 4; ++e) part[(long)s * P + base + j * 256 + e] = acc[j][e];
}

__global__ void k_fold(const double* part, int nsplit, double* out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    double x = 0;
    for (int s = 0; s < nsplit; ++s) x += part[s * P + i];
    out[i] = x;
  }
}

// contiguous read-only stream of both arrays (64 KiB per workgroup)
__global__ __launch_bounds__(256) void k_read(const f32x4* __restrict__ src, f32x4* __restrict__ out, long nw) {
  const G f32x4* s = (const G f32x4*)src;
  f32x4 acc = {0, 0, 0, 0};
  const long n0 = (long)blockIdx.x * 4096;
  for (long i = n0 + threadIdx.x; i < n0 + 4096 && i < nw; i += 256) acc += __builtin_nontemporal_load(s + i);
  if (acc.x == 1.2345f) out[threadIdx.x] = acc;
}

typedef void (*kfn)(const float*, const float*, double*, int);

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  float* uv;
  CHECK(hipMalloc(&uv, 2 * T * P * sizeof(float)));
  float* u = uv;
  float* v = uv + T * P;
  k_fill<<<8192, 256>>>(u, T * P, 1u);
  k_fill<<<8192, 256>>>(v, T * P, 2u);
  double *part, *out, *ref;
  CHECK(hipMalloc(&part, 16 * P * sizeof(double)));
  CHECK(hipMalloc(&out, P * sizeof(double)));
  CHECK(hipMalloc(&ref, P * sizeof(double)));
  f32x4* sink;
  CHECK(hipMalloc(&sink, 4096));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bytes = 2.0 * T * P * 4;
  std::vector<double> h_out(P), h_ref(P);

  struct Var { const char* name; kfn f; int W; };
  Var vs[] = {
      {"W1 U4 nt (library shape)", k_qm<1, 4, true>, 1},
      {"W1 U8 nt", k_qm<1, 8, true>, 1},
      {"W2 U4 nt", k_qm<2, 4, true>, 2},
      {"W4 U2 nt", k_qm<4, 2, true>, 4},
      {"W4 U4 nt", k_qm<4, 4, true>, 4},
      {"W8 U1 nt", k_qm<8, 1, true>, 8},
      {"W8 U2 nt", k_qm<8, 2, true>, 8},
      {"W1 U4 cached", k_qm<1, 4, false>, 1},
      {"W4 U2 cached", k_qm<4, 2, false>, 4},
  };
  const int splits[] = {1, 2, 3, 4, 6, 8};
  // interleaved rounds: every (variant, split) once per round, best of reps
  const int nv = sizeof(vs) / sizeof(vs[0]), ns = sizeof(splits) / sizeof(splits[0]);
  std::vector<float> best(nv * ns + 1, 1e30f);
  bool have_ref = false;
  for (int rep = 0; rep < reps + 1; ++rep) {
    {
      const long nw = 2 * T * P / 4;
      CHECK(hipEventRecord(e0));
      k_read<<<(unsigned)((nw + 4095) / 4096), 256>>>((const f32x4*)uv, sink, nw);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best[nv * ns]) best[nv * ns] = ms;
    }
    for (int i = 0; i < nv; ++i)
      for (int k = 0; k < ns; ++k) {
        const long bpt = (P + 1024L * vs[i].W - 1) / (1024L * vs[i].W);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(vs[i].f, dim3((unsigned)(bpt * splits[k])), dim3(256), 0, 0, u, v, part, splits[k]);
        k_fold<<<2048, 256>>>(part, splits[k], out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best[i * ns + k]) best[i * ns + k] = ms;
        if (rep == 0) {
          CHECK(hipMemcpy(h_out.data(), out, P * sizeof(double), hipMemcpyDeviceToHost));
          if (!have_ref) { h_ref = h_out; have_ref = true; }
          double md = 0;
          for (long p = 0; p < P; ++p) md = fmax(md, fabs(h_out[p] - h_ref[p]) / fmax(1e-300, fabs(h_ref[p])));
          if (md > 1e-12) printf("MISMATCH %s split %d: rel %g\n", vs[i].name, splits[k], md);
        }
      }
  }
  printf("read-only contiguous stream: %.3f ms %.0f GB/s\n", best[nv * ns], bytes / best[nv * ns] / 1e6);
  for (int i = 0; i < nv; ++i)
    for (int k = 0; k < ns; ++k)
      printf("%-26s split %d: %.3f ms %.0f GB/s (incl. fold)\n", vs[i].name, splits[k], best[i * ns + k],
             bytes / best[i * ns + k] / 1e6);
  return 0;
}
