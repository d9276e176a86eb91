// pieces_probe.hip -- development probe (not part of the library): the read
// pattern of the elided rechunk + mean (BASELINE config 3 "rechunk+reduce"):
// column sums (f64) of x (50000, 50000) f32 in row chunks of 1000, one
// piece per (row chunk i, 1000-column output block j), 1000 rows x 4000 B
// per piece (rows 200 KB apart; piece rows start mid 128-B line).  Variants:
// piece order (j-major = the library's task order, i-major = source order),
// block -> piece mapping (plain, XCD-contiguous runs so neighbouring pieces
// of one row band share an XCD's L2), non-temporal vs cached loads, and
// pieces per workgroup.  Every variant checks its sums against the first.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/pieces_probe tools/pieces_probe.hip
// Run:   tools/pieces_probe [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define G __attribute__((address_space(1)))
typedef float f32x4 __attribute__((ext_vector_type(4)));

static constexpr long NR = 50000, NC = 50000, RC = 1000, CB = 1000;
static constexpr long NI = NR / RC, NJ = NC / CB, NP = NI * NJ;

__global__ void k_fill(float* p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = (float)(h >> 8) * (1.0f / 16777216.0f);
  }
}

__device__ __forceinline__ long xcd_remap(long b, long nblk) {
  if (nblk < 8) return b;
  const long xcd = b & 7, q = nblk >> 3, r = nblk & 7, i = b >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + i;
}

// one workgroup = PPW consecutive pieces (in the chosen order); a thread owns
// 4 columns of a piece; U rows in flight.  part[i][col] = sum over the rows
// of row chunk i.
template <bool IMAJOR, bool REMAP, bool NT, int U, int PPW>
__global__ __launch_bounds__(256) void k_pieces(const float* __restrict__ x, double* __restrict__ part) {
  static_assert(RC % U == 0, "rows in flight must divide the row chunk (no reads past the array)");
  long g = blockIdx.x;
  if (REMAP) g = xcd_remap(g, gridDim.x);
  const int tid = threadIdx.x;
  const int pw = tid / (256 / PPW), lt = tid % (256 / PPW);
  const long piece = g * PPW + pw;
  const long i = IMAJOR ? piece / NJ : piece % NI;
  const long j = IMAJOR ? piece % NJ : piece / NI;
  for (long c4 = lt; c4 * 4 < CB; c4 += 256 / PPW) {
    const long col = j * CB + c4 * 4;
    const float* p = x + i * RC * NC + col;
    double acc[4] = {0, 0, 0, 0};
    for (long r = 0; r < RC; r += U) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const G f32x4* q = (const G f32x4*)(p + (r + u) * NC);
        v[u] = NT ? __builtin_nontemporal_load(q) : *q;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[0] += v[u].x; acc[1] += v[u].y; acc[2] += v[u].z; acc[3] += v[u].w;
      }
    }
    for (int e = 0; e < 4; ++e) part[i * NC + col + e] = acc[e];
  }
}

// the library's geometry for the same work (stream_body, W = 1): one task
// per 1000-column output block, its 50000 rows split S ways (contiguous row
// ranges crossing row chunks), a runtime row stride, partials per split
template <int U, int S>
__global__ __launch_bounds__(256) void k_libshape(const float* __restrict__ x, double* __restrict__ part,
                                                   long stride) {
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
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load((const G f32x4*)(p + u * stride));
    p += U * stride;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc[0] += v[u].x; acc[1] += v[u].y; acc[2] += v[u].z; acc[3] += v[u].w;
    }
  }
  for (; r < r1; ++r, p += stride) {
    const f32x4 v = __builtin_nontemporal_load((const G f32x4*)p);
    acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
  }
  for (int e = 0; e < 4; ++e) part[(long)s * NC + col + e] = acc[e];
}

// contiguous read-only stream of the same bytes (the ceiling)
__global__ __launch_bounds__(256) void k_read(const f32x4* __restrict__ x, long n4, double* out) {
  double a = 0;
  for (long k = blockIdx.x * 256L + threadIdx.x; k < n4; k += (long)gridDim.x * 256 * 4) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long q = k + (long)u * gridDim.x * 256;
      v[u] = q < n4 ? __builtin_nontemporal_load((const G f32x4*)(x + q)) : f32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) a += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (a == 12345.0) out[0] = a;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  float* x;
  double *part, *ref;
  CHECK(hipMalloc(&x, NR * NC * 4));
  CHECK(hipMalloc(&part, 64 * NC * 8));
  CHECK(hipMalloc(&ref, NI * NC * 8));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, x, NR * NC, 7u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<double> h0(NI * NC), h1(NI * NC);
  auto run = [&](const char* name, void (*k)(const float*, double*), int ppw, bool check_ref) {
    const long blocks = NP / ppw;
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, x, part);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    const char* ok = "";
    if (check_ref) {
      CHECK(hipMemcpy(ref, part, NI * NC * 8, hipMemcpyDeviceToDevice));
      CHECK(hipMemcpy(h0.data(), ref, NI * NC * 8, hipMemcpyDeviceToHost));
    } else {
      CHECK(hipMemcpy(h1.data(), part, NI * NC * 8, hipMemcpyDeviceToHost));
      ok = (h0 == h1) ? "" : "  MISMATCH";
    }
    printf("%-44s %.3f ms %6.0f GB/s%s\n", name, best, NR * NC * 4 / (best * 1e-3) / 1e9, ok);
    fflush(stdout);
  };
  {
    float best = 1e30f;
    double* dummy;
    CHECK(hipMalloc(&dummy, 8));
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_read, dim3(8192), dim3(256), 0, 0, (const f32x4*)x, NR * NC / 4, dummy);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    printf("%-44s %.3f ms %6.0f GB/s\n", "read-only contiguous stream", best, NR * NC * 4 / (best * 1e-3) / 1e9);
  }
  run("j-major plain nt U8 (library order)", k_pieces<false, false, true, 8, 1>, 1, true);
  run("j-major plain cached U8", k_pieces<false, false, false, 8, 1>, 1, false);
  run("i-major plain nt U8", k_pieces<true, false, true, 8, 1>, 1, false);
  run("i-major plain cached U8", k_pieces<true, false, false, 8, 1>, 1, false);
  run("i-major xcd-remap nt U8", k_pieces<true, true, true, 8, 1>, 1, false);
  run("i-major xcd-remap cached U8", k_pieces<true, true, false, 8, 1>, 1, false);
  run("i-major xcd-remap cached U10", k_pieces<true, true, false, 10, 1>, 1, false);
  run("i-major xcd-remap cached U4", k_pieces<true, true, false, 4, 1>, 1, false);
  run("i-major plain cached U8, 2 pieces/WG", k_pieces<true, false, false, 8, 2>, 2, false);
  run("i-major xcd-remap cached U8, 2 pieces/WG", k_pieces<true, true, false, 8, 2>, 2, false);
  run("i-major xcd-remap nt U8, 2 pieces/WG", k_pieces<true, true, true, 8, 2>, 2, false);
  run("i-major xcd-remap cached U20, 2 pieces/WG", k_pieces<true, true, false, 20, 2>, 2, false);
  run("j-major plain nt U8 (again)", k_pieces<false, false, true, 8, 1>, 1, false);
  auto runlib = [&](const char* name, void (*k)(const float*, double*, long), int S) {
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k, dim3(NJ * S), dim3(256), 0, 0, x, part, NC);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    printf("%-44s %.3f ms %6.0f GB/s\n", name, best, NR * NC * 4 / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  runlib("library shape U8, 19 splits (950 WGs)", k_libshape<8, 19>, 19);
  runlib("library shape U8, 50 splits (2500 WGs)", k_libshape<8, 50>, 50);
  runlib("library shape U8, 64 splits (3200 WGs)", k_libshape<8, 64>, 64);
  runlib("library shape U16, 19 splits", k_libshape<16, 19>, 19);
  return 0;
}
