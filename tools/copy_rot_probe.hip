// copy_rot_probe.hip -- development probe (not part of the library): the
// config 3 rechunk copy (50000^2 f32, (1000, N) row bands -> (N, 1000) column
// chunks, 2500 boxes of 1000 x 1000 sorted by source address, the library's
// flat-copy geometry) with the workgroup -> (box, block) order varied, on two
// placements of the target (first allocation, then a re-allocation).
//   order 0: library (box-major, block b of every box of a band in flight together)
//   order 1: block index rotated by box * rot (concurrent writes at different row offsets)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o tools/copy_rot_probe tools/copy_rot_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "cubed_amd.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define GA __attribute__((address_space(1)))
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

static constexpr long N = 50000, C = 1000;
static constexpr int kBlock = 256, UN = 4, SPB = 16;

__global__ void k_fill(unsigned* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    p[i] = (unsigned)i * 2654435761u;
}

template <int LD, int ST>  // LD: 0 cached, 1 non-temporal loads; ST: 0 non-temporal, 1 plain stores
__global__ __launch_bounds__(kBlock) void k_flat(const cubed_box_t* __restrict__ boxes, long nboxes, long bpb,
                                                 long rot) {
  const long g = blockIdx.x;
  const long bi = g / bpb;
  long blk = g % bpb;
  if (bi >= nboxes) return;
  if (rot) blk = (blk + bi * rot) % bpb;
  const cubed_box_t* __restrict__ B = boxes + bi;
  const unsigned nw = (unsigned)(B->extent[1] * 4 / 16);
  const long total = B->extent[0] * (long)nw;
  const long sstr = B->src_stride[0] * 4;
  const char* __restrict__ sbase = (const char*)(uintptr_t)B->src_base;
  GA u32x4* __restrict__ dst = (GA u32x4*)(uintptr_t)B->dst_base;
  constexpr int kSeg = 64 * UN;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long w_begin = blk * SPB * kSeg;
  long w_end = w_begin + SPB * kSeg;
  if (w_end > total) w_end = total;
  for (long i0 = w_begin + (long)wave * kSeg; i0 < w_end; i0 += (long)(kBlock / 64) * kSeg) {
    u32x4 v[UN];
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const long i = i0 + k * 64 + lane;
      if (i < w_end) {
        const unsigned r = (unsigned)i / nw, c = (unsigned)i - r * nw;
        const GA u32x4* q = (const GA u32x4*)(uintptr_t)(sbase + (long)r * sstr) + c;
        if constexpr (LD == 1) v[k] = __builtin_nontemporal_load(q);
        else v[k] = *q;
      }
    }
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const long i = i0 + k * 64 + lane;
      if (i < w_end) {
        if constexpr (ST == 1) dst[i] = v[k];
        else __builtin_nontemporal_store(v[k], dst + i);
      }
    }
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  char *x, *y;
  CHECK(hipMalloc(&x, N * N * 4));
  CHECK(hipMalloc(&y, N * N * 4));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (unsigned*)x, N * N);
  const long nb = (N / C) * (N / C);
  cubed_box_t* d_boxes;
  CHECK(hipMalloc(&d_boxes, nb * sizeof(cubed_box_t)));
  const long words = C * C * 4 / 16;
  long bpb = (words / (64 * UN) + SPB - 1) / SPB;
  bpb = (bpb + 7) / 8 * 8;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto build = [&](char* yy) {
    std::vector<cubed_box_t> h(nb);
    long k = 0;
    for (long j = 0; j < N / C; ++j)
      for (long i = 0; i < N / C; ++i) {
        cubed_box_t& b = h[k++];
        memset(&b, 0, sizeof(b));
        b.src_base = (int64_t)(uintptr_t)(x + (i * C * N + j * C) * 4);
        b.dst_base = (int64_t)(uintptr_t)(yy + (j * N * C + i * C * C) * 4);
        for (int d = 0; d < CUBED_MAX_DIMS; ++d) b.extent[d] = 1;
        b.extent[0] = C; b.extent[1] = C;
        b.src_stride[0] = N; b.src_stride[1] = 1;
        b.dst_stride[0] = C; b.dst_stride[1] = 1;
      }
    std::sort(h.begin(), h.end(), [](const cubed_box_t& a, const cubed_box_t& b) { return a.src_base < b.src_base; });
    CHECK(hipMemcpy(d_boxes, h.data(), nb * sizeof(cubed_box_t), hipMemcpyHostToDevice));
  };
  int variant = 0;  // 0: cached loads + NT stores (library), 1: NT loads, 2: plain stores, 3: NT loads + plain stores
  auto launch = [&](long rot) {
    switch (variant) {
      case 1: hipLaunchKernelGGL((k_flat<1, 0>), dim3(nb * bpb), dim3(kBlock), 0, 0, d_boxes, nb, bpb, rot); break;
      case 2: hipLaunchKernelGGL((k_flat<0, 1>), dim3(nb * bpb), dim3(kBlock), 0, 0, d_boxes, nb, bpb, rot); break;
      case 3: hipLaunchKernelGGL((k_flat<1, 1>), dim3(nb * bpb), dim3(kBlock), 0, 0, d_boxes, nb, bpb, rot); break;
      default: hipLaunchKernelGGL((k_flat<0, 0>), dim3(nb * bpb), dim3(kBlock), 0, 0, d_boxes, nb, bpb, rot); break;
    }
  };
  auto run = [&](const char* tag, long rot) {
    for (int w = 0; w < 2; ++w) launch(rot);
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch(rot);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-26s var %d rot %4ld  %.4f ms  %.0f GB/s moved\n", tag, variant, rot, ms, 2.0 * N * N * 4 / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  const long rots[] = {0, 1, 7, 37, bpb / 2, 0};
  printf("bpb %ld, y - x = %ld B\n", bpb, (long)(y - x));
  build(y);
  if (argc > 2) {  // load/store form sweep on both placements, rot 0
    build(y);
    for (variant = 0; variant < 4; ++variant) run("placement 1 (first y)", 0);
    char* y3;
    CHECK(hipMalloc(&y3, N * N * 4));
    CHECK(hipFree(y));
    build(y3);
    for (variant = 0; variant < 4; ++variant) run("placement 2 (second y)", 0);
    return 0;
  }
  for (long r : rots) run("placement 1 (first y)", r);
  char* y2;
  CHECK(hipMalloc(&y2, N * N * 4));
  CHECK(hipFree(y));
  printf("y2 - x = %ld B\n", (long)(y2 - x));
  build(y2);
  for (long r : rots) run("placement 2 (second y)", r);
  // correctness of the rotated order on the last placement: spot rows
  std::vector<unsigned> a(C), b(C);
  for (long j : {0L, 17L, 49L})
    for (long rr : {0L, 12345L, N - 1}) {
      CHECK(hipMemcpy(a.data(), x + (rr * N + j * C) * 4, C * 4, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(b.data(), y2 + (j * N * C + rr * C) * 4, C * 4, hipMemcpyDeviceToHost));
      if (memcmp(a.data(), b.data(), C * 4)) { printf("MISMATCH j %ld row %ld\n", j, rr); return 1; }
    }
  printf("check ok\n");
  // placement sweep: x and y carved from one pool at chosen offsets
  CHECK(hipFree(y2));
  CHECK(hipFree(x));
  char* pool;
  const long GB = 1L << 30;
  CHECK(hipMalloc(&pool, 64 * GB));
  const long offs[] = {0, 1L << 20, 1L << 30, 2L << 30, 4L << 30, 8L << 30, 12L << 30, 3L << 30, 5L << 30};
  for (int below = 0; below < 2; ++below)
    for (long off : offs) {
      x = below ? pool + 32 * GB : pool;
      char* yy = below ? x - N * N * 4 - off : x + N * N * 4 + off;
      yy = (char*)((uintptr_t)yy & ~(uintptr_t)255);
      hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (unsigned*)x, N * N);
      build(yy);
      char tag[64];
      snprintf(tag, sizeof(tag), "y %s x, gap %ld", below ? "below" : "above", off);
      run(tag, 0);
    }
  return 0;
}
