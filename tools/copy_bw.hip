// copy_bw.hip -- development probe (not part of the library): HBM copy
// variants on MI355X, for choosing the structure of the rechunk copy kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/copy_bw tools/copy_bw.hip
// Run:   tools/copy_bw [GiB]
//
// A: contiguous copy, one 4 KiB segment per wave-iteration, 4 x 16 B per lane
//    (the round-1 k_copy_flat structure), 64 KiB per workgroup.
// B: same, 8 x 16 B per lane in flight.
// C: persistent grid (CUs x 8 workgroups), each wave a contiguous run,
//    double-buffered registers: the next 4 x 16 B are loaded before the
//    current ones are stored.
// D: C with plain (temporal) loads/stores.
// R*: the config-3 rechunk pattern (f32 (50000, 50000) row chunks of 1000 rows
//    -> column chunks of 1000 cols) with A's structure (R1) and with whole
//    destination rows per wave walked as aligned 128-B source lines (R2).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int UN, bool NT, int WAVES = 4>
__global__ __launch_bounds__(WAVES * 64) void k_seg(const u32x4* __restrict__ src, u32x4* __restrict__ dst, long nw, long segs_per_block) {
  constexpr long kSeg = 64 * UN;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long w0 = (long)blockIdx.x * segs_per_block * kSeg;
  long w1 = w0 + segs_per_block * kSeg;
  if (w1 > nw) w1 = nw;
  const G u32x4* s = (const G u32x4*)src;
  G u32x4* d = (G u32x4*)dst;
  for (long i0 = w0 + wave * kSeg; i0 < w1; i0 += WAVES * kSeg) {
    u32x4 v[UN];
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const long i = i0 + k * 64 + lane;
      if (i < w1) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const long i = i0 + k * 64 + lane;
      if (i < w1) { if (NT) __builtin_nontemporal_store(v[k], d + i); else d[i] = v[k]; }
    }
  }
}

// read-only stream (xor-reduce, one store per lane) and write-only fill:
// the two halves of a copy measured alone
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ src, u32x4* __restrict__ out, long nw) {
  const G u32x4* s = (const G u32x4*)src;
  u32x4 acc = {0, 0, 0, 0};
  const long n0 = (long)blockIdx.x * 4096;
  for (long i = n0 + threadIdx.x; i < n0 + 4096 && i < nw; i += 256) acc ^= __builtin_nontemporal_load(s + i);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ dst, long nw) {
  G u32x4* d = (G u32x4*)dst;
  const long n0 = (long)blockIdx.x * 4096;
  const u32x4 v = {1u, 2u, 3u, (unsigned)blockIdx.x};
  for (long i = n0 + threadIdx.x; i < n0 + 4096 && i < nw; i += 256) __builtin_nontemporal_store(v, d + i);
}

// persistent: wave-contiguous runs, register double buffer
template <bool NT>
__global__ __launch_bounds__(256) void k_pers(const u32x4* __restrict__ src, u32x4* __restrict__ dst, long nw) {
  constexpr int UN = 4;
  constexpr long kSeg = 64 * UN;
  const long nwaves = (long)gridDim.x * 4;
  const long wv = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long nseg = (nw + kSeg - 1) / kSeg;
  const long per = (nseg + nwaves - 1) / nwaves;
  long s0 = wv * per, s1 = s0 + per;
  if (s1 > nseg) s1 = nseg;
  if (s0 >= s1) return;
  const G u32x4* s = (const G u32x4*)src;
  G u32x4* d = (G u32x4*)dst;
  auto ld = [&](long seg, u32x4 (&v)[UN]) {
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const long i = seg * kSeg + k * 64 + lane;
      if (i < nw) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
  };
  auto st = [&](long seg, const u32x4 (&v)[UN]) {
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const long i = seg * kSeg + k * 64 + lane;
      if (i < nw) { if (NT) __builtin_nontemporal_store(v[k], d + i); else d[i] = v[k]; }
    }
  };
  u32x4 a[UN], b[UN];
  ld(s0, a);
  long seg = s0;
  for (; seg + 1 < s1; seg += 2) {
    ld(seg + 1, b);
    st(seg, a);
    if (seg + 2 < s1) ld(seg + 2, a);
    st(seg + 1, b);
  }
  if (seg < s1) st(seg, a);
}

// rechunk pattern, A-structure: box = (piece i, target j): 1000 rows x 250 words,
// dst packed; walked as a flat run of destination words (round-1 k_copy_flat)
__global__ __launch_bounds__(256) void k_rflat(const char* __restrict__ src, char* __restrict__ dst, int N, int C, long segs_per_block) {
  constexpr int UN = 4;
  constexpr long kSeg = 64 * UN;
  const int nbj = N / C;
  const long wpb = (long)C * C / 4;  // words per box
  const long bpb = (wpb + segs_per_block * kSeg - 1) / (segs_per_block * kSeg);
  const long box = blockIdx.x / bpb, blk = blockIdx.x % bpb;
  const int i = box / nbj, j = box % nbj;
  const char* sb = src + ((long)i * C * N + (long)j * C) * 4;
  G u32x4* d = (G u32x4*)(dst + ((long)j * N * C + (long)i * C * C) * 4);
  const unsigned nw = C / 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long w0 = blk * segs_per_block * kSeg;
  long w1 = w0 + segs_per_block * kSeg;
  if (w1 > wpb) w1 = wpb;
  for (long i0 = w0 + wave * kSeg; i0 < w1; i0 += 4 * kSeg) {
    u32x4 v[UN];
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const long ii = i0 + k * 64 + lane;
      if (ii < w1) {
        const unsigned r = (unsigned)ii / nw, c = (unsigned)ii - r * nw;
        v[k] = __builtin_nontemporal_load((const G u32x4*)(sb + (long)r * N * 4) + c);
      }
    }
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const long ii = i0 + k * 64 + lane;
      if (ii < w1) __builtin_nontemporal_store(v[k], d + ii);
    }
  }
}

// rechunk pattern, source-row major: a workgroup owns RPB consecutive source
// rows of one row chunk and writes each row's N/C pieces (one per target
// chunk): every source line is read by one workgroup, in order.
template <int RPB>
__global__ __launch_bounds__(256) void k_rrow(const char* __restrict__ src, char* __restrict__ dst, int N, int C) {
  const long row0 = (long)blockIdx.x * RPB;
  const int nwr = N / 4;  // words per source row
  const int lanes = 256;
  for (int rr = 0; rr < RPB; ++rr) {
    const long row = row0 + rr;
    if (row >= N) return;
    const int i = row / C, rin = row % C;
    const G u32x4* s = (const G u32x4*)(src + row * (long)N * 4);
    u32x4 v[4];
    // 256 threads x 4 x 16 B = 16 KiB per pass, a row is 200000 B
    for (int w0 = 0; w0 < nwr; w0 += lanes * 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int w = w0 + k * lanes + threadIdx.x;
        if (w < nwr) v[k] = __builtin_nontemporal_load(s + w);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int w = w0 + k * lanes + threadIdx.x;
        if (w < nwr) {
          const int col = w * 4, j = col / C, cin = col % C;
          G u32x4* d = (G u32x4*)(dst + (((long)j * N * C) + ((long)i * C + rin) * C + cin) * 4);
          __builtin_nontemporal_store(v[k], d);
        }
      }
    }
  }
}

static float timeit(void (*launch)(void*), void* ctx, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  launch(ctx);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch(ctx);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

struct Ctx { void* src; void* dst; long nbytes; int N, C; long spb; int ncu; };

int main(int argc, char** argv) {
  int N = 50000, C = 1000;
  Ctx c;
  c.N = N; c.C = C;
  c.nbytes = (long)N * N * 4;
  CHECK(hipMalloc(&c.src, c.nbytes));
  CHECK(hipMalloc(&c.dst, c.nbytes));
  CHECK(hipMemset(c.src, 1, c.nbytes));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  c.ncu = p.multiProcessorCount;
  const long nw = c.nbytes / 16;
  const double gb = 2.0 * c.nbytes / 1e9;
  for (int round = 0; round < 2; ++round) {
    for (long spb : {16L, 64L}) {
      c.spb = spb;
      float ms = timeit([](void* x) { Ctx* c = (Ctx*)x; long nw = c->nbytes / 16; long per = c->spb * 256;
        hipLaunchKernelGGL((k_seg<4, true>), dim3((nw + per - 1) / per), dim3(256), 0, 0, (const u32x4*)c->src, (u32x4*)c->dst, nw, c->spb); }, &c, 5);
      printf("A contiguous UN4 nt spb%ld: %.3f ms %.0f GB/s\n", spb, ms, gb / ms * 1e3);
      ms = timeit([](void* x) { Ctx* c = (Ctx*)x; long nw = c->nbytes / 16; long per = c->spb * 512;
        hipLaunchKernelGGL((k_seg<8, true>), dim3((nw + per - 1) / per), dim3(256), 0, 0, (const u32x4*)c->src, (u32x4*)c->dst, nw, c->spb); }, &c, 5);
      printf("B contiguous UN8 nt spb%ld: %.3f ms %.0f GB/s\n", spb, ms, gb / ms * 1e3);
      ms = timeit([](void* x) { Ctx* c = (Ctx*)x; long nw = c->nbytes / 16; long per = c->spb * 256;
        hipLaunchKernelGGL((k_seg<4, false>), dim3((nw + per - 1) / per), dim3(256), 0, 0, (const u32x4*)c->src, (u32x4*)c->dst, nw, c->spb); }, &c, 5);
      printf("A' contiguous UN4 plain spb%ld: %.3f ms %.0f GB/s\n", spb, ms, gb / ms * 1e3);
    }
    {
      c.spb = 16;
      float ms = timeit([](void* x) { Ctx* c = (Ctx*)x; long nw = c->nbytes / 16; long per = c->spb * 256;
        hipLaunchKernelGGL((k_seg<4, true, 8>), dim3((nw + per - 1) / per), dim3(512), 0, 0, (const u32x4*)c->src, (u32x4*)c->dst, nw, c->spb); }, &c, 5);
      printf("E contiguous UN4 nt 512-thread WG spb16: %.3f ms %.0f GB/s\n", ms, gb / ms * 1e3);
      ms = timeit([](void* x) { Ctx* c = (Ctx*)x; long nw = c->nbytes / 16; long per = c->spb * 256;
        hipLaunchKernelGGL((k_seg<4, true, 16>), dim3((nw + per - 1) / per), dim3(1024), 0, 0, (const u32x4*)c->src, (u32x4*)c->dst, nw, c->spb); }, &c, 5);
      printf("E' contiguous UN4 nt 1024-thread WG spb16: %.3f ms %.0f GB/s\n", ms, gb / ms * 1e3);
      ms = timeit([](void* x) { Ctx* c = (Ctx*)x; long nw = c->nbytes / 16; long per = c->spb * 128;
        hipLaunchKernelGGL((k_seg<2, true, 4>), dim3((nw + per - 1) / per), dim3(256), 0, 0, (const u32x4*)c->src, (u32x4*)c->dst, nw, c->spb); }, &c, 5);
      printf("E'' contiguous UN2 nt spb16: %.3f ms %.0f GB/s\n", ms, gb / ms * 1e3);
      ms = timeit([](void* x) { Ctx* c = (Ctx*)x; CHECK(hipMemcpyAsync(c->dst, c->src, c->nbytes, hipMemcpyDeviceToDevice, 0)); }, &c, 5);
      printf("H hipMemcpyAsync D2D: %.3f ms %.0f GB/s\n", ms, gb / ms * 1e3);
      ms = timeit([](void* x) { Ctx* c = (Ctx*)x; long nw = c->nbytes / 16;
        hipLaunchKernelGGL(k_read, dim3((nw + 4095) / 4096), dim3(256), 0, 0, (const u32x4*)c->src, (u32x4*)c->dst, nw); }, &c, 5);
      printf("F read-only stream: %.3f ms %.0f GB/s (bytes read)\n", ms, gb / 2 / ms * 1e3);
      ms = timeit([](void* x) { Ctx* c = (Ctx*)x; long nw = c->nbytes / 16;
        hipLaunchKernelGGL(k_write, dim3((nw + 4095) / 4096), dim3(256), 0, 0, (u32x4*)c->dst, nw); }, &c, 5);
      printf("G write-only fill: %.3f ms %.0f GB/s (bytes written)\n", ms, gb / 2 / ms * 1e3);
    }
    for (int wpc : {4, 8, 16}) {
      c.spb = wpc;
      float ms = timeit([](void* x) { Ctx* c = (Ctx*)x;
        hipLaunchKernelGGL((k_pers<true>), dim3(c->ncu * c->spb), dim3(256), 0, 0, (const u32x4*)c->src, (u32x4*)c->dst, c->nbytes / 16); }, &c, 5);
      printf("C persistent dbuf nt %d WG/CU: %.3f ms %.0f GB/s\n", wpc, ms, gb / ms * 1e3);
      ms = timeit([](void* x) { Ctx* c = (Ctx*)x;
        hipLaunchKernelGGL((k_pers<false>), dim3(c->ncu * c->spb), dim3(256), 0, 0, (const u32x4*)c->src, (u32x4*)c->dst, c->nbytes / 16); }, &c, 5);
      printf("D persistent dbuf plain %d WG/CU: %.3f ms %.0f GB/s\n", wpc, ms, gb / ms * 1e3);
    }
    c.spb = 16;
    float ms = timeit([](void* x) { Ctx* c = (Ctx*)x; long nbox = (long)(c->N / c->C) * (c->N / c->C);
      long wpb = (long)c->C * c->C / 4; long bpb = (wpb + c->spb * 256 - 1) / (c->spb * 256);
      hipLaunchKernelGGL(k_rflat, dim3(nbox * bpb), dim3(256), 0, 0, (const char*)c->src, (char*)c->dst, c->N, c->C, c->spb); }, &c, 5);
    printf("R1 rechunk flat boxes spb16: %.3f ms %.0f GB/s\n", ms, gb / ms * 1e3);
    ms = timeit([](void* x) { Ctx* c = (Ctx*)x;
      hipLaunchKernelGGL((k_rrow<4>), dim3((c->N + 3) / 4), dim3(256), 0, 0, (const char*)c->src, (char*)c->dst, c->N, c->C); }, &c, 5);
    printf("R2 rechunk source rows (4 rows/WG): %.3f ms %.0f GB/s\n", ms, gb / ms * 1e3);
    ms = timeit([](void* x) { Ctx* c = (Ctx*)x;
      hipLaunchKernelGGL((k_rrow<1>), dim3(c->N), dim3(256), 0, 0, (const char*)c->src, (char*)c->dst, c->N, c->C); }, &c, 5);
    printf("R3 rechunk source rows (1 row/WG): %.3f ms %.0f GB/s\n", ms, gb / ms * 1e3);
  }
  return 0;
}
