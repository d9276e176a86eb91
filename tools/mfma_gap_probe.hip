// mfma_gap_probe.hip -- development probe (not part of the library).
//
// What one filler instruction costs inside the gap of a v_mfma_f32_32x32x16_bf16
// stream when ONE wave owns its SIMD (the 128 x 128-per-wave bf16 GEMM
// schedule the round-4 review asks for: 16 accumulators of 32 x 32 = 256
// AGPRs, 32 MFMAs per 32-deep K step, per step 8 ds_read_b128 (A), 16
// ds_read_b64_tr_b16 (B) and 8 global_load_lds pieces (this wave's quarter
// of a 256 x 256 x 32 stage)).  Each variant runs the same 32-MFMA step
// ITERS times with a different filler set placed one-per-gap by
// sched_barrier, on every CU at once (one 256-thread workgroup per CU,
// LDS sized to keep it alone); s_memtime around the loop gives cycles per
// MFMA (the floor is 32), HIP events the kernel time.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mfma_gap_probe tools/mfma_gap_probe.hip
// Run:   tools/mfma_gap_probe [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <utility>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#define L3 __attribute__((address_space(3)))
#define G1 __attribute__((address_space(1)))

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int LDS_BYTES = 96 * 1024;  // one workgroup per CU

// filler kinds per gap g (0..31) of a step
enum { F_NONE = 0, F_B128 = 1, F_TR = 2, F_GLDS = 4 };

// V: 0 bare | 1 b128 every gap | 2 tr every gap | 3 glds every 4th gap |
//    4 glds every 2nd gap | 5 the step's 24 reads (8 b128 + 16 tr) |
//    6 the full step (24 reads + 8 glds) | 7 full step + lgkmcnt/vmcnt wait +
//    s_barrier at the step's end (the real loop's step boundary) |
//    8 full step with the glds in the first 8 gaps | 9 full step, 2 fillers
//    per gap in the first 16 gaps then bare
template <int V>
__device__ __forceinline__ int filler(int g) {
  switch (V) {
    case 1: return F_B128;
    case 2: return F_TR;
    case 3: return (g % 4 == 0) ? F_GLDS : 0;
    case 4: return (g % 2 == 0) ? F_GLDS : 0;
    case 5: return (g % 4 == 0) ? F_B128 : F_TR * ((g % 4) != 3 || g < 0) ;  // 8 b128, 24 tr -> trimmed below
    case 6: case 7: return ((g % 4 == 0) ? F_B128 : ((g % 4 == 1 || g % 4 == 3) ? F_TR : F_GLDS));
    case 8: return (g < 8 ? F_GLDS : 0) | ((g % 4 == 0) ? F_B128 : ((g % 4 == 1 || g % 4 == 3) ? F_TR : 0));
    case 9: return g < 16 ? ((g % 2 == 0) ? (F_B128 | F_GLDS) : (F_TR)) : ((g % 2 == 0) ? F_TR : 0);
    case 10: return (g % 2 == 0) ? F_TR : 0;
    case 11: return (g % 2 == 0) ? F_B128 : 0;
    case 12: return F_B128 | F_TR;
    case 13: return (g % 2 == 0) ? F_B128 : ((g % 4 == 1) ? F_GLDS : 0);  // B^T step: 16 b128 + 8 glds
    case 14: return (g % 2 == 0) ? F_B128 : 0;                             // 16 b128 only
    default: return 0;
  }
}

template <int V>
__global__ __launch_bounds__(256, 1) void k_gap(const char* __restrict__ src, size_t src_mask, int iters,
                                                  unsigned long long* __restrict__ cyc, float* __restrict__ sink) {
  __shared__ __attribute__((aligned(1024))) char lds_[LDS_BYTES];
  L3 char* lds = (L3 char*)lds_;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};
  bf16x8 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    for (int e = 0; e < 8; ++e) {
      a[i][e] = (__bf16)(0.001f * (lane + e + i));
      b[i][e] = (__bf16)(0.002f * (lane - e + i));
    }
  }
  u32x4 rd = {0, 0, 0, 0};
  s16x4 rt = {0, 0, 0, 0};
  // the fragment addresses of the library's one-wave layout
  // (tools/gemm_bf16_experiments.h k_gemm_bf16_w4): A [256][64 B] rows, chunk
  // slot s of row r = k chunk s ^ ((r >> 2) & 3); B [32 k-rows][512 B], chunk
  // slot s of k-row r = col chunk s ^ 4 * (r & 3) -- both conflict-free
  const int ra_ = lane & 31;
  const uint32_t lb = (uint32_t)(uintptr_t)(lds + ra_ * 64 + 16 * (((lane >> 5)) ^ ((ra_ >> 2) & 3)));
  const int bq = lane >> 4, krow = (bq >> 1) * 8 + ((lane & 15) >> 2);
  const uint32_t lt = (uint32_t)(uintptr_t)(lds + 16384 + krow * 512 +
                                            16 * (((bq & 1) * 2 + ((lane & 3) >> 1)) ^ (4 * (krow & 3))) +
                                            8 * (lane & 1));
  size_t goff = ((size_t)(blockIdx.x * 4 + w) * 65536 + lane * 16) & src_mask;
  __syncthreads();
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; ++it) {
    // every read of a step lands in its own registers, consumed at the step's
    // end (the next step's fragments): the only lgkmcnt wait is there
    u32x4 ra[32];
    s16x4 rtt[32];
#pragma unroll
    for (int g = 0; g < 32; ++g) {
      const int mi = (g >> 1) & 3, ni = (g >> 3) & 3;
      acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      int f = filler<V>(g);
      if (V == 5) f = (g % 4 == 0) ? F_B128 : ((g % 4 == 1 || g % 4 == 3) ? F_TR : 0);
      if (f & F_B128)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ra[g]) : "v"(lb), "i"(0));
      else
        ra[g] = u32x4{0, 0, 0, 0};
      if (f & F_TR)
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(rtt[g]) : "v"(lt));
      else
        rtt[g] = s16x4{0, 0, 0, 0};
      if (f & F_GLDS) {
        __builtin_amdgcn_global_load_lds((const G1 void*)(uintptr_t)(src + goff),
                                         (L3 void*)(lds + w * 16384 + (g & 7) * 1024), 16, 0, 0);
        goff = (goff + 4096) & src_mask;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int g = 0; g < 32; ++g) {
      rd ^= ra[g];
      rt ^= rtt[g];
    }
    if (V == 7) {
      asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][lane & 15];
  s += (float)(rd[0] ^ rd[1] ^ rd[2] ^ rd[3]) * 1e-30f + (float)(rt[0] ^ rt[3]) * 1e-30f;
  sink[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
}

// Two waves per SIMD (512 threads, 256 registers per wave): each wave owns
// 128 x 64 (8 accumulators), a step = 16 MFMAs + this wave's fillers.  V2:
// 0 bare | 1 the wave's step reads (8 b128 + 8 tr, one per gap) | 2 reads +
// 4 glds (the wave's half of the stage) | 3 as 2 + lgkmcnt/vmcnt + s_barrier
template <int V2>
__global__ __launch_bounds__(512, 1) void k_gap2(const char* __restrict__ src, size_t src_mask, int iters,
                                                   unsigned long long* __restrict__ cyc, float* __restrict__ sink) {
  __shared__ __attribute__((aligned(1024))) char lds_[LDS_BYTES];
  L3 char* lds = (L3 char*)lds_;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  bf16x8 a[4], b[2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 8; ++e) a[i][e] = (__bf16)(0.001f * (lane + e + i));
#pragma unroll
  for (int i = 0; i < 2; ++i)
    for (int e = 0; e < 8; ++e) b[i][e] = (__bf16)(0.002f * (lane - e + i));
  u32x4 rd = {0, 0, 0, 0};
  s16x4 rt = {0, 0, 0, 0};
  const int ra_ = lane & 31;
  const uint32_t lb = (uint32_t)(uintptr_t)(lds + ra_ * 64 + 16 * (((lane >> 5)) ^ ((ra_ >> 2) & 3)));
  const int bq = lane >> 4, krow = (bq >> 1) * 8 + ((lane & 15) >> 2);
  const uint32_t lt = (uint32_t)(uintptr_t)(lds + 16384 + krow * 512 +
                                            16 * (((bq & 1) * 2 + ((lane & 3) >> 1)) ^ (4 * (krow & 3))) +
                                            8 * (lane & 1));
  size_t goff = ((size_t)(blockIdx.x * 8 + w) * 65536 + lane * 16) & src_mask;
  __syncthreads();
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; ++it) {
    u32x4 ra[16];
    s16x4 rtt[16];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int mi = (g >> 1) & 3, ni = (g >> 3) & 1;
      acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (V2 >= 1 && (g & 1) == 0)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ra[g]) : "v"(lb), "i"(0));
      else
        ra[g] = u32x4{0, 0, 0, 0};
      if (V2 >= 1 && (g & 1) == 1)
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(rtt[g]) : "v"(lt));
      else
        rtt[g] = s16x4{0, 0, 0, 0};
      if (V2 >= 2 && (g % 4) == 2) {
        __builtin_amdgcn_global_load_lds((const G1 void*)(uintptr_t)(src + goff),
                                         (L3 void*)(lds + (w & 3) * 16384 + (g & 7) * 1024), 16, 0, 0);
        goff = (goff + 4096) & src_mask;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      rd ^= ra[g];
      rt ^= rtt[g];
    }
    if (V2 == 3) {
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) s += acc[i][j][lane & 15];
  s += (float)(rd[0] ^ rd[1] ^ rd[2] ^ rd[3]) * 1e-30f + (float)(rt[0] ^ rt[3]) * 1e-30f;
  sink[blockIdx.x * 512 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

template <int V2>
void run2(const char* name, const char* src, size_t mask, int iters, int nblk, unsigned long long* d_cyc,
          float* d_sink) {
  hipLaunchKernelGGL(k_gap2<V2>, dim3(nblk), dim3(512), 0, 0, src, mask, iters, d_cyc, d_sink);  // warm
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_gap2<V2>, dim3(nblk), dim3(512), 0, 0, src, mask, iters, d_cyc, d_sink);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> c(nblk * 8);
  CHECK(hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost));
  std::sort(c.begin(), c.end());
  const double per = 32.0 * iters;  // two waves x 16 MFMAs per step on one SIMD
  const double flop = 32768.0 * 16 * iters * 8 * nblk;
  printf("%-44s cyc/MFMA/SIMD median %6.2f  p90 %6.2f  kernel %8.3f ms  %7.1f TF  (clk %.2f GHz)\n", name,
         c[c.size() / 2] / per, c[c.size() * 9 / 10] / per, ms, flop / (ms * 1e-3) / 1e12,
         c[c.size() / 2] / (ms * 1e-3) / 1e9);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

// ---- k_flow<F>: the w4l main loop's data flow without global memory
// semantics: two fragment sets, step p's 32 MFMAs read set X while this
// step's fillers read LDS into set Y (the next step's operands) -- no VALU
// consumes a read (k_gap above XORs every read into a sink after the step:
// 4 VALU per b128, which is what its "per filler" cycles mostly measured).
// F bits: 1 the 8 A ds_read_b128 | 2 the 16 B ds_read_b64_tr_b16 (or, with
// 16, 8 B ds_read_b128 from a B^T image laid out as A's, conflict-free) | 4 the 8 LDS-DMA pieces (+ one 64-bit
// source increment each, every 4th gap) | 8 s_waitcnt + s_barrier per step.
template <int J>
using ic = std::integral_constant<int, J>;
template <typename Fn, int... I>
__device__ __forceinline__ void seq_(Fn&& f, std::integer_sequence<int, I...>) {
  (f(ic<I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void seq(Fn&& f) {
  seq_(f, std::make_integer_sequence<int, N>{});
}
struct Fr {
  bf16x8 a[4][2], bt[4][2];
  s16x4 bl[4][2], bh[4][2];
};
template <int F>
__device__ __forceinline__ void flow_step(const Fr& X, Fr& Y, f32x16 (&acc)[4][4], uint32_t la, uint32_t lbt,
                                          const char* src, const char*& gp, size_t mask, L3 char* lds, int w) {
  seq<32>([&](auto G) {
    constexpr int g = decltype(G)::value, kh = g >> 4, mb = (g >> 2) & 3, nb = g & 3;
    if constexpr (F & 16) {
      acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(X.a[mb][kh], X.bt[nb][kh], acc[mb][nb], 0, 0, 0);
    } else {
      const bf16x8 b = __builtin_bit_cast(bf16x8, __builtin_shufflevector(X.bl[nb][kh], X.bh[nb][kh], 0, 1, 2, 3,
                                                                          4, 5, 6, 7));
      acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(X.a[mb][kh], b, acc[mb][nb], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    constexpr int r = g & 3, i = g >> 2;
    if constexpr (r == 0 && (F & 1)) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(Y.a[i & 3][i >> 2]) : "v"(la), "i"((i & 3) * 4096));
    } else if constexpr ((r == 1 || r == 3) && (F & 2)) {
      constexpr int j = 2 * i + (r == 3), jn = (j >> 1) & 3, jk = j >> 3;
      if constexpr (F & 16) {
        if constexpr (r == 1)  // B^T: one b128 per fragment
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(Y.bt[jn][jk]) : "v"(la), "i"(32768 + jn * 4096));
      } else if constexpr (j & 1) {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(Y.bh[jn][jk]) : "v"(lbt), "i"(jk * 8192 + 2048));
      } else {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(Y.bl[jn][jk]) : "v"(lbt), "i"(jk * 8192));
      }
    } else if constexpr (r == 2 && (F & 4)) {
      __builtin_amdgcn_global_load_lds((const G1 void*)gp, (L3 void*)(lds + 65536 + w * 8192 + (i & 7) * 1024), 16,
                                       0, 0);
      gp += 4096;  // one 64-bit increment per piece, as the library's sources
    }
    __builtin_amdgcn_sched_barrier(0);
  });
  if constexpr (F & 4) gp = src + ((size_t)(gp - src) & mask);
  if constexpr (F & 8) {
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int F>
__global__ __launch_bounds__(256, 1) void k_flow(const char* __restrict__ src, size_t src_mask, int iters,
                                                   unsigned long long* __restrict__ cyc, float* __restrict__ sink) {
  __shared__ __attribute__((aligned(1024))) char lds_[LDS_BYTES];
  L3 char* lds = (L3 char*)lds_;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < LDS_BYTES / 4; i += 256) ((L3 float*)lds)[i] = 0.001f * (i & 255);
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};
  Fr f0, f1;
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 2; ++k) {
      for (int e = 0; e < 8; ++e) f0.a[i][k][e] = f1.a[i][k][e] = (__bf16)(0.001f * (lane + e + i));
      f0.bl[i][k] = f1.bl[i][k] = s16x4{1, 2, 3, 4};
      f0.bh[i][k] = f1.bh[i][k] = s16x4{5, 6, 7, 8};
      f0.bt[i][k] = f1.bt[i][k] = f0.a[i][k];
    }
  // the library's conflict-free fragment addresses (gemm_bf16_w4l.h)
  const int ra = (w >> 1) * 128 + (lane & 31);
  const uint32_t la = (uint32_t)(uintptr_t)(lds + (ra & 127) * 128 + 16 * ((lane >> 5) ^ ((ra >> 1) & 7)));
  const int bq = lane >> 4, krow = (bq >> 1) * 8 + ((lane & 15) >> 2);
  const uint32_t lbt = (uint32_t)(uintptr_t)(lds + 16384 * 0 + krow * 512 +
                                             16 * ((((w & 1) * 16) + (bq & 1) * 2 + ((lane & 3) >> 1)) ^ (4 * (krow & 3))) +
                                             8 * (lane & 1));
  const char* gp = src + (((size_t)(blockIdx.x * 4 + w) * 65536 + lane * 16) & src_mask);
  __syncthreads();
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; it += 2) {
    flow_step<F>(f0, f1, acc, la, lbt, src, gp, src_mask, lds, w);
    flow_step<F>(f1, f0, acc, la, lbt, src, gp, src_mask, lds, w);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][lane & 15];
  sink[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
}

template <int F>
void runf(const char* name, const char* src, size_t mask, int iters, int nblk, unsigned long long* d_cyc,
          float* d_sink) {
  hipLaunchKernelGGL(k_flow<F>, dim3(nblk), dim3(256), 0, 0, src, mask, iters, d_cyc, d_sink);  // warm
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_flow<F>, dim3(nblk), dim3(256), 0, 0, src, mask, iters, d_cyc, d_sink);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> c(nblk * 4);
  CHECK(hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost));
  std::sort(c.begin(), c.end());
  const double per = 32.0 * iters;
  const double flop = 32768.0 * 32 * iters * 4 * nblk;
  printf("flow %-39s cyc/MFMA median %6.2f  p90 %6.2f  kernel %8.3f ms  %7.1f TF  (clk %.2f GHz)\n", name,
         c[c.size() / 2] / per, c[c.size() * 9 / 10] / per, ms, flop / (ms * 1e-3) / 1e12,
         c[c.size() / 2] / (ms * 1e-3) / 1e9);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

// ---- k_flow32<F>: the f32 one-wave step (gemm_f32_w4.h): 128
// v_mfma_f32_32x32x2_f32 over 16 accumulators, fragments f32x4 a[2][4] /
// b[2][4] read for the next step (F & 1: the 16 ds_read_b128, one per 4
// MFMAs in the first half), F & 4: 8 LDS-DMA pieces, F & 8: wait + barrier.
struct Fr32 {
  f32x4 a[2][4], b[2][4];
};

template <int F>
__device__ __forceinline__ void flow32_step(const Fr32& X, Fr32& Y, f32x16 (&acc)[4][4], uint32_t la,
                                            const char* src, const char*& gp, size_t mask, L3 char* lds, int w) {
  seq<128>([&](auto G) {
    constexpr int gi = decltype(G)::value, g = gi >> 6, j = (gi >> 4) & 3, rb = (gi >> 2) & 3, q = gi & 3;
    acc[rb][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(X.a[g][rb][j], X.b[g][j][q], acc[rb][q], 0, 0, 0);
    if constexpr ((F & 1) && gi < 64 && (gi & 3) == 0) {
      __builtin_amdgcn_sched_barrier(0);
      constexpr int e = gi >> 2;
      if constexpr (e < 8)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(Y.a[e >> 2][e & 3]) : "v"(la), "i"((e & 3) * 2048));
      else
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(Y.b[(e >> 2) & 1][e & 3]) : "v"(la), "i"(16384 + (e & 7) * 1024));
      __builtin_amdgcn_sched_barrier(0);
    } else if constexpr ((F & 4) && gi > 64 && (gi & 7) == 4) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_global_load_lds((const G1 void*)gp, (L3 void*)(lds + 65536 + w * 8192 + (gi & 7) * 1024), 16,
                                       0, 0);
      gp += 4096;
      __builtin_amdgcn_sched_barrier(0);
    }
  });
  if constexpr (F & 4) gp = src + ((size_t)(gp - src) & mask);
  if constexpr (F & 8) {
    asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int F>
__global__ __launch_bounds__(256, 1) void k_flow32(const char* __restrict__ src, size_t src_mask, int iters,
                                                     unsigned long long* __restrict__ cyc, float* __restrict__ sink) {
  __shared__ __attribute__((aligned(1024))) char lds_[LDS_BYTES];
  L3 char* lds = (L3 char*)lds_;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < LDS_BYTES / 4; i += 256) ((L3 float*)lds)[i] = 0.001f * (i & 255);
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};
  Fr32 f0, f1;
  for (int i = 0; i < 2; ++i)
    for (int k = 0; k < 4; ++k) {
      f0.a[i][k] = f1.a[i][k] = f32x4{0.5f, 0.25f, 0.125f, 1.f} * (float)(lane + k);
      f0.b[i][k] = f1.b[i][k] = f32x4{1.f, 2.f, 3.f, 4.f} * 0.001f;
    }
  const uint32_t la = (uint32_t)(uintptr_t)(lds + (lane & 31) * 64 + 16 * ((lane >> 5) ^ ((lane >> 2) & 3)));
  const char* gp = src + (((size_t)(blockIdx.x * 4 + w) * 65536 + lane * 16) & src_mask);
  __syncthreads();
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; it += 2) {
    flow32_step<F>(f0, f1, acc, la, src, gp, src_mask, lds, w);
    flow32_step<F>(f1, f0, acc, la, src, gp, src_mask, lds, w);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][lane & 15];
  sink[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
}

template <int F>
void runf32(const char* name, const char* src, size_t mask, int iters, int nblk, unsigned long long* d_cyc,
            float* d_sink) {
  hipLaunchKernelGGL(k_flow32<F>, dim3(nblk), dim3(256), 0, 0, src, mask, iters, d_cyc, d_sink);  // warm
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_flow32<F>, dim3(nblk), dim3(256), 0, 0, src, mask, iters, d_cyc, d_sink);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> c(nblk * 4);
  CHECK(hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost));
  std::sort(c.begin(), c.end());
  const double per = 128.0 * iters;
  const double flop = 4096.0 * 128 * iters * 4 * nblk;
  printf("flow32 %-37s cyc/MFMA median %6.2f  p90 %6.2f  kernel %8.3f ms  %7.1f TF  (clk %.2f GHz)\n", name,
         c[c.size() / 2] / per, c[c.size() * 9 / 10] / per, ms, flop / (ms * 1e-3) / 1e12,
         c[c.size() / 2] / (ms * 1e-3) / 1e9);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

template <int V>
void run(const char* name, const char* src, size_t mask, int iters, int nblk, unsigned long long* d_cyc,
         float* d_sink) {
  hipLaunchKernelGGL(k_gap<V>, dim3(nblk), dim3(256), 0, 0, src, mask, iters, d_cyc, d_sink);  // warm
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_gap<V>, dim3(nblk), dim3(256), 0, 0, src, mask, iters, d_cyc, d_sink);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> c(nblk * 4);
  CHECK(hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost));
  std::sort(c.begin(), c.end());
  const double per = 32.0 * iters;
  const double flop = 32768.0 * 32 * iters * 4 * nblk;
  printf("%-44s cyc/MFMA median %6.2f  p90 %6.2f  kernel %8.3f ms  %7.1f TF  (clk %.2f GHz)\n", name,
         c[c.size() / 2] / per, c[c.size() * 9 / 10] / per, ms, flop / (ms * 1e-3) / 1e12,
         c[c.size() / 2] / (ms * 1e-3) / 1e9);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  int dev = 0, ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int nblk = ncu;
  unsigned long long* d_cyc;
  float* d_sink;
  CHECK(hipMalloc(&d_cyc, nblk * 8 * 8));
  CHECK(hipMalloc(&d_sink, nblk * 512 * 4));
  // glds sources: L2-resident (4 MiB per XCD-ish) and HBM-streamed (1 GiB)
  for (size_t bytes : {(size_t)4 << 20, (size_t)1 << 30}) {
    char* src;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMemset(src, 1, bytes));
    const size_t mask = bytes - 1;
    printf("# %d CUs x 1 workgroup (4 waves, one per SIMD), %d steps of 32 MFMAs; glds source %zu MiB\n", ncu,
           iters, bytes >> 20);
    run<0>("bare 32x32x16 MFMAs", src, mask, iters, nblk, d_cyc, d_sink);
    run<1>("+1 ds_read_b128 every gap", src, mask, iters, nblk, d_cyc, d_sink);
    run<2>("+1 ds_read_b64_tr_b16 every gap", src, mask, iters, nblk, d_cyc, d_sink);
    run<3>("+1 glds16 every 4th gap (8/step)", src, mask, iters, nblk, d_cyc, d_sink);
    run<4>("+1 glds16 every 2nd gap (16/step)", src, mask, iters, nblk, d_cyc, d_sink);
    run<5>("step reads: 8 b128 + 16 tr, 1/gap", src, mask, iters, nblk, d_cyc, d_sink);
    run<6>("full step: 24 reads + 8 glds, 1/gap", src, mask, iters, nblk, d_cyc, d_sink);
    run<7>("full step + vmcnt/lgkmcnt + s_barrier", src, mask, iters, nblk, d_cyc, d_sink);
    run<8>("full step, glds in gaps 0-7", src, mask, iters, nblk, d_cyc, d_sink);
    run<9>("full step, 2/gap in gaps 0-15", src, mask, iters, nblk, d_cyc, d_sink);
    run<10>("+1 ds_read_b64_tr_b16 every 2nd gap", src, mask, iters, nblk, d_cyc, d_sink);
    run<11>("+1 ds_read_b128 every 2nd gap", src, mask, iters, nblk, d_cyc, d_sink);
    run<12>("+1 b128 + 1 tr every gap", src, mask, iters, nblk, d_cyc, d_sink);
    runf<0>("bare (two fragment sets)", src, mask, iters, nblk, d_cyc, d_sink);
    runf<1>("8 A b128 reads", src, mask, iters, nblk, d_cyc, d_sink);
    runf<2>("16 B tr_b16 reads", src, mask, iters, nblk, d_cyc, d_sink);
    runf<3>("24 reads (A + B)", src, mask, iters, nblk, d_cyc, d_sink);
    runf<4>("8 LDS-DMA pieces", src, mask, iters, nblk, d_cyc, d_sink);
    runf<7>("24 reads + 8 DMA", src, mask, iters, nblk, d_cyc, d_sink);
    runf<15>("24 reads + 8 DMA + wait/barrier", src, mask, iters, nblk, d_cyc, d_sink);
    runf<8>("wait/barrier only", src, mask, iters, nblk, d_cyc, d_sink);
    runf<19>("B^T: 16 b128 reads", src, mask, iters, nblk, d_cyc, d_sink);
    runf<31>("B^T: 16 b128 + 8 DMA + wait/barrier", src, mask, iters, nblk, d_cyc, d_sink);
    runf32<0>("f32 bare (128 MFMAs/step)", src, mask, iters / 4, nblk, d_cyc, d_sink);
    runf32<1>("f32 + 16 b128 reads", src, mask, iters / 4, nblk, d_cyc, d_sink);
    runf32<5>("f32 + reads + 8 DMA", src, mask, iters / 4, nblk, d_cyc, d_sink);
    runf32<13>("f32 + reads + DMA + wait/barrier", src, mask, iters / 4, nblk, d_cyc, d_sink);
    run<13>("B^T step: 16 b128 + 8 glds, 1/gap", src, mask, iters, nblk, d_cyc, d_sink);
    run<14>("16 b128 (every 2nd gap)", src, mask, iters, nblk, d_cyc, d_sink);
    if (argc > 2) {  // two waves per SIMD
      run2<0>("2 waves/SIMD: bare", src, mask, iters, nblk, d_cyc, d_sink);
      run2<1>("2 waves/SIMD: 8 b128 + 8 tr per wave-step", src, mask, iters, nblk, d_cyc, d_sink);
      run2<2>("2 waves/SIMD: + 4 glds per wave-step", src, mask, iters, nblk, d_cyc, d_sink);
      run2<3>("2 waves/SIMD: + waits + s_barrier", src, mask, iters, nblk, d_cyc, d_sink);
    }
    CHECK(hipFree(src));
  }
  return 0;
}
