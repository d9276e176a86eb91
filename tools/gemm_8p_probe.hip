// gemm_8p_probe.hip -- development probe (not part of the library): BASELINE
// config 5's bf16 chained GEMM (40000^2 in 5000^2 chunks, f32 out) on the
// library's packed operands, timed in ONE process on the one-wave kernel
// (k_gemm_bf16_w4p) and the two-waves-per-SIMD kernel (k_gemm_bf16_8p,
// csrc/gemm_bf16_8p.h), alternating; the outputs compared word for word.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude \
//          -o tools/gemm_8p_probe tools/gemm_8p_probe.hip
// Run:   tools/gemm_8p_probe [reps] [N] [out: 0 f32 / 1 bf16] [arms] -- arms 3: f32 INPUTS
//        (k_gemm_f32_w4p vs k_gemm_f32_8p)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

namespace cubed {
thread_local char g_err[512];
}
#include "../cubed_amd/csrc/gemm_chain.hip"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_fill(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float v = (float)(h >> 8) * (1.0f / 16777216.0f);  // U[0, 1) as config 5
    p[i] = (uint16_t)(__float_as_uint(v) >> 16);
  }
}

// pack A with all 8 rows' loads of a block issued before its stores (the
// library form unrolls by 2)
template <bool NTL = true, bool NTS = false>
__global__ __launch_bounds__(256) void k_pack_a8(const cubed_gemm_chain_t* __restrict__ tasks,
                                                 const cubed_gemm_seg_t* __restrict__ segs, PackPlan pp,
                                                 char* __restrict__ PA) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int64_t nkt = pp.kt1 - pp.kt0, nblk = pp.TM * nkt;
  const cubed_gemm_seg_t* __restrict__ sg0 = segs + tasks[0].seg0;
  const int sl = threadIdx.x & 7;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t mt = blk / nkt, kt = pp.kt0 + (blk - mt * nkt);
    const int64_t I0 = (mt * 256) / pp.cm, mb = (I0 + 1) * pp.cm;
    int64_t s0 = 0, ks0 = 0;
    if (kt * 64 < pp.K) seg_at(sg0, kt * 64, s0, ks0);
    char* dst = PA + mt * pp.apstride + kt * pp.akstride;
    uint4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = (threadIdx.x >> 3) + 32 * j, c = sl ^ ((r >> 1) & 7);
      const int64_t gm = mt * 256 + r, k = kt * 64 + c * 8;
      v[j] = uint4{0, 0, 0, 0};
      if (gm < pp.M && k < pp.K) {
        int64_t s = s0, ks = ks0;
        seg_at(sg0, k, s, ks);
        const bool hi = gm >= mb;
        const int64_t I = hi ? I0 + 1 : I0, lm = gm - I * pp.cm;
        const cubed_gemm_seg_t& S = segs[tasks[I * pp.tj].seg0 + s];
        const u32x4* src = (const u32x4*)((const char*)(uintptr_t)S.a + (lm * S.lda + (k - ks)) * 2);
        const u32x4 x = NTL ? __builtin_nontemporal_load(src) : *src;
        v[j] = uint4{x.x, x.y, x.z, x.w};
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = (threadIdx.x >> 3) + 32 * j;
      if constexpr (NTS) {
        const u32x4 x = {v[j].x, v[j].y, v[j].z, v[j].w};
        __builtin_nontemporal_store(x, (u32x4*)(dst + r * 128 + sl * 16));
      } else {
        *(uint4*)(dst + r * 128 + sl * 16) = v[j];
      }
    }
  }
}

__global__ void k_fill32(float* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = (float)(h >> 8) * (1.0f / 16777216.0f);
  }
}

__global__ void k_mismatch(const uint32_t* a, const uint32_t* b, int64_t n, unsigned long long* out) {
  unsigned long long c = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  atomicAdd(out, c);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  const int64_t N = argc > 2 ? atoll(argv[2]) : 40000, Cc = 5000, nb = N / Cc;
  const bool obf = argc > 3 && atoi(argv[3]) == 1;
  const bool f32in = argc > 4 && (atoi(argv[4]) == 3 || atoi(argv[4]) == 8);
  const int32_t in_code = f32in ? CUBED_F32 : CUBED_BF16;
  const int64_t al = 32;  // the executor's slot alignment (storage.SLOT_ALIGN)
  const int64_t slot_in = (Cc * Cc * (f32in ? 4 : 2) + al - 1) / al * al;
  const int64_t slot_out = (Cc * Cc * (obf ? 2 : 4) + al - 1) / al * al;
  char *A, *B, *C0, *C1;
  CHECK(hipMalloc(&A, slot_in * nb * nb));
  CHECK(hipMalloc(&B, slot_in * nb * nb));
  CHECK(hipMalloc(&C0, slot_out * nb * nb));
  CHECK(hipMalloc(&C1, slot_out * nb * nb));
  if (f32in) {
    k_fill32<<<4096, 256>>>((float*)A, slot_in * nb * nb / 4, 12345u);
    k_fill32<<<4096, 256>>>((float*)B, slot_in * nb * nb / 4, 777u);
  } else {
    k_fill<<<4096, 256>>>((uint16_t*)A, slot_in * nb * nb / 2, 12345u);
    k_fill<<<4096, 256>>>((uint16_t*)B, slot_in * nb * nb / 2, 777u);
  }
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
  const int32_t out_code = obf ? CUBED_BF16 : CUBED_F32;
  const int64_t wsb = cubed_gemm_pack_bytes(tasks.data(), nb, nb, segs.data(), segs.size(), in_code, out_code);
  if (wsb <= 0) { printf("pack_bytes: %s\n", g_err); return 1; }
  char* ws;
  CHECK(hipMalloc(&ws, wsb));
  PackPlan pp;
  GemmGrid gg;
  if (pack_plan(tasks.data(), nb, nb, segs.data(), segs.size(), in_code, out_code, pp, gg)) return 1;
  // the library entry: pack + w4p GEMM into C0 (the reference result)
  if (cubed_gemm_chain_packed(tasks.data(), dt0, nb, nb, segs.data(), ds, segs.size(), in_code, out_code, ws, wsb,
                              nullptr)) { printf("packed: %s\n", g_err); return 1; }
  CHECK(hipDeviceSynchronize());
  const char* PA = ws;
  const char* PB = ws + pp.TM * pp.pstride;
  const dim3 grid((unsigned)(pp.TM * pp.TN));
  const double flop = 2.0 * N * N * N;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  unsigned long long* dcnt;
  CHECK(hipMalloc(&dcnt, 8));
  unsigned long long* st;
  CHECK(hipMalloc(&st, (size_t)grid.x * 8 * 2 * 8));
  typedef void (*kfn)(const cubed_gemm_chain_t*, const char*, const char*, PackPlan, GemmGrid, unsigned long long*);
  unsigned* rctr;
  CHECK(hipMalloc(&rctr, 8 * 128));
  bool sync = false;  // pass the round counters (zeroed per launch) instead of stamps
  auto run = [&](const char* name, kfn f, int threads, bool stamp, int mfma_cyc, bool check) {
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipMemset(C1, 0, slot_out * nb * nb));
      CHECK(hipMemset(rctr, 0, 8 * 128));
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(f, grid, dim3(threads), 0, 0, dt1, PA, PB, pp, gg,
                         sync ? (unsigned long long*)rctr : stamp ? st : nullptr);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    printf("%-46s best %9.3f ms %7.1f TF", name, best, flop / best / 1e9);
    if (stamp) {
      const int nw = threads / 64;
      std::vector<unsigned long long> h((size_t)grid.x * nw * 2);
      CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
      double cyc = 0, units = 0;
      for (size_t i = 0; i < h.size(); i += 2) {
        cyc += (double)h[i];
        units += (double)h[i + 1];
      }
      // cycles per MFMA of ONE wave (w4p: 32 per step of 32x32x16; 8p: 16 per
      // phase of 16x16x32) and the clock from the mean wave's loop time
      const double per = mfma_cyc == 32 ? 32.0 : 16.0;
      printf("  loop %6.2f cyc per wave MFMA (ideal 32)  clock ~%.2f GHz", cyc / (units * per),
             (cyc / (h.size() / 2)) * ((double)grid.x / 256.0) / (best * 1e-3) / 1e9);
    }
    printf("\n");
    if (check) {
      CHECK(hipMemset(dcnt, 0, 8));
      k_mismatch<<<4096, 256>>>((const uint32_t*)C0, (const uint32_t*)C1, slot_out * nb * nb / 4, dcnt);
      unsigned long long c;
      CHECK(hipMemcpy(&c, dcnt, 8, hipMemcpyDeviceToHost));
      printf("   words differing from the library result: %llu of %lld\n", c, (long long)(slot_out * nb * nb / 4));
    }
    fflush(stdout);
  };
  printf("# N %lld chunk %lld, %s out, TM %lld TN %lld KTL %lld\n", (long long)N, (long long)Cc, obf ? "bf16" : "f32",
         (long long)pp.TM, (long long)pp.TN, (long long)pp.KTL);
  kfn w4p = obf ? (kfn)k_gemm_bf16_w4p<true> : (kfn)k_gemm_bf16_w4p<false>;
  kfn w4ps = obf ? (kfn)k_gemm_bf16_w4p<true, true> : (kfn)k_gemm_bf16_w4p<false, true>;
  kfn e8 = obf ? (kfn)k_gemm_bf16_8p<true> : (kfn)k_gemm_bf16_8p<false>;
  kfn e8s = obf ? (kfn)k_gemm_bf16_8p<true, true> : (kfn)k_gemm_bf16_8p<false, true>;
  const int arms = argc > 4 ? atoi(argv[4]) : 0;
  if (f32in) {  // f32 inputs: the library's one-wave w4p kernel (the two-wave f32 form,
    // gemm_f32_8p.h, lost: 943-959 ms vs 876; commit e0bc44c, profiles/r06_gemm_f32_8p.log)
    if (arms == 8) {  // tile rounds aligned per XCD (round_wait / round_done)
      run("f32 w4p (library)", (kfn)k_gemm_f32_w4p<false>, 256, false, 32, true);
      sync = true;
      run("f32 w4p rounds aligned", (kfn)k_gemm_f32_w4p<false, true, true>, 256, false, 32, true);
      sync = false;
      run("f32 w4p (library)", (kfn)k_gemm_f32_w4p<false>, 256, false, 32, false);
      sync = true;
      run("f32 w4p rounds aligned", (kfn)k_gemm_f32_w4p<false, true, true>, 256, false, 32, false);
      sync = false;
      return 0;
    }
    run("f32 w4p (lockstep XCD order)", (kfn)k_gemm_f32_w4p<false>, 256, false, 32, true);
    run("f32 w4p (contiguous XCD ranges)", (kfn)k_gemm_f32_w4p<false, false>, 256, false, 32, true);
    run("f32 w4p (lockstep XCD order)", (kfn)k_gemm_f32_w4p<false>, 256, false, 32, false);
    run("f32 w4p (contiguous XCD ranges)", (kfn)k_gemm_f32_w4p<false, false>, 256, false, 32, false);
    return 0;
  }
  {  // the library's packs, timed alone
    const int64_t na = pp.TM * pp.KTL, nbk = pp.TN * pp.KTL;
    const dim3 ga((unsigned)(na < 16384 ? na : 16384)), gb((unsigned)(nbk < 16384 ? nbk : 16384));
    char* PAw = ws;
    char* PBw = ws + pp.TM * pp.pstride;
    for (int r = 0; r < 3; ++r) {
      float ma, mb;
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_pack_a, ga, dim3(256), 0, 0, dt0, ds, pp, PAw);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ma, e0, e1));
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_pack_bt, gb, dim3(256), 0, 0, dt0, ds, pp, PBw);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&mb, e0, e1));
      const double bytes = (double)pp.TM * pp.pstride;  // written (read ~ the same)
      printf("pack A %.3f ms (%.0f GB/s moved)  pack B^T %.3f ms (%.0f GB/s moved)\n", ma, 2 * bytes / ma / 1e6, mb,
             2 * bytes / mb / 1e6);
    }
    char* PA2;
    CHECK(hipMalloc(&PA2, pp.TM * pp.pstride));
    typedef void (*pfn)(const cubed_gemm_chain_t*, const cubed_gemm_seg_t*, PackPlan, char*);
    const struct { const char* name; pfn f; int grid; } pv[] = {
        {"pack A, 8 loads in flight (nt loads)", k_pack_a8<true, false>, 16384},
        {"pack A, 8 loads in flight (plain)", k_pack_a8<false, false>, 16384},
        {"pack A, 8 loads in flight (plain, nt stores)", k_pack_a8<false, true>, 16384},
        {"pack A, 8 loads in flight (plain), grid 4096", k_pack_a8<false, false>, 4096},
        {"pack A, library, grid 4096", k_pack_a, 4096},
        {"pack A, library, grid 65536", k_pack_a, 65536},
    };
    for (const auto& v : pv)
      for (int r = 0; r < 3; ++r) {
        float ma;
        const dim3 g((unsigned)(na < v.grid ? na : v.grid));
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(v.f, g, dim3(256), 0, 0, dt0, ds, pp, PA2);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ma, e0, e1));
        printf("%-48s %.3f ms (%.0f GB/s moved)\n", v.name, ma, 2.0 * pp.TM * pp.pstride / ma / 1e6);
      }
    CHECK(hipMemset(dcnt, 0, 8));
    k_mismatch<<<4096, 256>>>((const uint32_t*)PAw, (const uint32_t*)PA2, pp.TM * pp.pstride / 4, dcnt);
    unsigned long long c;
    CHECK(hipMemcpy(&c, dcnt, 8, hipMemcpyDeviceToHost));
    printf("   words differing from the library pack: %llu\n", c);
    CHECK(hipFree(PA2));
  }
  run("w4p (library, one wave per SIMD)", w4p, 256, false, 32, true);
  run("8p  (two waves per SIMD, library form)", e8, 512, false, 16, true);
  if (arms == 0) {
    run("w4p stamped", w4ps, 256, true, 32, false);
    run("8p  stamped", e8s, 512, true, 16, false);
    run("w4p (again)", w4p, 256, false, 32, false);
    run("8p  (again)", e8, 512, false, 16, true);
    return 0;
  }
  if (arms == 4) {  // packing on a second stream while the 8p GEMM runs (into a separate image)
    char* ws2;
    CHECK(hipMalloc(&ws2, wsb));
    hipStream_t s2;
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t p0, p1, g1;
    CHECK(hipEventCreate(&p0));
    CHECK(hipEventCreate(&p1));
    CHECK(hipEventCreate(&g1));
    const int64_t na = pp.TM * pp.KTL, nbk = pp.TN * pp.KTL;
    kfn f = obf ? (kfn)k_gemm_bf16_8p<true> : (kfn)k_gemm_bf16_8p<false>;
    for (int pg : {16384, 2048, 512, 256}) {
      const dim3 ga((unsigned)(na < pg ? na : pg)), gb((unsigned)(nbk < pg ? nbk : pg));
      for (int order = 0; order < 2; ++order)
        for (int r = 0; r < 3; ++r) {
          CHECK(hipDeviceSynchronize());
          CHECK(hipEventRecord(e0, 0));
          CHECK(hipStreamWaitEvent(s2, e0, 0));
          if (order == 1) hipLaunchKernelGGL(f, grid, dim3(512), 0, 0, dt1, PA, PB, pp, gg, nullptr);
          CHECK(hipEventRecord(p0, s2));
          hipLaunchKernelGGL(k_pack_a, ga, dim3(256), 0, s2, dt0, ds, pp, ws2);
          hipLaunchKernelGGL(k_pack_bt, gb, dim3(256), 0, s2, dt0, ds, pp, ws2 + pp.TM * pp.pstride);
          CHECK(hipEventRecord(p1, s2));
          if (order == 0) hipLaunchKernelGGL(f, grid, dim3(512), 0, 0, dt1, PA, PB, pp, gg, nullptr);
          CHECK(hipEventRecord(g1, 0));
          CHECK(hipDeviceSynchronize());
          float mp, mg, mpp;
          CHECK(hipEventElapsedTime(&mp, e0, p1));
          CHECK(hipEventElapsedTime(&mpp, p0, p1));
          CHECK(hipEventElapsedTime(&mg, e0, g1));
          printf("concurrent pack grid %5d %s: packs done at %8.3f ms (own span %8.3f)  GEMM done at %8.3f ms\n", pg,
                 order ? "GEMM first" : "pack first", mp, mpp, mg);
          fflush(stdout);
        }
    }
    run("8p alone", f, 512, false, 16, false);
    return 0;
  }
#define ARM(NAME, V, G) run(NAME, obf ? (kfn)k_gemm_bf16_8p<true, false, V, G> : (kfn)k_gemm_bf16_8p<false, false, V, G>, 512, false, 16, true)
  if (arms == 7) {  // tile rounds aligned per XCD (round_wait / round_done)
    sync = true;
    ARM("8p rounds aligned", 512, 4);
    sync = false;
    run("8p  (library)", e8, 512, false, 16, false);
    sync = true;
    ARM("8p rounds aligned", 512, 4);
    sync = false;
    run("8p  (library)", e8, 512, false, 16, false);
    return 0;
  }
  if (arms == 10) {  // round alignment with slack (a round starts with 4 / 8 of the last unfinished)
    sync = true;
    ARM("8p rounds aligned", 512, 4);
    ARM("8p rounds aligned, slack 4", 512 | 1024, 4);
    ARM("8p rounds aligned, slack 8", 512 | 2048, 4);
    ARM("8p rounds aligned", 512, 4);
    ARM("8p rounds aligned, slack 4", 512 | 1024, 4);
    ARM("8p rounds aligned, slack 8", 512 | 2048, 4);
    sync = false;
    return 0;
  }
  if (arms == 5) {  // tile orders (the library form: xcd_lockstep, GM 4)
    ARM("8p contiguous XCD ranges GM 4 (round 5 order)", 64, 4);
    ARM("8p lockstep, contiguous tail", 128, 4);
    ARM("8p contiguous XCD ranges GM 4 (round 5 order)", 64, 4);
    ARM("8p lockstep, contiguous tail", 128, 4);
  } else if (arms == 2) {
    ARM("8p ABL no staging", 8, 4);
    ARM("8p ABL L2-resident staging", 16, 4);
    ARM("8p ABL no fragment reads", 32, 4);
    ARM("8p ABL neither staging nor reads", 40, 4);
  } else {
    ARM("8p VAR 1 (staging before the reads)", 1, 4);
    ARM("8p VAR 2 (setprio around MFMA clusters)", 2, 4);
    ARM("8p VAR 4 (group 1 static priority)", 4, 4);
    ARM("8p GM 8", 0, 8);
  }
  run("8p  (again)", e8, 512, false, 16, false);
  run("w4p (again)", w4p, 256, false, 32, false);
  return 0;
}
