// stream.hip -- streaming fast path of the fused chunk kernels (gfx950).
//
// Covers the hot shape of Cubed's reduction path: after canonicalisation a
// task is [one reduced dim] x [one packed kept dim] (or just the kept dim for
// a map), and every leaf is an array chunk stored in the VM's own dtype --
// e.g. the per-chunk `u * v -> _mean_func` of quad-means, fused with its
// merge/combine rounds into one pass over the time axis (chains.py).
// The host sets CUBED_MODE_STREAM only after checking that geometry
// (lowering.py:_stream_ok), so the kernel needs no per-element dtype or leaf
// kind dispatch and no odometer.
//
// Each thread owns 4 consecutive kept elements (16-byte loads for f32) and
// walks its slice of the reduced dim U rows at a time: the U x NL loads of a
// step are all issued before the first is consumed, so every wave keeps
// U*NL*1 KiB (f32) in flight -- enough bytes per CU to cover HBM latency at
// the occupancy this kernel gets.  Loads are non-temporal: a chunk row is
// read exactly once.  The accumulation order along the reduced dim is
// sequential per kept element (numpy's outer-axis add.reduce order), split
// ranges combine in order in k_finalize.  COUNT fields are the trip count,
// added once instead of per element.
#include "fused_common.h"

namespace cubed {

CUBED_DEV void ld4(float (&o)[4], const CUBED_G float* p) {
  const f32x4 v = __builtin_nontemporal_load((const CUBED_G f32x4*)p);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
CUBED_DEV void ld4(double (&o)[4], const CUBED_G double* p) {
  const f64x2 a = __builtin_nontemporal_load((const CUBED_G f64x2*)p);
  const f64x2 b = __builtin_nontemporal_load((const CUBED_G f64x2*)(p + 2));
  o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}
CUBED_DEV void ld4(int64_t (&o)[4], const CUBED_G int64_t* p) {
  const i64x2 a = __builtin_nontemporal_load((const CUBED_G i64x2*)p);
  const i64x2 b = __builtin_nontemporal_load((const CUBED_G i64x2*)(p + 2));
  o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}

template <int NL, typename V>
CUBED_DEV void set_leaves(Regs<V, 4>& regs, const V (&b)[NL][4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    regs.r0[j] = b[0][j];
    if constexpr (NL > 1) regs.r1[j] = b[1][j];
    if constexpr (NL > 2) regs.r2[j] = b[2][j];
    if constexpr (NL > 3) regs.r3[j] = b[3][j];
  }
}

template <typename V>
CUBED_DEV void accumulate_nocount(Acc (&acc)[CUBED_MAX_FIELDS][4], Regs<V, 4>& regs,
                                  const cubed_program_t& P) {
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f) {
    if (f < P.nfields && P.field_rop[f] != CUBED_R_COUNT) {
      V src[4];
      fetch(regs, P.field_src[f], src);
      const int rop = P.field_rop[f], ai = P.field_acc[f];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc_add<V>(acc[f][j], rop, ai, src[j]);
    }
  }
}

template <typename V, int NL, int U>
__global__ __launch_bounds__(kBlock) void k_stream(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t bpt, int32_t nsplit, Acc* __restrict__ ws, int64_t max_kept) {
  const cubed_program_t& P = *Pd;
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int64_t b = g % bpt;
  const int64_t rest = g / bpt;
  const int s = (int)(rest % nsplit);
  const int64_t t = rest / nsplit;
  if (t >= ntasks) return;
  const cubed_task_t* __restrict__ T = tasks + t;
  const int nr = P.nred;  // 0 (map) or 1
  const int64_t nk = T->extent[nr];
  const int64_t nrd = nr ? T->extent[0] : 1;
  const int64_t items = nk >> 2;
  const int64_t r0 = nrd * s / nsplit, r1 = nrd * (s + 1) / nsplit;

  const CUBED_G V* base[NL];
  int64_t rs[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    base[l] = (const CUBED_G V*)(uintptr_t)T->leaf_base[l];
    rs[l] = nr ? T->leaf_stride[l][0] : 0;
  }

  for (int64_t item = b * kBlock + threadIdx.x; item < items; item += bpt * kBlock) {
    const int64_t k = item * 4;
    int64_t ooff[CUBED_MAX_OUTS];
#pragma unroll
    for (int o = 0; o < CUBED_MAX_OUTS; ++o) ooff[o] = k;
    Regs<V, 4> regs;
    if (P.nfields == 0) {
      V buf[NL][4];
#pragma unroll
      for (int l = 0; l < NL; ++l) ld4(buf[l], base[l] + k);
      set_leaves<NL, V>(regs, buf);
      run_vm<V, 4>(regs, P.insns, P.ninsns, P);
#pragma unroll
      for (int o = 0; o < CUBED_MAX_OUTS; ++o) {
        if (o < P.nouts) {
          V X[4];
          fetch(regs, P.out_src[o], X);
          stv<V, 4>((char*)T->out_base[o], ooff[o], P.out_dtype[o], X);
        }
      }
      continue;
    }
    Acc acc[CUBED_MAX_FIELDS][4];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[f][j] = acc_init(P.field_rop[f], P.field_acc[f]);

    const CUBED_G V* p[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) p[l] = base[l] + k + r0 * rs[l];
    int64_t r = r0;
    for (; r + U <= r1; r += U) {
      V buf[U][NL][4];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int l = 0; l < NL; ++l) ld4(buf[u][l], p[l] + u * rs[l]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        set_leaves<NL, V>(regs, buf[u]);
        run_vm<V, 4>(regs, P.insns, P.ninsns, P);
        accumulate_nocount<V>(acc, regs, P);
      }
#pragma unroll
      for (int l = 0; l < NL; ++l) p[l] += U * rs[l];
    }
    for (; r < r1; ++r) {
      V buf[NL][4];
#pragma unroll
      for (int l = 0; l < NL; ++l) ld4(buf[l], p[l]);
      set_leaves<NL, V>(regs, buf);
      run_vm<V, 4>(regs, P.insns, P.ninsns, P);
      accumulate_nocount<V>(acc, regs, P);
#pragma unroll
      for (int l = 0; l < NL; ++l) p[l] += rs[l];
    }
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
      if (f < P.nfields && P.field_rop[f] == CUBED_R_COUNT)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[f][j].i += r1 - r0;

    if (nsplit == 1) {
      finish<4>(P, T, acc, ooff);
    } else {
      Acc* w = ws + ((int64_t)(s * ntasks + t) * max_kept + k) * P.nfields;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
          if (f < P.nfields) w[j * P.nfields + f] = acc[f][j];
    }
  }
}

template <typename V>
void launch_stream(const cubed_program_t& P, const cubed_program_t* dP, const LaunchPlan& L, const cubed_task_t* d_tasks,
                   int64_t ntasks, int64_t max_kept, Acc* ws, hipStream_t st) {
  constexpr int U = sizeof(V) == 4 ? 4 : 2;
  const dim3 grid = grid_of(L.blocks);
  switch (P.nleaves) {
    case 1: hipLaunchKernelGGL((k_stream<V, 1, U>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, L.nsplit, ws, max_kept); break;
    case 2: hipLaunchKernelGGL((k_stream<V, 2, U>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, L.nsplit, ws, max_kept); break;
    case 3: hipLaunchKernelGGL((k_stream<V, 3, U>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, L.nsplit, ws, max_kept); break;
    default: hipLaunchKernelGGL((k_stream<V, 4, U>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, L.nsplit, ws, max_kept); break;
  }
}

template void launch_stream<float>(const cubed_program_t&, const cubed_program_t*, const LaunchPlan&, const cubed_task_t*,
                                   int64_t, int64_t, Acc*, hipStream_t);
template void launch_stream<double>(const cubed_program_t&, const cubed_program_t*, const LaunchPlan&, const cubed_task_t*,
                                    int64_t, int64_t, Acc*, hipStream_t);
template void launch_stream<int64_t>(const cubed_program_t&, const cubed_program_t*, const LaunchPlan&, const cubed_task_t*,
                                     int64_t, int64_t, Acc*, hipStream_t);

}  // namespace cubed
