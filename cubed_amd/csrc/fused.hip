// fused.hip -- grouped launches of fused Cubed chunk programs on gfx950.
//
// One launch runs every task (output chunk) of one fused pipeline, i.e. the
// whole `for m in pipeline.mappable: apply_blockwise(m, config)` loop of the
// reference executor (runtime/executors/python.py:26-29 over
// primitive/blockwise.py:61-84), with the chunk function lowered to a
// cubed_program_t.  Three kernel shapes:
//
//   A (mode 0): reduced dims first.  A thread owns VEC consecutive kept
//      elements (coalesced along the innermost kept dim) and walks the
//      reduced dims sequentially -- the order numpy uses for an outer-axis
//      add.reduce, so outer-axis sums are bit-identical to the reference.
//      With nred == 0 this is the elementwise (map) kernel.
//   B (mode 1): reduced dims last (innermost dim reduced).  A workgroup owns
//      one kept element; lanes stride the reduced range (coalesced), then a
//      64-wide shuffle tree + LDS across the 4 waves.
//   split: when a launch would not fill 256 CUs, the reduced range is split
//      over workgroups that write partial accumulators to the workspace;
//      k_finalize combines them in split order and runs the epilogue.
#include "fused_common.h"
#include <stdio.h>
#include <string.h>

namespace cubed {

thread_local char g_err[512];
static void set_err(const char* m) { snprintf(g_err, sizeof(g_err), "%s", m); }

// Load leaf l (VEC elements) at element offset `off`; `inner` is the leaf's
// stride along the dim the VEC elements run on (0 = broadcast, 1 = packed).
template <typename V, int VEC>
CUBED_DEV void load_leaf(V (&o)[VEC], const cubed_program_t& P,
                         const cubed_task_t* T, int l, int64_t off,
                         int64_t inner) {
  const int kind = P.leaf_kind[l];
  if (kind == CUBED_LEAF_ARRAY) {
    const char* base = (const char*)T->leaf_base[l];
    const int dt = P.leaf_dtype[l];
    if (VEC == 1 || inner == 1) {
      ldv<V, VEC>(o, base, off, dt);
    } else if (inner == 0) {
      const V v = ld1<V>(base + off * dt_size(dt), dt);
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = v;
    } else {
      const int sz = dt_size(dt);
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = ld1<V>(base + (off + j * inner) * sz, dt);
    }
  } else if (kind == CUBED_LEAF_PHILOX) {
    if (VEC == 4 && inner == 1 && (off & 3) == 0) {
      const uint64_t b = (uint64_t)(off >> 2) + 1ull;
      P4 r = philox4x64_10(b, 0ull, T->key_lo, T->key_hi);
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = (V)u64_to_unit(r.x[j]);
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = (V)philox_at(T->key_lo, T->key_hi, off + j * inner);
    }
  } else if (kind == CUBED_LEAF_IOTA) {
    const int64_t b = T->leaf_base[l] + off;
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = (V)(b + j * inner);
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = (V)T->block_offset;
  }
}

template <typename V, int VEC>
CUBED_DEV void load_leaves(Regs<V, VEC>& regs, const cubed_program_t& P,
                           const cubed_task_t* T, const int64_t (&off)[CUBED_MAX_LEAVES],
                           const int64_t (&inner)[CUBED_MAX_LEAVES]) {
  const int nl = P.nleaves;
  if (nl > 0) load_leaf<V, VEC>(regs.r0, P, T, 0, off[0], inner[0]);
  if (nl > 1) load_leaf<V, VEC>(regs.r1, P, T, 1, off[1], inner[1]);
  if (nl > 2) load_leaf<V, VEC>(regs.r2, P, T, 2, off[2], inner[2]);
  if (nl > 3) load_leaf<V, VEC>(regs.r3, P, T, 3, off[3], inner[3]);
}

// ------------------------------------------------------------------ kernel A
template <typename V, int VEC>
__global__ __launch_bounds__(kBlock) void k_fused_a(
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
  const int nd = P.ndim, nr = P.nred;

  int64_t nk = 1, nrd = 1;
  for (int d = 0; d < nd; ++d) { if (d < nr) nrd *= T->extent[d]; else nk *= T->extent[d]; }
  const int64_t items = nk / VEC;
  // split range of the reduced index
  const int64_t r0 = nrd * s / nsplit, r1 = nrd * (s + 1) / nsplit;

  int64_t inner[CUBED_MAX_LEAVES];
#pragma unroll
  for (int l = 0; l < CUBED_MAX_LEAVES; ++l) inner[l] = T->leaf_stride[l][nd - 1];

  for (int64_t item = b * kBlock + threadIdx.x; item < items; item += bpt * kBlock) {
    int64_t loff[CUBED_MAX_LEAVES] = {0, 0, 0, 0};
    int64_t ooff[CUBED_MAX_OUTS] = {0, 0};
    int64_t k = item * VEC;
    const int64_t kflat = k;
#pragma unroll
    for (int d = CUBED_MAX_DIMS - 1; d >= 0; --d) {
      if (d < nd && d >= nr) {
        int64_t q, c;
        divmod64(k, T->extent[d], q, c);
        k = q;
#pragma unroll
        for (int l = 0; l < CUBED_MAX_LEAVES; ++l) loff[l] += c * T->leaf_stride[l][d];
#pragma unroll
        for (int o = 0; o < CUBED_MAX_OUTS; ++o) ooff[o] += c * T->out_stride[o][d];
      }
    }
    Regs<V, VEC> regs;
    if (P.nfields == 0) {
      load_leaves<V, VEC>(regs, P, T, loff, inner);
      run_vm<V, VEC>(regs, P.insns, P.ninsns, P);
#pragma unroll
      for (int o = 0; o < CUBED_MAX_OUTS; ++o) {
        if (o < P.nouts) {
          V X[VEC];
          fetch(regs, P.out_src[o], X);
          stv<V, VEC>((char*)T->out_base[o], ooff[o], P.out_dtype[o], X);
        }
      }
      continue;
    }
    Acc acc[CUBED_MAX_FIELDS][VEC];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[f][j] = acc_init(P.field_rop[f], P.field_acc[f]);

    // reduced coordinates of r0 (odometer over dims [0, nr))
    int64_t cr[CUBED_MAX_DIMS];
    int64_t roff[CUBED_MAX_LEAVES] = {0, 0, 0, 0};
    {
      int64_t rr = r0;
#pragma unroll
      for (int d = CUBED_MAX_DIMS - 1; d >= 0; --d) {
        cr[d] = 0;
        if (d < nr) {
          int64_t q, c;
          divmod64(rr, T->extent[d], q, c);
          rr = q; cr[d] = c;
#pragma unroll
          for (int l = 0; l < CUBED_MAX_LEAVES; ++l) roff[l] += c * T->leaf_stride[l][d];
        }
      }
    }
    for (int64_t r = r0; r < r1; ++r) {
      int64_t off[CUBED_MAX_LEAVES];
#pragma unroll
      for (int l = 0; l < CUBED_MAX_LEAVES; ++l) off[l] = loff[l] + roff[l];
      load_leaves<V, VEC>(regs, P, T, off, inner);
      run_vm<V, VEC>(regs, P.insns, P.ninsns, P);
      accumulate<V, VEC>(acc, regs, P);
      // advance the odometer
      bool carry = true;
#pragma unroll
      for (int d = CUBED_MAX_DIMS - 1; d >= 0; --d) {
        if (carry && d < nr) {
          cr[d] += 1;
#pragma unroll
          for (int l = 0; l < CUBED_MAX_LEAVES; ++l) roff[l] += T->leaf_stride[l][d];
          if (cr[d] == T->extent[d] && d > 0) {
            cr[d] = 0;
#pragma unroll
            for (int l = 0; l < CUBED_MAX_LEAVES; ++l) roff[l] -= T->extent[d] * T->leaf_stride[l][d];
          } else {
            carry = false;
          }
        }
      }
    }
    if (nsplit == 1) {
      finish<VEC>(P, T, acc, ooff);
    } else {
      Acc* w = ws + ((int64_t)(s * ntasks + t) * max_kept + kflat) * P.nfields;
#pragma unroll
      for (int j = 0; j < VEC; ++j)
#pragma unroll
        for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
          if (f < P.nfields) w[j * P.nfields + f] = acc[f][j];
    }
  }
}

// ------------------------------------------------------------------ kernel B
template <typename V, int VEC>
__global__ __launch_bounds__(kBlock) void k_fused_b(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, int32_t nsplit, Acc* __restrict__ ws) {
  const cubed_program_t& P = *Pd;
  __shared__ Acc red[kBlock / 64][CUBED_MAX_FIELDS];
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int s = (int)(g % nsplit);
  const int64_t rest = g / nsplit;
  const int64_t k = rest % max_kept;
  const int64_t t = rest / max_kept;
  if (t >= ntasks) return;
  const cubed_task_t* __restrict__ T = tasks + t;
  const int nd = P.ndim, nr = P.nred, nkd = nd - nr;
  int64_t nk = 1, nrd = 1;
  for (int d = 0; d < nd; ++d) { if (d < nkd) nk *= T->extent[d]; else nrd *= T->extent[d]; }
  if (k >= nk) return;

  int64_t loff[CUBED_MAX_LEAVES] = {0, 0, 0, 0};
  int64_t ooff[CUBED_MAX_OUTS] = {0, 0};
  {
    int64_t kk = k;
#pragma unroll
    for (int d = CUBED_MAX_DIMS - 1; d >= 0; --d) {
      if (d < nkd) {
        int64_t q, c;
        divmod64(kk, T->extent[d], q, c);
        kk = q;
#pragma unroll
        for (int l = 0; l < CUBED_MAX_LEAVES; ++l) loff[l] += c * T->leaf_stride[l][d];
#pragma unroll
        for (int o = 0; o < CUBED_MAX_OUTS; ++o) ooff[o] += c * T->out_stride[o][d];
      }
    }
  }
  int64_t inner[CUBED_MAX_LEAVES];
#pragma unroll
  for (int l = 0; l < CUBED_MAX_LEAVES; ++l) inner[l] = T->leaf_stride[l][nd - 1];

  // split range, aligned to VEC (the innermost reduced extent is a multiple of VEC)
  int64_t r0 = nrd * s / nsplit, r1 = nrd * (s + 1) / nsplit;
  r0 -= r0 % VEC; r1 -= r1 % VEC;
  if (s == nsplit - 1) r1 = nrd;

  Acc acc[CUBED_MAX_FIELDS][VEC];
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[f][j] = acc_init(P.field_rop[f], P.field_acc[f]);

  Regs<V, VEC> regs;
  for (int64_t p = r0 + (int64_t)threadIdx.x * VEC; p < r1; p += (int64_t)kBlock * VEC) {
    int64_t off[CUBED_MAX_LEAVES];
#pragma unroll
    for (int l = 0; l < CUBED_MAX_LEAVES; ++l) off[l] = loff[l];
    int64_t rr = p;
#pragma unroll
    for (int d = CUBED_MAX_DIMS - 1; d >= 0; --d) {
      if (d < nd && d >= nkd) {
        int64_t q, c;
        if (d == nkd) { q = 0; c = rr; } else divmod64(rr, T->extent[d], q, c);
        rr = q;
#pragma unroll
        for (int l = 0; l < CUBED_MAX_LEAVES; ++l) off[l] += c * T->leaf_stride[l][d];
      }
    }
    load_leaves<V, VEC>(regs, P, T, off, inner);
    run_vm<V, VEC>(regs, P.insns, P.ninsns, P);
    accumulate<V, VEC>(acc, regs, P);
  }
  // combine VEC lanes, then the 64-wide wave, then the 4 waves
  Acc a[CUBED_MAX_FIELDS];
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f) {
    a[f] = acc[f][0];
#pragma unroll
    for (int j = 1; j < VEC; ++j) a[f] = acc_combine(a[f], acc[f][j], P.field_rop[f], P.field_acc[f]);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
      a[f] = acc_combine(a[f], shfl_xor_acc(a[f], m), P.field_rop[f], P.field_acc[f]);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) red[wave][f] = a[f];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc fin[CUBED_MAX_FIELDS][1];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) {
      Acc x = red[0][f];
#pragma unroll
      for (int w = 1; w < kBlock / 64; ++w) x = acc_combine(x, red[w][f], P.field_rop[f], P.field_acc[f]);
      fin[f][0] = x;
    }
    if (nsplit == 1) {
      finish<1>(P, T, fin, ooff);
    } else {
      Acc* w = ws + ((int64_t)(s * ntasks + t) * max_kept + k) * P.nfields;
#pragma unroll
      for (int f = 0; f < CUBED_MAX_FIELDS; ++f) if (f < P.nfields) w[f] = fin[f][0];
    }
  }
}

// ---------------------------------------------------------------- finalize
// Combine nsplit partial accumulators (in split order) for every kept
// element and run the epilogue.  kept dims are [kd0, kd1) of the task.
__global__ __launch_bounds__(kBlock) void k_finalize(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, int32_t nsplit, const Acc* __restrict__ ws, int kd0, int kd1) {
  const cubed_program_t& P = *Pd;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t t = i / max_kept, k = i % max_kept;
  if (t >= ntasks) return;
  const cubed_task_t* __restrict__ T = tasks + t;
  int64_t nk = 1;
  for (int d = kd0; d < kd1; ++d) nk *= T->extent[d];
  if (k >= nk) return;
  int64_t ooff[CUBED_MAX_OUTS] = {0, 0};
  int64_t kk = k;
  for (int d = kd1 - 1; d >= kd0; --d) {
    int64_t q, c;
    divmod64(kk, T->extent[d], q, c);
    kk = q;
    for (int o = 0; o < CUBED_MAX_OUTS; ++o) ooff[o] += c * T->out_stride[o][d];
  }
  Acc fin[CUBED_MAX_FIELDS][1];
  for (int f = 0; f < P.nfields && f < CUBED_MAX_FIELDS; ++f) {
    Acc x = ws[(t * max_kept + k) * P.nfields + f];
    for (int s = 1; s < nsplit; ++s)
      x = acc_combine(x, ws[(((int64_t)s * ntasks + t) * max_kept + k) * P.nfields + f],
                      P.field_rop[f], P.field_acc[f]);
    fin[f][0] = x;
  }
  finish<1>(P, T, fin, ooff);
}

static LaunchPlan plan_launch(const cubed_program_t* P, int64_t ntasks, int64_t max_kept,
                              int64_t max_red) {
  LaunchPlan L;
  L.kernel = P->mode & 3;
  L.vec = (P->mode & 4) ? 4 : 1;
  L.nsplit = 1;
  L.bpt = 1;
  const int64_t target = 2048;  // ~8 workgroups per CU
  if (L.kernel == 0) {
    const int64_t items = (max_kept + L.vec - 1) / L.vec;
    L.bpt = (items + kBlock - 1) / kBlock;
    if (L.bpt < 1) L.bpt = 1;
    if (L.bpt > 65536) L.bpt = 65536;
    const int64_t base = ntasks * L.bpt;
    if (P->nfields > 0 && base < target && max_red >= 64) {
      int64_t s = (target + base - 1) / base;
      if (s > max_red / 16) s = max_red / 16;
      if (s > 4096) s = 4096;
      if (s > 1) L.nsplit = (int32_t)s;
    }
    L.blocks = ntasks * L.nsplit * L.bpt;
  } else {
    const int64_t base = ntasks * max_kept;
    if (base < target && max_red >= 8192) {
      int64_t s = (target + base - 1) / base;
      if (s > max_red / 4096) s = max_red / 4096;
      if (s > 4096) s = 4096;
      if (s > 1) L.nsplit = (int32_t)s;
    }
    L.blocks = ntasks * max_kept * L.nsplit;
  }
  L.ws_bytes = L.nsplit > 1 ? (int64_t)L.nsplit * ntasks * max_kept * P->nfields * (int64_t)sizeof(Acc) : 0;
  return L;
}

dim3 grid_of(int64_t blocks) {
  if (blocks <= 0x7fffffff) return dim3((unsigned)blocks, 1, 1);
  const int64_t y = (blocks + 0x7fffffff - 1) / 0x7fffffff;
  return dim3(0x7fffffffu, (unsigned)y, 1);
}

template <typename V>
static void launch_fused(const cubed_program_t& P, const cubed_program_t* dP, const LaunchPlan& L, const cubed_task_t* d_tasks,
                         int64_t ntasks, int64_t max_kept, Acc* ws, hipStream_t st) {
  const dim3 grid = grid_of(L.blocks);
  if (P.mode & CUBED_MODE_STREAM) {
    launch_stream<V>(P, dP, L, d_tasks, ntasks, max_kept, ws, st);
  } else if (L.kernel == 0) {
    if (L.vec == 4)
      hipLaunchKernelGGL((k_fused_a<V, 4>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, L.nsplit, ws, max_kept);
    else
      hipLaunchKernelGGL((k_fused_a<V, 1>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, L.nsplit, ws, max_kept);
  } else {
    if (L.vec == 4)
      hipLaunchKernelGGL((k_fused_b<V, 4>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, max_kept, L.nsplit, ws);
    else
      hipLaunchKernelGGL((k_fused_b<V, 1>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, max_kept, L.nsplit, ws);
  }
}

}  // namespace cubed

using namespace cubed;

extern "C" int64_t cubed_fused_workspace_bytes(const cubed_program_t* prog, int64_t ntasks,
                                               int64_t max_kept, int64_t max_red) {
  if (!prog || ntasks <= 0) return 0;
  return plan_launch(prog, ntasks, max_kept, max_red).ws_bytes;
}

extern "C" int cubed_fused_chunks(const cubed_program_t* prog, const cubed_program_t* d_prog,
                                  const cubed_task_t* d_tasks,
                                  int64_t ntasks, int64_t max_kept, int64_t max_red,
                                  void* d_workspace, int64_t workspace_bytes, void* stream) {
  if (!prog || !d_prog || (!d_tasks && ntasks > 0)) { set_err("cubed_fused_chunks: null argument"); return CUBED_E_ARG; }
  if (ntasks == 0) return 0;
  const cubed_program_t& P = *prog;
  if (P.ndim < 1 || P.ndim > CUBED_MAX_DIMS || P.nred < 0 || P.nred > P.ndim ||
      P.nleaves < 0 || P.nleaves > CUBED_MAX_LEAVES || P.nfields < 0 ||
      P.nfields > CUBED_MAX_FIELDS || P.nouts < 1 || P.nouts > CUBED_MAX_OUTS ||
      P.ninsns < 0 || P.ninsns > CUBED_MAX_INSNS || P.nepi > CUBED_MAX_EPI) {
    set_err("cubed_fused_chunks: program header out of range");
    return CUBED_E_ARG;
  }
  if ((P.mode & 3) == 1 && P.nfields == 0) { set_err("cubed_fused_chunks: kernel B needs a reduction"); return CUBED_E_ARG; }
  if ((P.mode & CUBED_MODE_STREAM) &&
      ((P.mode & 3) != 0 || !(P.mode & 4) || P.nred > 1 || P.ndim != P.nred + 1 || P.nleaves < 1)) {
    set_err("cubed_fused_chunks: stream mode needs kernel A, VEC=4, one kept dim and <= 1 reduced dim");
    return CUBED_E_LAYOUT;
  }
  if (P.mode & CUBED_MODE_STREAM) {
    const int want = P.vtype == CUBED_V_F32 ? CUBED_F32 : P.vtype == CUBED_V_F64 ? CUBED_F64 : CUBED_I64;
    for (int l = 0; l < P.nleaves; ++l)
      if (P.leaf_kind[l] != CUBED_LEAF_ARRAY || P.leaf_dtype[l] != want) {
        set_err("cubed_fused_chunks: stream mode needs array leaves in the vtype's dtype");
        return CUBED_E_LAYOUT;
      }
  }
  if (max_kept <= 0 || max_red <= 0) { set_err("cubed_fused_chunks: empty task bounds"); return CUBED_E_ARG; }
  const LaunchPlan L = plan_launch(&P, ntasks, max_kept, max_red);
  if (L.ws_bytes > 0 && (d_workspace == nullptr || workspace_bytes < L.ws_bytes)) {
    set_err("cubed_fused_chunks: workspace too small");
    return CUBED_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  Acc* ws = (Acc*)d_workspace;
  switch (P.vtype) {
    case CUBED_V_F32: launch_fused<float>(P, d_prog, L, d_tasks, ntasks, max_kept, ws, st); break;
    case CUBED_V_F64: launch_fused<double>(P, d_prog, L, d_tasks, ntasks, max_kept, ws, st); break;
    case CUBED_V_I64: launch_fused<int64_t>(P, d_prog, L, d_tasks, ntasks, max_kept, ws, st); break;
    default: set_err("cubed_fused_chunks: bad vtype"); return CUBED_E_DTYPE;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err(hipGetErrorString(e)); return (int)e; }
  if (L.nsplit > 1) {
    const int kd0 = (L.kernel == 0) ? P.nred : 0;
    const int kd1 = (L.kernel == 0) ? P.ndim : P.ndim - P.nred;
    const int64_t n = ntasks * max_kept;
    hipLaunchKernelGGL(k_finalize, grid_of((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st,
                       d_prog, d_tasks, ntasks, max_kept, L.nsplit, (const Acc*)ws, kd0, kd1);
    e = hipGetLastError();
    if (e != hipSuccess) { set_err(hipGetErrorString(e)); return (int)e; }
  }
  return 0;
}

extern "C" const char* cubed_last_error(void) { return g_err; }
extern "C" int cubed_abi_version(void) { return CUBED_ABI_VERSION; }
extern "C" int cubed_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
