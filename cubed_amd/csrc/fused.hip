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
#include "kernels.h"
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

namespace cubed {

thread_local char g_err[512];
void set_error(const char* m) { snprintf(g_err, sizeof(g_err), "%s", m); }
static void set_err(const char* m) { set_error(m); }

// ------------------------------------------------------------------ kernel A
template <typename V, int VEC>
__global__ __launch_bounds__(kBlock) void k_fused_a(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t bpt, int32_t nsplit, Acc* __restrict__ ws, int64_t max_kept) {
  fused_a_body<V, VEC>(*Pd, tasks, ntasks, bpt, nsplit, ws, max_kept);
}

// ------------------------------------------------------------------ kernel B
template <typename V, int VEC>
__global__ __launch_bounds__(kBlock) void k_fused_b(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, int32_t nsplit, Acc* __restrict__ ws) {
  fused_b_body<V, VEC>(*Pd, tasks, ntasks, max_kept, nsplit, ws);
}

// ---------------------------------------------------------------- finalize
// Combine nsplit partial accumulators (in split order) for every kept
// element and run the epilogue.  kept dims are [kd0, kd1) of the task.
__global__ __launch_bounds__(kBlock) void k_finalize(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, int32_t nsplit, const Acc* __restrict__ ws, int kd0, int kd1) {
  finalize_body(*Pd, tasks, ntasks, max_kept, nsplit, ws, kd0, kd1);
}

// Partials mode: combine splits into SoA per-field partials (kernels.h).
__global__ __launch_bounds__(kBlock) void k_collect(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, int32_t nsplit, const Acc* __restrict__ ws, Acc* __restrict__ soa, int kd0, int kd1) {
  collect_body(*Pd, tasks, ntasks, max_kept, nsplit, ws, soa, kd0, kd1);
}

__global__ __launch_bounds__(kBlock) void k_finish_soa(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, int kd0, int kd1) {
  finish_soa_body(*Pd, tasks, ntasks, max_kept, soa, kd0, kd1);
}

__global__ __launch_bounds__(kBlock) void k_finish_groups(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, const int64_t* __restrict__ gs, int64_t ngroups,
    int kd0, int kd1) {
  finish_groups_body(*Pd, tasks, ntasks, max_kept, soa, gs, ngroups, kd0, kd1);
}

__global__ __launch_bounds__(kBlock) void k_combine_groups(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, const int64_t* __restrict__ gs, int64_t ngroups,
    int64_t max_kept_out, Acc* __restrict__ out, int kd0, int kd1) {
  combine_groups_body(*Pd, tasks, ntasks, max_kept, soa, gs, ngroups, max_kept_out, out, kd0, kd1);
}

__global__ __launch_bounds__(kBlock) void k_fold_groups(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, const int64_t* __restrict__ gs, int64_t ngroups,
    Acc* __restrict__ out, int kd0, int kd1, const cubed_program_t* __restrict__ Pfin,
    const cubed_task_t* __restrict__ fin_tasks) {
  fold_groups_body<false>(*Pd, tasks, ntasks, max_kept, soa, gs, ngroups, out, kd0, kd1, Pfin, fin_tasks);
}

__global__ __launch_bounds__(kBlock) void k_fold_groups_split(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, const int64_t* __restrict__ gs, int64_t ngroups,
    int64_t nsplit, Acc* __restrict__ out_split, Acc* __restrict__ out, int kd0, int kd1,
    const cubed_program_t* __restrict__ Pfin, const cubed_task_t* __restrict__ fin_tasks) {
  fold_groups_split_body<false>(*Pd, tasks, ntasks, max_kept, soa, gs, ngroups, nsplit, out_split, out, kd0, kd1,
                                Pfin, fin_tasks);
}

__global__ __launch_bounds__(kBlock) void k_combine_parts(
    const cubed_program_t* __restrict__ Pd, const Acc* __restrict__ parts, int32_t nparts, int64_t n,
    Acc* __restrict__ out) {
  combine_parts_body(*Pd, parts, nparts, n, out);
}

void kept_dims(const cubed_program_t& P, int& kd0, int& kd1) {
  const bool a = (P.mode & 3) == 0;
  kd0 = a ? P.nred : 0;
  kd1 = a ? P.ndim : P.ndim - P.nred;
}

int launch_collect(const cubed_program_t& P, const cubed_program_t* dP, const LaunchPlan& L,
                   const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept, Acc* ws_base,
                   hipStream_t st) {
  int kd0, kd1;
  kept_dims(P, kd0, kd1);
  const int64_t n = ntasks * max_kept;
  hipLaunchKernelGGL(k_collect, grid_of((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, dP, d_tasks,
                     ntasks, max_kept, L.nsplit, (const Acc*)(ws_base + L.soa_elems), ws_base, kd0, kd1);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
  return 0;
}

// Split factor for a reduction whose un-split grid has `base` workgroups:
// enough workgroups to fill the chip (`resident` = 256 CUs x 8 resident
// 256-thread groups at the specialised kernels' occupancy), rounded so the
// last round of workgroups is nearly full (a 1.5-round grid idles half the
// chip for its last third).  Deterministic in its arguments, so the
// workspace size the host queries matches the launch.
static int64_t choose_split(int64_t base, int64_t max_split, int64_t resident) {
  if (max_split < 2) return 1;
  if (max_split > 4096) max_split = 4096;
  int64_t best = 1;
  double best_eff = 0.0;
  for (int64_t s = 1; s <= max_split && s <= 64; ++s) {
    const int64_t blocks = base * s;
    if (blocks < (resident * 9) / 10) continue;
    const int64_t rounds = (blocks + resident - 1) / resident;
    const double eff = (double)blocks / (double)(rounds * resident);
    if (eff >= 0.9) return s;
    if (eff > best_eff) { best_eff = eff; best = s; }
  }
  if (best_eff == 0.0) {
    // few, long tasks (e.g. one output block): as many splits as one round
    // of resident workgroups holds -- rounding up would start a second round
    // for a handful of workgroups and double the kernel's time
    int64_t s = resident / base;
    if (s < 1) s = 1;
    return s > max_split ? max_split : s;
  }
  return best;
}

// Kept VEC groups per thread of a streaming JIT kernel: the host picks W
// (lowering.py _stream_groups) and records it in the mode bits, so the JIT
// cache key, the kernel and the grid agree.
int stream_groups(const cubed_program_t& P) {
  return (P.mode & CUBED_MODE_STREAM_W4) ? 4 : (P.mode & CUBED_MODE_STREAM_W2) ? 2 : 1;
}

// Streaming launches: a grid that fills the CUs without splitting the
// reduced dim runs unsplit (a time split costs more than the occupancy it
// adds: config 2 W = 2 unsplit 6.81 TB/s vs 6.02 for the round-2 3-way
// split, profiles/r02_stream_ab.log); smaller grids split toward ONE
// workgroup per CU (256): with the split fold in the last-arriving
// workgroup (round 4) one long row walk per CU beats 2-12 shorter ones --
// config 1 0.452 ms (256) / 0.479 (512) / 0.498 (1024) / 0.511 (2048), the
// per-rank share of config 3 0.204 / 0.221 / 0.242 / 0.292, a grid of 384
// or 160 (not whole rounds of 256) slower than either neighbour
// (profiles/r04_split_sweep.log).
static int64_t g_stream_target = 256;  // cubed_stream_split_target() (probes)
static int64_t g_stream_force_split = 0;  // cubed_stream_force_split() (probes: split full grids too)

LaunchPlan plan_launch(const cubed_program_t* P, int64_t ntasks, int64_t max_kept,
                              int64_t max_red, int stream_w) {
  LaunchPlan L;
  L.kernel = P->mode & 3;
  L.vec = (P->mode & 4) ? 4 : 1;
  L.nsplit = 1;
  L.balanced = 0;
  L.bpt = 1;
  const int64_t target = 2048;  // ~8 workgroups per CU
  if (P->mode & CUBED_MODE_STREAM) {
    // stream_body: whole waves of W groups of 4 kept elements per thread
    const int64_t W = stream_w;
    const int64_t slots = ((max_kept + 256 * W - 1) / (256 * W)) * 64;
    L.bpt = (slots + kBlock - 1) / kBlock;
    if (L.bpt < 1) L.bpt = 1;
    if (L.bpt > 65536) L.bpt = 65536;
    const int64_t base = ntasks * L.bpt;
    // bytes of loads one workgroup keeps in flight: U rows x leaves x W
    // groups x 4 elements per lane; below ~96 KiB per CU the grid cannot
    // cover HBM latency (the per-rank share of the elided rechunk + mean:
    // 350 one-leaf f32 workgroups = 44 KiB per CU, 2.9 TB/s unsplit)
    const int isz = P->vtype == CUBED_V_F32 ? 4 : 8;
    const int64_t inflight = (int64_t)kBlock * stream_unroll(isz, P->nleaves) * P->nleaves * W * 4 * isz;
    if (P->nfields > 0 && base * inflight < (int64_t)256 * 96 * 1024 && max_red >= 64)
      L.nsplit = (int32_t)choose_split(base, max_red / 16, g_stream_target);
    else if (P->nfields > 0 && g_stream_force_split > 1 && max_red >= 16 * g_stream_force_split)
      L.nsplit = (int32_t)g_stream_force_split;  // probes only (cubed_stream_force_split)
    // a multiple of 8 workgroups (the surplus exits at once): stream_body
    // maps them to XCD-contiguous runs
    L.blocks = (ntasks * L.nsplit * L.bpt + 7) / 8 * 8;
    // every task the same reduced extent (the host's CUBED_MODE_STREAM_EVEN):
    // exactly the target's workgroups, each an equal run of (task, column
    // block, row) units (stream_body's balanced split) -- a uniform split
    // of 49 column blocks x 5 keeps 245 of 256 CUs busy
    const int64_t G = g_stream_target / 8 * 8;
    const int64_t units = base * max_red;
    if (L.nsplit > 1 && (P->mode & CUBED_MODE_STREAM_EVEN) && G >= 8 && units / G >= 64 &&
        L.bpt * kBlock >= slots) {
      const int64_t minlen = units / G;
      L.nsplit = (int32_t)((max_red + minlen - 1) / minlen + 1);
      L.balanced = 1;
      L.blocks = G;
    }
  } else if (L.kernel == 0) {
    const int64_t items = (max_kept + L.vec - 1) / L.vec;
    L.bpt = (items + kBlock - 1) / kBlock;
    if (L.bpt < 1) L.bpt = 1;
    if (L.bpt > 65536) L.bpt = 65536;
    const int64_t base = ntasks * L.bpt;
    if (P->nfields > 0 && base < target && max_red >= 64) {
      L.nsplit = (int32_t)choose_split(base, max_red / 16, target);
    }
    L.blocks = ntasks * L.nsplit * L.bpt;
  } else {
    const int64_t base = ntasks * max_kept;
    if (base < target && max_red >= 8192) {
      // whole rounds of workgroups, >= 4 of them: rows of one launch can
      // differ a lot in size (pieces of a task cut at chunk boundaries), and
      // with several rounds the short ones no longer leave a ragged tail
      L.nsplit = (int32_t)choose_split(base, max_red / 4096, 4 * target);
    }
    L.blocks = ntasks * max_kept * L.nsplit;
  }
  const bool partials = (P->mode & CUBED_MODE_PARTIALS) != 0;
  L.soa_elems = partials ? (int64_t)P->nfields * ntasks * max_kept : 0;
  L.ws_bytes = (L.nsplit > 1 || partials)
                   ? (L.soa_elems + (int64_t)L.nsplit * ntasks * max_kept * P->nfields) * (int64_t)sizeof(Acc)
                   : 0;
  if ((P->mode & CUBED_MODE_STREAM) && P->nfields > 0 && L.nsplit > 1) {
    // stream_body's arrival counters: one uint32 per (task, column block)
    const int64_t W = stream_w;
    const int64_t slots = ((max_kept + 256 * W - 1) / (256 * W)) * 64;
    L.ws_bytes += ntasks * ((slots + kBlock - 1) / kBlock) * 4;
  }
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

int check_program(const cubed_program_t& P) {
  if (P.ndim < 1 || P.ndim > CUBED_MAX_DIMS || P.nred < 0 || P.nred > P.ndim ||
      P.nleaves < 0 || P.nleaves > CUBED_MAX_LEAVES || P.nfields < 0 ||
      P.nfields > CUBED_MAX_FIELDS || P.nouts < 1 || P.nouts > CUBED_MAX_OUTS ||
      P.ninsns < 0 || P.ninsns > CUBED_MAX_INSNS || P.nepi > CUBED_MAX_EPI) {
    set_err("cubed_fused_chunks: program header out of range");
    return CUBED_E_ARG;
  }
  const bool triple = P.nfields > 0 && triple_rop(P.field_rop[0]);
  if (triple && (P.nfields != 3 || P.field_rop[1] != CUBED_R_VAR_MEAN || P.field_rop[2] != CUBED_R_VAR_M2 ||
                 P.field_acc[0] != 1 || P.field_acc[1] != 0 || P.field_acc[2] != 0)) {
    set_err("cubed_fused_chunks: a var triple is fields {n (i64), mu (f64), M2 (f64)}");
    return CUBED_E_ARG;
  }
  for (int f = 0; f < P.nfields; ++f) {
    const int rop = P.field_rop[f];
    const bool partner = rop == CUBED_R_PAIR_INDEX || rop == CUBED_R_PAIR_IMAG;
    const bool tpartner = rop == CUBED_R_VAR_MEAN || rop == CUBED_R_VAR_M2;
    const bool pair_ok = f == 0 ? (!pair_rop(rop) || (P.nfields == 2 &&
                                   P.field_rop[1] == (rop == CUBED_R_CPROD ? CUBED_R_PAIR_IMAG : CUBED_R_PAIR_INDEX)))
                                : (partner == pair_rop(P.field_rop[0]));
    if (rop < CUBED_R_SUM || rop > CUBED_R_VAR_M2 || (f == 0 && (partner || tpartner)) || !pair_ok ||
        (f > 0 && tpartner != triple) || (f > 0 && triple_rop(rop))) {
      set_err("cubed_fused_chunks: bad reduction op (pair / triple leads need their partners)");
      return CUBED_E_ARG;
    }
  }
  if ((P.mode & CUBED_MODE_PARTIALS) && P.nfields == 0) { set_err("cubed_fused_chunks: partials mode needs a reduction"); return CUBED_E_ARG; }
  if ((P.mode & 3) == 1 && P.nfields == 0) { set_err("cubed_fused_chunks: kernel B needs a reduction"); return CUBED_E_ARG; }
  if ((P.mode & CUBED_MODE_STREAM) &&
      ((P.mode & 3) != 0 || !(P.mode & 4) || P.nred > 2 || P.ndim != P.nred + 1 || P.nleaves < 1)) {
    set_err("cubed_fused_chunks: stream mode needs kernel A, VEC=4, one kept dim and <= 2 reduced dims");
    return CUBED_E_LAYOUT;
  }
  if ((P.mode & CUBED_MODE_HOST_COUNT) && !(P.mode & CUBED_MODE_PARTIALS)) {
    set_err("cubed_fused_chunks: host-provided counts need partials mode");
    return CUBED_E_ARG;
  }
  if (P.mode & CUBED_MODE_OWNER_MAJOR) {
    int stored = 0;
    for (int f = 0; f < P.nfields; ++f) stored += P.field_rop[f] != CUBED_R_COUNT;
    const int64_t mko = P.consts[CUBED_MAX_CONSTS - 3].i, w = P.consts[CUBED_MAX_CONSTS - 2].i,
                  l = P.consts[CUBED_MAX_CONSTS - 1].i;
    if (!(P.mode & CUBED_MODE_STREAM) || !(P.mode & CUBED_MODE_PARTIALS) || !(P.mode & CUBED_MODE_HOST_COUNT) ||
        stored != 1 || mko < 1 || w < 1 || l < 1) {
      set_err("cubed_fused_chunks: owner-major partials need stream + partials + host counts, one stored field "
              "and mko, W, L >= 1");
      return CUBED_E_ARG;
    }
  }
  if ((P.mode & (CUBED_MODE_STREAM_W2 | CUBED_MODE_STREAM_W4)) &&
      (!(P.mode & CUBED_MODE_STREAM) || (P.mode & CUBED_MODE_STREAM_W2 && P.mode & CUBED_MODE_STREAM_W4))) {
    set_err("cubed_fused_chunks: stream group bits need stream mode (one of W2 / W4)");
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
  return 0;
}

}  // namespace cubed

using namespace cubed;

extern "C" int64_t cubed_fused_workspace_bytes(const cubed_program_t* prog, int64_t ntasks,
                                               int64_t max_kept, int64_t max_red) {
  if (!prog || ntasks <= 0) return 0;
  // enough for the interpreted (W = 1) and the JIT streaming grid
  const int64_t a = plan_launch(prog, ntasks, max_kept, max_red).ws_bytes;
  const int64_t b = (prog->mode & CUBED_MODE_STREAM)
                        ? plan_launch(prog, ntasks, max_kept, max_red, stream_groups(*prog)).ws_bytes
                        : 0;
  return a > b ? a : b;
}

extern "C" int cubed_fused_chunks(const cubed_program_t* prog, const cubed_program_t* d_prog,
                                  const cubed_task_t* d_tasks,
                                  int64_t ntasks, int64_t max_kept, int64_t max_red,
                                  void* d_workspace, int64_t workspace_bytes, void* stream) {
  if (!prog || !d_prog || (!d_tasks && ntasks > 0)) { set_err("cubed_fused_chunks: null argument"); return CUBED_E_ARG; }
  if (ntasks == 0) return 0;
  const cubed_program_t& P = *prog;
  if (int rc = check_program(P)) return rc;
  if (max_kept <= 0 || max_red <= 0) { set_err("cubed_fused_chunks: empty task bounds"); return CUBED_E_ARG; }
  const LaunchPlan L = plan_launch(&P, ntasks, max_kept, max_red);
  if (L.ws_bytes > 0 && (d_workspace == nullptr || workspace_bytes < L.ws_bytes)) {
    set_err("cubed_fused_chunks: workspace too small");
    return CUBED_E_WORKSPACE;
  }
  if (!owner_major_fits(P, L.soa_elems)) {
    set_err("cubed_fused_chunks: owner-major slots exceed the SoA block");
    return CUBED_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  Acc* ws = (Acc*)d_workspace + L.soa_elems;  // partials mode: SoA block first
  switch (P.vtype) {
    case CUBED_V_F32: launch_fused<float>(P, d_prog, L, d_tasks, ntasks, max_kept, ws, st); break;
    case CUBED_V_F64: launch_fused<double>(P, d_prog, L, d_tasks, ntasks, max_kept, ws, st); break;
    case CUBED_V_I64: launch_fused<int64_t>(P, d_prog, L, d_tasks, ntasks, max_kept, ws, st); break;
    default: set_err("cubed_fused_chunks: bad vtype"); return CUBED_E_DTYPE;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err(hipGetErrorString(e)); return (int)e; }
  // streaming kernels fold their splits and write SoA partials themselves
  if (P.mode & CUBED_MODE_STREAM) return 0;
  if (P.mode & CUBED_MODE_PARTIALS)
    return launch_collect(P, d_prog, L, d_tasks, ntasks, max_kept, (Acc*)d_workspace, st);
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

extern "C" int cubed_fused_finish(const cubed_program_t* prog, const cubed_program_t* d_prog,
                                  const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept,
                                  const void* d_partials, void* stream) {
  if (!prog || !d_prog || !d_partials || (!d_tasks && ntasks > 0)) { set_err("cubed_fused_finish: null argument"); return CUBED_E_ARG; }
  if (ntasks == 0) return 0;
  if (int rc = check_program(*prog)) return rc;
  if (prog->nfields == 0 || max_kept <= 0) { set_err("cubed_fused_finish: not a reduction"); return CUBED_E_ARG; }
  int kd0, kd1;
  kept_dims(*prog, kd0, kd1);
  const int64_t n = ntasks * max_kept;
  hipLaunchKernelGGL(k_finish_soa, grid_of((n + kBlock - 1) / kBlock), dim3(kBlock), 0, (hipStream_t)stream,
                     d_prog, d_tasks, ntasks, max_kept, (const Acc*)d_partials, kd0, kd1);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err(hipGetErrorString(e)); return (int)e; }
  return 0;
}

extern "C" int cubed_fused_finish_groups(const cubed_program_t* prog, const cubed_program_t* d_prog,
                                         const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept,
                                         const void* d_partials, const int64_t* d_group_start,
                                         int64_t ngroups, void* stream) {
  if (!prog || !d_prog || !d_partials || !d_group_start || (!d_tasks && ntasks > 0)) {
    set_err("cubed_fused_finish_groups: null argument");
    return CUBED_E_ARG;
  }
  if (ntasks == 0 || ngroups == 0) return 0;
  if (int rc = check_program(*prog)) return rc;
  if (prog->nfields == 0 || max_kept <= 0 || ngroups > ntasks) { set_err("cubed_fused_finish_groups: bad shape"); return CUBED_E_ARG; }
  int kd0, kd1;
  kept_dims(*prog, kd0, kd1);
  const int64_t n = ngroups * max_kept;
  hipLaunchKernelGGL(k_finish_groups, grid_of((n + kBlock - 1) / kBlock), dim3(kBlock), 0, (hipStream_t)stream,
                     d_prog, d_tasks, ntasks, max_kept, (const Acc*)d_partials, d_group_start, ngroups, kd0, kd1);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err(hipGetErrorString(e)); return (int)e; }
  return 0;
}

extern "C" int cubed_combine_groups(const cubed_program_t* prog, const cubed_program_t* d_prog,
                                    const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept,
                                    const void* d_row_partials, const int64_t* d_group_start,
                                    int64_t ngroups, int64_t max_kept_out, void* d_group_partials,
                                    void* stream) {
  if (!prog || !d_prog || !d_row_partials || !d_group_start || !d_group_partials ||
      (!d_tasks && ntasks > 0)) {
    set_err("cubed_combine_groups: null argument");
    return CUBED_E_ARG;
  }
  if (ngroups == 0) return 0;
  if (int rc = check_program(*prog)) return rc;
  if (prog->nfields == 0 || max_kept <= 0 || max_kept_out <= 0 || ngroups > ntasks) {
    set_err("cubed_combine_groups: bad shape");
    return CUBED_E_ARG;
  }
  int kd0, kd1;
  kept_dims(*prog, kd0, kd1);
  const int64_t n = ngroups * max_kept_out;
  hipLaunchKernelGGL(k_combine_groups, grid_of((n + kBlock - 1) / kBlock), dim3(kBlock), 0, (hipStream_t)stream,
                     d_prog, d_tasks, ntasks, max_kept, (const Acc*)d_row_partials, d_group_start, ngroups,
                     max_kept_out, (Acc*)d_group_partials, kd0, kd1);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err(hipGetErrorString(e)); return (int)e; }
  return 0;
}

extern "C" int64_t cubed_fold_groups_splits(int64_t ngroups, int64_t max_rows_per_group, int64_t max_kept) {
  // fewer groups than ~2 per CU: cut each group's rows x max_kept SoA
  // entries into runs of >= 512 (2 per thread), toward 1024 workgroups.
  // (The vorticity's one-group fold of 98K entries takes 39 us with 195 runs,
  // 49 with 32, 40 with 10: a fixed chain of dependent first touches --
  // tables, partials, counter, epilogue program, output -- not the entries.)
  if (ngroups <= 0 || max_rows_per_group < 1 || max_kept < 1 || ngroups >= 512) return 1;
  const int64_t per_group = (1024 + ngroups - 1) / ngroups;
  const int64_t by_size = max_rows_per_group * max_kept / 512;
  const int64_t s = per_group < by_size ? per_group : by_size;
  return s > 1 ? s : 1;
}

extern "C" int cubed_fold_groups(const cubed_program_t* prog, const cubed_program_t* d_prog,
                                 const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept,
                                 const void* d_row_partials, const int64_t* d_group_start,
                                 int64_t ngroups, void* d_group_partials, int64_t nsplit,
                                 void* d_split_ws, const cubed_program_t* fin, const cubed_program_t* d_fin,
                                 const cubed_task_t* d_fin_tasks, void* stream) {
  if (!prog || !d_prog || !d_row_partials || !d_group_start || !d_group_partials ||
      (!d_tasks && ntasks > 0) || (nsplit > 1 && !d_split_ws) || (!fin != !d_fin) || (fin && !d_fin_tasks)) {
    set_err("cubed_fold_groups: null argument");
    return CUBED_E_ARG;
  }
  if (ngroups == 0) return 0;
  if (int rc = check_program(*prog)) return rc;
  if (fin) {
    if (int rc = check_program(*fin)) return rc;
    if (fin->nfields != prog->nfields || fin->nred != fin->ndim) {
      set_err("cubed_fold_groups: the epilogue program must reduce every dim over the same fields");
      return CUBED_E_ARG;
    }
  }
  if (prog->nfields == 0 || max_kept <= 0 || ngroups > ntasks || nsplit < 1) { set_err("cubed_fold_groups: bad shape"); return CUBED_E_ARG; }
  int kd0, kd1;
  kept_dims(*prog, kd0, kd1);
  if (nsplit > 1) {
    hipLaunchKernelGGL(k_fold_groups_split, grid_of(ngroups * nsplit), dim3(kBlock), 0, (hipStream_t)stream,
                       d_prog, d_tasks, ntasks, max_kept, (const Acc*)d_row_partials, d_group_start, ngroups,
                       nsplit, (Acc*)d_split_ws, (Acc*)d_group_partials, kd0, kd1, d_fin, d_fin_tasks);
  } else {
    hipLaunchKernelGGL(k_fold_groups, grid_of(ngroups), dim3(kBlock), 0, (hipStream_t)stream, d_prog, d_tasks,
                       ntasks, max_kept, (const Acc*)d_row_partials, d_group_start, ngroups,
                       (Acc*)d_group_partials, kd0, kd1, d_fin, d_fin_tasks);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err(hipGetErrorString(e)); return (int)e; }
  return 0;
}

extern "C" int cubed_combine_partials(const cubed_program_t* prog, const cubed_program_t* d_prog,
                                      const void* d_parts, int32_t nparts, int64_t n, void* d_out,
                                      void* stream) {
  if (!prog || !d_prog || !d_parts || !d_out || nparts < 1 || n < 0) { set_err("cubed_combine_partials: bad argument"); return CUBED_E_ARG; }
  if (n == 0) return 0;
  if (prog->nfields < 1 || prog->nfields > CUBED_MAX_FIELDS) { set_err("cubed_combine_partials: not a reduction"); return CUBED_E_ARG; }
  hipLaunchKernelGGL(k_combine_parts, grid_of((n + kBlock - 1) / kBlock), dim3(kBlock), 0, (hipStream_t)stream,
                     d_prog, (const Acc*)d_parts, nparts, n, (Acc*)d_out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err(hipGetErrorString(e)); return (int)e; }
  return 0;
}

extern "C" int64_t cubed_stream_force_split(int64_t nsplit) {
  const int64_t prev = g_stream_force_split;
  if (nsplit >= 0) g_stream_force_split = nsplit;
  return prev;
}

extern "C" int64_t cubed_stream_split_target(int64_t workgroups) {
  const int64_t prev = g_stream_target;
  if (workgroups > 0) g_stream_target = workgroups;
  return prev;
}

extern "C" const char* cubed_last_error(void) { return g_err; }
extern "C" int cubed_abi_version(void) { return CUBED_ABI_VERSION; }
extern "C" int cubed_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
