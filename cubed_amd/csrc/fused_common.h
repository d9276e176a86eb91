// fused_common.h -- pieces shared by the generic fused kernels (fused.hip)
// and the streaming fast path (stream.hip).
#pragma once
#include "vm.h"

// Program hooks: the ahead-of-time kernels interpret P's instruction lists;
// runtime-specialised builds (jit.cpp) define these to generated
// straight-line functions before including this header.
#ifndef CUBED_RUN_PROLOGUE
#define CUBED_RUN_PROLOGUE(V, VEC, regs) run_vm<V, VEC>(regs, P.insns, P.ninsns, P)
#endif
#ifndef CUBED_RUN_EPILOGUE
#define CUBED_RUN_EPILOGUE(VEC, regs) run_vm<double, VEC>(regs, P.epi, P.nepi, P)
#endif

namespace cubed {

CUBED_DEV void divmod64(int64_t a, int64_t b, int64_t& q, int64_t& r) {
  if (((uint64_t)a | (uint64_t)b) < 0x100000000ull) {
    const uint32_t qa = (uint32_t)a / (uint32_t)b;
    q = qa; r = a - (int64_t)qa * b;
  } else {
    q = a / b; r = a - q * b;
  }
}

template <typename V, int VEC>
CUBED_DEV void accumulate(Acc (&acc)[CUBED_MAX_FIELDS][VEC], Regs<V, VEC>& regs,
                          const cubed_program_t& P) {
  V src[CUBED_MAX_FIELDS][VEC];
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
    if (f < P.nfields) fetch(regs, P.field_src[f], src[f]);
  fields_add<V, VEC>(acc, src, P);
}

// Epilogue + store of VEC reduced elements.
template <int VEC>
CUBED_DEV void finish(const cubed_program_t& P, const cubed_task_t* T,
                      const Acc (&acc)[CUBED_MAX_FIELDS][VEC],
                      const int64_t (&ooff)[CUBED_MAX_OUTS]) {
  if (P.nepi >= 0) {
    Regs<double, VEC> er;
#pragma unroll
    for (int j = 0; j < VEC; ++j) { er.r0[j] = 0; er.r1[j] = 0; er.r2[j] = 0; er.r3[j] = 0; er.r4[j] = 0; er.r5[j] = 0; }
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) {
      if (f < P.nfields) {
        double X[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) X[j] = P.field_acc[f] ? (double)acc[f][j].i : acc[f][j].f;
        put(er, f, X);
      }
    }
    CUBED_RUN_EPILOGUE(VEC, er);
#pragma unroll
    for (int o = 0; o < CUBED_MAX_OUTS; ++o) {
      if (o < P.nouts) {
        double X[VEC];
        fetch(er, P.out_src[o], X);
        stv<double, VEC>((char*)T->out_base[o], ooff[o], P.out_dtype[o], X);
      }
    }
  } else {
#pragma unroll
    for (int o = 0; o < CUBED_MAX_OUTS; ++o) {
      if (o < P.nouts) {
        const int f = P.out_src[o];
        if (P.field_acc[f]) {
          int64_t X[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) X[j] = acc[f][j].i;
          stv<int64_t, VEC>((char*)T->out_base[o], ooff[o], P.out_dtype[o], X);
        } else {
          double X[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) X[j] = acc[f][j].f;
          stv<double, VEC>((char*)T->out_base[o], ooff[o], P.out_dtype[o], X);
        }
      }
    }
  }
}

// Rows in flight per lane in the streaming kernel: about 128 B of loads per
// lane whatever the leaf count (a 1-leaf mean needs twice the rows of a
// 2-leaf quad-means product to keep the same bytes in flight).
__host__ __device__ constexpr int stream_unroll(int itemsize, int nleaves) {
  return itemsize == 4 ? (nleaves <= 1 ? 8 : nleaves == 2 ? 4 : 2)
                       : (nleaves <= 1 ? 4 : 2);
}

#ifndef __HIPCC_RTC__
// ---------------------------------------------------------------- launch plan
struct LaunchPlan {
  int kernel;     // 0 = A, 1 = B
  int vec;        // 1 or 4
  int64_t bpt;    // A: blocks per task per split
  int32_t nsplit;  // split slots (balanced: the most contributors of one column block)
  int32_t balanced;  // stream: CUBED_MODE_STREAM_EVEN's balanced split (kernel gets -nsplit)
  int64_t soa_elems;  // partials mode: SoA per-field partials at the workspace start
  int64_t ws_bytes;
  int64_t blocks;
};

// stream_impl.h: the streaming fast path (mode bit CUBED_MODE_STREAM), one
// instantiation per (value type, split variant) in stream_*.hip
template <typename V, bool SPLIT>
void launch_stream_v(const cubed_program_t& P, const cubed_program_t* dP, const LaunchPlan& L,
                     const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept, Acc* ws, hipStream_t st);
template <typename V>
void launch_stream(const cubed_program_t& P, const cubed_program_t* dP, const LaunchPlan& L, const cubed_task_t* d_tasks,
                   int64_t ntasks, int64_t max_kept, Acc* ws, hipStream_t st) {
  if (L.nsplit > 1 && P.nfields > 0)
    launch_stream_v<V, true>(P, dP, L, d_tasks, ntasks, max_kept, ws, st);
  else
    launch_stream_v<V, false>(P, dP, L, d_tasks, ntasks, max_kept, ws, st);
}

dim3 grid_of(int64_t blocks);
// stream_w: kept VEC groups per thread of a streaming launch (1 for the
// interpreted kernels of stream.hip, stream_groups(P) for JIT kernels)
LaunchPlan plan_launch(const cubed_program_t* P, int64_t ntasks, int64_t max_kept, int64_t max_red,
                       int stream_w = 1);
// Streaming JIT kernels: kept VEC groups per thread (1, 2 or 4; fused.hip)
int stream_groups(const cubed_program_t& P);
int check_program(const cubed_program_t& P);
void kept_dims(const cubed_program_t& P, int& kd0, int& kd1);
int launch_collect(const cubed_program_t& P, const cubed_program_t* dP, const LaunchPlan& L,
                   const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept, Acc* ws_base,
                   hipStream_t st);  // 0 or a CUBED_E_* code (message set)
void set_error(const char* msg);

// CUBED_MODE_OWNER_MAJOR: every owner-major slot (W x L groups of mko) lies
// inside the launch's SoA block
inline bool owner_major_fits(const cubed_program_t& P, int64_t soa_elems) {
  if (!(P.mode & CUBED_MODE_OWNER_MAJOR)) return true;
  const int64_t mko = P.consts[CUBED_MAX_CONSTS - 3].i, w = P.consts[CUBED_MAX_CONSTS - 2].i,
                l = P.consts[CUBED_MAX_CONSTS - 1].i;
  return mko * w * l <= soa_elems;
}

#endif  // __HIPCC_RTC__

}  // namespace cubed
