// stream_impl.h -- streaming fast path of the fused chunk kernels (gfx950),
// instantiated per value type and split variant by stream_{f32,f64,i64}{,_split}.hip.
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
// ranges combine in split order in the last-arriving workgroup (the _split
// variant, kernels.h).  COUNT fields are the trip count,
// added once instead of per element.
#include "kernels.h"

namespace cubed {

template <typename V, int NL, int U, bool SPLIT>
__global__ __launch_bounds__(kBlock) void k_stream(
    const cubed_program_t* __restrict__ Pd, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t bpt, int32_t nsplit, Acc* __restrict__ ws, int64_t max_kept) {
  stream_body<V, NL, U, 1, SPLIT>(*Pd, tasks, ntasks, bpt, nsplit, ws, max_kept);
}

// The interpreted kernels are the fallback / cross-check of the JIT ones
// (CUBED_AMD_JIT=0): two rows in flight instead of stream_unroll()'s 2-8
// keeps each a few copies of the interpreter instead of up to 8 (build time);
// the accumulation order per element -- and so every result bit -- is the same.
template <typename V, bool SPLIT>
void launch_stream_v(const cubed_program_t& P, const cubed_program_t* dP, const LaunchPlan& L,
                     const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept, Acc* ws, hipStream_t st) {
  const dim3 grid = grid_of(L.blocks);
  const int32_t ns = L.balanced ? -L.nsplit : L.nsplit;  // balanced split: -slots
  switch (P.nleaves) {
    case 1: hipLaunchKernelGGL((k_stream<V, 1, 2, SPLIT>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, ns, ws, max_kept); break;
    case 2: hipLaunchKernelGGL((k_stream<V, 2, 2, SPLIT>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, ns, ws, max_kept); break;
    case 3: hipLaunchKernelGGL((k_stream<V, 3, 2, SPLIT>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, ns, ws, max_kept); break;
    default: hipLaunchKernelGGL((k_stream<V, 4, 2, SPLIT>), grid, dim3(kBlock), 0, st, dP, d_tasks, ntasks, L.bpt, ns, ws, max_kept); break;
  }
}

// one TU per (value type, split variant): stream_{f32,f64,i64}{,_split}.hip
// compile in parallel; launch_stream (fused.hip) picks the variant
template void launch_stream_v<CUBED_STREAM_V, CUBED_STREAM_SPLIT>(
    const cubed_program_t&, const cubed_program_t*, const LaunchPlan&, const cubed_task_t*, int64_t, int64_t,
    Acc*, hipStream_t);

}  // namespace cubed
