// copy_random.hip -- Philox chunk generation and strided box copies.
//
// cubed_random_chunks replaces the per-task numpy call of cubed/random.py:31-36
// (Generator(Philox(key=root_seed + block_offset)).random(shape)): one thread
// produces one Philox4x64-10 block = 4 consecutive doubles, stored as two
// 16-byte stores, so a chunk is written at HBM rate.
//
// cubed_copy_boxes replaces copy_read_to_write (primitive/rechunk.py:187-192)
// and the map_direct region reads (core/ops.py:481,784): every (source chunk
// x target chunk) intersection is one box.  Rechunk never permutes axes, so
// both views of a box are C-ordered sub-boxes of the same index space and the
// innermost run is contiguous on both sides: the row kernel moves each row
// with 16/8/4/1-byte lanes.  Boxes whose innermost runs differ (after the host
// drops unit dims -- e.g. (1,N) chunks -> (N,1) chunks) go through a 64x64
// LDS tile so both the read and the write stay coalesced.
#include <cstdlib>
#include "common.h"
#include <stdio.h>

namespace cubed {
extern thread_local char g_err[512];
}
using namespace cubed;

static int fail(const char* m) { snprintf(g_err, sizeof(g_err), "%s", m); return CUBED_E_ARG; }

__global__ __launch_bounds__(kBlock) void k_random(const int64_t* __restrict__ outs,
                                                   const int64_t* __restrict__ counts,
                                                   const uint64_t* __restrict__ keys,
                                                   int64_t ntasks, int64_t bpt) {
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int64_t t = g / bpt, b = g % bpt;
  if (t >= ntasks) return;
  CUBED_G double* __restrict__ out = (CUBED_G double*)(uintptr_t)outs[t];
  const int64_t n = counts[t];
  const uint64_t k0 = keys[2 * t], k1 = keys[2 * t + 1];
  const int64_t nblk = (n + 3) >> 2;
  for (int64_t i = b * kBlock + threadIdx.x; i < nblk; i += bpt * kBlock) {
    P4 r = philox4x64_10((uint64_t)i + 1ull, 0ull, k0, k1);
    const int64_t e = i << 2;
    if (e + 4 <= n && (((uintptr_t)(out + e)) & 15) == 0) {
      f64x2 a, c;
      a.x = u64_to_unit(r.x[0]); a.y = u64_to_unit(r.x[1]);
      c.x = u64_to_unit(r.x[2]); c.y = u64_to_unit(r.x[3]);
      ((CUBED_G f64x2*)(out + e))[0] = a;
      ((CUBED_G f64x2*)(out + e))[1] = c;
    } else {
      for (int j = 0; j < 4 && e + j < n; ++j) out[e + j] = u64_to_unit(r.x[j]);
    }
  }
}

extern "C" int cubed_random_chunks(const int64_t* d_out_ptrs, const int64_t* d_counts,
                                   const uint64_t* d_keys, int64_t ntasks, int64_t max_count,
                                   void* stream) {
  if (ntasks == 0) return 0;
  if (!d_out_ptrs || !d_counts || !d_keys || max_count < 0) return fail("cubed_random_chunks: bad argument");
  const int64_t nblk = (max_count + 3) / 4;
  int64_t bpt = (nblk + kBlock - 1) / kBlock;
  if (bpt < 1) bpt = 1;
  if (bpt > 16384) bpt = 16384;
  const int64_t blocks = ntasks * bpt;
  dim3 grid(blocks <= 0x7fffffff ? (unsigned)blocks : 0x7fffffffu,
            blocks <= 0x7fffffff ? 1u : (unsigned)((blocks + 0x7ffffffe) / 0x7fffffff));
  hipLaunchKernelGGL(k_random, grid, dim3(kBlock), 0, (hipStream_t)stream, d_out_ptrs, d_counts,
                     d_keys, ntasks, bpt);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}

// ------------------------------------------------------------------ box copies
// Row kernel: rows = product of all but the innermost extent.  A work unit
// is one segment of up to kSeg W-byte words (4 KiB with 16-B lanes) of one
// row, so long contiguous rows (whole-chunk moves) spread over many waves and
// short rows (rechunk pieces) are one unit each.  Template W = lane width in
// bytes.
template <int W, int UN>
__global__ __launch_bounds__(kBlock) void k_copy_rows(const cubed_box_t* __restrict__ boxes,
                                                      int64_t nboxes, int32_t ndim, int32_t isz,
                                                      int64_t bpb, int64_t units_per_block) {
  using T = typename conditional<W == 16, u32x4,
            typename conditional<W == 8, uint64_t,
            typename conditional<W == 4, uint32_t, uint8_t>::type>::type>::type;
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int64_t bi = g / bpb, blk = g % bpb;
  if (bi >= nboxes) return;
  const cubed_box_t* __restrict__ B = boxes + bi;
  const int nd = ndim;
  int64_t nrows = 1;
  for (int d = 0; d < nd - 1; ++d) nrows *= B->extent[d];
  const int64_t rowbytes = B->extent[nd - 1] * isz;
  const int64_t nw = rowbytes / W;
  constexpr int kSeg = 64 * UN;  // words per work unit
  const int64_t nseg = (nw + kSeg - 1) / kSeg;
  const int64_t units = nrows * nseg;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t u_begin = blk * units_per_block;
  int64_t u_end = u_begin + units_per_block;
  if (u_end > units) u_end = units;
  for (int64_t u = u_begin + wave; u < u_end; u += kBlock / 64) {
    const int64_t row = u / nseg, seg = u - row * nseg;
    // decompose the row index over dims [0, nd-1)
    int64_t so = 0, dof = 0, rr = row;
    for (int d = nd - 2; d >= 0; --d) {
      const int64_t e = B->extent[d];
      const int64_t c = rr % e;
      rr /= e;
      so += c * B->src_stride[d];
      dof += c * B->dst_stride[d];
    }
    const CUBED_G T* __restrict__ src = (const CUBED_G T*)(uintptr_t)(B->src_base + so * isz);
    CUBED_G T* __restrict__ dst = (CUBED_G T*)(uintptr_t)(B->dst_base + dof * isz);
    const int64_t w0 = seg * kSeg;
    const int64_t w1 = (w0 + kSeg < nw) ? w0 + kSeg : nw;
    // 4 lane-widths per step, all loads issued before the first store
    // (4 x W bytes in flight per lane); bytes are touched once: non-temporal
    for (int64_t i0 = w0; i0 < w1; i0 += UN * 64) {
      T v[UN];
#pragma unroll
      for (int k = 0; k < UN; ++k) {
        const int64_t i = i0 + k * 64 + lane;
        if (i < w1) v[k] = __builtin_nontemporal_load(src + i);
      }
#pragma unroll
      for (int k = 0; k < UN; ++k) {
        const int64_t i = i0 + k * 64 + lane;
        if (i < w1) __builtin_nontemporal_store(v[k], dst + i);
      }
    }
  }
}

// Flat-destination kernel for 2-d boxes whose destination is packed
// (dst row stride == row length): the box is walked as one contiguous run of
// W-byte destination words, so every wave writes kSeg aligned consecutive
// words whatever the row length (rechunk pieces of 4000-B rows no longer end
// in partial lines per wave); each lane finds its source row by one 32-bit
// division (host guarantees < 2^31 words per box).
template <int W, int UN, bool NTL = true>
__global__ __launch_bounds__(kBlock) void k_copy_flat(const cubed_box_t* __restrict__ boxes,
                                                      int64_t nboxes, int32_t isz, int64_t bpb,
                                                      int64_t segs_per_block) {
  using T = typename conditional<W == 16, u32x4,
            typename conditional<W == 8, uint64_t,
            typename conditional<W == 4, uint32_t, uint8_t>::type>::type>::type;
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int64_t bi = g / bpb, blk = g % bpb;
  if (bi >= nboxes) return;
  const cubed_box_t* __restrict__ B = boxes + bi;
  const uint32_t nw = (uint32_t)(B->extent[1] * isz / W);
  const int64_t total = B->extent[0] * (int64_t)nw;
  const int64_t sstr = B->src_stride[0] * isz;
  const char* __restrict__ sbase = (const char*)(uintptr_t)B->src_base;
  CUBED_G T* __restrict__ dst = (CUBED_G T*)(uintptr_t)B->dst_base;
  constexpr int kSeg = 64 * UN;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t w_begin = blk * segs_per_block * kSeg;
  int64_t w_end = w_begin + segs_per_block * kSeg;
  if (w_end > total) w_end = total;
  for (int64_t i0 = w_begin + (int64_t)wave * kSeg; i0 < w_end; i0 += (int64_t)(kBlock / 64) * kSeg) {
    T v[UN];
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const int64_t i = i0 + k * 64 + lane;
      if (i < w_end) {
        const uint32_t r = (uint32_t)i / nw, c = (uint32_t)i - r * nw;
        const CUBED_G T* __restrict__ src = (const CUBED_G T*)(uintptr_t)(sbase + (int64_t)r * sstr);
        if constexpr (NTL) v[k] = __builtin_nontemporal_load(src + c);
        else v[k] = src[c];
      }
    }
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const int64_t i = i0 + k * 64 + lane;
      if (i < w_end) __builtin_nontemporal_store(v[k], dst + i);
    }
  }
}

// 64x64 LDS tile transpose-copy for 2-d boxes whose contiguous axes differ:
// src contiguous along dim 1, dst contiguous along dim 0 (host arranges).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_copy_tile(const cubed_box_t* __restrict__ boxes,
                                                      int64_t nboxes, int64_t tiles_per_box) {
  __shared__ T tile[64][65];
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int64_t bi = g / tiles_per_box, ti = g % tiles_per_box;
  if (bi >= nboxes) return;
  const cubed_box_t* __restrict__ B = boxes + bi;
  const int64_t e0 = B->extent[0], e1 = B->extent[1];
  const int64_t nt1 = (e1 + 63) / 64;
  const int64_t t0 = (ti / nt1) * 64, t1 = (ti % nt1) * 64;
  if (t0 >= e0) return;
  const CUBED_G T* __restrict__ src = (const CUBED_G T*)(uintptr_t)B->src_base;
  CUBED_G T* __restrict__ dst = (CUBED_G T*)(uintptr_t)B->dst_base;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int64_t i0 = t0 + r, i1 = t1 + tx;
    if (i0 < e0 && i1 < e1) tile[r][tx] = src[i0 * B->src_stride[0] + i1 * B->src_stride[1]];
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int64_t i1 = t1 + r, i0 = t0 + tx;
    if (i0 < e0 && i1 < e1) dst[i0 * B->dst_stride[0] + i1 * B->dst_stride[1]] = tile[tx][r];
  }
}

// Generic element gather (any strides, any itemsize); used for odd layouts.
__global__ __launch_bounds__(kBlock) void k_copy_elems(const cubed_box_t* __restrict__ boxes,
                                                       int64_t nboxes, int32_t ndim, int32_t isz,
                                                       int64_t bpb) {
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int64_t bi = g / bpb, blk = g % bpb;
  if (bi >= nboxes) return;
  const cubed_box_t* __restrict__ B = boxes + bi;
  int64_t n = 1;
  for (int d = 0; d < ndim; ++d) n *= B->extent[d];
  for (int64_t i = blk * kBlock + threadIdx.x; i < n; i += bpb * kBlock) {
    int64_t so = 0, dof = 0, rr = i;
    for (int d = ndim - 1; d >= 0; --d) {
      const int64_t e = B->extent[d];
      const int64_t c = rr % e;
      rr /= e;
      so += c * B->src_stride[d];
      dof += c * B->dst_stride[d];
    }
    const char* s = (const char*)B->src_base + so * isz;
    char* dd = (char*)B->dst_base + dof * isz;
    switch (isz) {
      case 1: *(uint8_t*)dd = *(const uint8_t*)s; break;
      case 2: *(uint16_t*)dd = *(const uint16_t*)s; break;
      case 4: *(uint32_t*)dd = *(const uint32_t*)s; break;
      case 8: *(uint64_t*)dd = *(const uint64_t*)s; break;
      default: for (int j = 0; j < isz; ++j) dd[j] = s[j]; break;
    }
  }
}

static dim3 grid2(int64_t blocks) {
  if (blocks <= 0x7fffffff) return dim3((unsigned)blocks, 1, 1);
  return dim3(0x7fffffffu, (unsigned)((blocks + 0x7ffffffe) / 0x7fffffff), 1);
}

extern "C" int cubed_copy_boxes(const cubed_box_t* d_boxes, int64_t nboxes, int32_t ndim,
                                int32_t itemsize, int32_t path, int32_t lane_bytes,
                                int64_t work, int64_t row_bytes, void* stream) {
  if (nboxes == 0) return 0;
  if (!d_boxes) return fail("cubed_copy_boxes: null box table");
  hipStream_t st = (hipStream_t)stream;
  const int isz = itemsize;
  const int width = lane_bytes;
  const int nd = ndim;
  const int64_t max_box_elems = work;
  if (nd < 1 || nd > CUBED_MAX_DIMS || isz < 1) return fail("cubed_copy_boxes: bad ndim/itemsize");
  if (path == 2) {
    if (nd != 2) return fail("cubed_copy_boxes: tile path needs 2-d boxes");
    // max_box_elems carries tiles per box for this path
    const int64_t tpb = max_box_elems;
    const dim3 grid = grid2(nboxes * tpb);
    switch (isz) {
      case 1: hipLaunchKernelGGL(k_copy_tile<uint8_t>, grid, dim3(kBlock), 0, st, d_boxes, nboxes, tpb); break;
      case 2: hipLaunchKernelGGL(k_copy_tile<uint16_t>, grid, dim3(kBlock), 0, st, d_boxes, nboxes, tpb); break;
      case 4: hipLaunchKernelGGL(k_copy_tile<uint32_t>, grid, dim3(kBlock), 0, st, d_boxes, nboxes, tpb); break;
      case 8: hipLaunchKernelGGL(k_copy_tile<uint64_t>, grid, dim3(kBlock), 0, st, d_boxes, nboxes, tpb); break;
      default: return fail("cubed_copy_boxes: tile path itemsize");
    }
  } else if (path == 1) {
    int64_t bpb = (max_box_elems + kBlock * 4 - 1) / (kBlock * 4);
    if (bpb < 1) bpb = 1;
    if (bpb > 65536) bpb = 65536;
    hipLaunchKernelGGL(k_copy_elems, grid2(nboxes * bpb), dim3(kBlock), 0, st, d_boxes, nboxes, nd, isz, bpb);
  } else if (path == 3) {
    // flat: work = max destination words per box (< 2^31), 16 segments of
    // 64*UN words per workgroup (64 KiB with 16-B lanes)
    if (nd != 2) return fail("cubed_copy_boxes: flat path needs 2-d boxes");
    if (max_box_elems <= 0 || max_box_elems >= ((int64_t)1 << 31)) return fail("cubed_copy_boxes: flat path box size");
    constexpr int UN = 4;
    // segments per workgroup (16 = 64 KiB with 16-B lanes)
    const int64_t spb = 16;
    const int64_t nseg = (max_box_elems + 64 * UN - 1) / (64 * UN);
    int64_t bpb = (nseg + spb - 1) / spb;
    // a multiple of 8 workgroups per box: workgroup i of box b and of box
    // b+1 -- the same rows of the next piece of the source rows when the
    // host orders boxes by source address -- run on the same XCD (round-robin
    // dispatch) at nearly the same time, so the 128-B line a 4000-B piece
    // boundary splits is fetched into that XCD's L2 once, not twice
    if (nboxes > 1) bpb = (bpb + 7) / 8 * 8;
    const dim3 grid = grid2(nboxes * bpb);
    // cached source loads for 16-B lanes: a 4000-B piece row starts and ends
    // mid-line, and the neighbouring piece (next box, same XCD) finds the
    // shared lines in L2 -- non-temporal loads let them go: PMC fetch 1.078x
    // -> 1.004x algorithmic, config 3 copy 3.81 -> 3.71 ms
    // (profiles/r02_stream_ab.log)
    if (width == 16) {
      hipLaunchKernelGGL((k_copy_flat<16, UN, false>), grid, dim3(kBlock), 0, st, d_boxes, nboxes, isz, bpb, spb);
    } else switch (width) {
      case 8: hipLaunchKernelGGL((k_copy_flat<8, UN>), grid, dim3(kBlock), 0, st, d_boxes, nboxes, isz, bpb, spb); break;
      case 4: hipLaunchKernelGGL((k_copy_flat<4, UN>), grid, dim3(kBlock), 0, st, d_boxes, nboxes, isz, bpb, spb); break;
      default: hipLaunchKernelGGL((k_copy_flat<1, UN>), grid, dim3(kBlock), 0, st, d_boxes, nboxes, isz, bpb, spb); break;
    }
  } else {
    // rows: max_box_elems = max rows per box, row_bytes = longest row; work
    // units are <= 4 KiB row segments; aim ~64 KB per workgroup
    const int64_t max_rows = max_box_elems;
    // 4 x 16-B loads in flight per lane (2 and 8 measured the same, as did
    // plain vs non-temporal accesses: 5.5-5.75 TB/s read+write on MI355X)
    constexpr int UN = 4;
    const int64_t seg_bytes = (int64_t)64 * UN * width;
    const int64_t nseg = row_bytes > 0 ? (row_bytes + seg_bytes - 1) / seg_bytes : 1;
    const int64_t unit_bytes = row_bytes > 0 && row_bytes < seg_bytes ? row_bytes : seg_bytes;
    int64_t rpb = (65536 + unit_bytes - 1) / unit_bytes;
    if (rpb < 4) rpb = 4;
    if (rpb > 4096) rpb = 4096;
    int64_t bpb = (max_rows * nseg + rpb - 1) / rpb;
    if (bpb < 1) bpb = 1;
    const dim3 grid = grid2(nboxes * bpb);
    switch (width) {
      case 16: hipLaunchKernelGGL((k_copy_rows<16, UN>), grid, dim3(kBlock), 0, st, d_boxes, nboxes, nd, isz, bpb, rpb); break;
      case 8: hipLaunchKernelGGL((k_copy_rows<8, UN>), grid, dim3(kBlock), 0, st, d_boxes, nboxes, nd, isz, bpb, rpb); break;
      case 4: hipLaunchKernelGGL((k_copy_rows<4, UN>), grid, dim3(kBlock), 0, st, d_boxes, nboxes, nd, isz, bpb, rpb); break;
      default: hipLaunchKernelGGL((k_copy_rows<1, UN>), grid, dim3(kBlock), 0, st, d_boxes, nboxes, nd, isz, bpb, rpb); break;
    }

  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { snprintf(g_err, sizeof(g_err), "%s", hipGetErrorString(e)); return (int)e; }
  return 0;
}
