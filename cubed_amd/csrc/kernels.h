// kernels.h -- device bodies of the fused chunk kernels (gfx950).
//
// Each body takes the fused program as `const cubed_program_t& P`.  The
// ahead-of-time kernels (fused.hip, stream.hip) bind P to a device-memory
// copy read through the scalar cache; the runtime-specialised kernels
// (jit.cpp) bind it to a compile-time constant, so every switch of the
// interpreter folds away and the body compiles to straight-line code.
//
#pragma once
#include "fused_common.h"

namespace cubed {

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
CUBED_DEV void fused_a_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t bpt, int32_t nsplit, Acc* __restrict__ ws, int64_t max_kept) {
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
    int64_t ooff[CUBED_MAX_OUTS] = {};
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
      CUBED_RUN_PROLOGUE(V, VEC, regs);
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
    if (r1 > r0) {  // (an empty task -- a rank without chunks of this block -- has extent 0)
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
      CUBED_RUN_PROLOGUE(V, VEC, regs);
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
    if (nsplit == 1 && !(P.mode & CUBED_MODE_PARTIALS)) {
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
CUBED_DEV void fused_b_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, int32_t nsplit, Acc* __restrict__ ws) {
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
  int64_t ooff[CUBED_MAX_OUTS] = {};
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

  // Two-level walk of the split's flattened reduced range: outer reduced
  // index o (dims [nkd, nd-1), decomposed once per o), inner dim nd-1 strided
  // by the workgroup (no per-element index decomposition).
  Regs<V, VEC> regs;
  const int64_t nin = T->extent[nd - 1];
  const int64_t stepw = (int64_t)kBlock * VEC;
  if (nin < 2 * stepw) {
    // short inner rows: one flattened walk keeps every lane busy
    for (int64_t p = r0 + (int64_t)threadIdx.x * VEC; p < r1; p += stepw) {
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
      CUBED_RUN_PROLOGUE(V, VEC, regs);
      accumulate<V, VEC>(acc, regs, P);
    }
  }
  for (int64_t o = nin ? r0 / nin : 0; nin >= 2 * stepw && o * nin < r1; ++o) {
    const int64_t lo = (r0 > o * nin ? r0 - o * nin : 0);
    const int64_t hi = (r1 < (o + 1) * nin ? r1 - o * nin : nin);
    int64_t ooffs[CUBED_MAX_LEAVES];
#pragma unroll
    for (int l = 0; l < CUBED_MAX_LEAVES; ++l) ooffs[l] = loff[l];
    int64_t rr = o;
#pragma unroll
    for (int d = CUBED_MAX_DIMS - 2; d >= 0; --d) {
      if (d < nd - 1 && d >= nkd) {
        int64_t q, c;
        if (d == nkd) { q = 0; c = rr; } else divmod64(rr, T->extent[d], q, c);
        rr = q;
#pragma unroll
        for (int l = 0; l < CUBED_MAX_LEAVES; ++l) ooffs[l] += c * T->leaf_stride[l][d];
      }
    }
    for (int64_t i = lo + (int64_t)threadIdx.x * VEC; i < hi; i += stepw) {
      int64_t off[CUBED_MAX_LEAVES];
#pragma unroll
      for (int l = 0; l < CUBED_MAX_LEAVES; ++l) off[l] = ooffs[l] + i * inner[l];
      load_leaves<V, VEC>(regs, P, T, off, inner);
      CUBED_RUN_PROLOGUE(V, VEC, regs);
      accumulate<V, VEC>(acc, regs, P);
    }
  }
  // combine VEC lanes, then the 64-wide wave, then the 4 waves
  Acc a[CUBED_MAX_FIELDS];
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f) a[f] = acc[f][0];
#pragma unroll
  for (int j = 1; j < VEC; ++j) {
    Acc b[CUBED_MAX_FIELDS];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) b[f] = acc[f][j];
    fields_combine(a, b, P);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    Acc b[CUBED_MAX_FIELDS];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) b[f] = shfl_xor_acc(a[f], m);
    fields_combine(a, b, P);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) red[wave][f] = a[f];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc x[CUBED_MAX_FIELDS];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) x[f] = red[0][f];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) fields_combine(x, red[w], P);
    Acc fin[CUBED_MAX_FIELDS][1];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) fin[f][0] = x[f];
    if (nsplit == 1 && !(P.mode & CUBED_MODE_PARTIALS)) {
      finish<1>(P, T, fin, ooff);
    } else {
      Acc* w = ws + ((int64_t)(s * ntasks + t) * max_kept + k) * P.nfields;
#pragma unroll
      for (int f = 0; f < CUBED_MAX_FIELDS; ++f) if (f < P.nfields) w[f] = fin[f][0];
    }
  }
}

// The fields of element i of a SoA partial block (field stride n); fields
// past P.nfields hold the identity.
CUBED_DEV void soa_load(const cubed_program_t& P, const Acc* __restrict__ soa, int64_t n, int64_t i,
                        Acc (&x)[CUBED_MAX_FIELDS]) {
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
    x[f] = f < P.nfields ? soa[f * n + i] : acc_init(P.field_rop[f], P.field_acc[f]);
}

// ---------------------------------------------------------------- finalize
// Fold the nsplit split partials of element (t, k) in split order into
// x[f]: batches of 8 splits are loaded before they are combined, so a
// thread keeps 8 x nfields loads in flight instead of one (the finalize of a
// 100-way split read one dependent partial at a time).  Same order, same bits.
CUBED_DEV void fold_splits_of(const cubed_program_t& P, const Acc* __restrict__ ws, int32_t nsplit,
                              int64_t ntasks, int64_t t, int64_t max_kept, int64_t k,
                              Acc (&x)[CUBED_MAX_FIELDS]) {
  const int nf = P.nfields;
  const int64_t sstride = ntasks * max_kept * nf;
  const Acc* __restrict__ p = ws + (t * max_kept + k) * nf;
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
    if (f < nf) x[f] = p[f];
  int s = 1;
  for (; s + 8 <= nsplit; s += 8) {
    Acc v[8][CUBED_MAX_FIELDS];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
        if (f < nf) v[u][f] = p[(int64_t)(s + u) * sstride + f];
#pragma unroll
    for (int u = 0; u < 8; ++u) fields_combine(x, v[u], P);
  }
  for (; s < nsplit; ++s) {
    Acc v[CUBED_MAX_FIELDS];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
      if (f < nf) v[f] = p[(int64_t)s * sstride + f];
    fields_combine(x, v, P);
  }
}

CUBED_DEV void finalize_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, int32_t nsplit, const Acc* __restrict__ ws, int kd0, int kd1) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t t = i / max_kept, k = i % max_kept;
  if (t >= ntasks) return;
  const cubed_task_t* __restrict__ T = tasks + t;
  int64_t nk = 1;
  for (int d = kd0; d < kd1; ++d) nk *= T->extent[d];
  if (k >= nk) return;
  int64_t ooff[CUBED_MAX_OUTS] = {};
  int64_t kk = k;
  for (int d = kd1 - 1; d >= kd0; --d) {
    int64_t q, c;
    divmod64(kk, T->extent[d], q, c);
    kk = q;
    for (int o = 0; o < CUBED_MAX_OUTS; ++o) ooff[o] += c * T->out_stride[o][d];
  }
  Acc x[CUBED_MAX_FIELDS];
  fold_splits_of(P, ws, nsplit, ntasks, t, max_kept, k, x);
  Acc fin[CUBED_MAX_FIELDS][1];
  for (int f = 0; f < P.nfields && f < CUBED_MAX_FIELDS; ++f) fin[f][0] = x[f];
  finish<1>(P, T, fin, ooff);
}

// ---------------------------------------------------------------- partials (multi-GPU)
// CUBED_MODE_PARTIALS: the reduce kernels above always leave their
// accumulators in the split workspace; collect_body combines the splits (in
// split order) and writes one SoA block per field, soa[f][t][k], with the
// reduction identity in the padding k >= nk of edge tasks, so every rank's
// block has the same layout and can be summed / gathered by RCCL.
CUBED_DEV void collect_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, int32_t nsplit, const Acc* __restrict__ ws, Acc* __restrict__ soa,
    int kd0, int kd1) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t t = i / max_kept, k = i % max_kept;
  if (t >= ntasks) return;
  const cubed_task_t* __restrict__ T = tasks + t;
  int64_t nk = 1;
  for (int d = kd0; d < kd1; ++d) nk *= T->extent[d];
  const int64_t n = ntasks * max_kept;
  Acc x[CUBED_MAX_FIELDS];
  if (k < nk) fold_splits_of(P, ws, nsplit, ntasks, t, max_kept, k, x);
  for (int f = 0; f < P.nfields && f < CUBED_MAX_FIELDS; ++f)
    if (!(P.mode & CUBED_MODE_HOST_COUNT) || P.field_rop[f] != CUBED_R_COUNT)
      soa[f * n + i] = k < nk ? x[f] : acc_init(P.field_rop[f], P.field_acc[f]);
}

// Epilogue + store from combined SoA partials (the last step of a reduction
// whose partials were combined across GPUs).
CUBED_DEV void finish_soa_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, int kd0, int kd1) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t t = i / max_kept, k = i % max_kept;
  if (t >= ntasks) return;
  const cubed_task_t* __restrict__ T = tasks + t;
  int64_t nk = 1;
  for (int d = kd0; d < kd1; ++d) nk *= T->extent[d];
  if (k >= nk) return;
  int64_t ooff[CUBED_MAX_OUTS] = {};
  int64_t kk = k;
  for (int d = kd1 - 1; d >= kd0; --d) {
    int64_t q, c;
    divmod64(kk, T->extent[d], q, c);
    kk = q;
    for (int o = 0; o < CUBED_MAX_OUTS; ++o) ooff[o] += c * T->out_stride[o][d];
  }
  const int64_t n = ntasks * max_kept;
  Acc fin[CUBED_MAX_FIELDS][1];
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
    fin[f][0] = f < P.nfields ? soa[f * n + i] : acc_init(CUBED_R_NONE, 0);
  finish<1>(P, T, fin, ooff);
}

// Grouped finish: tasks [gs[g], gs[g+1]) are pieces of one output box (a
// task split where its inputs straddle source chunks along a reduced dim);
// their SoA partials are combined in piece order and the first piece's
// output views receive the epilogue.
CUBED_DEV void finish_groups_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, const int64_t* __restrict__ gs, int64_t ngroups,
    int kd0, int kd1) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t g = i / max_kept, k = i % max_kept;
  if (g >= ngroups) return;
  const int64_t t0 = gs[g], t1 = gs[g + 1];
  const cubed_task_t* __restrict__ T = tasks + t0;
  int64_t nk = 1;
  for (int d = kd0; d < kd1; ++d) nk *= T->extent[d];
  if (k >= nk) return;
  int64_t ooff[CUBED_MAX_OUTS] = {};
  int64_t kk = k;
  for (int d = kd1 - 1; d >= kd0; --d) {
    int64_t q, c;
    divmod64(kk, T->extent[d], q, c);
    kk = q;
    for (int o = 0; o < CUBED_MAX_OUTS; ++o) ooff[o] += c * T->out_stride[o][d];
  }
  const int64_t n = ntasks * max_kept;
  Acc x[CUBED_MAX_FIELDS];
  soa_load(P, soa, n, t0 * max_kept + k, x);
  for (int64_t t = t0 + 1; t < t1; ++t) {
    Acc y[CUBED_MAX_FIELDS];
    soa_load(P, soa, n, t * max_kept + k, y);
    fields_combine(x, y, P);
  }
  Acc fin[CUBED_MAX_FIELDS][1];
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f) fin[f][0] = x[f];
  finish<1>(P, T, fin, ooff);
}

// Per-group combine without the epilogue (multi-GPU pieces): rows
// [gs[g], gs[g+1]) of the row partials fold, in row order, into
// out[f][g][k] (max_kept_out per group, identity past a group's extent) --
// the same layout on every rank, for the cross-rank combine.
CUBED_DEV void combine_groups_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, const int64_t* __restrict__ gs, int64_t ngroups,
    int64_t max_kept_out, Acc* __restrict__ out, int kd0, int kd1) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t g = i / max_kept_out, k = i % max_kept_out;
  if (g >= ngroups) return;
  const int64_t t0 = gs[g], t1 = gs[g + 1];
  const cubed_task_t* __restrict__ T = tasks + t0;
  int64_t nk = 1;
  for (int d = kd0; d < kd1; ++d) nk *= T->extent[d];
  const int64_t n = ntasks * max_kept, no = ngroups * max_kept_out;
  Acc x[CUBED_MAX_FIELDS];
  if (k < nk) {
    soa_load(P, soa, n, t0 * max_kept + k, x);
    for (int64_t t = t0 + 1; t < t1; ++t) {
      Acc y[CUBED_MAX_FIELDS];
      soa_load(P, soa, n, t * max_kept + k, y);
      fields_combine(x, y, P);
    }
  } else {
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) x[f] = acc_init(P.field_rop[f], P.field_acc[f]);
  }
  for (int f = 0; f < P.nfields && f < CUBED_MAX_FIELDS; ++f) out[f * no + i] = x[f];
}

// Split accumulators shared between workgroups (a column block's splits, a
// fold group's runs): agent-scope relaxed atomics, i.e. stores written
// through to memory and loads that miss the (per-XCD, non-coherent) L2.
CUBED_DEV void store_through(Acc* p, Acc v) {
  __hip_atomic_store(&p->i, v.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
CUBED_DEV Acc load_through(const Acc* p) {
  Acc v;
  v.i = __hip_atomic_load(&p->i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return v;
}

// Workgroup fold of per-thread accumulators (64-wide shuffle tree, then the
// waves in order through LDS); the result lands in thread 0's x.
CUBED_DEV void block_fold(const cubed_program_t& P, Acc (&a)[CUBED_MAX_FIELDS],
                          Acc (&red)[kBlock / 64][CUBED_MAX_FIELDS], Acc (&x)[CUBED_MAX_FIELDS]) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    Acc b[CUBED_MAX_FIELDS];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) b[f] = shfl_xor_acc(a[f], m);
    fields_combine(a, b, P);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) red[wave][f] = a[f];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) x[f] = red[0][f];
    for (int w = 1; w < kBlock / 64; ++w) fields_combine(x, red[w], P);
  }
}

// A fold group's result (thread 0): stored to out[f][g] and, with an
// epilogue program (the lifted reduction's, nred = ndim), finished into the
// group's output (fin_tasks[g], one element) right here.
// The epilogue program is first copied into LDS by the whole workgroup (one
// round trip): the interpreter's chain of dependent program reads then costs
// LDS latency instead of a global-memory trip each (the separate finish
// launch this replaces took 7 us for ONE element).
CUBED_DEV void stage_program(cubed_program_t& dst, const cubed_program_t* __restrict__ src) {
  static_assert(sizeof(cubed_program_t) % 16 == 0, "program struct in 16-byte units");
  for (int i = threadIdx.x; i < (int)(sizeof(cubed_program_t) / 16); i += kBlock)
    reinterpret_cast<uint4*>(&dst)[i] = reinterpret_cast<const uint4*>(src)[i];
  __syncthreads();
}
CUBED_DEV void fold_group_done(const cubed_program_t& P, Acc (&x)[CUBED_MAX_FIELDS], Acc* __restrict__ out,
                               int64_t ngroups, int64_t g, const cubed_program_t* Pfin,
                               const cubed_task_t* __restrict__ fin_tasks) {
  for (int f = 0; f < P.nfields && f < CUBED_MAX_FIELDS; ++f) out[f * ngroups + g] = x[f];
  if (Pfin) {
    Acc fin[CUBED_MAX_FIELDS][1];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f) fin[f][0] = x[f];
    int64_t ooff[CUBED_MAX_OUTS] = {};
    finish<1>(*Pfin, fin_tasks + g, fin, ooff);
  }
}

// Full reductions run "lifted": the innermost reduced dims are walked as if
// kept (kernel A / streaming, one lane per element, rows in flight), leaving
// per-element partials; this fold then reduces each group's rows AND kept
// elements to one accumulator per field: one workgroup per group, a strided
// pass per thread, then the 64-wide shuffle tree and LDS across the waves.
// FIN_MAIN (the JIT fold, cubed_fold_groups_compiled): the epilogue is the
// main program's own (constant-folded, no LDS staging); fin_tasks gives the
// outputs.
template <bool FIN_MAIN = false>
CUBED_DEV void fold_groups_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, const int64_t* __restrict__ gs, int64_t ngroups,
    Acc* __restrict__ out, int kd0, int kd1, const cubed_program_t* __restrict__ Pfin,
    const cubed_task_t* __restrict__ fin_tasks) {
  __shared__ Acc red[kBlock / 64][CUBED_MAX_FIELDS];
  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  if (g >= ngroups) return;
  const int64_t n = ntasks * max_kept;
  Acc a[CUBED_MAX_FIELDS];
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f) a[f] = acc_init(P.field_rop[f], P.field_acc[f]);
  // the group's rows are one flat run of SoA entries: partials mode leaves
  // the identity past every task's kept extent (collect_body, stream_body)
  for (int64_t e = gs[g] * max_kept + threadIdx.x; e < gs[g + 1] * max_kept; e += kBlock) {
    Acc y[CUBED_MAX_FIELDS];
    soa_load(P, soa, n, e, y);
    fields_combine(a, y, P);
  }
  Acc x[CUBED_MAX_FIELDS];
  block_fold(P, a, red, x);
  if constexpr (FIN_MAIN) {
    if (threadIdx.x == 0) fold_group_done(P, x, out, ngroups, g, &P, fin_tasks);
  } else {
    __shared__ __attribute__((aligned(16))) cubed_program_t pfin;
    if (Pfin) stage_program(pfin, Pfin);
    if (threadIdx.x == 0) fold_group_done(P, x, out, ngroups, g, Pfin ? &pfin : nullptr, fin_tasks);
  }
}

// Split fold for few groups of many elements (e.g. one scalar over 720
// source chunks' per-element partials): a group's SoA entries are the flat
// run [gs[g], gs[g+1]) x max_kept, cut
// into nsplit equal runs; workgroup (g, s) folds run s and leaves its result
// in out_split[f][g][s] (write-through), and the LAST of the group's nsplit
// workgroups to arrive (arrival counter per group, self-resetting) folds the
// nsplit results and finishes the group: one launch.  A fixed
// (shape-determined) order, so deterministic.
template <bool FIN_MAIN = false>
CUBED_DEV void fold_groups_split_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t max_kept, const Acc* __restrict__ soa, const int64_t* __restrict__ gs, int64_t ngroups,
    int64_t nsplit, Acc* __restrict__ out_split, Acc* __restrict__ out, int kd0, int kd1,
    const cubed_program_t* __restrict__ Pfin, const cubed_task_t* __restrict__ fin_tasks) {
  __shared__ Acc red[kBlock / 64][CUBED_MAX_FIELDS];
  __shared__ int last_arrival;
  const int64_t b = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  if (b >= ngroups * nsplit) return;
  const int64_t g = b / nsplit, sp = b - g * nsplit;
  const int64_t n = ntasks * max_kept;
  const int64_t base = gs[g] * max_kept, E = (gs[g + 1] - gs[g]) * max_kept;
  const int64_t e0 = base + E * sp / nsplit, e1 = base + E * (sp + 1) / nsplit;
  Acc a[CUBED_MAX_FIELDS];
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f) a[f] = acc_init(P.field_rop[f], P.field_acc[f]);
  // (a flat run: the identity past every task's kept extent, see above;
  // runs of ~2 entries per thread -- an 8-deep batched form measured 58 us
  // against 39 for the vorticity fold)
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kBlock) {
    Acc y[CUBED_MAX_FIELDS];
    soa_load(P, soa, n, e, y);
    fields_combine(a, y, P);
  }
  Acc x[CUBED_MAX_FIELDS];
  block_fold(P, a, red, x);
  const int64_t ns = ngroups * nsplit;
  uint32_t* cnt = (uint32_t*)(out_split + (int64_t)P.nfields * ns);
  if (threadIdx.x == 0) {
    for (int f = 0; f < P.nfields && f < CUBED_MAX_FIELDS; ++f) store_through(&out_split[f * ns + b], x[f]);
    // the stores complete before the arrival counts (MI355X_MICROARCH.md
    // "Correctness boundaries": write-through stores, drained, then the count)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(cnt + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int lastv = old == (uint32_t)(nsplit - 1);
    if (lastv) __hip_atomic_store(cnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_arrival = lastv;
  }
  __syncthreads();
  if (!last_arrival) return;
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f) a[f] = acc_init(P.field_rop[f], P.field_acc[f]);
  for (int64_t s = threadIdx.x; s < nsplit; s += kBlock) {
    Acc y[CUBED_MAX_FIELDS];
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
      y[f] = f < P.nfields ? load_through(&out_split[f * ns + g * nsplit + s]) : acc_init(P.field_rop[f], P.field_acc[f]);
    fields_combine(a, y, P);
  }
  __syncthreads();  // red is reused
  block_fold(P, a, red, x);
  if constexpr (FIN_MAIN) {
    if (threadIdx.x == 0) fold_group_done(P, x, out, ngroups, g, &P, fin_tasks);
  } else {
    __shared__ __attribute__((aligned(16))) cubed_program_t pfin;
    if (Pfin) stage_program(pfin, Pfin);
    if (threadIdx.x == 0) fold_group_done(P, x, out, ngroups, g, Pfin ? &pfin : nullptr, fin_tasks);
  }
}

// Combine nparts SoA partial blocks (e.g. all-gathered from the ranks) in
// part order: out[f][i] = part0 (+) part1 (+) ...  Used for the fields RCCL
// cannot reduce with numpy's semantics (max/min with NaN, prod, any/all).
CUBED_DEV void combine_parts_body(const cubed_program_t& P, const Acc* __restrict__ parts,
                                  int32_t nparts, int64_t n, Acc* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t block = (int64_t)P.nfields * n;
  Acc x[CUBED_MAX_FIELDS];
  soa_load(P, parts, n, i, x);
  for (int r = 1; r < nparts; ++r) {
    Acc y[CUBED_MAX_FIELDS];
    soa_load(P, parts + r * block, n, i, y);
    fields_combine(x, y, P);
  }
  for (int f = 0; f < P.nfields && f < CUBED_MAX_FIELDS; ++f) out[f * n + i] = x[f];
}

// ---------------------------------------------------------------- streaming fast path
CUBED_DEV void ld4(float (&o)[4], const CUBED_G float* p) {
  const f32x4 v = __builtin_nontemporal_load((const CUBED_G f32x4*)p);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
CUBED_DEV void ld4(double (&o)[4], const CUBED_G double* p) {
  const f64x2 a = __builtin_nontemporal_load((const CUBED_G f64x2*)p);
  const f64x2 b = __builtin_nontemporal_load((const CUBED_G f64x2*)(p + 2));
  o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}
// Cached form for leaves re-read along the reduced dim (reduced stride 0:
// a broadcast operand such as x in a[1:] * x): non-temporal loads would send
// every re-read back to HBM.
template <typename V>
CUBED_DEV void ld4c(V (&o)[4], const CUBED_G V* p) {
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = p[j];
}
template <>
CUBED_DEV void ld4c<float>(float (&o)[4], const CUBED_G float* p) {
  const f32x4 v = *(const CUBED_G f32x4*)p;
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <>
CUBED_DEV void ld4c<double>(double (&o)[4], const CUBED_G double* p) {
  const f64x2 a = *(const CUBED_G f64x2*)p;
  const f64x2 b = *(const CUBED_G f64x2*)(p + 2);
  o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}
CUBED_DEV void ld4(int64_t (&o)[4], const CUBED_G int64_t* p) {
  const i64x2 a = __builtin_nontemporal_load((const CUBED_G i64x2*)p);
  const i64x2 b = __builtin_nontemporal_load((const CUBED_G i64x2*)(p + 2));
  o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}

// 8-byte elements: a thread's 4 kept elements are two pairs dk apart (the
// lane-interleaved mapping of stream_body), each pair one 16-byte load, so
// every load instruction of a wave reads 1 KiB contiguous.
template <typename V>
CUBED_DEV void ld4h(V (&o)[4], const CUBED_G V* p, int64_t dk) {
  using P2 = typename conditional<__is_same(V, double), f64x2, i64x2>::type;
  // non-temporal: measured 7 % faster than cached loads on config 1 and the
  // vorticity pieces (each byte is read once)
#ifdef CUBED_LD64_CACHED
  const P2 a = *((const CUBED_G P2*)p);
  const P2 b = *((const CUBED_G P2*)(p + dk));
#else
  const P2 a = __builtin_nontemporal_load((const CUBED_G P2*)p);
  const P2 b = __builtin_nontemporal_load((const CUBED_G P2*)(p + dk));
#endif
  o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}
template <typename V>
CUBED_DEV void ld4ch(V (&o)[4], const CUBED_G V* p, int64_t dk) {
  o[0] = p[0]; o[1] = p[1]; o[2] = p[dk]; o[3] = p[dk + 1];
}

template <typename V>
CUBED_DEV void ld4s(V (&o)[4], const CUBED_G V* p, bool streamed) {
  if (streamed) ld4(o, p); else ld4c<V>(o, p);
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
  V src[CUBED_MAX_FIELDS][4];
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
    if (f < P.nfields) fetch(regs, P.field_src[f], src[f]);
  fields_add<V, 4, true>(acc, src, P);
}

// Rows [lo, hi) of W kept VEC groups (group j at element offset go[j], pair
// distance dk[j] for 8-byte elements, gv[j] = inside the kept extent): U rows
// x W groups of loads in flight, then the program and the accumulation per
// group; MIXED: some leaves are re-read (cached loads).  p[l] points at the
// row's element 0.
template <typename V, int NL, int U, int W, bool MIXED>
CUBED_DEV void stream_rows(Acc (&acc)[W][CUBED_MAX_FIELDS][4], Regs<V, 4>& regs,
                           const cubed_program_t& P, const CUBED_G V* (&p)[NL],
                           const int64_t (&rs)[NL], int64_t lo, int64_t hi,
                           const int64_t (&go)[W], const int64_t (&dk)[W], const bool (&gv)[W]) {
  constexpr bool IL = sizeof(V) == 8;
  int64_t r = lo;
  // one group's 4 elements of leaf l at row pointer q
  auto ld_group = [&](V (&o)[4], const CUBED_G V* q, int j) {
    if (!gv[j]) {
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (V)0;
      return;
    }
    if constexpr (IL) ld4h<V>(o, q + go[j], dk[j]);
    else ld4(o, q + go[j]);
  };
  // leaves with reduced stride 0 (broadcast operands) are loop-invariant:
  // loaded once here instead of once per row
  V inv[W][NL][4];
  if (MIXED && lo < hi) {
#pragma unroll
    for (int j = 0; j < W; ++j)
#pragma unroll
      for (int l = 0; l < NL; ++l)
        if (rs[l] == 0) {
          if (!gv[j]) {
#pragma unroll
            for (int e = 0; e < 4; ++e) inv[j][l][e] = (V)0;
          } else if constexpr (IL) {
            ld4ch<V>(inv[j][l], p[l] + go[j], dk[j]);
          } else {
            ld4c<V>(inv[j][l], p[l] + go[j]);
          }
        }
  }
  auto load_batch = [&](V (&buf)[U][W][NL][4]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < W; ++j)
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          if (MIXED && rs[l] == 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) buf[u][j][l][e] = inv[j][l][e];
          } else {
            ld_group(buf[u][j][l], p[l] + u * rs[l], j);
          }
        }
#pragma unroll
    for (int l = 0; l < NL; ++l) p[l] += U * rs[l];
  };
  auto reduce_batch = [&](V (&buf)[U][W][NL][4]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < W; ++j) {
        set_leaves<NL, V>(regs, buf[u][j]);
        CUBED_RUN_PROLOGUE(V, 4, regs);
        accumulate_nocount<V>(acc[j], regs, P);
      }
  };
  // (a software-pipelined form -- batch r + U loading while batch r reduces --
  // and U = 2 / 8 measured equal or slower on quad-means, config 1 and
  // vorticity: profiles/r02_stream_ab.log)
  for (; r + U <= hi; r += U) {
    V buf[U][W][NL][4];
    load_batch(buf);
    reduce_batch(buf);
  }

  for (; r < hi; ++r) {
    V buf[W][NL][4];
#pragma unroll
    for (int j = 0; j < W; ++j)
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        if (MIXED && rs[l] == 0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) buf[j][l][e] = inv[j][l][e];
        } else {
          ld_group(buf[j][l], p[l], j);
        }
      }
#pragma unroll
    for (int j = 0; j < W; ++j) {
      set_leaves<NL, V>(regs, buf[j]);
      CUBED_RUN_PROLOGUE(V, 4, regs);
      accumulate_nocount<V>(acc[j], regs, P);
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) p[l] += rs[l];
  }
}

// W: kept VEC groups per thread (stream_groups()).  The 64 lanes of a wave
// own a block of 256 * W consecutive kept elements: group j of lane L starts
// at block + 256 j + 4 L (4-byte elements: every 16-byte load instruction of
// the wave reads 1 KiB contiguous), or for 8-byte elements at
// block + 256 j + 2 L as the pairs (k, k+1), (k+128, k+129) (again 1 KiB per
// instruction); a last partial 256-element run of 8-byte elements falls back
// to 4 consecutive elements per lane (dk = 2).  W = 1 is the round-2 mapping.
// SPLIT: the kernel variant for nsplit > 1 (the split handshake and fold);
// the unsplit variant carries none of it (same registers as a plain stream).
template <typename V, int NL, int U, int W = 1, bool SPLIT = false>
CUBED_DEV void stream_body(
    const cubed_program_t& P, const cubed_task_t* __restrict__ tasks, int64_t ntasks,
    int64_t bpt, int32_t nsplit, Acc* __restrict__ ws, int64_t max_kept) {
  // XCD-contiguous runs: dispatch is round-robin over the 8 XCDs, so
  // workgroup g runs logical index (g % 8) * (G / 8) + g / 8 -- each XCD
  // walks one contiguous run of (task, split, column block), and the column
  // blocks either side of a 128-B line a misaligned row splits share its L2
  // (the launcher pads the grid to a multiple of 8; the surplus exits).
  // Vorticity -2 %, config 1 -0.8 %, others equal (profiles/r03_stream_xcd_ab.log)
  const int64_t G = (int64_t)gridDim.x * gridDim.y;
  int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);
  // nr = 0 (map), 1 (rows) or 2 (chunks x rows: a reduction chain whose
  // chunks sit at a slot stride that is not the rows' own continuation)
  const int nr = P.nred;
  auto nrd_of = [&](const cubed_task_t* T) {
    return (nr == 2 ? T->extent[0] : 1) * (nr ? T->extent[nr - 1] : 1);
  };
  // One segment: rows [lo, hi) of column block b of task t, split slot s of
  // nsp (lo < 0: the uniform split's range of slot s).
  auto segment = [&](int64_t t, int64_t b, int s, int nsp, int64_t lo, int64_t hi) {
  const cubed_task_t* __restrict__ T = tasks + t;
  const int64_t nk = T->extent[nr];
  const int64_t nrow = nr ? T->extent[nr - 1] : 1;
  const int64_t nq = nr == 2 ? T->extent[0] : 1;
  const int64_t nrd = nq * nrow;
  // thread slots: whole waves of W groups each
  const int64_t slots = ((nk + 256 * W - 1) / (256 * W)) * 64;
  // (a balanced run is clamped to the task's own extent: the host promises
  // equal extents, the clamp keeps a broken promise inside the task)
  const int64_t r0 = lo < 0 ? nrd * s / nsp : (lo < nrd ? lo : nrd);
  const int64_t r1 = lo < 0 ? nrd * (s + 1) / nsp : (hi < nrd ? hi : nrd);

  const CUBED_G V* base[NL];
  int64_t rs[NL], qs[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    base[l] = (const CUBED_G V*)(uintptr_t)T->leaf_base[l];
    rs[l] = nr ? T->leaf_stride[l][nr - 1] : 0;
    qs[l] = nr == 2 ? T->leaf_stride[l][0] : 0;
  }

  // leaves re-read along the rows (stride 0) take cached loads; the common
  // all-streamed case keeps the loop free of per-leaf branches
  bool all_streamed = true;
#pragma unroll
  for (int l = 0; l < NL; ++l) all_streamed = all_streamed && rs[l] != 0;

  constexpr bool IL = sizeof(V) == 8;
  // a wave's W groups of 4 kept elements (the lane-interleaved mapping above)
  auto groups_of = [&](int64_t it, int64_t (&go)[W], int64_t (&dk)[W], bool (&gv)[W]) {
    const int64_t wb = (it >> 6) * (256 * W);
    const int lane = (int)(it & 63);
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const int64_t sub = wb + 256 * j;
      if (IL && sub + 256 <= nk) {
        go[j] = sub + 2 * lane;
        dk[j] = 128;
      } else {
        go[j] = sub + 4 * lane;
        dk[j] = 2;
      }
      gv[j] = go[j] + 4 <= nk || (dk[j] == 128);
    }
  };
  if (P.nfields == 0) {
    for (int64_t it = b * kBlock + threadIdx.x; it < slots; it += bpt * kBlock) {
      int64_t go[W], dk[W];
      bool gv[W];
      groups_of(it, go, dk, gv);
      Regs<V, 4> regs;
#pragma unroll
      for (int j = 0; j < W; ++j) {
        if (!gv[j]) continue;
        V buf[NL][4];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          if constexpr (IL) ld4h<V>(buf[l], base[l] + go[j], dk[j]);
          else ld4(buf[l], base[l] + go[j]);
        }
        set_leaves<NL, V>(regs, buf);
        CUBED_RUN_PROLOGUE(V, 4, regs);
#pragma unroll
        for (int o = 0; o < CUBED_MAX_OUTS; ++o) {
          if (o < P.nouts) {
            V X[4];
            fetch(regs, P.out_src[o], X);
            if constexpr (IL) {
              V X0[2] = {X[0], X[1]}, X1[2] = {X[2], X[3]};
              stv<V, 2>((char*)T->out_base[o], go[j], P.out_dtype[o], X0);
              stv<V, 2>((char*)T->out_base[o], go[j] + dk[j], P.out_dtype[o], X1);
            } else {
              stv<V, 4>((char*)T->out_base[o], go[j], P.out_dtype[o], X);
            }
          }
        }
      }
    }
    return;
  }

  // ---- reductions.  Three endings per kept element:
  //  * unsplit: the epilogue (or, in partials mode, the SoA partials) here;
  //  * split: every workgroup leaves its split's accumulators in the
  //    workspace, and the LAST workgroup of the nsplit splits of one column
  //    block to arrive (a per-(task, block) arrival counter) folds them in
  //    split order -- k_finalize's order, so the same bits -- and finishes.
  //    No second launch.  COUNT fields are never stored: every split counts
  //    its own trip count, the fold takes the whole reduced extent.
  // Workspace layout: [SoA partials (partials mode)] [split accumulators]
  // [arrival counters, uint32 per (task, column block)]; the counters start at
  // zero (the host zeroes the workspace once) and the last arrival resets
  // its counter, so they are zero again after every launch.
  const bool partials = (P.mode & CUBED_MODE_PARTIALS) != 0;
  const int nf = P.nfields;
  const int64_t nsoa = ntasks * max_kept;
  const int64_t nslots = nsplit < 0 ? -nsplit : nsplit;  // split slots in the workspace
  Acc* __restrict__ soa = ws - (int64_t)nf * nsoa;
  const int64_t slots_max = ((max_kept + 256 * W - 1) / (256 * W)) * 64;
  const int64_t nblk = (slots_max + kBlock - 1) / kBlock;
  uint32_t* __restrict__ cnt = (uint32_t*)(ws + (int64_t)nslots * nsoa * nf);
  __shared__ int last_arrival;
  // partials mode writes every element < max_kept (the identity past an
  // edge task's extent), so every column block of max_kept takes part
  const int64_t wslots = partials ? slots_max : slots;
  auto store_soa = [&](int64_t el, const Acc (&x)[CUBED_MAX_FIELDS], bool valid) {
    if (el >= max_kept) return;
    if (P.mode & CUBED_MODE_OWNER_MAJOR) {
      // straight into the reduce-scatter's owner-major order (dist.ScatterCombine):
      // group g's elements to rank g % W's slot g / W
      const int64_t mko = P.consts[CUBED_MAX_CONSTS - 3].i, wr = P.consts[CUBED_MAX_CONSTS - 2].i,
                    lr = P.consts[CUBED_MAX_CONSTS - 1].i;
      const int64_t i = t * max_kept + el, g = i / mko;
      Acc* __restrict__ d = soa + ((g % wr) * lr + g / wr) * mko + (i - g * mko);
#pragma unroll
      for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
        if (f < nf && P.field_rop[f] != CUBED_R_COUNT) *d = valid ? x[f] : acc_init(P.field_rop[f], P.field_acc[f]);
      return;
    }
#pragma unroll
    for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
      if (f < nf && (!(P.mode & CUBED_MODE_HOST_COUNT) || P.field_rop[f] != CUBED_R_COUNT))
        soa[f * nsoa + t * max_kept + el] = valid ? x[f] : acc_init(P.field_rop[f], P.field_acc[f]);
  };
  // (block-uniform trip count: the arrival handshake below has barriers)
  for (int64_t bb = b * kBlock; bb < wslots; bb += bpt * kBlock) {
    const int64_t it = bb + threadIdx.x;
    int64_t go[W], dk[W];
    bool gv[W];
    groups_of(it, go, dk, gv);
    bool any = false;
#pragma unroll
    for (int j = 0; j < W; ++j) any = any || gv[j];
    Regs<V, 4> regs;
    Acc acc[W][CUBED_MAX_FIELDS][4];
#pragma unroll
    for (int j = 0; j < W; ++j)
#pragma unroll
      for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[j][f][e] = acc_init(P.field_rop[f], P.field_acc[f]);

    // flattened reduced range [r0, r1) = (chunk q, row) pairs in order
    for (int64_t q = nrow ? r0 / nrow : 0; any && q < nq && q * nrow < r1; ++q) {
      const int64_t lo = (r0 > q * nrow ? r0 : q * nrow) - q * nrow;
      const int64_t hi = (r1 < (q + 1) * nrow ? r1 : (q + 1) * nrow) - q * nrow;
      const CUBED_G V* p[NL];
#pragma unroll
      for (int l = 0; l < NL; ++l) p[l] = base[l] + q * qs[l] + lo * rs[l];
      if (all_streamed)
        stream_rows<V, NL, U, W, false>(acc, regs, P, p, rs, lo, hi, go, dk, gv);
      else
        stream_rows<V, NL, U, W, true>(acc, regs, P, p, rs, lo, hi, go, dk, gv);
    }

    if constexpr (SPLIT) {
      Acc* __restrict__ w = ws + ((int64_t)(s * ntasks + t) * max_kept) * nf;
#pragma unroll
      for (int j = 0; j < W; ++j) {
        if (!gv[j]) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t el = go[j] + (e >> 1) * dk[j] + (e & 1);
#pragma unroll
          for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
            if (f < nf && P.field_rop[f] != CUBED_R_COUNT) store_through(&w[el * nf + f], acc[j][f][e]);
        }
      }
      // Handshake without L2 maintenance (MI355X_MICROARCH.md "Correctness
      // boundaries", the sc1 form): the accumulators above are write-through
      // stores (agent-scope relaxed atomics: sc1) -- the 8 XCDs' L2s are not
      // coherent with each other, and an agent-scope release/acquire fence
      // would write back and invalidate this XCD's whole L2 per workgroup
      // (measured 2x slower on the per-rank share).  Every storing wave
      // drains its stores (vmcnt(0)) before the barrier, so they are complete
      // before one lane counts the arrival; the fold reads them with sc1
      // loads after the second barrier.
      // (inline asm: the builtin form was dropped by the wait-count pass,
      // which does not order stores before a barrier)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t* c = cnt + t * nblk + bb / kBlock;
        const uint32_t old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int lastv = old == (uint32_t)(nsp - 1);
        if (lastv) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_arrival = lastv;
      }
      __syncthreads();
      if (!last_arrival) continue;
      // the other splits' accumulators: read past this XCD's L2 (load_through)
      // fold splits 0..nsplit-1 in order (this workgroup's own included).
      // The loads are agent-scope atomics, which keep their program order:
      // every load of a batch (4 splits x 4 elements) is issued before the
      // first combine, so a batch costs one memory round trip
      const int64_t sstride = nsoa * nf;
      auto stored = [&](int f) { return f < nf && P.field_rop[f] != CUBED_R_COUNT; };
#pragma unroll
      for (int j = 0; j < W; ++j) {
        if (!gv[j]) continue;
        const Acc* __restrict__ pe[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          pe[e] = ws + ((int64_t)t * max_kept + go[j] + (e >> 1) * dk[j] + (e & 1)) * nf;
        Acc x[4][CUBED_MAX_FIELDS];
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
            x[e][f] = stored(f) ? load_through(pe[e] + f) : acc_init(P.field_rop[f], P.field_acc[f]);
        int sp = 1;
        for (; sp + 4 <= nsp; sp += 4) {
          Acc v[4][4][CUBED_MAX_FIELDS];
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
              for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
                v[u][e][f] = stored(f) ? load_through(pe[e] + (int64_t)(sp + u) * sstride + f)
                                       : acc_init(P.field_rop[f], P.field_acc[f]);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int u = 0; u < 4; ++u) fields_combine(x[e], v[u][e], P);
        }
        for (; sp < nsp; ++sp) {
          Acc v[4][CUBED_MAX_FIELDS];
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
              v[e][f] = stored(f) ? load_through(pe[e] + (int64_t)sp * sstride + f)
                                  : acc_init(P.field_rop[f], P.field_acc[f]);
#pragma unroll
          for (int e = 0; e < 4; ++e) fields_combine(x[e], v[e], P);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int f = 0; f < CUBED_MAX_FIELDS; ++f) {
            if (f < nf && P.field_rop[f] == CUBED_R_COUNT) x[e][f].i = nrd;
            acc[j][f][e] = x[e][f];
          }
      }
    } else {
#pragma unroll
      for (int j = 0; j < W; ++j)
#pragma unroll
        for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
          if (f < nf && P.field_rop[f] == CUBED_R_COUNT)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[j][f][e].i += r1 - r0;
    }

#pragma unroll
    for (int j = 0; j < W; ++j) {
      if (partials) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t el = go[j] + (e >> 1) * dk[j] + (e & 1);
          Acc x[CUBED_MAX_FIELDS];
#pragma unroll
          for (int f = 0; f < CUBED_MAX_FIELDS; ++f) x[f] = acc[j][f][e];
          store_soa(el, x, gv[j]);
        }
        continue;
      }
      if (!gv[j]) continue;
      int64_t ooff[CUBED_MAX_OUTS];
#pragma unroll
      for (int o = 0; o < CUBED_MAX_OUTS; ++o) ooff[o] = go[j];
      if constexpr (IL) {
        Acc a0[CUBED_MAX_FIELDS][2], a1[CUBED_MAX_FIELDS][2];
#pragma unroll
        for (int f = 0; f < CUBED_MAX_FIELDS; ++f) {
          a0[f][0] = acc[j][f][0]; a0[f][1] = acc[j][f][1];
          a1[f][0] = acc[j][f][2]; a1[f][1] = acc[j][f][3];
        }
        int64_t o1[CUBED_MAX_OUTS];
#pragma unroll
        for (int o = 0; o < CUBED_MAX_OUTS; ++o) o1[o] = ooff[o] + dk[j];
        finish<2>(P, T, a0, ooff);
        finish<2>(P, T, a1, o1);
      } else {
        finish<4>(P, T, acc[j], ooff);
      }
    }
  }
  };

  // Balanced split (SPLIT variant, nsplit < 0 = -slots; the host's
  // CUBED_MODE_STREAM_EVEN: every task the same reduced extent): the (task,
  // column block, row) units of the launch, in that order, are cut into G
  // equal runs, one per workgroup -- a run may end in one column block and
  // continue in the next, so every CU streams the same number of rows (a
  // uniform split leaves G mod blocks CUs idle: 11 of 256 for 49 column
  // blocks).  Column block c's contributors are the workgroups whose runs
  // meet it, in row order: slot g - owner(first row); the last to arrive
  // folds them in that order.  One call site of segment() (it is inlined).
  const bool bal = SPLIT && nsplit < 0;
  int64_t nru = 1, Ut = 1, u = 0, S1 = 0;
  if (bal) {
    nru = nrd_of(tasks);
    Ut = ntasks * bpt * nru;
    u = g * Ut / G;
    S1 = (g + 1) * Ut / G;
    if (u >= S1) return;
  } else if (g / bpt / nsplit >= ntasks) {
    return;
  }
  for (;;) {
    int64_t t, b, lo = -1, hi = -1;
    int s, nsp = nsplit;
    if (bal) {
      const int64_t c = u / nru;
      lo = u - c * nru;
      hi = S1 - c * nru < nru ? S1 - c * nru : nru;
      const int64_t first = ((c * nru + 1) * G - 1) / Ut, last = (((c + 1) * nru) * G - 1) / Ut;
      t = c / bpt;
      b = c % bpt;
      s = (int)(g - first);
      nsp = (int)(last - first + 1);
      u = c * nru + hi;
    } else {
      b = g % bpt;
      const int64_t rest = g / bpt;
      s = (int)(rest % nsplit);
      t = rest / nsplit;
    }
    segment(t, b, s, nsp, lo, hi);
    if (!bal || u >= S1) break;
  }
}

}  // namespace cubed
