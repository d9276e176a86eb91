// vm.h -- the per-element program interpreter of the fused chunk kernels.
//
// A fused Cubed pipeline (elementwise chain -> optional reduction ->
// epilogue, see DESIGN.md "Fused chunk programs") is lowered on the host to
// a short two-address program over CUBED_NREGS registers, each holding VEC
// consecutive elements of the thread.  The opcode and the register operands
// are wave-uniform (they live in the kernel-argument segment and are read
// with scalar loads), so every switch below is a scalar branch: the VALU
// only executes the selected op on the VEC elements.  Register operands are
// resolved by fetch/op/write-back switches so the register file stays in
// VGPRs (a runtime-indexed array would be demoted to scratch).
#pragma once
#include "common.h"

namespace cubed {

template <typename V, int VEC>
struct Regs {
  V r0[VEC], r1[VEC], r2[VEC], r3[VEC], r4[VEC], r5[VEC];
};

#define CUBED_REG_SWITCH(idx, STMT) \
  switch (idx) {                    \
    case 0: { auto& R = regs.r0; STMT; } break; \
    case 1: { auto& R = regs.r1; STMT; } break; \
    case 2: { auto& R = regs.r2; STMT; } break; \
    case 3: { auto& R = regs.r3; STMT; } break; \
    case 4: { auto& R = regs.r4; STMT; } break; \
    default: { auto& R = regs.r5; STMT; } break; \
  }

template <typename V, int VEC>
CUBED_DEV void fetch(const Regs<V, VEC>& regs, int idx, V (&X)[VEC]) {
  CUBED_REG_SWITCH(idx, { _Pragma("unroll") for (int j = 0; j < VEC; ++j) X[j] = R[j]; })
}
template <typename V, int VEC>
CUBED_DEV void put(Regs<V, VEC>& regs, int idx, const V (&X)[VEC]) {
  CUBED_REG_SWITCH(idx, { _Pragma("unroll") for (int j = 0; j < VEC; ++j) R[j] = X[j]; })
}
#define CUBED_EACH(EXPR) _Pragma("unroll") for (int j = 0; j < VEC; ++j) { const V x = X[j]; (void)x; X[j] = (EXPR); }
#define CUBED_EACH2(EXPR) _Pragma("unroll") for (int j = 0; j < VEC; ++j) { const V x = X[j]; const V y = Y[j]; X[j] = (EXPR); }

// CAST: round the value (of source dtype s) to dtype t, keeping it in V.
template <typename V>
CUBED_DEV V cast_val(V x, int t, int s) {
  if (t == CUBED_BOOL) return (x != (V)0) ? (V)1 : (V)0;
  if constexpr (is_same_v<V, int64_t>) {
    switch (t) {
      case CUBED_I8: return (int64_t)(int8_t)x;
      case CUBED_I16: return (int64_t)(int16_t)x;
      case CUBED_I32: return (int64_t)(int32_t)x;
      case CUBED_U8: return (int64_t)(uint8_t)x;
      case CUBED_U16: return (int64_t)(uint16_t)x;
      case CUBED_U32: return (int64_t)(uint32_t)x;
      default: return x;
    }
  } else {
    switch (t) {
      case CUBED_F32: return (V)(float)x;
      case CUBED_F64: return x;
      case CUBED_F16: return (V)(float)(_Float16)x;
      case CUBED_BF16: return (V)bf16_to_f32(f32_to_bf16((float)x));
      default: break;
    }
    // integer targets: float sources truncate toward zero, then wrap
    int64_t i = dt_is_float(s) ? f2i64((double)x) : f2i64((double)x);
    switch (t) {
      case CUBED_I8: return (V)(int8_t)i;
      case CUBED_I16: return (V)(int16_t)i;
      case CUBED_I32: return (V)(int32_t)i;
      case CUBED_U8: return (V)(uint8_t)i;
      case CUBED_U16: return (V)(uint16_t)i;
      case CUBED_U32: return (V)(uint32_t)i;
      case CUBED_U64: return (V)(uint64_t)i;
      default: return (V)i;
    }
  }
}

template <typename V, int VEC>
CUBED_DEV void unary(int op, V (&X)[VEC]) {
  if constexpr (is_same_v<V, int64_t>) {
    switch (op) {
      case CUBED_OP_NEG: CUBED_EACH((int64_t)(0ull - (uint64_t)x)); break;
      case CUBED_OP_ABS: CUBED_EACH(x < 0 ? (int64_t)(0ull - (uint64_t)x) : x); break;
      case CUBED_OP_LNOT: CUBED_EACH((int64_t)(x == 0)); break;
      case CUBED_OP_BNOT: CUBED_EACH(~x); break;
      case CUBED_OP_SIGN: CUBED_EACH((int64_t)((x > 0) - (x < 0))); break;
      case CUBED_OP_SQUARE: CUBED_EACH((int64_t)((uint64_t)x * (uint64_t)x)); break;
      case CUBED_OP_ISNAN: case CUBED_OP_ISINF: case CUBED_OP_SIGNBIT: CUBED_EACH((int64_t)(op == CUBED_OP_SIGNBIT ? (x < 0) : 0)); break;
      case CUBED_OP_ISFINITE: CUBED_EACH((int64_t)1); break;
      default: break;  // floor/ceil/trunc/rint/positive of ints are identities
    }
  } else {
    switch (op) {
      case CUBED_OP_NEG: CUBED_EACH(-x); break;
      case CUBED_OP_ABS: CUBED_EACH(fabs(x)); break;
      case CUBED_OP_SQRT: CUBED_EACH(sqrt(x)); break;
      case CUBED_OP_EXP: CUBED_EACH(exp(x)); break;
      case CUBED_OP_LOG: CUBED_EACH(log(x)); break;
      case CUBED_OP_SIN: CUBED_EACH(sin(x)); break;
      case CUBED_OP_COS: CUBED_EACH(cos(x)); break;
      case CUBED_OP_TAN: CUBED_EACH(tan(x)); break;
      case CUBED_OP_TANH: CUBED_EACH(tanh(x)); break;
      case CUBED_OP_FLOOR: CUBED_EACH(floor(x)); break;
      case CUBED_OP_CEIL: CUBED_EACH(ceil(x)); break;
      case CUBED_OP_TRUNC: CUBED_EACH(trunc(x)); break;
      case CUBED_OP_RINT: CUBED_EACH(rint(x)); break;
      case CUBED_OP_ISNAN: CUBED_EACH((V)(x != x)); break;
      case CUBED_OP_ISINF: CUBED_EACH((V)(isinf(x) ? 1 : 0)); break;
      case CUBED_OP_ISFINITE: CUBED_EACH((V)(isfinite(x) ? 1 : 0)); break;
      case CUBED_OP_LNOT: CUBED_EACH((V)(x == (V)0)); break;
      case CUBED_OP_BNOT: CUBED_EACH((V)(~f2i64((double)x))); break;
      case CUBED_OP_SIGN: CUBED_EACH(x > 0 ? (V)1 : (x < 0 ? (V)-1 : (x == 0 ? (V)0 : x))); break;
      case CUBED_OP_SQUARE: CUBED_EACH(x * x); break;
      case CUBED_OP_RECIP: CUBED_EACH((V)1 / x); break;
      case CUBED_OP_LOG1P: CUBED_EACH(log1p(x)); break;
      case CUBED_OP_EXPM1: CUBED_EACH(expm1(x)); break;
      case CUBED_OP_LOG2: CUBED_EACH(log2(x)); break;
      case CUBED_OP_LOG10: CUBED_EACH(log10(x)); break;
      case CUBED_OP_SINH: CUBED_EACH(sinh(x)); break;
      case CUBED_OP_COSH: CUBED_EACH(cosh(x)); break;
      case CUBED_OP_ASIN: CUBED_EACH(asin(x)); break;
      case CUBED_OP_ACOS: CUBED_EACH(acos(x)); break;
      case CUBED_OP_ATAN: CUBED_EACH(atan(x)); break;
      case CUBED_OP_ASINH: CUBED_EACH(asinh(x)); break;
      case CUBED_OP_ACOSH: CUBED_EACH(acosh(x)); break;
      case CUBED_OP_ATANH: CUBED_EACH(atanh(x)); break;
      case CUBED_OP_EXP2: CUBED_EACH(exp2(x)); break;
      case CUBED_OP_SIGNBIT: CUBED_EACH((V)(signbit(x) ? 1 : 0)); break;
      default: break;
    }
  }
}

template <typename V, int VEC>
CUBED_DEV void binary(int op, V (&X)[VEC], const V (&Y)[VEC]) {
  if constexpr (is_same_v<V, int64_t>) {
    switch (op) {
      case CUBED_OP_ADD: CUBED_EACH2((int64_t)((uint64_t)x + (uint64_t)y)); break;
      case CUBED_OP_SUB: CUBED_EACH2((int64_t)((uint64_t)x - (uint64_t)y)); break;
      case CUBED_OP_MUL: CUBED_EACH2((int64_t)((uint64_t)x * (uint64_t)y)); break;
      case CUBED_OP_FLOORDIV: CUBED_EACH2(ifloordiv(x, y)); break;
      case CUBED_OP_MOD: CUBED_EACH2(imod(x, y)); break;
      case CUBED_OP_POW: CUBED_EACH2(ipow(x, y)); break;
      case CUBED_OP_MAX: case CUBED_OP_FMAX: CUBED_EACH2(x > y ? x : y); break;
      case CUBED_OP_MIN: case CUBED_OP_FMIN: CUBED_EACH2(x < y ? x : y); break;
      case CUBED_OP_EQ: CUBED_EACH2((int64_t)(x == y)); break;
      case CUBED_OP_NE: CUBED_EACH2((int64_t)(x != y)); break;
      case CUBED_OP_LT: CUBED_EACH2((int64_t)(x < y)); break;
      case CUBED_OP_LE: CUBED_EACH2((int64_t)(x <= y)); break;
      case CUBED_OP_GT: CUBED_EACH2((int64_t)(x > y)); break;
      case CUBED_OP_GE: CUBED_EACH2((int64_t)(x >= y)); break;
      case CUBED_OP_LAND: CUBED_EACH2((int64_t)((x != 0) && (y != 0))); break;
      case CUBED_OP_LOR: CUBED_EACH2((int64_t)((x != 0) || (y != 0))); break;
      case CUBED_OP_LXOR: CUBED_EACH2((int64_t)((x != 0) != (y != 0))); break;
      case CUBED_OP_BAND: CUBED_EACH2(x & y); break;
      case CUBED_OP_BOR: CUBED_EACH2(x | y); break;
      case CUBED_OP_BXOR: CUBED_EACH2(x ^ y); break;
      case CUBED_OP_SHL: CUBED_EACH2((y < 0 || y > 63) ? (int64_t)0 : (int64_t)((uint64_t)x << y)); break;
      case CUBED_OP_SHR: CUBED_EACH2((y < 0 || y > 63) ? (x < 0 ? (int64_t)-1 : (int64_t)0) : (x >> y)); break;
      default: break;
    }
  } else {
    switch (op) {
      case CUBED_OP_ADD: CUBED_EACH2(x + y); break;
      case CUBED_OP_SUB: CUBED_EACH2(x - y); break;
      case CUBED_OP_MUL: CUBED_EACH2(x * y); break;
      case CUBED_OP_DIV: CUBED_EACH2(x / y); break;
      case CUBED_OP_FLOORDIV: { _Pragma("unroll") for (int j = 0; j < VEC; ++j) { V m; X[j] = npy_divmod<V>(X[j], Y[j], &m); } } break;
      case CUBED_OP_MOD: { _Pragma("unroll") for (int j = 0; j < VEC; ++j) { V m; npy_divmod<V>(X[j], Y[j], &m); X[j] = m; } } break;
      case CUBED_OP_POW: CUBED_EACH2(pow(x, y)); break;
      case CUBED_OP_MAX: CUBED_EACH2(npy_max<V>(x, y)); break;
      case CUBED_OP_MIN: CUBED_EACH2(npy_min<V>(x, y)); break;
      case CUBED_OP_FMAX: CUBED_EACH2(fmax(x, y)); break;
      case CUBED_OP_FMIN: CUBED_EACH2(fmin(x, y)); break;
      case CUBED_OP_EQ: CUBED_EACH2((V)(x == y)); break;
      case CUBED_OP_NE: CUBED_EACH2((V)(x != y)); break;
      case CUBED_OP_LT: CUBED_EACH2((V)(x < y)); break;
      case CUBED_OP_LE: CUBED_EACH2((V)(x <= y)); break;
      case CUBED_OP_GT: CUBED_EACH2((V)(x > y)); break;
      case CUBED_OP_GE: CUBED_EACH2((V)(x >= y)); break;
      case CUBED_OP_LAND: CUBED_EACH2((V)((x != 0) && (y != 0))); break;
      case CUBED_OP_LOR: CUBED_EACH2((V)((x != 0) || (y != 0))); break;
      case CUBED_OP_LXOR: CUBED_EACH2((V)((x != 0) != (y != 0))); break;
      case CUBED_OP_BAND: CUBED_EACH2((V)(f2i64((double)x) & f2i64((double)y))); break;
      case CUBED_OP_BOR: CUBED_EACH2((V)(f2i64((double)x) | f2i64((double)y))); break;
      case CUBED_OP_BXOR: CUBED_EACH2((V)(f2i64((double)x) ^ f2i64((double)y))); break;
      case CUBED_OP_ATAN2: CUBED_EACH2(atan2(x, y)); break;
      case CUBED_OP_HYPOT: CUBED_EACH2(hypot(x, y)); break;
      case CUBED_OP_COPYSIGN: CUBED_EACH2(copysign(x, y)); break;
      case CUBED_OP_LOGADDEXP: CUBED_EACH2(npy_logaddexp<V>(x, y)); break;
      case CUBED_OP_LOGADDEXP2: CUBED_EACH2(npy_logaddexp2<V>(x, y)); break;
      default: break;
    }
  }
}

// Run `n` instructions.  consts: the program's constant pool.
template <typename V, int VEC>
CUBED_DEV void run_vm(Regs<V, VEC>& regs, const cubed_insn_t* ins, int n,
                      const cubed_program_t& P) {
  for (int i = 0; i < n; ++i) {
    const cubed_insn_t I = ins[i];
    const int op = I.op;
    V X[VEC];
    if (op == CUBED_OP_CONST) {
      V c;
      if constexpr (is_same_v<V, int64_t>) c = P.consts[I.imm].i;
      else c = (V)P.consts[I.imm].f;
#pragma unroll
      for (int j = 0; j < VEC; ++j) X[j] = c;
      put(regs, I.a, X);
      continue;
    }
    if (op == CUBED_OP_MOV) {
      fetch(regs, I.b, X);
      put(regs, I.a, X);
      continue;
    }
    fetch(regs, I.a, X);
    if (op == CUBED_OP_CAST) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) X[j] = cast_val<V>(X[j], I.t, I.imm);
    } else if (op == CUBED_OP_WHERE) {
      V Y[VEC], C[VEC];
      fetch(regs, I.b, Y);
      fetch(regs, I.c, C);
#pragma unroll
      for (int j = 0; j < VEC; ++j) X[j] = (C[j] != (V)0) ? X[j] : Y[j];
    } else if (op >= CUBED_OP_ADD) {
      V Y[VEC];
      fetch(regs, I.b, Y);
      binary<V, VEC>(op, X, Y);
    } else {
      unary<V, VEC>(op, X);
    }
    put(regs, I.a, X);
  }
}


// ---------------------------------------------------------------- static form
// One instruction with every operand a compile-time constant: the form the
// runtime-specialised kernels (jit.cpp) are generated in.  Register operands
// resolve to named registers at compile time and the op switch folds, so a
// program compiles to straight-line VALU code with no scratch and no branches.
template <int I, typename V, int VEC>
CUBED_DEV V (&regref(Regs<V, VEC>& r))[VEC] {
  if constexpr (I == 0) return r.r0;
  else if constexpr (I == 1) return r.r1;
  else if constexpr (I == 2) return r.r2;
  else if constexpr (I == 3) return r.r3;
  else if constexpr (I == 4) return r.r4;
  else return r.r5;
}

template <int OP, int A, int B, int C, int T, int IMM, typename V, int VEC>
CUBED_DEV void sinsn(Regs<V, VEC>& regs, const cubed_program_t& P) {
  V (&X)[VEC] = regref<A>(regs);
  if constexpr (OP == CUBED_OP_CONST) {
    V c;
    if constexpr (is_same_v<V, int64_t>) c = P.consts[IMM].i;
    else c = (V)P.consts[IMM].f;
#pragma unroll
    for (int j = 0; j < VEC; ++j) X[j] = c;
  } else if constexpr (OP == CUBED_OP_MOV) {
    const V (&Y)[VEC] = regref<B>(regs);
#pragma unroll
    for (int j = 0; j < VEC; ++j) X[j] = Y[j];
  } else if constexpr (OP == CUBED_OP_CAST) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) X[j] = cast_val<V>(X[j], T, IMM);
  } else if constexpr (OP == CUBED_OP_WHERE) {
    V Y[VEC], Cn[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) { Y[j] = regref<B>(regs)[j]; Cn[j] = regref<C>(regs)[j]; }
#pragma unroll
    for (int j = 0; j < VEC; ++j) X[j] = (Cn[j] != (V)0) ? X[j] : Y[j];
  } else if constexpr (OP >= CUBED_OP_ADD) {
    V Y[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) Y[j] = regref<B>(regs)[j];
    binary<V, VEC>(OP, X, Y);
  } else {
    unary<V, VEC>(OP, X);
  }
}

// ---------------------------------------------------------------- reductions
union Acc { double f; int64_t i; };

CUBED_DEV Acc acc_init(int rop, int acc_i) {
  Acc a;
  switch (rop) {
    case CUBED_R_MAX: if (acc_i) a.i = INT64_MIN; else a.f = -__builtin_inf(); break;
    case CUBED_R_MIN: if (acc_i) a.i = INT64_MAX; else a.f = __builtin_inf(); break;
    case CUBED_R_NANMAX: case CUBED_R_NANMIN: if (acc_i) a.i = (rop == CUBED_R_NANMAX ? INT64_MIN : INT64_MAX); else a.f = __builtin_nan(""); break;
    case CUBED_R_PROD: case CUBED_R_NANPROD: if (acc_i) a.i = 1; else a.f = 1.0; break;
    case CUBED_R_ALL: a.i = 1; break;
    case CUBED_R_SUM: case CUBED_R_NANSUM: if (acc_i) a.i = 0; else a.f = -0.0; break;
    // pairs: {value, index} starts at the weakest value with no index, so
    // any element (even -inf / INT64_MIN) takes its place; {re, im} at 1 + 0j
    case CUBED_R_ARGMAX: if (acc_i) a.i = INT64_MIN; else a.f = -__builtin_inf(); break;
    case CUBED_R_ARGMIN: if (acc_i) a.i = INT64_MAX; else a.f = __builtin_inf(); break;
    case CUBED_R_PAIR_INDEX: a.i = INT64_MAX; break;
    case CUBED_R_CPROD: a.f = 1.0; break;
    case CUBED_R_PAIR_IMAG: a.f = 0.0; break;
    // var triples start empty: {n = 0, mu = 0, M2 = 0}
    case CUBED_R_VAR: case CUBED_R_VARC: a.i = 0; break;
    case CUBED_R_VAR_MEAN: case CUBED_R_VAR_M2: a.f = 0.0; break;
    default: a.i = 0; break;
  }
  return a;
}

// ---- pair reductions: field 0 leads, field 1 is its partner
// argmax/argmin {value, index}: numpy's rule -- the first NaN wins, else the
// larger (smaller) value, ties to the smaller index (an order-free choice,
// so every combine tree gives the same pair).  cprod {re, im}: the complex
// product (ar*br - ai*bi, ar*bi + ai*br), unfused like npymath's nc_prod.
__host__ __device__ inline bool pair_rop(int rop) { return rop == CUBED_R_ARGMAX || rop == CUBED_R_ARGMIN || rop == CUBED_R_CPROD; }

CUBED_DEV void pair_combine(Acc& a0, Acc& a1, Acc b0, Acc b1, int rop, int acc_i) {
  if (rop == CUBED_R_CPROD) {
#pragma clang fp contract(off)
    const double re = a0.f * b0.f - a1.f * b1.f;
    const double im = a0.f * b1.f + a1.f * b0.f;
    a0.f = re; a1.f = im;
    return;
  }
  const bool mx = rop == CUBED_R_ARGMAX;
  bool take;
  if (acc_i) {
    take = (mx ? b0.i > a0.i : b0.i < a0.i) || (b0.i == a0.i && b1.i < a1.i);
  } else {
    const bool an = a0.f != a0.f, bn = b0.f != b0.f;
    take = an ? (bn && b1.i < a1.i)
              : (bn || (mx ? b0.f > a0.f : b0.f < a0.f) || (b0.f == a0.f && b1.i < a1.i));
  }
  if (take) { a0 = b0; a1 = b1; }
}

// ---- var triples {n, mu, M2} (field 0 leads; include/cubed_amd.h cubed_rop)
__host__ __device__ inline bool triple_rop(int rop) { return rop == CUBED_R_VAR || rop == CUBED_R_VARC; }

// Chan, Golub & LeVeque's pairwise update: {n, mu, M2} (+)= {nb, mb, Mb}.
// An empty side leaves the other unchanged (so identities and empty tasks
// fold away exactly); NaN / inf propagate through d as in numpy's var.
CUBED_DEV void var_combine(Acc& n, Acc& mu, Acc& m2, int64_t nb, double mb, double Mb) {
#pragma clang fp contract(off)
  if (nb == 0) return;
  if (n.i == 0) { n.i = nb; mu.f = mb; m2.f = Mb; return; }
  const int64_t na = n.i, nn = na + nb;
  const double d = mb - mu.f;
  const double fb = (double)nb / (double)nn;
  mu.f = mu.f + d * fb;
  m2.f = m2.f + Mb + d * d * ((double)na * fb);
  n.i = nn;
}

// Welford's update: fold one value x into {n, mu, M2}
CUBED_DEV void var_add(Acc& n, Acc& mu, Acc& m2, double x) {
#pragma clang fp contract(off)
  n.i += 1;
  const double d = x - mu.f;
  mu.f = mu.f + d / (double)n.i;
  m2.f = m2.f + d * (x - mu.f);
}

// the same with the count's reciprocal given: the elements of one VEC group
// fold the same rows, so one f64 division serves the group
CUBED_DEV void var_add_inv(Acc& n, Acc& mu, Acc& m2, double x, int64_t n1, double inv) {
#pragma clang fp contract(off)
  n.i = n1;
  const double d = x - mu.f;
  mu.f = mu.f + d * inv;
  m2.f = m2.f + d * (x - mu.f);
}

template <typename V>
CUBED_DEV void pair_add(Acc& a0, Acc& a1, int rop, int acc_i, V v0, V v1) {
  Acc b0, b1;
  if (rop == CUBED_R_CPROD) { b0.f = (double)v0; b1.f = (double)v1; }
  else {
    if (acc_i) b0.i = to_i64(v0); else b0.f = (double)v0;
    b1.i = to_i64(v1);
  }
  pair_combine(a0, a1, b0, b1, rop, acc_i);
}

// fold one value into an accumulator
template <typename V>
CUBED_DEV void acc_add(Acc& a, int rop, int acc_i, V v) {
  switch (rop) {
    case CUBED_R_SUM:
      if (acc_i) a.i = (int64_t)((uint64_t)a.i + (uint64_t)to_i64(v)); else a.f += (double)v; break;
    case CUBED_R_NANSUM:
      if (acc_i) a.i += to_i64(v); else if (v == v) a.f += (double)v; break;
    case CUBED_R_COUNT: a.i += 1; break;
    case CUBED_R_COUNT_NONNAN: a.i += (v == v) ? 1 : 0; break;
    case CUBED_R_MAX:
      if (acc_i) { int64_t w = to_i64(v); a.i = w > a.i ? w : a.i; } else a.f = npy_max<double>(a.f, (double)v); break;
    case CUBED_R_MIN:
      if (acc_i) { int64_t w = to_i64(v); a.i = w < a.i ? w : a.i; } else a.f = npy_min<double>(a.f, (double)v); break;
    case CUBED_R_NANMAX:
      if (acc_i) { int64_t w = to_i64(v); a.i = w > a.i ? w : a.i; }
      else if (v == v) a.f = (a.f != a.f || (double)v > a.f) ? (double)v : a.f; break;
    case CUBED_R_NANMIN:
      if (acc_i) { int64_t w = to_i64(v); a.i = w < a.i ? w : a.i; }
      else if (v == v) a.f = (a.f != a.f || (double)v < a.f) ? (double)v : a.f; break;
    case CUBED_R_PROD:
      if (acc_i) a.i = (int64_t)((uint64_t)a.i * (uint64_t)to_i64(v)); else a.f *= (double)v; break;
    case CUBED_R_NANPROD:
      if (acc_i) a.i = (int64_t)((uint64_t)a.i * (uint64_t)to_i64(v)); else if (v == v) a.f *= (double)v; break;
    case CUBED_R_ANY: a.i |= (v != (V)0) ? 1 : 0; break;
    case CUBED_R_ALL: a.i &= (v != (V)0) ? 1 : 0; break;
    default: break;
  }
}

// combine two partial accumulators
CUBED_DEV Acc acc_combine(Acc a, Acc b, int rop, int acc_i) {
  Acc r;
  switch (rop) {
    case CUBED_R_SUM: case CUBED_R_NANSUM:
      if (acc_i) r.i = (int64_t)((uint64_t)a.i + (uint64_t)b.i); else r.f = a.f + b.f; break;
    case CUBED_R_COUNT: case CUBED_R_COUNT_NONNAN: r.i = a.i + b.i; break;
    case CUBED_R_MAX: if (acc_i) r.i = a.i > b.i ? a.i : b.i; else r.f = npy_max<double>(a.f, b.f); break;
    case CUBED_R_MIN: if (acc_i) r.i = a.i < b.i ? a.i : b.i; else r.f = npy_min<double>(a.f, b.f); break;
    case CUBED_R_NANMAX:
      if (acc_i) r.i = a.i > b.i ? a.i : b.i;
      else r.f = (a.f != a.f) ? b.f : ((b.f != b.f) ? a.f : (a.f > b.f ? a.f : b.f)); break;
    case CUBED_R_NANMIN:
      if (acc_i) r.i = a.i < b.i ? a.i : b.i;
      else r.f = (a.f != a.f) ? b.f : ((b.f != b.f) ? a.f : (a.f < b.f ? a.f : b.f)); break;
    case CUBED_R_PROD: case CUBED_R_NANPROD:
      if (acc_i) r.i = (int64_t)((uint64_t)a.i * (uint64_t)b.i); else r.f = a.f * b.f; break;
    case CUBED_R_ANY: r.i = a.i | b.i; break;
    case CUBED_R_ALL: r.i = a.i & b.i; break;
    default: r = a; break;
  }
  return r;
}

CUBED_DEV Acc shfl_xor_acc(Acc a, int m) {
  Acc r;
  r.i = __shfl_xor((long long)a.i, m, 64);
  return r;
}

// x (+)= y over all fields of P (a pair program combines its two fields as
// one; its partner rop leaves acc_combine a no-op)
CUBED_DEV void fields_combine(Acc (&x)[CUBED_MAX_FIELDS], const Acc (&y)[CUBED_MAX_FIELDS],
                              const cubed_program_t& P) {
  if (triple_rop(P.field_rop[0])) {
    var_combine(x[0], x[1], x[2], y[0].i, y[1].f, y[2].f);
    return;
  }
  if (pair_rop(P.field_rop[0])) {
    pair_combine(x[0], x[1], y[0], y[1], P.field_rop[0], P.field_acc[0]);
    return;
  }
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f)
    if (f < P.nfields) x[f] = acc_combine(x[f], y[f], P.field_rop[f], P.field_acc[f]);
}

// fold the field values src[f][j] of VEC elements into acc[f][j]; SKIP_COUNT:
// the streaming kernel adds CUBED_R_COUNT fields once per run instead
template <typename V, int VEC, bool SKIP_COUNT = false>
CUBED_DEV void fields_add(Acc (&acc)[CUBED_MAX_FIELDS][VEC], const V (&src)[CUBED_MAX_FIELDS][VEC],
                          const cubed_program_t& P) {
  if (triple_rop(P.field_rop[0])) {
    if (P.field_rop[0] == CUBED_R_VAR) {
      if constexpr (VEC > 1) {
        // (every element of the group has folded the same number of values)
        const int64_t n1 = acc[0][0].i + 1;
        const double inv = 1.0 / (double)n1;
#pragma unroll
        for (int j = 0; j < VEC; ++j) var_add_inv(acc[0][j], acc[1][j], acc[2][j], (double)src[0][j], n1, inv);
      } else {
        var_add(acc[0][0], acc[1][0], acc[2][0], (double)src[0][0]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        var_combine(acc[0][j], acc[1][j], acc[2][j], to_i64(src[0][j]), (double)src[1][j], (double)src[2][j]);
    }
    return;
  }
  if (pair_rop(P.field_rop[0])) {
#pragma unroll
    for (int j = 0; j < VEC; ++j)
      pair_add<V>(acc[0][j], acc[1][j], P.field_rop[0], P.field_acc[0], src[0][j], src[1][j]);
    return;
  }
#pragma unroll
  for (int f = 0; f < CUBED_MAX_FIELDS; ++f) {
    if (f < P.nfields && !(SKIP_COUNT && P.field_rop[f] == CUBED_R_COUNT)) {
      const int rop = P.field_rop[f], ai = P.field_acc[f];
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc_add<V>(acc[f][j], rop, ai, src[f][j]);
    }
  }
}

}  // namespace cubed
