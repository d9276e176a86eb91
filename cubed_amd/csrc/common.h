// common.h -- device helpers shared by the libcubed_amd kernels (gfx950).
//
// Element loads/stores for every cubed_dtype, the numpy-compatible scalar
// semantics of the VM ops (npy_divmod, NaN-propagating maximum, ...), and
// the Philox4x64-10 generator numpy uses for Generator.random().
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#endif
#include "cubed_amd.h"

#define CUBED_DEV __device__ __forceinline__

// Device addresses arrive as int64 in the task tables; casting them to
// address_space(1) pointers makes the compiler emit global_load/store
// (SGPR base + offset addressing) instead of flat accesses.
#define CUBED_G __attribute__((address_space(1)))
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int64_t i64x2 __attribute__((ext_vector_type(2)));

template <typename T>
CUBED_DEV const CUBED_G T* gload_ptr(const char* p) { return (const CUBED_G T*)(uintptr_t)p; }
template <typename T>
CUBED_DEV CUBED_G T* gstore_ptr(char* p) { return (CUBED_G T*)(uintptr_t)p; }

namespace cubed {

// minimal type traits (hipRTC builds have no <type_traits>)
template <typename A, typename B> struct is_same_t { static constexpr bool value = false; };
template <typename A> struct is_same_t<A, A> { static constexpr bool value = true; };
template <typename A, typename B> inline constexpr bool is_same_v = is_same_t<A, B>::value;
template <bool C, typename A, typename B> struct conditional { using type = A; };
template <typename A, typename B> struct conditional<false, A, B> { using type = B; };

static constexpr int kBlock = 256;  // 4 waves of 64

CUBED_DEV bool dt_is_float(int dt) {
  return dt == CUBED_F32 || dt == CUBED_F64 || dt == CUBED_F16 || dt == CUBED_BF16;
}

__host__ __device__ inline int dt_size(int dt) {
  switch (dt) {
    case CUBED_BOOL: case CUBED_I8: case CUBED_U8: return 1;
    case CUBED_I16: case CUBED_U16: case CUBED_F16: case CUBED_BF16: return 2;
    case CUBED_I32: case CUBED_U32: case CUBED_F32: return 4;
    default: return 8;
  }
}

// ---------------------------------------------------------------- scalar I/O
CUBED_DEV float bf16_to_f32(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }

// float -> bfloat16, round to nearest even (NaN stays a quiet NaN)
CUBED_DEV uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Read one element of dtype dt at p and convert to V.
template <typename V>
CUBED_DEV V ld1(const char* p, int dt) {
  switch (dt) {
    case CUBED_BOOL: return (V)(*gload_ptr<uint8_t>(p) != 0);
    case CUBED_I8: return (V)(*gload_ptr<int8_t>(p));
    case CUBED_I16: return (V)(*gload_ptr<int16_t>(p));
    case CUBED_I32: return (V)(*gload_ptr<int32_t>(p));
    case CUBED_I64: return (V)(*gload_ptr<int64_t>(p));
    case CUBED_U8: return (V)(*gload_ptr<uint8_t>(p));
    case CUBED_U16: return (V)(*gload_ptr<uint16_t>(p));
    case CUBED_U32: return (V)(*gload_ptr<uint32_t>(p));
    case CUBED_U64: return (V)(*gload_ptr<uint64_t>(p));
    case CUBED_F32: return (V)(*gload_ptr<float>(p));
    case CUBED_F64: return (V)(*gload_ptr<double>(p));
    case CUBED_F16: return (V)(float)(*gload_ptr<_Float16>(p));
    case CUBED_BF16: return (V)bf16_to_f32(*gload_ptr<uint16_t>(p));
  }
  return (V)0;
}

// float -> int conversion with defined results for NaN/out of range (x86
// cvttsd2si behaviour: the "integer indefinite" value).
CUBED_DEV int64_t f2i64(double x) {
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)x;
}

template <typename V>
CUBED_DEV int64_t to_i64(V x) {
  if constexpr (is_same_v<V, int64_t>) return x;
  else return f2i64((double)x);
}

// Convert V to dtype dt and write it at p.
template <typename V>
CUBED_DEV void st1(char* p, int dt, V v) {
  switch (dt) {
    case CUBED_BOOL: *gstore_ptr<uint8_t>(p) = (v != (V)0) ? 1 : 0; return;
    case CUBED_I8: *gstore_ptr<int8_t>(p) = (int8_t)to_i64(v); return;
    case CUBED_I16: *gstore_ptr<int16_t>(p) = (int16_t)to_i64(v); return;
    case CUBED_I32: *gstore_ptr<int32_t>(p) = (int32_t)to_i64(v); return;
    case CUBED_I64: *gstore_ptr<int64_t>(p) = to_i64(v); return;
    case CUBED_U8: *gstore_ptr<uint8_t>(p) = (uint8_t)to_i64(v); return;
    case CUBED_U16: *gstore_ptr<uint16_t>(p) = (uint16_t)to_i64(v); return;
    case CUBED_U32: *gstore_ptr<uint32_t>(p) = (uint32_t)to_i64(v); return;
    case CUBED_U64:
      if constexpr (is_same_v<V, int64_t>) *gstore_ptr<uint64_t>(p) = (uint64_t)v;
      else *gstore_ptr<uint64_t>(p) = ((double)v >= 9223372036854775808.0)
                               ? (uint64_t)((double)v)
                               : (uint64_t)to_i64(v);
      return;
    case CUBED_F32: *gstore_ptr<float>(p) = (float)v; return;
    case CUBED_F64: *gstore_ptr<double>(p) = (double)v; return;
    case CUBED_F16: *gstore_ptr<_Float16>(p) = (_Float16)v; return;
    case CUBED_BF16: *gstore_ptr<uint16_t>(p) = f32_to_bf16((float)v); return;
  }
}

// ---------------------------------------------------------------- vector I/O
// VEC consecutive elements starting at element offset `off` (contiguous,
// aligned to VEC*itemsize; the host checks alignment before choosing VEC>1).
template <typename V, int VEC>
CUBED_DEV void ldv(V (&o)[VEC], const char* base, int64_t off, int dt) {
  if constexpr (VEC == 1) {
    o[0] = ld1<V>(base + off * dt_size(dt), dt);
  } else {
    static_assert(VEC == 4, "VEC is 1 or 4");
    switch (dt) {
      case CUBED_F32: {
        f32x4 v = *gload_ptr<f32x4>(base + off * 4);
        o[0] = (V)v.x; o[1] = (V)v.y; o[2] = (V)v.z; o[3] = (V)v.w; return;
      }
      case CUBED_F64: {
        const CUBED_G f64x2* q = gload_ptr<f64x2>(base + off * 8);
        f64x2 a = q[0], b = q[1];
        o[0] = (V)a.x; o[1] = (V)a.y; o[2] = (V)b.x; o[3] = (V)b.y; return;
      }
      case CUBED_I32: {
        i32x4 v = *gload_ptr<i32x4>(base + off * 4);
        o[0] = (V)v.x; o[1] = (V)v.y; o[2] = (V)v.z; o[3] = (V)v.w; return;
      }
      case CUBED_U32: {
        u32x4 v = *gload_ptr<u32x4>(base + off * 4);
        o[0] = (V)v.x; o[1] = (V)v.y; o[2] = (V)v.z; o[3] = (V)v.w; return;
      }
      case CUBED_I64: case CUBED_U64: {
        const CUBED_G i64x2* q = gload_ptr<i64x2>(base + off * 8);
        i64x2 a = q[0], b = q[1];
        if (dt == CUBED_I64) { o[0] = (V)a.x; o[1] = (V)a.y; o[2] = (V)b.x; o[3] = (V)b.y; }
        else { o[0] = (V)(uint64_t)a.x; o[1] = (V)(uint64_t)a.y; o[2] = (V)(uint64_t)b.x; o[3] = (V)(uint64_t)b.y; }
        return;
      }
      default: {
        const int sz = dt_size(dt);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = ld1<V>(base + (off + j) * sz, dt);
        return;
      }
    }
  }
}

template <typename V, int VEC>
CUBED_DEV void stv(char* base, int64_t off, int dt, const V (&v)[VEC]) {
  if constexpr (VEC == 1) {
    st1<V>(base + off * dt_size(dt), dt, v[0]);
  } else if constexpr (VEC == 2) {
    if (dt == CUBED_F64) {
      f64x2 a; a.x = (double)v[0]; a.y = (double)v[1];
      *gstore_ptr<f64x2>(base + off * 8) = a;
    } else {
      const int sz = dt_size(dt);
      st1<V>(base + off * sz, dt, v[0]);
      st1<V>(base + (off + 1) * sz, dt, v[1]);
    }
  } else {
    switch (dt) {
      case CUBED_F32: {
        f32x4 w; w.x = (float)v[0]; w.y = (float)v[1]; w.z = (float)v[2]; w.w = (float)v[3];
        *gstore_ptr<f32x4>(base + off * 4) = w; return;
      }
      case CUBED_F64: {
        CUBED_G f64x2* q = gstore_ptr<f64x2>(base + off * 8);
        f64x2 a, b; a.x = (double)v[0]; a.y = (double)v[1]; b.x = (double)v[2]; b.y = (double)v[3];
        q[0] = a; q[1] = b; return;
      }
      default: {
        const int sz = dt_size(dt);
#pragma unroll
        for (int j = 0; j < 4; ++j) st1<V>(base + (off + j) * sz, dt, v[j]);
        return;
      }
    }
  }
}

// ---------------------------------------------------------------- Philox
// numpy's Philox4x64-10 (bit_generator "Philox"): counter incremented
// before each block, so element e of a fresh stream is word e%4 of
// philox(ctr = e/4 + 1, key); Generator.random() = (u64 >> 11) * 2^-53.
struct P4 { uint64_t x[4]; };

CUBED_DEV P4 philox4x64_10(uint64_t c0, uint64_t c1, uint64_t k0, uint64_t k1) {
  uint64_t x0 = c0, x1 = c1, x2 = 0, x3 = 0;
  const uint64_t M0 = 0xD2E7470EE14C6C93ull, M1 = 0xCA5A826395121157ull;
  const uint64_t W0 = 0x9E3779B97F4A7C15ull, W1 = 0xBB67AE8584CAA73Bull;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t hi0 = __umul64hi(M0, x0), lo0 = M0 * x0;
    const uint64_t hi1 = __umul64hi(M1, x2), lo1 = M1 * x2;
    const uint64_t y0 = hi1 ^ x1 ^ k0;
    const uint64_t y2 = hi0 ^ x3 ^ k1;
    x0 = y0; x1 = lo1; x2 = y2; x3 = lo0;
    k0 += W0; k1 += W1;
  }
  P4 r; r.x[0] = x0; r.x[1] = x1; r.x[2] = x2; r.x[3] = x3;
  return r;
}

CUBED_DEV double u64_to_unit(uint64_t u) {
  return (double)(u >> 11) * (1.0 / 9007199254740992.0);
}

// element e of the stream (block counter e/4+1 carried into word 1)
CUBED_DEV double philox_at(uint64_t k0, uint64_t k1, int64_t e) {
  const uint64_t b = (uint64_t)(e >> 2) + 1ull;
  P4 r = philox4x64_10(b, b == 0 ? 1ull : 0ull, k0, k1);
  const int w = (int)(e & 3);
  const uint64_t u = w == 0 ? r.x[0] : (w == 1 ? r.x[1] : (w == 2 ? r.x[2] : r.x[3]));
  return u64_to_unit(u);
}

// ---------------------------------------------------------------- numpy ops
template <typename F>
CUBED_DEV F npy_divmod(F a, F b, F* mod_out) {
  F mod = fmod(a, b);
  if (!b) { *mod_out = mod; return a / b; }
  F div = (a - mod) / b;
  if (mod) {
    if ((b < 0) != (mod < 0)) { mod += b; div -= (F)1; }
  } else {
    mod = copysign((F)0, b);
  }
  F floordiv;
  if (div) {
    floordiv = floor(div);
    if (div - floordiv > (F)0.5) floordiv += (F)1;
  } else {
    floordiv = copysign((F)0, a / b);
  }
  *mod_out = mod;
  return floordiv;
}

CUBED_DEV int64_t ifloordiv(int64_t a, int64_t b) {
  if (b == 0) return 0;
  if (b == -1 && a == INT64_MIN) return INT64_MIN;
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
  return q;
}
CUBED_DEV int64_t imod(int64_t a, int64_t b) {
  if (b == 0) return 0;
  if (b == -1) return 0;
  int64_t r = a % b;
  if (r != 0 && ((r < 0) != (b < 0))) r += b;
  return r;
}
CUBED_DEV int64_t ipow(int64_t b, int64_t e) {
  if (e < 0) return 0;
  uint64_t r = 1, x = (uint64_t)b;
  while (e) { if (e & 1) r *= x; x *= x; e >>= 1; }
  return (int64_t)r;
}

template <typename F>
CUBED_DEV F npy_max(F a, F b) { return (a >= b || a != a) ? a : b; }
template <typename F>
CUBED_DEV F npy_min(F a, F b) { return (a <= b || a != a) ? a : b; }

template <typename F>
CUBED_DEV F npy_logaddexp(F x, F y) {
  if (x == y) return x + (F)0.69314718055994530942;
  F t = x - y;
  if (t > 0) return x + log1p(exp(-t));
  if (t <= 0) return y + log1p(exp(t));
  return t;
}
template <typename F>
CUBED_DEV F npy_logaddexp2(F x, F y) {
  if (x == y) return x + (F)1;
  F t = x - y;
  if (t > 0) return x + log1p(exp2(-t)) * (F)1.44269504088896340736;
  if (t <= 0) return y + log1p(exp2(t)) * (F)1.44269504088896340736;
  return t;
}

}  // namespace cubed
