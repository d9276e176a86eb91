"""Array API dtypes and promotion (the reference's array_api/dtypes.py,
copied there from numpy.array_api; restated here as data)."""

import numpy as np

int8 = np.dtype("int8")
int16 = np.dtype("int16")
int32 = np.dtype("int32")
int64 = np.dtype("int64")
uint8 = np.dtype("uint8")
uint16 = np.dtype("uint16")
uint32 = np.dtype("uint32")
uint64 = np.dtype("uint64")
float32 = np.dtype("float32")
float64 = np.dtype("float64")
complex64 = np.dtype("complex64")
complex128 = np.dtype("complex128")
bool = np.dtype("bool")
# bfloat16 is not an array API (or numpy) dtype and the reference has none
# (cubed/array_api/dtypes.py:14-37); it is offered for the MFMA chunk GEMMs
# (BASELINE config 5 "bf16").  Carried as ir.bfloat16; compute() returns its
# values widened exactly to float32.
from ..ir import bfloat16  # noqa: E402

_all_dtypes = (int8, int16, int32, int64, uint8, uint16, uint32, uint64, float32, float64,
               complex64, complex128, bool, bfloat16)
_boolean_dtypes = (bool,)
_real_floating_dtypes = (float32, float64, bfloat16)
_floating_dtypes = (float32, float64, bfloat16, complex64, complex128)
_complex_floating_dtypes = (complex64, complex128)
_integer_dtypes = (int8, int16, int32, int64, uint8, uint16, uint32, uint64)
_signed_integer_dtypes = (int8, int16, int32, int64)
_unsigned_integer_dtypes = (uint8, uint16, uint32, uint64)
_integer_or_boolean_dtypes = (bool,) + _integer_dtypes
_real_numeric_dtypes = (float32, float64, bfloat16) + _integer_dtypes
_numeric_dtypes = (float32, float64, bfloat16, complex64, complex128) + _integer_dtypes

_dtype_categories = {
    "all": _all_dtypes,
    "real numeric": _real_numeric_dtypes,
    "numeric": _numeric_dtypes,
    "integer": _integer_dtypes,
    "integer or boolean": _integer_or_boolean_dtypes,
    "boolean": _boolean_dtypes,
    "real floating-point": _floating_dtypes,
    "complex floating-point": _complex_floating_dtypes,
    "floating-point": _floating_dtypes,
}


def _promote(t1, t2):
    """Array API type promotion: within a kind by size; signed+unsigned to
    the next signed size that holds both; no cross-kind promotion except
    the float/complex lattice."""
    t1, t2 = np.dtype(t1), np.dtype(t2)
    if t1 == t2:
        return t1
    if t1 == bfloat16 or t2 == bfloat16:
        # bf16 joins the float lattice below float32 (bf16 + f32 -> f32)
        o = t2 if t1 == bfloat16 else t1
        if o.kind in "fc":
            return o
        raise TypeError(f"{t1} and {t2} cannot be type promoted together")
    k1, k2 = t1.kind, t2.kind
    if k1 == "b" or k2 == "b":
        raise TypeError(f"{t1} and {t2} cannot be type promoted together")
    if k1 in "iu" and k2 in "iu":
        if k1 == k2:
            return t1 if t1.itemsize >= t2.itemsize else t2
        s, u = (t1, t2) if k1 == "i" else (t2, t1)
        if u.itemsize < s.itemsize:
            return s
        if u.itemsize == 8:
            raise TypeError(f"{t1} and {t2} cannot be type promoted together")
        return np.dtype(f"int{u.itemsize * 16}")
    if k1 in "fc" and k2 in "fc":
        return np.result_type(t1, t2)
    raise TypeError(f"{t1} and {t2} cannot be type promoted together")


def _result_type(type1, type2):
    return _promote(type1, type2)
