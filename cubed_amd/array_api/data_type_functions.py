"""Data type functions (mirrors cubed/array_api/data_type_functions.py)."""

from dataclasses import dataclass

import numpy as np

from .. import ir
from ..core import CoreArray
from .dtypes import (
    _all_dtypes,
    _boolean_dtypes,
    _complex_floating_dtypes,
    _integer_dtypes,
    _numeric_dtypes,
    _real_floating_dtypes,
    _result_type,
    _signed_integer_dtypes,
    _unsigned_integer_dtypes,
)


def astype(x, dtype, /, *, copy=True):
    """map_blocks(_astype) (data_type_functions.py:22-29): one CAST in the
    fused program (numpy astype semantics: float->int truncates)."""
    from ..core.ops import map_blocks

    dtype = np.dtype(dtype)
    if not copy and dtype == x.dtype:
        return x
    prog = ir.elementwise_program("astype", [x.dtype], [x.ndim], dtype)
    return map_blocks(prog, x, dtype=dtype)


def can_cast(from_, to, /):
    if isinstance(from_, CoreArray):
        from_ = from_.dtype
    elif from_ not in _all_dtypes:
        raise TypeError(f"{from_=}, but should be an array_api array or dtype")
    if to not in _all_dtypes:
        raise TypeError(f"{to=}, but should be a dtype")
    try:
        return to == _result_type(from_, to)
    except TypeError:
        return False


@dataclass
class finfo_object:
    bits: int
    eps: float
    max: float
    min: float
    smallest_normal: float
    dtype: np.dtype


@dataclass
class iinfo_object:
    bits: int
    max: int
    min: int
    dtype: np.dtype


def finfo(type, /):
    fi = np.finfo(type)
    return finfo_object(fi.bits, float(fi.eps), float(fi.max), float(fi.min),
                        float(fi.smallest_normal), fi.dtype)


def iinfo(type, /):
    ii = np.iinfo(type)
    return iinfo_object(ii.bits, ii.max, ii.min, ii.dtype)


def isdtype(dtype, kind):
    if isinstance(kind, tuple):
        return any(isdtype(dtype, k) for k in kind)
    if isinstance(kind, str):
        table = {
            "bool": _boolean_dtypes, "signed integer": _signed_integer_dtypes,
            "unsigned integer": _unsigned_integer_dtypes, "integral": _integer_dtypes,
            "real floating": _real_floating_dtypes, "complex floating": _complex_floating_dtypes,
            "numeric": _numeric_dtypes,
        }
        if kind not in table:
            raise ValueError(f"Unrecognized data type kind: {kind!r}")
        return dtype in table[kind]
    if kind in _all_dtypes:
        return dtype == kind
    raise TypeError(f"'kind' must be a dtype, str, or tuple of dtypes and strs, not {type(kind).__name__}")


def result_type(*arrays_and_dtypes):
    A = []
    for a in arrays_and_dtypes:
        if isinstance(a, CoreArray):
            a = a.dtype
        elif isinstance(a, np.ndarray) or a not in _all_dtypes:
            raise TypeError("result_type() inputs must be array_api arrays or dtypes")
        A.append(a)
    if len(A) == 0:
        raise ValueError("at least one array or dtype is required")
    t = A[0]
    for t2 in A[1:]:
        t = _result_type(t, t2)
    return t
