"""NaN-ignoring reductions (cubed/nan_functions.py:21-77)."""

import numpy as np

from .array_api.dtypes import (
    _numeric_dtypes,
    _signed_integer_dtypes,
    _unsigned_integer_dtypes,
    complex64,
    complex128,
    float32,
    float64,
    int64,
    uint64,
)
from .chunkfuncs import NumpyReduction, _nanmean_aggregate, _nanmean_combine, _nanmean_func
from .core import reduction

_np_nansum = NumpyReduction("nansum", "nansum")


def nanmean(x, /, *, axis=None, keepdims=False):
    """Arithmetic mean along ``axis`` ignoring NaNs: fields n = count of
    non-NaN (int64), total = nansum (float64)."""
    dtype = x.dtype
    intermediate_dtype = [("n", np.int64), ("total", np.float64)]
    return reduction(x, _nanmean_func, combine_func=_nanmean_combine,
                     aggegrate_func=_nanmean_aggregate, axis=axis,
                     intermediate_dtype=intermediate_dtype, dtype=dtype, keepdims=keepdims)


def nansum(x, /, *, axis=None, dtype=None, keepdims=False):
    """Sum treating NaNs as zero."""
    if x.dtype not in _numeric_dtypes:
        raise TypeError("Only numeric dtypes are allowed in nansum")
    if dtype is None:
        if x.dtype in _signed_integer_dtypes:
            dtype = int64
        elif x.dtype in _unsigned_integer_dtypes:
            dtype = uint64
        elif x.dtype == float32:
            dtype = float64
        elif x.dtype == complex64:
            dtype = complex128
        else:
            dtype = x.dtype
    return reduction(x, _np_nansum, axis=axis, dtype=dtype, keepdims=keepdims,
                     extra_func_kwargs=dict(dtype=dtype))
