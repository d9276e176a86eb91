"""Statistical functions (cubed/array_api/statistical_functions.py:22-156).

``mean`` keeps the reference's structured ``{n: int64, total: float64}``
intermediate (stored SoA in HBM) and its reduction rounds; the chunk
functions are the program builders of cubed_amd.chunkfuncs."""

import numpy as np

from ..chunkfuncs import (NumpyReduction, _mean_aggregate, _mean_combine, _mean_func, _var_combine,
                          _var_func, _VarAggregate)
from ..core import reduction
from .dtypes import (
    _numeric_dtypes,
    _real_floating_dtypes,
    _real_numeric_dtypes,
    _signed_integer_dtypes,
    _unsigned_integer_dtypes,
    complex64,
    complex128,
    float32,
    float64,
    int64,
    uint64,
)

_np_max = NumpyReduction("max", "max")
_np_min = NumpyReduction("min", "min")
_np_sum = NumpyReduction("sum", "sum")
_np_prod = NumpyReduction("prod", "prod")


def max(x, /, *, axis=None, keepdims=False):
    if x.dtype not in _real_numeric_dtypes:
        raise TypeError("Only real numeric dtypes are allowed in max")
    return reduction(x, _np_max, axis=axis, dtype=x.dtype, keepdims=keepdims)


def min(x, /, *, axis=None, keepdims=False):
    if x.dtype not in _real_numeric_dtypes:
        raise TypeError("Only real numeric dtypes are allowed in min")
    return reduction(x, _np_min, axis=axis, dtype=x.dtype, keepdims=keepdims)


def mean(x, /, *, axis=None, keepdims=False, use_new_impl=False):
    if x.dtype not in _real_floating_dtypes:
        raise TypeError("Only real floating-point dtypes are allowed in mean")
    dtype = x.dtype
    intermediate_dtype = [("n", np.int64), ("total", np.float64)]
    extra_func_kwargs = dict(dtype=intermediate_dtype)
    return reduction(x, _mean_func, combine_func=_mean_combine, aggegrate_func=_mean_aggregate,
                     axis=axis, intermediate_dtype=intermediate_dtype, dtype=dtype,
                     keepdims=keepdims, use_new_impl=use_new_impl,
                     extra_func_kwargs=extra_func_kwargs)


def _default_sum_dtype(dt):
    if dt in _signed_integer_dtypes:
        return int64
    if dt in _unsigned_integer_dtypes:
        return uint64
    if dt == float32:
        return float64
    if dt == complex64:
        return complex128
    return dt


def prod(x, /, *, axis=None, dtype=None, keepdims=False):
    if x.dtype not in _numeric_dtypes:
        raise TypeError("Only numeric dtypes are allowed in prod")
    if dtype is None:
        dtype = _default_sum_dtype(x.dtype)
    return reduction(x, _np_prod, axis=axis, dtype=dtype, keepdims=keepdims,
                     extra_func_kwargs=dict(dtype=dtype))


def sum(x, /, *, axis=None, dtype=None, keepdims=False):
    if x.dtype not in _numeric_dtypes:
        raise TypeError("Only numeric dtypes are allowed in sum")
    if dtype is None:
        dtype = _default_sum_dtype(x.dtype)
    return reduction(x, _np_sum, axis=axis, dtype=dtype, keepdims=keepdims,
                     extra_func_kwargs=dict(dtype=dtype))


def _var_std(x, axis, correction, keepdims, use_new_impl, sqrt):
    if x.dtype not in _real_floating_dtypes:
        raise TypeError(f"Only real floating-point dtypes are allowed in {'std' if sqrt else 'var'}")
    intermediate_dtype = [("n", np.int64), ("mu", np.float64), ("M2", np.float64)]
    return reduction(x, _var_func, combine_func=_var_combine,
                     aggegrate_func=_VarAggregate(correction, sqrt), axis=axis,
                     intermediate_dtype=intermediate_dtype, dtype=x.dtype, keepdims=keepdims,
                     use_new_impl=use_new_impl, extra_func_kwargs=dict(dtype=intermediate_dtype))


def var(x, /, *, axis=None, correction=0.0, keepdims=False, use_new_impl=False):
    """Array API ``var`` (not in the reference v0.12.0, api_status.md:74):
    one fused pass of the {n, mu, M2} triple reduction (Welford per element,
    Chan's update across chunks, merge rounds and GPUs) in f64, then
    M2 / max(n - correction, 0), cast to x's dtype.  Matches numpy's
    ``var(ddof=correction)`` computed in f64."""
    return _var_std(x, axis, correction, keepdims, use_new_impl, sqrt=False)


def std(x, /, *, axis=None, correction=0.0, keepdims=False, use_new_impl=False):
    """Array API ``std`` (api_status.md:72): the square root of ``var``'s
    aggregate, same single pass."""
    return _var_std(x, axis, correction, keepdims, use_new_impl, sqrt=True)
