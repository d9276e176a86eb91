"""Linear algebra (cubed/array_api/linear_algebra_functions.py:13-155).

matmul = blockwise over (i, k, j) with a chunk GEMM per task (MFMA for f32)
writing a (m, 1, n) partial, then a sum reduction over the k axis
(``_sum_wo_cat``) -- the same DAG as the reference."""

from numbers import Integral
from typing import Iterable

import numpy as np

from .. import ir
from ..chunkfuncs import _chunk_sum
from ..core import blockwise, reduction, squeeze
from .data_type_functions import result_type
from .dtypes import _numeric_dtypes
from .manipulation_functions import expand_dims


def matmul(x1, x2, /):
    if x1.dtype not in _numeric_dtypes or x2.dtype not in _numeric_dtypes:
        raise TypeError("Only numeric dtypes are allowed in matmul")
    if x1.ndim == 0 or x2.ndim == 0:
        raise ValueError("matmul does not support 0-dimensional arrays.")
    x1_is_1d = x1.ndim == 1
    if x1_is_1d:
        x1 = expand_dims(x1, axis=0)
    x2_is_1d = x2.ndim == 1
    if x2_is_1d:
        x2 = expand_dims(x2, axis=-1)
    if x1.ndim < x2.ndim:
        x1 = expand_dims(x1, axis=tuple(range(x2.ndim - x1.ndim)))
    elif x1.ndim > x2.ndim:
        x2 = expand_dims(x2, axis=tuple(range(x1.ndim - x2.ndim)))
    out_ind = tuple(range(x1.ndim + 1))
    x1_ind = tuple(range(x1.ndim))
    x2_ind = tuple(range(x1.ndim - 2)) + (x1_ind[-1], x1.ndim)
    dtype = result_type(x1, x2)
    out = blockwise(ir.MatmulProgram(out_dtype=np.dtype(dtype)), out_ind, x1, x1_ind, x2, x2_ind,
                    adjust_chunks={x1_ind[-1]: 1}, dtype=dtype)
    out = _sum_wo_cat(out, axis=-2, dtype=dtype)
    if x1_is_1d:
        out = squeeze(out, -2)
    if x2_is_1d:
        out = squeeze(out, -1)
    return out


def _sum_wo_cat(a, axis=None, dtype=None):
    if a.shape[axis] == 1:
        return squeeze(a, axis)
    return reduction(a, _chunk_sum, axis=axis, dtype=dtype, extra_func_kwargs=dict(dtype=dtype))


def matrix_transpose(x, /):
    if x.ndim < 2:
        raise ValueError("x must be at least 2-dimensional for matrix_transpose")
    from .manipulation_functions import permute_dims

    axes = list(range(x.ndim))
    axes[-1], axes[-2] = axes[-2], axes[-1]
    return permute_dims(x, axes)


def outer(x1, x2, /):
    prog = ir.ExprProgram(
        ndim=2, nargs=2,
        outputs=ir.apply_op("multiply", [ir.Arg(0, x1.dtype, (0,)), ir.Arg(1, x2.dtype, (1,))],
                            result_type(x1, x2)),
        out_axes=(0, 1), name="outer")
    return blockwise(prog, "ij", x1, "i", x2, "j", dtype=result_type(x1, x2))


def tensordot(x1, x2, /, *, axes=2):
    from .statistical_functions import sum

    if x1.dtype not in _numeric_dtypes or x2.dtype not in _numeric_dtypes:
        raise TypeError("Only numeric dtypes are allowed in tensordot")
    if isinstance(axes, Iterable):
        x1_axes, x2_axes = axes
    else:
        x1_axes = tuple(range(x1.ndim - axes, x1.ndim))
        x2_axes = tuple(range(0, axes))
    if isinstance(x1_axes, Integral):
        x1_axes = (x1_axes,)
    if isinstance(x2_axes, Integral):
        x2_axes = (x2_axes,)
    x1_axes, x2_axes = tuple(x1_axes), tuple(x2_axes)
    dtype = result_type(x1, x2)
    x1_ind = list(range(x1.ndim))
    x2_ind = list(range(x1.ndim, x1.ndim + x2.ndim))
    out_ind = x1_ind + x2_ind
    adjust_chunks = {}
    for a1, a2 in zip(x1_axes, x2_axes):
        out_ind.remove(x2_ind[a2])
        x2_ind[a2] = x1_ind[a1]
        adjust_chunks[x1_ind[a1]] = lambda c: 1
    out = blockwise(ir.TensordotProgram(axes=(x1_axes, x2_axes), out_dtype=np.dtype(dtype)),
                    out_ind, x1, x1_ind, x2, x2_ind, dtype=dtype, adjust_chunks=adjust_chunks)
    return sum(out, axis=x1_axes, dtype=dtype)


def vecdot(x1, x2, /, *, axis=-1):
    if x1.dtype not in _numeric_dtypes or x2.dtype not in _numeric_dtypes:
        raise TypeError("Only numeric dtypes are allowed in vecdot")
    return tensordot(x1, x2, axes=((axis,), (axis,)))
