"""Creation functions (cubed/array_api/creation_functions.py).

asarray -> VirtualInMemoryArray (0-d ones fold into kernel constants),
full/ones/zeros -> VirtualFullArray (constants), empty -> VirtualEmptyArray,
arange/linspace/eye -> map_blocks over an Iota leaf (global index)."""

import math
from typing import TYPE_CHECKING, Iterable

import numpy as np

from .. import ir
from ..core import Plan, gensym
from ..core.ops import map_blocks
from ..storage import virtual_empty, virtual_full, virtual_in_memory, virtual_offsets
from ..utils import normalize_chunks, normalize_shape, to_chunksize

if TYPE_CHECKING:
    from .array_object import Array


def _Array():
    from .array_object import Array

    return Array


def asarray(obj, /, *, dtype=None, device=None, copy=None, chunks="auto", spec=None) -> "Array":
    a = obj
    Array = _Array()
    if isinstance(a, Array):
        return a
    if type(a).__module__.split(".")[0] == "xarray" and hasattr(a, "data"):  # pragma: no cover
        return asarray(a.data)
    if not isinstance(getattr(a, "shape", None), Iterable):
        a = np.asarray(a, dtype=dtype)
    else:
        a = np.asarray(a)
        if dtype is not None:
            a = a.astype(dtype)
    if dtype is None:
        dtype = a.dtype
    from ..ir import check_input_dtype

    check_input_dtype(a.dtype)
    chunksize = to_chunksize(normalize_chunks(chunks, shape=a.shape, dtype=dtype)) if a.ndim else ()
    name = gensym()
    target = virtual_in_memory(a, chunks=chunksize)
    plan = Plan._new(name, "asarray", target)
    return Array(name, target, spec, plan)


def empty(shape, *, dtype=None, device=None, chunks="auto", spec=None) -> "Array":
    shape = normalize_shape(shape)
    return empty_virtual_array(shape, dtype=dtype, device=device, chunks=chunks, spec=spec,
                               hidden=False)


def empty_like(x, /, *, dtype=None, device=None, chunks=None, spec=None) -> "Array":
    return empty(**_like_args(x, dtype, device, chunks, spec))


def empty_virtual_array(shape, *, dtype=None, device=None, chunks="auto", spec=None,
                        hidden=True) -> "Array":
    if dtype is None:
        dtype = np.float64
    chunksize = to_chunksize(normalize_chunks(chunks, shape=shape, dtype=dtype)) if len(shape) else ()
    name = gensym()
    target = virtual_empty(shape, dtype=dtype, chunks=chunksize)
    plan = Plan._new(name, "empty", target, hidden=hidden)
    return _Array()(name, target, spec, plan)


def full(shape, fill_value, *, dtype=None, device=None, chunks="auto", spec=None) -> "Array":
    shape = normalize_shape(shape)
    if dtype is None:
        if isinstance(fill_value, bool):
            dtype = np.bool_
        elif isinstance(fill_value, int):
            dtype = np.int64
        elif isinstance(fill_value, float):
            dtype = np.float64
        else:
            raise TypeError("Invalid input to full")
    chunksize = to_chunksize(normalize_chunks(chunks, shape=shape, dtype=dtype)) if len(shape) else ()
    name = gensym()
    target = virtual_full(shape, fill_value, dtype=dtype, chunks=chunksize)
    plan = Plan._new(name, "full", target)
    return _Array()(name, target, spec, plan)


def full_like(x, /, fill_value, *, dtype=None, device=None, chunks=None, spec=None) -> "Array":
    return full(fill_value=fill_value, **_like_args(x, dtype, device, chunks, spec))


def ones(shape, *, dtype=None, device=None, chunks="auto", spec=None) -> "Array":
    if dtype is None:
        dtype = np.float64
    return full(shape, 1, dtype=dtype, device=device, chunks=chunks, spec=spec)


def ones_like(x, /, *, dtype=None, device=None, chunks=None, spec=None) -> "Array":
    return ones(**_like_args(x, dtype, device, chunks, spec))


def zeros(shape, *, dtype=None, device=None, chunks="auto", spec=None) -> "Array":
    if dtype is None:
        dtype = np.float64
    return full(shape, 0, dtype=dtype, device=device, chunks=chunks, spec=spec)


def zeros_like(x, /, *, dtype=None, device=None, chunks=None, spec=None) -> "Array":
    return zeros(**_like_args(x, dtype, device, chunks, spec))


def offsets_virtual_array(shape, spec=None) -> "Array":
    name = gensym()
    target = virtual_offsets(shape)
    plan = Plan._new(name, "block_ids", target, hidden=True)
    return _Array()(name, target, spec, plan)


def _iota_program(chunks, expr_of_index, out_dtype):
    """map_blocks program over an empty template (arg 0) whose output is a
    function of the global indices (Iota leaves)."""
    ndim = len(chunks)
    e = expr_of_index([ir.Iota(d, 0, tuple(range(ndim)), chunks) for d in range(ndim)])
    return ir.ExprProgram(ndim=ndim, nargs=1, outputs=ir.cast(e, out_dtype),
                          out_axes=tuple(range(ndim)), name="iota")


def arange(start, /, stop=None, step=1, *, dtype=None, device=None, chunks="auto",
           spec=None) -> "Array":
    """arange via map_blocks (creation_functions.py:23-51): element i of
    the result is start + i * step, computed in the output dtype."""
    if stop is None:
        start, stop = 0, start
    num = int(max(math.ceil((stop - start) / step), 0))
    if dtype is None:
        dtype = np.arange(start, stop, step * num if num else step).dtype
    dtype = np.dtype(dtype)
    chunks = normalize_chunks(chunks, shape=(num,), dtype=dtype)

    def expr(ix):
        ct = np.dtype(np.float64) if dtype.kind == "f" or isinstance(step, float) or \
            isinstance(start, float) else np.dtype(np.int64)
        i = ir.cast(ix[0], ct)
        return ir.Binary("add", ir.Const(start, ct), ir.Binary("multiply", i, ir.Const(step, ct), ct), ct)

    return map_blocks(_iota_program(chunks, expr, dtype), dtype=dtype, chunks=chunks, spec=spec)


def linspace(start, stop, /, num, *, dtype=None, device=None, endpoint=True, chunks="auto",
             spec=None) -> "Array":
    range_ = stop - start
    div = (num - 1) if endpoint else num
    if div == 0:
        div = 1
    step = float(range_) / div
    if dtype is None:
        dtype = np.float64
    if num == 0:
        return asarray(0.0, dtype=dtype, spec=spec)
    chunks = normalize_chunks(chunks, shape=(num,), dtype=dtype)

    def expr(ix):
        f64 = np.dtype(np.float64)
        i = ir.cast(ix[0], f64)
        return ir.Binary("add", ir.Const(float(start), f64),
                         ir.Binary("multiply", i, ir.Const(step, f64), f64), f64)

    return map_blocks(_iota_program(chunks, expr, dtype), dtype=dtype, chunks=chunks, spec=spec)


def eye(n_rows, n_cols=None, /, *, k=0, dtype=None, device=None, chunks="auto",
        spec=None) -> "Array":
    if n_cols is None:
        n_cols = n_rows
    if dtype is None:
        dtype = np.float64
    shape = (n_rows, n_cols)
    chunks = normalize_chunks(chunks, shape=shape, dtype=dtype)

    def expr(ix):
        i64 = np.dtype(np.int64)
        diag = ir.Binary("subtract", ix[1], ix[0], i64)
        return ir.Binary("equal", diag, ir.Const(k, i64), np.dtype(np.bool_))

    return map_blocks(_iota_program(chunks, expr, dtype), dtype=dtype, chunks=chunks, spec=spec)


def tril(x, /, *, k=0) -> "Array":
    from .searching_functions import where

    if x.ndim < 2:
        raise ValueError("x must be at least 2-dimensional for tril")
    mask = _tri_mask(x.shape[-2], x.shape[-1], k, x.chunks[-2:], x.spec)
    return where(mask, x, zeros_like(x))


def triu(x, /, *, k=0) -> "Array":
    from .searching_functions import where

    if x.ndim < 2:
        raise ValueError("x must be at least 2-dimensional for triu")
    mask = _tri_mask(x.shape[-2], x.shape[-1], k - 1, x.chunks[-2:], x.spec)
    return where(mask, zeros_like(x), x)


def _tri_mask(N, M, k, chunks, spec):
    """mask[i, j] = i >= j - k, as one iota program."""
    chunks = normalize_chunks(chunks, shape=(N, M))

    def expr(ix):
        i64 = np.dtype(np.int64)
        return ir.Binary("greater_equal", ix[0], ir.Binary("subtract", ix[1], ir.Const(k, i64), i64),
                         np.dtype(np.bool_))

    return map_blocks(_iota_program(chunks, expr, np.bool_), dtype=np.bool_, chunks=chunks, spec=spec)


def _like_args(x, dtype=None, device=None, chunks=None, spec=None):
    if dtype is None:
        dtype = x.dtype
    if chunks is None:
        chunks = x.chunks
    if spec is None:
        spec = x.spec
    return dict(shape=x.shape, dtype=dtype, device=device, chunks=chunks, spec=spec)


def meshgrid(*arrays, indexing="xy"):
    """array_api/creation_functions.py:228-256: each 1-d input indexed with
    new axes, then broadcast together (views of index/broadcast programs)."""
    from .manipulation_functions import broadcast_arrays

    if len({a.dtype for a in arrays}) > 1:
        raise ValueError("meshgrid inputs must all have the same dtype")
    if indexing not in ("ij", "xy"):
        raise ValueError("`indexing` must be `'ij'` or `'xy'`")
    arrs = list(arrays)
    if indexing == "xy" and len(arrs) > 1:
        arrs[0], arrs[1] = arrs[1], arrs[0]
    grid = []
    for i in range(len(arrs)):
        s = [None] * len(arrs)
        s[i] = slice(None)
        grid.append(arrs[i][tuple(s)])
    grid = list(broadcast_arrays(*grid))
    if indexing == "xy" and len(arrs) > 1:
        grid[0], grid[1] = grid[1], grid[0]
    return grid
