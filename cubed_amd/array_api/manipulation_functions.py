"""Manipulation functions needed by the hot path (broadcast_to,
expand_dims, permute_dims, squeeze) -- cubed/array_api/manipulation_functions.py
:35-69, :155-170, :188-207.  Each is a map/blockwise whose program only
re-maps axes, so it fuses into its neighbours' kernels."""

import numpy as np

from .. import ir
from ..core import squeeze  # noqa: F401
from ..core import blockwise, unify_chunks
from ..core.ops import elemwise, map_blocks, validate_axis
from ..utils import normalize_chunks
from .creation_functions import empty


def broadcast_arrays(*arrays):
    inds = [list(reversed(range(x.ndim))) for x in arrays]
    args = []
    for a, i in zip(arrays, inds):
        args += [a, tuple(i)]
    _, args = unify_chunks(*args)
    shape = np.broadcast_shapes(*(e.shape for e in args))
    chunks = _broadcast_chunks(*(e.chunks for e in args))
    return tuple(broadcast_to(e, shape=shape, chunks=chunks) for e in args)


def _broadcast_chunks(*chunkss):
    if not chunkss:
        return ()
    n = max(len(c) for c in chunkss)
    out = []
    for i in range(n):
        cands = [c[i - (n - len(c))] for c in chunkss if i - (n - len(c)) >= 0]
        non1 = [c for c in cands if c != (1,)]
        out.append(non1[0] if non1 else cands[0])
    return tuple(out)


def broadcast_to(x, /, shape, *, chunks=None):
    shape = tuple(shape)
    if x.shape == shape and (chunks is None or chunks == x.chunks):
        return x
    ndim_new = len(shape) - x.ndim
    if ndim_new < 0 or any(new != old for new, old in zip(shape[ndim_new:], x.shape) if old != 1):
        raise ValueError(f"cannot broadcast shape {x.shape} to shape {shape}")
    if chunks is None:
        xchunks = normalize_chunks(x.chunks, x.shape, dtype=x.dtype)
        chunks = tuple((1,) * s for s in shape[:ndim_new]) + tuple(
            bd if old > 1 else ((1,) * new if new > 0 else (0,))
            for bd, old, new in zip(xchunks, x.shape, shape[ndim_new:]))
    else:
        chunks = normalize_chunks(chunks, shape, dtype=x.dtype, previous_chunks=x.chunks)
        for old_bd, new_bd in zip(x.chunks, chunks[ndim_new:]):
            if old_bd != new_bd and old_bd != (1,):
                raise ValueError(
                    f"cannot broadcast chunks {x.chunks} to chunks {chunks}: new chunks must either "
                    "be along a new dimension or a dimension of size 1")
    template = empty(shape, dtype=np.int8, chunks=chunks, spec=x.spec)
    n = len(shape)
    prog = ir.ExprProgram(ndim=n, nargs=2,
                          outputs=ir.Arg(0, x.dtype, ir.right_aligned_axes(x.ndim, n)),
                          out_axes=tuple(range(n)), name="broadcast_to")
    return elemwise(prog, x, template, dtype=x.dtype)


def expand_dims(x, /, *, axis):
    if not isinstance(axis, tuple):
        axis = (axis,)
    ndim_new = len(axis) + x.ndim
    axis = validate_axis(axis, ndim_new)
    chunks_it = iter(x.chunks)
    chunks = tuple(1 if i in axis else next(chunks_it) for i in range(ndim_new))
    # space = input dims; new unit output dims have no space dim
    out_axes, k = [], 0
    for i in range(ndim_new):
        if i in axis:
            out_axes.append(None)
        else:
            out_axes.append(k)
            k += 1
    prog = ir.ExprProgram(ndim=x.ndim, nargs=1, outputs=ir.Arg(0, x.dtype, tuple(range(x.ndim))),
                          out_axes=tuple(out_axes), name="expand_dims")
    return map_blocks(prog, x, dtype=x.dtype, chunks=chunks, new_axis=axis)


def permute_dims(x, /, axes):
    if axes:
        if len(axes) != x.ndim:
            raise ValueError("axes don't match array")
    else:
        axes = tuple(range(x.ndim))[::-1]
    axes = tuple(d + x.ndim if d < 0 else d for d in axes)
    extra_projected_mem = x.chunkmem
    # output dim j = input dim axes[j]; space = output dims
    arg_axes = [None] * x.ndim
    for j, a in enumerate(axes):
        arg_axes[a] = j
    prog = ir.ExprProgram(ndim=x.ndim, nargs=1, outputs=ir.Arg(0, x.dtype, tuple(arg_axes)),
                          out_axes=tuple(range(x.ndim)), name="permute_dims")
    return blockwise(prog, axes, x, tuple(range(x.ndim)), dtype=x.dtype,
                     extra_projected_mem=extra_projected_mem)


def moveaxis(x, source, destination, /):
    src = tuple(validate_axis(s, x.ndim) for s in (source if isinstance(source, (tuple, list)) else (source,)))
    dst = tuple(validate_axis(d, x.ndim) for d in (destination if isinstance(destination, (tuple, list)) else (destination,)))
    if len(src) != len(dst):
        raise ValueError("`source` and `destination` arguments must have the same number of elements")
    order = [n for n in range(x.ndim) if n not in src]
    for d, s in sorted(zip(dst, src)):
        order.insert(d, s)
    return permute_dims(x, order)
