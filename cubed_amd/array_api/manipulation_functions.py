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


def concat(arrays, /, *, axis=0):
    """array_api/manipulation_functions.py:76-104: a map_direct whose output
    blocks (chunked like ``arrays[0]``) read regions of every input; lowered
    to one box-copy launch (or a scratch gather when fused)."""
    from ..core.ops import ConcatRegions, map_direct
    from ..utils import to_chunksize

    if not arrays:
        raise ValueError("Need array(s) to concat")
    arrays = list(arrays)
    if axis is None:
        arrays = [flatten(a) for a in arrays]
        axis = 0
    a = arrays[0]
    axis = validate_axis(axis, a.ndim)
    # nxp.concat promotes and the write casts back to a.dtype
    arrays = [x if x.dtype == a.dtype else _astype(x, a.dtype) for x in arrays]
    offsets = [0]
    for x in arrays:
        offsets.append(offsets[-1] + x.shape[axis])
    shape = a.shape[:axis] + (offsets[-1],) + a.shape[axis + 1:]
    chunks = normalize_chunks(to_chunksize(a.chunks), shape=shape, dtype=a.dtype)
    return map_direct(ConcatRegions(chunks, axis, offsets), *arrays, shape=shape, dtype=a.dtype,
                      chunks=chunks, extra_projected_mem=a.chunkmem)


def _astype(x, dtype):
    from .data_type_functions import astype

    return astype(x, dtype)


def stack(arrays, /, *, axis=0):
    """array_api/manipulation_functions.py:278-312: output block i along the
    new axis is block-for-block arrays[i] with a unit dim inserted."""
    from ..core.ops import general_blockwise

    if not arrays:
        raise ValueError("Need array(s) to stack")
    a = arrays[0]
    axis = validate_axis(axis, a.ndim + 1)
    # the reference reads arrays[i]'s chunk (i's own chunking) into a's
    # chunk shape; matching chunks (and dtype) first keeps that well defined
    arrays = [x if x.dtype == a.dtype else _astype(x, a.dtype) for x in arrays]
    arrays = [x if x.chunks == a.chunks else x.rechunk(a.chunks) for x in arrays]
    shape = a.shape[:axis] + (len(arrays),) + a.shape[axis:]
    chunks = a.chunks[:axis] + ((1,) * len(arrays),) + a.chunks[axis:]
    names = [x.name for x in arrays]

    def block_function(out_key):
        c = out_key[1:]
        return ((names[c[axis]], *(c[:axis] + c[axis + 1:])),)

    n = a.ndim + 1
    leaf_axes = tuple(d if d < axis else d + 1 for d in range(a.ndim))
    prog = ir.ExprProgram(ndim=n, nargs=1, outputs=ir.Arg(0, a.dtype, leaf_axes),
                          out_axes=tuple(range(n)), name="stack")
    return general_blockwise(prog, block_function, *arrays, shape=shape, dtype=a.dtype,
                             chunks=chunks)


def flatten(x):
    return reshape(x, (-1,))


def reshape(x, /, shape, *, copy=None):
    """array_api/manipulation_functions.py:210-246 (dask's reshape): rechunk
    so every input block maps to one output block, then reinterpret each
    C-order chunk with the output extents (a flat copy, no arithmetic)."""
    import math as _m

    from ..utils import to_chunksize

    shape = tuple(shape)
    known = [s for s in shape if s != -1]
    if len(known) != len(shape):
        if len(shape) - len(known) > 1:
            raise ValueError("can only specify one unknown dimension")
        if len(shape) == 1 and x.ndim == 1:
            return x
        missing = x.size // _m.prod(known)
        shape = tuple(missing if s == -1 else s for s in shape)
    if _m.prod(shape) != x.size:
        raise ValueError("total size of new array must be unchanged")
    if x.shape == shape:
        return x
    if x.npartitions == 1:
        return reshape_chunks(x, shape, tuple((d,) for d in shape))
    inchunks, outchunks = reshape_rechunk(x.shape, shape, x.chunks)
    x2 = x.rechunk(to_chunksize(inchunks))
    return reshape_chunks(x2, shape, outchunks)


def reshape_chunks(x, shape, chunks):
    import math as _m

    from ..core.ops import general_blockwise
    from ..utils import block_id_to_offset, offset_to_block_id

    if _m.prod(shape) != x.size:
        raise ValueError("total size of new array must be unchanged")
    outchunks = normalize_chunks(chunks, shape=shape, dtype=x.dtype)
    template = empty(shape, dtype=x.dtype, chunks=chunks, spec=x.spec)
    out_nb = tuple(len(c) for c in outchunks)
    in_nb = x.numblocks
    if _m.prod(out_nb) != _m.prod(in_nb):
        raise ValueError(f"reshape: {in_nb} input blocks cannot map onto {out_nb} output blocks")

    def block_function(out_key):
        oc = out_key[1:]
        ic = offset_to_block_id(block_id_to_offset(oc, out_nb), in_nb)
        return ((x.name, *ic), (template.name, *oc))

    n = len(shape)
    leaf = ir.ReshapeArg(0, x.dtype, tuple(range(n)), in_numblocks=tuple(in_nb),
                         out_chunks=tuple(outchunks))
    prog = ir.ExprProgram(ndim=n, nargs=2, outputs=leaf, out_axes=tuple(range(n)), name="reshape")
    return general_blockwise(prog, block_function, x, template, shape=shape, dtype=x.dtype,
                             chunks=outchunks)


def reshape_rechunk(inshape, outshape, inchunks):
    """Input chunks to rechunk to, and the resulting output chunks, so that a
    reshape maps blocks one to one (restates dask's reshape_rechunk,
    vendor/dask/array/reshape.py:20-98, used at manipulation_functions.py
    :241).  Dims are matched from the right: equal extents keep their
    chunks; a run of input dims merging into one output dim keeps chunking
    only on its leftmost dim (the others whole); one input dim splitting into
    a run of output dims is chunked in multiples of the run's inner size."""
    import math as _m

    res_in = [None] * len(inshape)
    res_out = [None] * len(outshape)
    i, o = len(inshape) - 1, len(outshape) - 1
    while i >= 0 or o >= 0:
        din, dout = inshape[i], outshape[o]
        if din == dout:
            res_in[i] = res_out[o] = inchunks[i]
            i -= 1
            o -= 1
        elif din == 1:
            res_in[i] = (1,)
            i -= 1
        elif dout == 1:
            res_out[o] = (1,)
            o -= 1
        elif din < dout:  # input dims left..i merge into output dim o
            left = i - 1
            while left >= 0 and _m.prod(inshape[left:i + 1]) < dout:
                left -= 1
            if _m.prod(inshape[left:i + 1]) != dout:
                raise NotImplementedError(_UNEVEN)
            if all(len(inchunks[k]) == inshape[k] for k in range(i)):
                # all lower dims chunked by 1: blocks just move around
                for k in range(i + 1):
                    res_in[k] = inchunks[k]
                res_out[o] = inchunks[i] * _m.prod(len(c) for c in inchunks[left:i])
            else:
                for k in range(left + 1, i + 1):
                    res_in[k] = (inshape[k],)
                nsplit = _m.prod(len(c) for c in inchunks[left + 1:i + 1])
                res_in[left] = _expand_chunks(inchunks[left], nsplit)
                inner = _m.prod(inshape[left + 1:i + 1])
                res_out[o] = tuple(inner * c for c in res_in[left])
            o -= 1
            i = left - 1
        else:  # input dim i splits into output dims left..o
            left = o - 1
            while left >= 0 and _m.prod(outshape[left:o + 1]) < din:
                left -= 1
            if _m.prod(outshape[left:o + 1]) != din:
                raise NotImplementedError(_UNEVEN)
            inner = _m.prod(outshape[left + 1:o + 1])
            res_in[i] = _contract_chunks(inchunks[i], inner)
            for k in range(left + 1, o + 1):
                res_out[k] = (outshape[k],)
            res_out[left] = tuple(c // inner for c in res_in[i])
            o = left - 1
            i -= 1
    return tuple(res_in), tuple(res_out)


_UNEVEN = ("reshape only supports merging or splitting existing dimensions evenly "
           "(e.g. (6, 5, 4) -> (3, 2, 5, 4) or (30, 4), not (4, 5, 6)); reshape in "
           "several passes instead")


def _expand_chunks(chunks, factor):
    """Split each chunk into about ``factor`` pieces (sizes >= 1)."""
    if factor == 1:
        return tuple(chunks)
    out = []
    for c in chunks:
        part = max(c / factor, 1)
        rest = c
        while rest >= 2 * part:
            out.append(int(part))
            rest -= int(part)
        if rest:
            out.append(rest)
    return tuple(out)


def _contract_chunks(chunks, factor):
    """Chunks that are all multiples of ``factor``: each chunk is cut down to
    a multiple and its remainder carried into the next one."""
    if sum(chunks) % factor:
        raise NotImplementedError(_UNEVEN)
    out, carry = [], 0
    for c in chunks:
        c += carry
        carry = c % factor
        if c - carry:
            out.append(c - carry)
    return tuple(out)
