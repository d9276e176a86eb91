"""Core ops: the public blockwise / reduction / rechunk API.

Mirrors cubed/core/ops.py (from_array :40, blockwise :185-302,
general_blockwise :305-356, elemwise :359-371, index :374-517, map_blocks
:520-643, map_direct :646-699, rechunk :702-758, merge_chunks :761-787,
reduction :790-903, reduction_new/partial_reduce/tree_reduce :906-1090,
squeeze :1156, unify_chunks :1172-1219) with the same signatures, chunk
inference, projected-memory errors and reduction rounds.  What changes is the
chunk function: each op attaches an IR program (cubed_amd/ir.py) so the
MI355X executor can lower the pipeline to one kernel launch.
"""

from __future__ import annotations

import builtins
import math
import numbers
from functools import partial
from itertools import product
from numbers import Integral, Number
from typing import TYPE_CHECKING, Any, Sequence, Union

import numpy as np

from .. import ir
from ..chunkfuncs import ChunkMap, ChunkReduction, as_chunk_reduction
from ..primitive.blockwise import blockwise as primitive_blockwise
from ..primitive.blockwise import general_blockwise as primitive_general_blockwise
from ..primitive.rechunk import rechunk as primitive_rechunk
from ..storage import DeviceArray, HostArray
from ..utils import (
    chunk_memory,
    common_blockdim,
    get_item,
    normalize_chunks,
    offset_to_block_id,
    to_chunksize,
)
from .array import CoreArray, check_array_specs, compute, gensym
from .plan import Plan, new_temp_path

if TYPE_CHECKING:
    from ..array_api.array_object import Array


def _Array():
    from ..array_api.array_object import Array

    return Array


# ------------------------------------------------------------------ sources


def from_array(x, chunks="auto", asarray=None, spec=None) -> "Array":
    """Create an array from an in-memory array-like; chunks are uploaded to
    HBM by the executor (reference: map_blocks(_from_array), core/ops.py:40-85)."""
    if isinstance(x, CoreArray):
        raise ValueError("Array is already a Cubed array. Use 'asarray' or 'rechunk' instead.")
    from ..ir import check_input_dtype

    check_input_dtype(x.dtype)
    previous_chunks = getattr(x, "chunks", None)
    outchunks = normalize_chunks(chunks, x.shape, dtype=x.dtype, previous_chunks=previous_chunks)
    host = HostArray(np.asarray(x) if (asarray or asarray is None) else x, to_chunksize(outchunks) if x.ndim else ())
    name = gensym()
    from .array import CoreArray as _CA  # noqa: F401

    spec = spec or _default_spec()
    target = DeviceArray(x.shape, x.dtype, to_chunksize(outchunks) if x.ndim else (), name=name)
    op = upload_op(host, target, spec)
    plan = Plan._new(name, "from_array", target, op, False)
    return _Array()(name, target, spec, plan)


def _default_spec():
    from ..spec import Spec

    return Spec(None, allowed_mem=200_000_000, reserved_mem=100_000_000)


def upload_stage(item, *, config=None):
    raise TypeError("uploads run only through the MI355X executor")


class UploadSpec:
    def __init__(self, source: HostArray, target: DeviceArray):
        self.source = source
        self.target = target


def upload_op(host: HostArray, target: DeviceArray, spec):
    from ..primitive.types import PrimitiveOperation
    from ..runtime.types import CubedPipeline

    pipeline = CubedPipeline(upload_stage, gensym("upload"), [], UploadSpec(host, target))
    projected = spec.reserved_mem + 2 * chunk_memory(target.dtype, target.chunks)
    return PrimitiveOperation(pipeline=pipeline, target_array=target, projected_mem=projected,
                              allowed_mem=spec.allowed_mem, reserved_mem=spec.reserved_mem,
                              num_tasks=target.nchunks, fusable=False)


def from_zarr(store, spec=None) -> "Array":
    from .. import zarr_io

    return zarr_io.from_zarr(store, spec=spec)


def store(sources, targets, executor=None, **kwargs):
    from .. import zarr_io

    return zarr_io.store(sources, targets, executor=executor, **kwargs)


def to_zarr(x, store, executor=None, **kwargs):
    from .. import zarr_io

    return zarr_io.to_zarr(x, store, executor=executor, **kwargs)


# ------------------------------------------------------------------ lowering of callables


def _lower_callable(func, arrays, inds, out_ind, dtype, kwargs):
    """IR program for ``func`` called on chunks of ``arrays`` laid out by
    ``inds`` in the output space ``out_ind``.  Numpy ufuncs lower to
    expressions; everything else becomes an OpaqueProgram (the executor then
    refuses the plan)."""
    if isinstance(func, ir.Program):
        return func
    if isinstance(func, _BlockIdFunc):
        # the last argument is the block-offsets array map_blocks appended
        meta = tuple((np.dtype(a.dtype), a.ndim) for a in arrays[:-1])
        return ir.PerBlockProgram(func=func.func, kwargs=dict(kwargs), args_meta=meta,
                                  inds=tuple(inds[:-1]), out_ind=tuple(out_ind), dtype=dtype,
                                  nargs=len(arrays))
    if isinstance(func, partial) and not func.args:
        base = func.func
        kwargs = {**func.keywords, **kwargs}
    else:
        base = func
    name = ir.NUMPY_ELEMENTWISE.get(base)
    if name is not None and not kwargs:
        space = len(out_ind)
        pos = {idx: i for i, idx in enumerate(out_ind)}
        args = []
        for i, (a, ind) in enumerate(zip(arrays, inds)):
            if ind is None or any(idx not in pos for idx in ind):
                return ir.OpaqueProgram(func=func, nargs=len(arrays))
            args.append(ir.Arg(i, a.dtype, tuple(pos[idx] for idx in ind)))
        try:
            e = ir.apply_op(name, args, dtype)
        except NotImplementedError:
            return ir.OpaqueProgram(func=func, nargs=len(arrays))
        return ir.ExprProgram(ndim=space, nargs=len(args), outputs=e,
                              out_axes=tuple(range(space)), name=name)
    # a numpy reduction applied per chunk with keepdims (map_blocks(np.max,
    # x, axis=0, keepdims=True)): the per-chunk reduce program of reduction()
    red = as_chunk_reduction(base)
    if red is not None and len(arrays) == 1 and kwargs.get("keepdims") and \
            set(kwargs) <= {"axis", "keepdims", "dtype"} and tuple(inds[0] or ()) == tuple(out_ind):
        ax = kwargs.get("axis")
        nd = arrays[0].ndim
        ax = tuple(range(nd)) if ax is None else tuple(a % nd for a in (ax if isinstance(ax, tuple) else (ax,)))
        extra = {"dtype": kwargs["dtype"]} if kwargs.get("dtype") is not None else {}
        try:
            return red.program(nd, arrays[0].dtype, ax, keepdims=True, **extra)
        except (NotImplementedError, TypeError, ValueError):
            pass
    from ..tracing import trace_callable

    traced = trace_callable(func, arrays, inds, out_ind, dtype, kwargs)
    if traced is not None:
        return traced
    return ir.OpaqueProgram(func=func, nargs=len(arrays))


# ------------------------------------------------------------------ blockwise


def blockwise(func, out_ind, *args: Any, dtype=None, adjust_chunks=None, new_axes=None,
              align_arrays=True, target_store=None, extra_func_kwargs=None, **kwargs) -> "Array":
    arrays = args[::2]
    assert len(arrays) > 0
    new_axes = new_axes or {}
    new = (set(out_ind) - {a for arg in args[1::2] if arg is not None for a in arg}
           - set(new_axes or ()))
    if new:
        raise ValueError("Unknown dimension", new)
    if align_arrays:
        chunkss, arrays = unify_chunks(*args)
    else:
        chunkss = {}
        for arg, ind in zip(arrays, args[1::2]):
            arg_chunks = normalize_chunks(arg.chunks, shape=arg.shape, dtype=arg.dtype)
            for c, i in zip(arg_chunks, ind):
                if i not in chunkss or len(c) > len(chunkss[i]):
                    chunkss[i] = c
    for k, v in new_axes.items():
        if not isinstance(v, tuple):
            v = (v,)
        chunkss[k] = v
    chunks = [chunkss[i] for i in out_ind]
    if adjust_chunks:
        for i, ind in enumerate(out_ind):
            if ind in adjust_chunks:
                aj = adjust_chunks[ind]
                if callable(aj):
                    chunks[i] = tuple(map(aj, chunks[i]))
                elif isinstance(aj, numbers.Integral):
                    chunks[i] = tuple(aj for _ in chunks[i])
                elif isinstance(aj, (tuple, list)):
                    if len(aj) != len(chunks[i]):
                        raise ValueError(
                            f"Dimension {i} has {len(chunks[i])} blocks, adjust_chunks "
                            f"specified with {len(aj)} blocks")
                    chunks[i] = tuple(aj)
                else:
                    raise NotImplementedError("adjust_chunks values must be callable, int, or tuple")
    _chunks = tuple(chunks)
    shape = tuple(map(sum, _chunks))

    zargs = list(args)
    zargs[::2] = [a.zarray_maybe_lazy for a in arrays]
    in_names = [a.name for a in arrays]
    extra_source_arrays = kwargs.pop("extra_source_arrays", [])
    source_arrays = list(arrays) + list(extra_source_arrays)
    extra_projected_mem = kwargs.pop("extra_projected_mem", 0)
    fusable = kwargs.pop("fusable", True)

    program = _lower_callable(func, arrays, args[1::2], out_ind, dtype,
                              {**kwargs, **(extra_func_kwargs or {})})
    name = gensym()
    spec = check_array_specs(arrays)
    if target_store is None:
        target_store = new_temp_path(name=name, spec=spec)
    op = primitive_blockwise(
        program, out_ind, *zargs, allowed_mem=spec.allowed_mem, reserved_mem=spec.reserved_mem,
        extra_projected_mem=extra_projected_mem, target_store=target_store, shape=shape,
        dtype=dtype, chunks=_chunks, new_axes=new_axes, in_names=in_names, out_name=name,
        extra_func_kwargs=extra_func_kwargs, fusable=fusable)
    if isinstance(op.target_array, DeviceArray):
        op.target_array.name = name
    plan = Plan._new(name, "blockwise", op.target_array, op, False, *source_arrays)
    return _Array()(name, op.target_array, spec, plan)


def general_blockwise(func, block_function, *arrays, shape, dtype, chunks, target_store=None,
                      extra_func_kwargs=None, **kwargs) -> "Array":
    assert len(arrays) > 0
    zargs = [a.zarray_maybe_lazy for a in arrays]
    in_names = [a.name for a in arrays]
    extra_source_arrays = kwargs.pop("extra_source_arrays", [])
    source_arrays = list(arrays) + list(extra_source_arrays)
    extra_projected_mem = kwargs.pop("extra_projected_mem", 0)
    name = gensym()
    spec = check_array_specs(arrays)
    if target_store is None:
        target_store = new_temp_path(name=name, spec=spec)
    program = func if isinstance(func, ir.Program) else ir.OpaqueProgram(func=func, nargs=len(arrays))
    op = primitive_general_blockwise(
        program, block_function, *zargs, allowed_mem=spec.allowed_mem,
        reserved_mem=spec.reserved_mem, extra_projected_mem=extra_projected_mem,
        target_store=target_store, shape=shape, dtype=dtype, chunks=chunks, in_names=in_names,
        extra_func_kwargs=extra_func_kwargs)
    if isinstance(op.target_array, DeviceArray):
        op.target_array.name = name
    plan = Plan._new(name, "blockwise", op.target_array, op, False, *source_arrays)
    return _Array()(name, op.target_array, spec, plan)


def elemwise(func, *args: "Array", dtype=None) -> "Array":
    """Apply an elementwise op to broadcast array arguments.  ``func`` is an
    op name (ir.UNARY_OPS / ir.BINARY_OPS / "where") or a numpy ufunc."""
    shapes = [arg.shape for arg in args]
    out_ndim = len(np.broadcast_shapes(*shapes))
    expr_inds = tuple(range(out_ndim))[::-1]
    if dtype is None:
        raise ValueError("dtype must be specified for elemwise")
    opname = func if isinstance(func, str) else ir.NUMPY_ELEMENTWISE.get(func)
    if opname is not None:
        program = ir.elementwise_program(opname, [a.dtype for a in args],
                                         [a.ndim for a in args], dtype)
    else:
        program = func
    pairs = []
    for a in args:
        pairs += [a, tuple(range(a.ndim)[::-1])]
    return blockwise(program, expr_inds, *pairs, dtype=dtype)


# ------------------------------------------------------------------ index


def _is_int(x):
    return isinstance(x, (Integral, np.integer)) and not isinstance(x, bool)


def index(x, key):
    """Subset an array along one or more axes (basic indexing: slices with
    step >= 1, integers, None, Ellipsis, and one integer list)."""
    if not isinstance(key, tuple):
        key = (key,)
    if all(isinstance(ind, slice) and ind == slice(None) for ind in key):
        return x
    where_none = [i for i, ind in enumerate(key) if ind is None]
    for i, a in enumerate(where_none):
        n = sum(_is_int(ind) for ind in key[:a])
        if n:
            where_none[i] -= n
    key = tuple(ind for ind in key if ind is not None)
    selection = tuple(
        s.compute().tolist() if isinstance(s, CoreArray) else s for s in key)
    selection = tuple(s.tolist() if isinstance(s, np.ndarray) else s for s in selection)
    # replace ellipsis
    if any(s is Ellipsis for s in selection):
        i = [k for k, s in enumerate(selection) if s is Ellipsis][0]
        n_missing = x.ndim - (len(selection) - 1)
        selection = selection[:i] + (slice(None),) * n_missing + selection[i + 1:]
    selection = selection + (slice(None),) * (x.ndim - len(selection))
    if any(isinstance(s, slice) and s.step is not None and s.step < 1 for s in selection):
        raise NotImplementedError(f"Slice step must be >= 1: {key}")
    if sum(isinstance(s, list) for s in selection) > 1:
        raise NotImplementedError("Only one integer array index is allowed.")

    # normalized selection + output geometry (zarr OrthogonalIndexer semantics)
    norm = []
    shape, chunks, merged = [], [], []
    for d, s in enumerate(selection):
        n = x.shape[d]
        dcl = x.chunksize[d]
        if isinstance(s, slice):
            start, stop, step = s.indices(n)
            length = max(0, (stop - start + (step - 1)) // step)
            norm.append(slice(start, stop, step))
            shape.append(length)
            cl = max(dcl // step, 1)
            chunks.append(cl)
            if step == 1 or dcl // step < 1:
                merged.append(dcl)
            else:
                merged.append((dcl // step) * step)
        elif isinstance(s, list):
            lst = [int(v) + n if int(v) < 0 else int(v) for v in s]
            norm.append(lst)
            shape.append(len(lst))
            chunks.append(dcl)
            merged.append(dcl)
        elif _is_int(s):
            v = int(s)
            if v < 0:
                v += n
            if not 0 <= v < n:
                raise IndexError(f"index {s} is out of bounds for axis {d} with size {n}")
            norm.append(v)
        else:
            raise NotImplementedError(f"unsupported index {s!r}")
    shape = tuple(shape)
    target_chunks = normalize_chunks(tuple(chunks), shape, dtype=x.dtype)
    extra_projected_mem = x.chunkmem
    out = map_direct(
        _read_index_region(norm, target_chunks), x, shape=shape, dtype=x.dtype,
        chunks=target_chunks, extra_projected_mem=extra_projected_mem,
        target_chunks=target_chunks, selection=tuple(norm))
    merged = tuple(merged)
    if tuple(chunks) != merged:
        out = merge_chunks(out, merged)
    for axis in where_none:
        from ..array_api.manipulation_functions import expand_dims

        out = expand_dims(out, axis=axis)
    return out


class _read_index_region:
    """Region of ``x`` that output block ``block_id`` of ``x[selection]``
    reads (core/ops.py:489-517 _target_chunk_selection)."""

    def __init__(self, selection, target_chunks):
        self.selection = selection
        self.target_chunks = target_chunks

    def __call__(self, block_id):
        sel = []
        i = 0
        for s in self.selection:
            if isinstance(s, slice):
                starts = [s.start]
                for c in self.target_chunks[i]:
                    starts.append(starts[-1] + c * s.step)
                j = block_id[i]
                sel.append(slice(starts[j], starts[j + 1], s.step))
                i += 1
            elif isinstance(s, list):
                st = [0]
                for c in self.target_chunks[i]:
                    st.append(st[-1] + c)
                j = block_id[i]
                sel.append(s[st[j]:st[j + 1]])
                i += 1
            else:
                sel.append(s)
        return tuple(sel)


# ------------------------------------------------------------------ map_blocks


class _BlockIdProgram:
    """Marker for program builders that need the task's block id: the
    builder gets ``block_arg`` = index of the offsets argument."""

    def __init__(self, build, nargs_without_offsets):
        self.build = build
        self.nargs = nargs_without_offsets


def map_blocks(func, *args: "Array", dtype=None, chunks=None, drop_axis=[], new_axis=None,
               spec=None, **kwargs) -> "Array":
    """Apply a function to corresponding blocks from multiple input arrays."""
    if len(args) == 0:
        from ..array_api.creation_functions import empty_virtual_array

        shape = tuple(map(sum, chunks))
        args = (empty_virtual_array(shape, dtype=dtype, chunks=chunks, spec=spec),)
    if isinstance(func, _BlockIdProgram) or _has_block_id(func):
        from ..array_api.creation_functions import offsets_virtual_array

        arg0 = args[0]
        offsets = offsets_virtual_array(arg0.numblocks, arg0.spec)
        new_args = args + (offsets,)
        if isinstance(func, _BlockIdProgram):
            func = func.build(len(args))
        else:
            func = _BlockIdFunc(func)
        return _map_blocks(func, *new_args, dtype=dtype, chunks=chunks, drop_axis=drop_axis,
                           new_axis=new_axis, **kwargs)
    return _map_blocks(func, *args, dtype=dtype, chunks=chunks, drop_axis=drop_axis,
                       new_axis=new_axis, **kwargs)


class _BlockIdFunc:
    """A user function taking ``block_id``: lowered per block (PerBlockProgram)."""

    def __init__(self, func):
        self.func = func


def _has_block_id(func) -> bool:
    import inspect

    if isinstance(func, (ir.Program, ChunkMap, ChunkReduction)):
        return False
    try:
        return "block_id" in inspect.signature(func).parameters
    except (TypeError, ValueError):
        return False


def _map_blocks(func, *args: "Array", dtype=None, chunks=None, drop_axis=[], new_axis=None,
                **kwargs) -> "Array":
    new_axes = {}
    if isinstance(drop_axis, Number):
        drop_axis = [drop_axis]
    if isinstance(new_axis, Number):
        new_axis = [new_axis]
    arrs = args
    argpairs = [(a, tuple(range(a.ndim))[::-1]) if isinstance(a, CoreArray) else (a, None)
                for a in args]
    out_ind = tuple(range(max(a.ndim for a in arrs)))[::-1] if arrs else ()
    if drop_axis:
        ndim_out = len(out_ind)
        if any(i < -ndim_out or i >= ndim_out for i in drop_axis):
            raise ValueError(f"drop_axis out of range (drop_axis={drop_axis}, but output is {ndim_out}d).")
        drop_axis = [i % ndim_out for i in drop_axis]
        out_ind = tuple(x for i, x in enumerate(out_ind) if i not in drop_axis)
    if new_axis is None and chunks is not None and len(out_ind) < len(chunks):
        new_axis = range(len(chunks) - len(out_ind))
    if new_axis:
        temp_out_ind = list(out_ind)
        for ax in sorted(new_axis):
            n = len(temp_out_ind) + len(drop_axis)
            temp_out_ind.insert(ax, n)
            new_axes[n] = chunks[ax] if chunks is not None else 1
        out_ind = tuple(temp_out_ind)
        if max(new_axis) > max(out_ind):
            raise ValueError("New_axis values do not fill in all dimensions")
    if chunks is not None:
        if len(chunks) != len(out_ind):
            raise ValueError(f"Provided chunks have {len(chunks)} dims; expected {len(out_ind)} dims")
        adjust_chunks = dict(zip(out_ind, chunks))
    else:
        adjust_chunks = None
    pairs = []
    for a, ind in argpairs:
        pairs += [a, ind]
    return blockwise(func, out_ind, *pairs, dtype=dtype, adjust_chunks=adjust_chunks,
                     new_axes=new_axes, align_arrays=False, **kwargs)


def map_direct(func, *args: "Array", shape, dtype, chunks, extra_projected_mem, spec=None,
               **kwargs) -> "Array":
    """Apply ``func`` over the blocks of a new array, reading side inputs
    directly.  ``func(block_id) -> region`` of the first side input (the only
    form the MI355X lowering needs: merge_chunks and index)."""
    from ..array_api.creation_functions import empty_virtual_array

    if spec is None and len(args) > 0 and hasattr(args[0], "spec"):
        spec = args[0].spec
    out = empty_virtual_array(shape, dtype=dtype, chunks=chunks, spec=spec)
    kwargs.pop("target_chunks", None)
    kwargs.pop("selection", None)
    ndim = len(shape)
    src = args[0]
    region_fn = func
    # space dims of the region: source dims not removed by integer indexing
    sel = getattr(func, "selection", None)
    if sel is not None:
        axes, k = [], 0
        for s in sel:
            if _is_int(s):
                axes.append(None)
            else:
                axes.append(k)
                k += 1
        axes = tuple(axes)
    else:
        axes = tuple(range(src.ndim))

    def build(block_arg):
        if isinstance(region_fn, ConcatRegions):
            leaf = ir.Concat(src.name, np.dtype(dtype), tuple(range(ndim)), region_fn, block_arg,
                             sources=tuple(a.zarray_maybe_lazy for a in args), axis=region_fn.axis)
        else:
            leaf = ir.Region(src.name, src.dtype, axes, region_fn, block_arg,
                             target=src.zarray_maybe_lazy)
        return ir.ExprProgram(ndim=ndim, nargs=block_arg + 1, outputs=leaf,
                              out_axes=tuple(range(ndim)), name="map_direct")

    return map_blocks(_BlockIdProgram(build, 1), out, dtype=dtype, chunks=chunks,
                      extra_source_arrays=args, extra_projected_mem=extra_projected_mem,
                      fusable=False, **kwargs)


class ConcatRegions:
    """Regions read by output block ``block_id`` of ``concat(arrays, axis)``
    (_read_concat_chunk / _array_slices, array_api/manipulation_functions.py
    :107-132): a list of (array index, region of that array, offset along
    ``axis`` inside the output block).  The block spans
    [block_id[axis] * chunk, + its extent) of the concatenated axis."""

    def __init__(self, out_chunks, axis, offsets):
        self.out_chunks = out_chunks
        self.axis = axis
        self.offsets = offsets

    def __call__(self, block_id):
        from bisect import bisect

        starts = [tuple(np.cumsum((0,) + c[:-1])) for c in self.out_chunks]
        base = [slice(int(starts[d][b]), int(starts[d][b]) + self.out_chunks[d][b])
                for d, b in enumerate(block_id)]
        ax = self.axis
        lo, hi = base[ax].start, base[ax].stop
        parts = []
        pos = lo
        while pos < hi:
            i = bisect(self.offsets, pos) - 1
            stop = min(hi, self.offsets[i + 1])
            if stop > pos:
                region = list(base)
                region[ax] = slice(pos - self.offsets[i], stop - self.offsets[i], 1)
                parts.append((i, tuple(region), pos - lo))
            pos = stop
        return parts


# ------------------------------------------------------------------ rechunk / merge


def rechunk(x, chunks, target_store=None):
    normalized_chunks = normalize_chunks(chunks, x.shape, dtype=x.dtype)
    if x.chunks == normalized_chunks:
        return x
    target_chunks = to_chunksize(normalized_chunks)
    name = gensym()
    spec = x.spec
    if target_store is None:
        target_store = new_temp_path(name=name, spec=spec)
    name_int = f"{name}-int"
    temp_store = new_temp_path(name=name_int, spec=spec)
    ops = primitive_rechunk(x.zarray_maybe_lazy, target_chunks=target_chunks,
                            allowed_mem=spec.allowed_mem, reserved_mem=spec.reserved_mem,
                            target_store=target_store, temp_store=temp_store)
    Array = _Array()
    if len(ops) == 1:
        op = ops[0]
        op.target_array.name = name
        plan = Plan._new(name, "rechunk", op.target_array, op, False, x)
        return Array(name, op.target_array, spec, plan)
    op1 = ops[0]
    op1.target_array.name = name_int
    plan1 = Plan._new(name_int, "rechunk", op1.target_array, op1, False, x)
    x_int = Array(name_int, op1.target_array, spec, plan1)
    op2 = ops[1]
    op2.target_array.name = name
    plan2 = Plan._new(name, "rechunk", op2.target_array, op2, False, x_int)
    return Array(name, op2.target_array, spec, plan2)


class _merged_region:
    def __init__(self, target_chunks):
        self.target_chunks = target_chunks

    def __call__(self, block_id):
        return get_item(self.target_chunks, block_id)


def merge_chunks(x, chunks):
    target_chunksize = chunks
    if len(target_chunksize) != x.ndim:
        raise ValueError(
            f"Chunks {target_chunksize} must have same number of dimensions as array ({x.ndim})")
    if not all(c1 % c0 == 0 for c0, c1 in zip(x.chunksize, target_chunksize)):
        raise ValueError(f"Chunks {target_chunksize} must be a multiple of array's chunks {x.chunksize}")
    target_chunks = normalize_chunks(chunks, x.shape, dtype=x.dtype)
    return map_direct(_merged_region(target_chunks), x, shape=x.shape, dtype=x.dtype,
                      chunks=target_chunks, extra_projected_mem=0, target_chunks=target_chunks)


# ------------------------------------------------------------------ reductions


def _reduction_program(func, ndim, in_dtype, axis, extra_func_kwargs):
    r = as_chunk_reduction(func)
    if r is None:
        return ir.OpaqueProgram(func=func, nargs=1)
    return r.program(ndim, in_dtype, axis, keepdims=True, **(extra_func_kwargs or {}))


def _map_program(func, ndim, in_dtype, out_dtype):
    if isinstance(func, ChunkMap):
        return func.program(ndim, in_dtype, out_dtype)
    name = ir.NUMPY_ELEMENTWISE.get(func)
    if name is not None:
        return ir.elementwise_program(name, [in_dtype], [ndim], out_dtype)
    return ir.OpaqueProgram(func=func, nargs=1)


def reduction(x: "Array", func, combine_func=None, aggegrate_func=None, axis=None,
              intermediate_dtype=None, dtype=None, keepdims=False, use_new_impl=False,
              split_every=None, extra_func_kwargs=None) -> "Array":
    """Apply a function to reduce an array along one or more axes
    (core/ops.py:790-903: per-chunk reduce, then merge+combine rounds sized by
    allowed_mem, then aggregate / squeeze / astype)."""
    if use_new_impl:
        return reduction_new(x, func, combine_func, aggegrate_func, axis, intermediate_dtype,
                             dtype, keepdims, split_every, extra_func_kwargs)
    if combine_func is None:
        combine_func = func
    if axis is None:
        axis = tuple(range(x.ndim))
    if isinstance(axis, Integral):
        axis = (axis,)
    axis = validate_axis(axis, x.ndim)
    if intermediate_dtype is None:
        intermediate_dtype = dtype
    inds = tuple(range(x.ndim))
    result = x
    allowed_mem = x.spec.allowed_mem
    max_mem = allowed_mem - x.spec.reserved_mem

    adjust_chunks = {i: (1,) * len(c) if i in axis else c for i, c in enumerate(result.chunks)}
    prog = _reduction_program(func, x.ndim, x.dtype, axis, extra_func_kwargs)
    result = blockwise(prog, inds, result, inds, dtype=intermediate_dtype,
                       adjust_chunks=adjust_chunks)

    while any(n > 1 for i, n in enumerate(result.numblocks) if i in axis):
        target_chunks = list(result.chunksize)
        chunk_mem = chunk_memory(intermediate_dtype, result.chunksize)
        for i, s in enumerate(result.shape):
            if i in axis:
                assert result.chunksize[i] == 1
                if len(axis) > 1:
                    target_chunks[i] = min(s, x.chunksize[i])
                else:
                    target_chunk_size = (max_mem - chunk_mem) // (chunk_mem * 4)
                    if target_chunk_size <= 1:
                        raise ValueError(
                            f"Not enough memory for reduction. Increase allowed_mem ({allowed_mem}) "
                            "or decrease chunk size")
                    target_chunks[i] = min(s, target_chunk_size)
        if all(target_chunks[i] == result.chunksize[i] for i in axis):
            # multi-axis with unit source chunks along a reduced axis: the
            # per-axis target above would merge nothing (and loop forever);
            # merge along the first unfinished axis by the memory bound
            i = next(i for i in axis if result.numblocks[i] > 1)
            target_chunk_size = (max_mem - chunk_mem) // (chunk_mem * 4)
            if target_chunk_size <= 1:
                raise ValueError(
                    f"Not enough memory for reduction. Increase allowed_mem ({allowed_mem}) "
                    "or decrease chunk size")
            target_chunks[i] = min(result.shape[i], target_chunk_size)
        result = merge_chunks(result, tuple(target_chunks))
        if any(s > 1 for i, s in enumerate(result.chunksize) if i in axis):
            adjust_chunks = {i: (1,) * len(c) if i in axis else c for i, c in enumerate(result.chunks)}
            prog = _reduction_program(combine_func, x.ndim, result.dtype, axis, extra_func_kwargs)
            result = blockwise(prog, inds, result, inds, dtype=intermediate_dtype,
                               adjust_chunks=adjust_chunks)

    if aggegrate_func is not None:
        result = map_blocks(_map_program(aggegrate_func, result.ndim, result.dtype, dtype),
                            result, dtype=dtype)
    if not keepdims:
        axis_to_squeeze = tuple(i for i in axis if result.shape[i] == 1)
        if len(axis_to_squeeze) > 0:
            result = squeeze(result, axis_to_squeeze)
    from ..array_api import astype

    return astype(result, dtype, copy=False)


def reduction_new(x: "Array", func, combine_func=None, aggegrate_func=None, axis=None,
                  intermediate_dtype=None, dtype=None, keepdims=False, split_every=None,
                  extra_func_kwargs=None) -> "Array":
    """Tree reduction with ``split_every`` (core/ops.py:906-963)."""
    if combine_func is None:
        combine_func = func
    if axis is None:
        axis = tuple(range(x.ndim))
    if isinstance(axis, Integral):
        axis = (axis,)
    axis = validate_axis(axis, x.ndim)
    if intermediate_dtype is None:
        intermediate_dtype = dtype
    split_every = _normalize_split_every(split_every, axis)
    result = partial_reduce(
        x, partial(combine_func, **(extra_func_kwargs or {})),
        initial_func=partial(func, axis=axis, keepdims=True, **(extra_func_kwargs or {})),
        split_every=split_every, dtype=intermediate_dtype)
    result = tree_reduce(result, partial(combine_func, **(extra_func_kwargs or {})), axis=axis,
                         dtype=intermediate_dtype, split_every=split_every)
    if aggegrate_func is not None:
        result = map_blocks(_map_program(aggegrate_func, result.ndim, result.dtype, dtype),
                            result, dtype=dtype)
    if not keepdims:
        axis_to_squeeze = tuple(i for i in axis if result.shape[i] == 1)
        if len(axis_to_squeeze) > 0:
            result = squeeze(result, axis_to_squeeze)
    from ..array_api import astype

    return astype(result, dtype, copy=False)


def _normalize_split_every(split_every, axis):
    split_every = split_every or 4
    if isinstance(split_every, dict):
        split_every = {k: split_every.get(k, 2) for k in axis}
    elif isinstance(split_every, Integral):
        n = builtins.max(int(split_every ** (1 / (len(axis) or 1))), 2)
        split_every = dict.fromkeys(axis, n)
    else:
        raise ValueError("split_every must be a int or a dict")
    return split_every


def tree_reduce(x, func, axis, dtype, split_every=None):
    """Apply a reduction function repeatedly across multiple axes."""
    if axis is None:
        axis = tuple(range(x.ndim))
    if isinstance(axis, Integral):
        axis = (axis,)
    axis = validate_axis(axis, x.ndim)
    split_every = _normalize_split_every(split_every, axis)
    depth = 0
    for i, n in enumerate(x.numblocks):
        if i in split_every and split_every[i] != 1:
            depth = int(builtins.max(depth, math.ceil(math.log(n, split_every[i]))))
    for _ in range(depth):
        x = partial_reduce(x, func, split_every=split_every, dtype=dtype)
    return x


def partial_reduce(x, func, initial_func=None, split_every=None, dtype=None):
    """Reduce groups of ``split_every`` blocks per axis into one block."""
    chunks = [(1,) * math.ceil(len(c) / split_every[i]) if i in split_every else c
              for (i, c) in enumerate(x.chunks)]
    shape = tuple(map(sum, chunks))
    axis = tuple(ax for ax in split_every.keys())

    def block_function(out_key):
        out_coords = out_key[1:]
        in_keys = [list(range(bi * split_every.get(i, 1),
                              min((bi + 1) * split_every.get(i, 1), x.numblocks[i])))
                   for i, bi in enumerate(out_coords)]
        return (iter([(x.name,) + tuple(p) for p in product(*in_keys)]),)

    extra_projected_mem = x.chunkmem
    # the task reduces the concatenation of its blocks: initial_func's
    # reduction over the merged view (fields compose, e.g. mean's n/total)
    r = as_chunk_reduction(initial_func if initial_func is not None else func)
    if r is None:
        prog = ir.OpaqueProgram(func=func, nargs=1)
    else:
        kw = {"dtype": dtype} if dtype is not None and not _has_bound_dtype(r) else {}
        prog = r.program(x.ndim, x.dtype, axis, keepdims=True, **kw)
    return general_blockwise(prog, block_function, x, shape=shape, dtype=dtype, chunks=chunks,
                             extra_projected_mem=extra_projected_mem)


def _has_bound_dtype(r) -> bool:
    kw = getattr(r, "kw", None)
    return bool(kw) and "dtype" in kw


def squeeze(x, /, axis):
    if not isinstance(axis, tuple):
        axis = (axis,)
    if any(x.shape[i] != 1 for i in axis):
        raise ValueError("cannot squeeze axis with size other than one")
    axis = validate_axis(axis, x.ndim)
    chunks = tuple(c for i, c in enumerate(x.chunks) if i not in axis)
    prog = ir.ExprProgram(ndim=x.ndim, nargs=1,
                          outputs=ir.Arg(0, x.dtype, tuple(range(x.ndim))) if not x.dtype.names else
                          tuple((f, ir.Arg(0, x.dtype[f], tuple(range(x.ndim)), field=f))
                                for f in x.dtype.names),
                          out_axes=tuple(d for d in range(x.ndim) if d not in axis), name="squeeze")
    return map_blocks(prog, x, dtype=x.dtype, chunks=chunks, drop_axis=axis)


def arg_reduction(x, /, arg_func, axis=None, *, keepdims=False):
    """argmax / argmin along one axis or over the whole array
    (core/ops.py:1093-1153).

    The reference's first map (_arg_map_func) turns each block into {i, v}
    with the block-offset index, then ``reduction`` combines the pairs with
    _arg_combine.  Here every ELEMENT is a {v, i} pair -- its value key and
    its global index (the flat C-order index when axis is None, which the
    reference gets from reshape) -- built inside the reduce kernel's program
    and reduced in one fused pass with the pair op argmax / argmin
    (chunkfuncs.ArgReduction): the first NaN wins, else the larger (smaller)
    value, ties to the smaller index, as numpy.  Value keys: floats as f64
    (exact), bool / ints as int64, uint64 with the sign bit flipped
    (order-preserving)."""
    from ..array_api import creation_functions as cf
    from ..array_api import manipulation_functions as mf
    from ..array_api import elementwise_functions as ef
    from ..chunkfuncs import ArgReduction, _arg_aggregate

    if x.ndim == 0:
        x = mf.expand_dims(x, axis=0)
        axis, keepdims = 0, False
    if axis is not None:
        axis = validate_axis(axis, x.ndim)
        if isinstance(axis, tuple):
            if len(axis) != 1:
                raise ValueError("argmax/argmin take a single axis")
            axis = axis[0]
    if (x.size if axis is None else x.shape[axis]) == 0:
        raise ValueError(f"attempt to get {arg_func} of an empty sequence")

    def index_along(d):
        """The index along dim d, broadcastable against x."""
        idx = cf.arange(x.shape[d], dtype=np.int64, chunks=(x.chunks[d],), spec=x.spec)
        for e in range(x.ndim):
            if e != d:
                idx = mf.expand_dims(idx, axis=e)
        return idx

    if axis is None and x.ndim > 1:
        idx = None
        for d in range(x.ndim):
            stride = int(np.prod(x.shape[d + 1:], dtype=np.int64))
            term = ef.multiply(index_along(d), cf.asarray(np.int64(stride), spec=x.spec))
            idx = term if idx is None else ef.add(idx, term)
        red_axis = None
    else:
        red_axis = 0 if axis is None else axis
        idx = index_along(red_axis)

    dt = np.dtype(x.dtype)
    n = x.ndim
    v = ir.Arg(0, dt, tuple(range(n)))
    if ir.is_float(dt):
        vdt = np.dtype(np.float64)
        key = ir.cast(v, vdt)
    else:
        vdt = np.dtype(np.int64)
        key = ir.cast(v, vdt)
        if dt == np.uint64:
            key = ir.Binary("bitwise_xor", key, ir.Const(np.int64(np.iinfo(np.int64).min), vdt), vdt)
    intermediate = [("v", vdt), ("i", np.int64)]
    prog = ir.ExprProgram(ndim=n, nargs=2,
                          outputs=(("v", key), ("i", ir.Arg(1, np.dtype(np.int64), tuple(range(n))))),
                          out_axes=tuple(range(n)), name=f"{arg_func}_pairs")
    inds = tuple(range(n))[::-1]
    pairs = blockwise(prog, inds, x, inds, idx, inds, dtype=intermediate)
    r = ArgReduction(arg_func)
    return reduction(pairs, r, combine_func=r, aggegrate_func=_arg_aggregate, axis=red_axis,
                     intermediate_dtype=intermediate, dtype=np.int64, keepdims=keepdims)


def unify_chunks(*args: "Array", **kwargs):
    if not args:
        return {}, []
    arginds = [(args[i], args[i + 1]) for i in range(0, len(args), 2)]
    arrays, inds = zip(*arginds)
    if all(ind is None for ind in inds):
        return {}, list(arrays)
    if all(ind == inds[0] for ind in inds) and all(a.chunks == arrays[0].chunks for a in arrays):
        return dict(zip(inds[0], arrays[0].chunks)), list(arrays)
    # broadcast dimensions: per index, the common refinement of the chunkings
    groups = {}
    for a, ind in arginds:
        if ind is None:
            continue
        for c, i in zip(a.chunks, ind):
            groups.setdefault(i, set()).add(c)
    chunkss = {}
    for i, cs in groups.items():
        cs2 = cs - {(1,)} if len(cs) > 1 else cs
        chunkss[i] = common_blockdim(cs2)
    out = []
    for a, ind in arginds:
        if ind is None:
            out.append(a)
            continue
        chunks = tuple(chunkss[j] if a.shape[n] > 1 else (a.shape[n],) for n, j in enumerate(ind))
        if chunks != a.chunks and all(a.chunks):
            out.append(rechunk(a, to_chunksize(chunks)))
        else:
            out.append(a)
    return chunkss, out


def validate_axis(axis, ndim):
    if isinstance(axis, (tuple, list)):
        return tuple(validate_axis(ax, ndim) for ax in axis)
    if not isinstance(axis, Integral):
        raise TypeError(f"Axis value must be an integer, got {axis}")
    if axis < -ndim or axis >= ndim:
        raise np.exceptions.AxisError(axis, ndim) if hasattr(np, "exceptions") else ValueError(axis)
    if axis < 0:
        axis += ndim
    return axis
