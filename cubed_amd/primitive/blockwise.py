"""Blockwise primitive: task descriptors and their fusion.

Mirrors cubed/primitive/blockwise.py: ``BlockwiseSpec`` (:34-58),
``blockwise``/``general_blockwise`` with the projected-memory check
(:106-320, check :282-300), fusion ``can_fuse_*``/``peak_projected_mem``/
``fuse``/``fuse_multiple`` (:326-508) and the dask-style block-key mapping
(``make_blockwise_function``, :514-592, dask ``_get_coord_mapping``
vendor/dask/blockwise.py:10-101).  The differences: ``function`` is an IR
``Program`` (cubed_amd/ir.py) and fusion composes programs; targets are
HBM ``DeviceArray``s.
"""

from __future__ import annotations

import itertools
import math
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import ir
from ..runtime.types import CubedPipeline
from ..storage import DeviceArray
from ..utils import chunk_memory, gensym_factory, normalize_chunks, split_into, to_chunksize
from .types import CubedArrayProxy, MemoryModeller, PrimitiveOperation

gensym = gensym_factory("apply_blockwise")


@dataclass(frozen=True)
class BlockwiseSpec:
    """How to run blockwise on an array.

    block_function : output chunk key -> input chunk keys (one entry per arg;
        nested lists / iterators for contractions and partial reductions)
    function : the chunk ``Program`` (ir.ExprProgram / MatmulProgram / ...)
    function_nargs : number of array args of ``function``
    reads_map : input proxies keyed by array name
    write : output proxy
    """

    block_function: Callable[..., Any]
    function: Any
    function_nargs: int
    reads_map: Dict[str, CubedArrayProxy]
    write: CubedArrayProxy


class OutputBlocks:
    """Re-iterable ``mappable``: every output block key as a list."""

    def __init__(self, numblocks: Sequence[int]):
        self.numblocks = tuple(numblocks)

    def __iter__(self):
        return map(list, itertools.product(*[range(n) for n in self.numblocks]))

    def __len__(self):
        return math.prod(self.numblocks)


def apply_blockwise(out_key, *, config: BlockwiseSpec) -> None:
    """Stage function marker for blockwise pipelines.  The GPU executor
    lowers whole pipelines; a per-task host call has no implementation."""
    raise TypeError("blockwise pipelines run only through the MI355X executor")


def blockwise(
    func,
    out_ind,
    *args,
    allowed_mem: int,
    reserved_mem: int,
    target_store,
    shape,
    dtype,
    chunks,
    new_axes=None,
    in_names=None,
    out_name=None,
    extra_projected_mem: int = 0,
    extra_func_kwargs=None,
    fusable: bool = True,
    **kwargs,
):
    """Index-notation blockwise (``out_ind`` and (array, ind) pairs)."""
    arrays = args[::2]
    array_names = in_names or [f"in_{i}" for i in range(len(arrays))]
    inds = args[1::2]
    numblocks = {}
    for name, array in zip(array_names, arrays):
        nc = normalize_chunks(array.chunks, shape=array.shape, dtype=array.dtype)
        numblocks[name] = tuple(len(c) for c in nc)
    argpairs = list(zip(array_names, inds))
    block_function = make_blockwise_key_function(
        out_name or "out", out_ind, argpairs, numblocks=numblocks, new_axes=new_axes)
    return general_blockwise(
        func, block_function, *arrays, allowed_mem=allowed_mem, reserved_mem=reserved_mem,
        target_store=target_store, shape=shape, dtype=dtype, chunks=chunks,
        in_names=in_names, extra_projected_mem=extra_projected_mem,
        extra_func_kwargs=extra_func_kwargs, fusable=fusable, **kwargs)


def general_blockwise(
    func,
    block_function,
    *arrays,
    allowed_mem: int,
    reserved_mem: int,
    target_store,
    shape,
    dtype,
    chunks,
    in_names=None,
    extra_projected_mem: int = 0,
    extra_func_kwargs=None,
    fusable: bool = True,
    **kwargs,
):
    """Blockwise with an explicit ``block_function``."""
    array_names = in_names or [f"in_{i}" for i in range(len(arrays))]
    array_map = dict(zip(array_names, arrays))
    chunks = normalize_chunks(chunks, shape=shape, dtype=dtype)
    chunksize = to_chunksize(chunks) if len(shape) else ()
    if isinstance(target_store, DeviceArray):
        target_array = target_store
    else:
        target_array = DeviceArray(shape, dtype, chunksize, name=target_store)

    program = func if isinstance(func, ir.Program) else ir.OpaqueProgram(func=func, nargs=len(arrays))
    read_proxies = {name: CubedArrayProxy(a, a.chunks) for name, a in array_map.items()}
    write_proxy = CubedArrayProxy(target_array, chunksize)
    spec = BlockwiseSpec(block_function, program, len(arrays), read_proxies, write_proxy)

    # projected memory (primitive/blockwise.py:282-300): a compressed and an
    # uncompressed copy of every input and of the output chunk
    projected_mem = reserved_mem + extra_projected_mem
    for a in arrays:
        projected_mem += chunk_memory(a.dtype, a.chunks) * 2
    projected_mem += chunk_memory(dtype, chunksize) * 2
    if projected_mem > allowed_mem:
        raise ValueError(
            f"Projected blockwise memory ({projected_mem}) exceeds allowed_mem ({allowed_mem}), "
            f"including reserved_mem ({reserved_mem})"
        )
    numblocks_out = tuple(len(c) for c in chunks)
    pipeline = CubedPipeline(apply_blockwise, gensym("apply_blockwise"),
                             OutputBlocks(numblocks_out), spec)
    return PrimitiveOperation(
        pipeline=pipeline, target_array=target_array, projected_mem=projected_mem,
        allowed_mem=allowed_mem, reserved_mem=reserved_mem,
        num_tasks=math.prod(numblocks_out), fusable=fusable)


# ---------------------------------------------------------------- fusion


def is_fuse_candidate(op: PrimitiveOperation) -> bool:
    return op.pipeline.function is apply_blockwise


def can_fuse_primitive_ops(op1: PrimitiveOperation, op2: PrimitiveOperation) -> bool:
    if is_fuse_candidate(op1) and is_fuse_candidate(op2):
        return op1.num_tasks == op2.num_tasks
    return False


def can_fuse_multiple_primitive_ops(op: PrimitiveOperation, *preds: PrimitiveOperation) -> bool:
    if is_fuse_candidate(op) and all(is_fuse_candidate(p) for p in preds):
        if peak_projected_mem(preds) > op.allowed_mem:
            return False
        return all(op.num_tasks == p.num_tasks for p in preds)
    return False


def peak_projected_mem(ops) -> int:
    """Peak projected memory of running ``ops`` in order, keeping outputs."""
    mm = MemoryModeller()
    for p in ops:
        mm.allocate(p.projected_mem)
        chunkmem = chunk_memory(p.target_array.dtype, p.target_array.chunks)
        mm.free(p.projected_mem - chunkmem)
    return mm.peak_mem


def _fuse_program(consumer, producers, nargs):
    try:
        return ir.fuse_programs(consumer, producers, nargs)
    except ir.FusionError as e:
        return ir.OpaqueProgram(func=f"unfusable ({e})", nargs=sum(nargs))


def fuse(op1: PrimitiveOperation, op2: PrimitiveOperation) -> PrimitiveOperation:
    """Fuse two blockwise ops (op2 consumes op1's output)."""
    assert op1.num_tasks == op2.num_tasks
    p1, p2 = op1.pipeline, op2.pipeline

    def fused_block_function(out_key):
        return p1.config.block_function(*p2.config.block_function(out_key))

    if isinstance(p1.config.function, (ir.MatmulProgram, ir.TensordotProgram)):
        # chunk GEMMs do not fuse into an expression program: keep the GEMM's
        # output geometry as scratch and run the consumer program over it
        program = ir.GemmThenProgram(gemm=p1.config.function, gemm_block_function=p1.config.block_function,
                                     gemm_reads=p1.config.reads_map, gemm_target=op1.target_array,
                                     then=p2.config.function, then_block_function=p2.config.block_function,
                                     nargs=p1.config.function_nargs)
    else:
        program = _fuse_program(p2.config.function, [p1.config.function], [p1.config.function_nargs])
        if isinstance(program, ir.OpaqueProgram) and \
                isinstance(p1.config.function, (ir.ExprProgram, ir.PerBlockProgram)) \
                and isinstance(p2.config.function, ir.ExprProgram):
            # not expressible as one program (e.g. a consumer of a chunk
            # reshape): one task still runs both, through op1's chunk
            program = ir.GemmThenProgram(gemm=p1.config.function, gemm_block_function=p1.config.block_function,
                                         gemm_reads=p1.config.reads_map, gemm_target=op1.target_array,
                                         then=p2.config.function, then_block_function=p2.config.block_function,
                                         nargs=p1.config.function_nargs, name="seq")
    spec = BlockwiseSpec(fused_block_function, program, p1.config.function_nargs,
                         p1.config.reads_map, p2.config.write)
    pipeline = CubedPipeline(apply_blockwise, gensym("fused_apply_blockwise"), p2.mappable, spec)
    return PrimitiveOperation(
        pipeline=pipeline, target_array=op2.target_array,
        projected_mem=max(op1.projected_mem, op2.projected_mem),
        allowed_mem=op2.allowed_mem, reserved_mem=op2.reserved_mem,
        num_tasks=op2.num_tasks, fusable=True)


def fuse_multiple(op: PrimitiveOperation, *preds: Optional[PrimitiveOperation]) -> PrimitiveOperation:
    """Fuse an op with its (fusable) predecessors; None = unfused input."""
    assert all(op.num_tasks == p.num_tasks for p in preds if p is not None)
    pipeline = op.pipeline
    pred_pipelines = [p.pipeline if p is not None else None for p in preds]
    pred_nargs = [pp.config.function_nargs if pp is not None else 1 for pp in pred_pipelines]

    def apply_block(pp, arg):
        if pp is None:
            return (arg,)
        return pp.config.block_function(arg)

    # Unlike the reference (which groups the keys per predecessor with
    # split_into so its composed closure can unpack them), fused programs
    # take a flat argument list: the concatenation of the groups.
    def fused_block_function(out_key):
        args = pipeline.config.block_function(out_key)
        return [item for pp, a in zip(pred_pipelines, args) for item in apply_block(pp, a)]

    producers = [pp.config.function if pp is not None else None for pp in pred_pipelines]
    program = _fuse_program(pipeline.config.function, producers, pred_nargs)
    reads = dict(pipeline.config.reads_map)
    for pp in pred_pipelines:
        if pp is not None:
            reads.update(pp.config.reads_map)
    spec = BlockwiseSpec(fused_block_function, program, sum(pred_nargs),
                         reads, pipeline.config.write)
    fused = CubedPipeline(apply_blockwise, gensym("fused_apply_blockwise"), pipeline.mappable, spec)
    projected = max(op.projected_mem, peak_projected_mem([p for p in preds if p is not None]))
    return PrimitiveOperation(
        pipeline=fused, target_array=op.target_array, projected_mem=projected,
        allowed_mem=op.allowed_mem, reserved_mem=op.reserved_mem,
        num_tasks=op.num_tasks, fusable=True)


# ---------------------------------------------------------------- block keys


def _broadcast_dims(argpairs, numblocks):
    dims: Dict[Any, set] = {}
    for name, ind in argpairs:
        if ind is None:
            continue
        for i, nb in zip(ind, numblocks[name]):
            dims.setdefault(i, set()).add(nb)
    out = {}
    for i, vals in dims.items():
        vals2 = vals - {1} if len(vals) > 1 else vals
        if len(vals2) != 1:
            raise ValueError(f"Shapes do not align {dims}")
        out[i] = next(iter(vals2))
    return out


def make_blockwise_key_function(output, out_ind, argpairs, numblocks, new_axes=None):
    """out key ('out', i, j, ...) -> per-arg chunk keys.

    An arg index that is an output index takes the output coordinate (0 when
    the arg has a single block there: broadcasting); an index missing from
    the output (a contraction) expands to a list over all its blocks, nested
    per dummy index (dask's lol_product)."""
    new_axes = new_axes or {}
    dims = _broadcast_dims(argpairs, numblocks)
    for k, v in new_axes.items():
        dims[k] = len(v) if isinstance(v, tuple) else 1
    out_pos = {idx: i for i, idx in enumerate(out_ind)}

    def key_for(name, ind, coords):
        per_dim = []
        for idx, nb in zip(ind, numblocks[name]):
            if nb == 1:
                per_dim.append(0)
            elif idx in out_pos:
                per_dim.append(coords[out_pos[idx]])
            else:
                per_dim.append(list(range(dims[idx])))
        return _lol_product((name,), per_dim)

    def block_function(out_key):
        coords = out_key[1:]
        res = []
        for name, ind in argpairs:
            if ind is None:
                res.append(name)
            else:
                res.append(key_for(name, ind, coords))
        if res and isinstance(res[0], list):
            res = list(_flatten(res))
        return res

    return block_function


def _lol_product(head, values):
    if not values:
        return head
    if isinstance(values[0], list):
        return [_lol_product(head + (x,), values[1:]) for x in values[0]]
    return _lol_product(head + (values[0],), values[1:])


def _flatten(seq):
    for item in seq:
        if isinstance(item, list):
            yield from _flatten(item)
        else:
            yield item
