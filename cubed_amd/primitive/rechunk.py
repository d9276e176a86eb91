"""Rechunk primitive: plan (read / intermediate / write chunks) and ops.

Mirrors cubed/primitive/rechunk.py:23-220 (``rechunk``, ``_setup_array_rechunk``,
``ChunkKeys``, ``copy_read_to_write``) and restates the single-stage plan of
the vendored rechunker (cubed/vendor/rechunker/algorithm.py:14-95
``consolidate_chunks``, :200-365 ``multistage_rechunking_plan`` with
min_mem = itemsize, which always stops at one stage): write chunks are the
target chunks consolidated up to ``max_mem``; read chunks are the source
chunks consolidated (only along axes where the write chunk is larger) up to
``max_mem``; the intermediate chunks are their elementwise minimum.  The
plan's chunk shapes are pinned against the reference planner in
tests/golden/rechunk_plans.json.

On the GPU the chunk shapes only decide the task counts and the DAG shape
(kept identical to the reference); the data movement is one box-copy launch
per op over all (source chunk x target chunk) intersections.
"""

from __future__ import annotations

import itertools
import math
from math import ceil, prod
from typing import List, Optional, Sequence, Tuple

from ..runtime.types import CubedPipeline
from ..storage import DeviceArray
from ..utils import gensym_factory
from .types import CubedArrayProxy, CubedCopySpec, PrimitiveOperation

gensym = gensym_factory("copy_read_to_write")


def consolidate_chunks(shape: Sequence[int], chunks: Sequence[int], itemsize: int, max_mem: int,
                       chunk_limits: Optional[Sequence[Optional[int]]] = None) -> Tuple[int, ...]:
    """Grow ``chunks`` (last axis first) up to ``max_mem`` bytes, bounded per
    axis by ``chunk_limits`` (None: do not grow this axis, -1: no limit)."""
    ndim = len(shape)
    if chunk_limits is None:
        chunk_limits = shape
    if len(chunk_limits) != ndim:
        raise ValueError("chunk_limits must have one entry per axis")
    limits = {}
    for ax, cl in enumerate(chunk_limits):
        if cl is None:
            continue
        if cl == -1:
            limits[ax] = shape[ax]
        elif chunks[ax] <= cl <= shape[ax]:
            limits[ax] = cl
        elif cl > shape[ax]:
            limits[ax] = shape[ax]
        else:
            raise ValueError(f"Invalid chunk_limits {chunk_limits}.")
    chunk_mem = itemsize * prod(chunks)
    if chunk_mem > max_mem:
        raise ValueError(f"chunk_mem {chunk_mem} > max_mem {max_mem}")
    headroom = max_mem / chunk_mem
    new = list(chunks)
    for ax in sorted(limits)[::-1]:
        upper = min(shape[ax], limits[ax])
        new[ax] = upper
        mem = itemsize * prod(new)
        if max_mem / mem > 1:
            headroom = max_mem / mem
        else:
            new[ax] = min(int(chunks[ax] * int(headroom)), upper)
            headroom = max_mem / (itemsize * prod(new))
        assert headroom >= 1
    return tuple(new)


def rechunking_plan(shape: Sequence[int], source_chunks: Sequence[int],
                    target_chunks: Sequence[int], itemsize: int, max_mem: int,
                    consolidate_reads: bool = True, consolidate_writes: bool = True):
    """(read_chunks, int_chunks, write_chunks) of a single-stage rechunk."""
    ndim = len(shape)
    if len(source_chunks) != ndim:
        raise ValueError(f"source_chunks {source_chunks} must have length {ndim}")
    if len(target_chunks) != ndim:
        raise ValueError(f"target_chunks {target_chunks} must have length {ndim}")
    src_mem = itemsize * prod(source_chunks)
    tgt_mem = itemsize * prod(target_chunks)
    if src_mem > max_mem:
        raise ValueError(f"Source chunk memory ({src_mem}) exceeds max_mem ({max_mem})")
    if tgt_mem > max_mem:
        raise ValueError(f"Target chunk memory ({tgt_mem}) exceeds max_mem ({max_mem})")
    if max_mem < itemsize:
        raise ValueError(f"max_mem ({max_mem}) cannot be smaller than min_mem ({itemsize})")
    if consolidate_writes:
        write = consolidate_chunks(shape, target_chunks, itemsize, max_mem)
    else:
        write = tuple(target_chunks)
    if consolidate_reads:
        limits = [wc if wc > sc else None for sc, wc in zip(source_chunks, write)]
        read = consolidate_chunks(shape, source_chunks, itemsize, max_mem, limits)
    else:
        read = tuple(source_chunks)
    inter = tuple(min(r, w) for r, w in zip(read, write))
    return read, inter, write


def total_chunks(shape, chunks) -> int:
    return prod(ceil(s / c) for s, c in zip(shape, chunks))


class ChunkKeys:
    """Re-iterable keys (lists of slices) covering ``shape`` in ``chunks``."""

    def __init__(self, shape, chunks):
        self.shape = tuple(shape)
        self.chunks = tuple(chunks)

    def __iter__(self):
        ranges = [range(math.ceil(s / c)) for s, c in zip(self.shape, self.chunks)]
        for idx in itertools.product(*ranges):
            yield [slice(c * i, min(c * (i + 1), s)) for i, s, c in zip(idx, self.shape, self.chunks)]

    def __len__(self):
        return total_chunks(self.shape, self.chunks)


def copy_read_to_write(chunk_key, *, config: CubedCopySpec) -> None:
    """Stage function marker for rechunk copies (lowered to box copies)."""
    raise TypeError("rechunk copies run only through the MI355X executor")


def rechunk(source, target_chunks, allowed_mem: int, reserved_mem: int, target_store,
            temp_store=None) -> List[PrimitiveOperation]:
    """Change the chunking of an array (1 op, or 2 through an intermediate)."""
    rechunker_max_mem = (allowed_mem - reserved_mem) // 4
    projected_mem = allowed_mem
    shape = tuple(int(x) for x in source.shape)
    read_chunks, int_chunks, write_chunks = rechunking_plan(
        shape, source.chunks, target_chunks, source.dtype.itemsize, rechunker_max_mem)
    target_chunks = tuple(int(x) for x in target_chunks)
    target = DeviceArray(shape, source.dtype, target_chunks, name=target_store)
    read_proxy = CubedArrayProxy(source, read_chunks)
    write_proxy = CubedArrayProxy(target, write_chunks)
    if read_chunks == write_chunks:
        spec = CubedCopySpec(read_proxy, write_proxy)
        return [_spec_to_op(spec, target, projected_mem, allowed_mem, reserved_mem,
                            total_chunks(shape, write_chunks))]
    if temp_store is None:
        raise ValueError("A temporary store location must be provided.")
    intermediate = DeviceArray(shape, source.dtype, int_chunks, name=temp_store)
    int_proxy = CubedArrayProxy(intermediate, int_chunks)
    spec1 = CubedCopySpec(read_proxy, int_proxy)
    op1 = _spec_to_op(spec1, intermediate, projected_mem, allowed_mem, reserved_mem,
                      total_chunks(shape, int_chunks))
    spec2 = CubedCopySpec(int_proxy, write_proxy)
    op2 = _spec_to_op(spec2, target, projected_mem, allowed_mem, reserved_mem,
                      total_chunks(shape, write_chunks))
    return [op1, op2]


def _spec_to_op(spec, target, projected_mem, allowed_mem, reserved_mem, num_tasks):
    shape = spec.read.array.shape
    pipeline = CubedPipeline(copy_read_to_write, gensym("copy_read_to_write"),
                             ChunkKeys(shape, spec.write.chunks), spec)
    return PrimitiveOperation(pipeline=pipeline, target_array=target, projected_mem=projected_mem,
                              allowed_mem=allowed_mem, reserved_mem=reserved_mem,
                              num_tasks=num_tasks, fusable=False, write_chunks=spec.write.chunks)
