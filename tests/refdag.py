"""Test infrastructure: DAGs of the reference cubed's shape without the
reference (it cannot be imported in this image: zarr, toolz, array_api_compat
are absent).

The stand-ins below carry the class names and attributes the reference's
executor interface exposes (runtime/types.py CubedPipeline, primitive/types.py
PrimitiveOperation / CubedArrayProxy / CubedCopySpec, primitive/blockwise.py
BlockwiseSpec, storage/zarr.py LazyZarrArray, storage/virtual.py virtual
arrays), and stage / chunk functions that report the reference's module
names, built the way the reference builds them: ``functools.partial`` keyword
binding (primitive/blockwise.py:272-273), map_blocks' block_id wrapper
(core/ops.py:531-560), ``fuse``'s closure (primitive/blockwise.py:368-417)
and ``random``'s Philox chunk function (random.py:13-36).  They are API-shape
fixtures for tests/test_reference_dag.py, not copies of reference code.
"""

from __future__ import annotations

import functools
import itertools
from dataclasses import dataclass
from typing import Any, Callable, Dict

import networkx as nx
import numpy as np


# -- storage ------------------------------------------------------------------
class LazyZarrArray:
    def __init__(self, shape, dtype, chunks, store, fill_value=None):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.chunks = tuple(chunks)
        self.store = store
        self.fill_value = fill_value
        self.nbytes = int(np.prod(shape)) * self.dtype.itemsize


class VirtualEmptyArray:
    def __init__(self, shape, dtype, chunks):
        self.shape, self.dtype, self.chunks = tuple(shape), np.dtype(dtype), tuple(chunks)


class VirtualOffsetsArray:
    def __init__(self, shape):
        self.shape, self.dtype, self.chunks = tuple(shape), np.dtype(np.int32), (1,) * len(shape)
        self.ndim = len(shape)


class VirtualInMemoryArray:
    def __init__(self, array, chunks):
        self.array = np.asarray(array)
        self.shape, self.dtype, self.chunks = self.array.shape, self.array.dtype, tuple(chunks)


# -- pipeline / op types -------------------------------------------------------
@dataclass(frozen=True)
class CubedPipeline:
    function: Callable[..., Any]
    name: str
    mappable: Any
    config: Any


@dataclass(frozen=True)
class PrimitiveOperation:
    pipeline: CubedPipeline
    target_array: Any
    projected_mem: int
    allowed_mem: int
    reserved_mem: int
    num_tasks: int
    fusable: bool = True


class CubedArrayProxy:
    def __init__(self, array, chunks):
        self.array, self.chunks = array, chunks


@dataclass(frozen=True)
class CubedCopySpec:
    read: CubedArrayProxy
    write: CubedArrayProxy


@dataclass(frozen=True)
class BlockwiseSpec:
    block_function: Callable[..., Any]
    function: Callable[..., Any]
    function_nargs: int
    reads_map: Dict[str, CubedArrayProxy]
    write: CubedArrayProxy


def _stage(name, module):
    def f(*a, **k):
        raise AssertionError("reference stage functions never run on the MI355X executor")

    f.__name__ = f.__qualname__ = name
    f.__module__ = module
    return f


apply_blockwise = _stage("apply_blockwise", "cubed.primitive.blockwise")
copy_read_to_write = _stage("copy_read_to_write", "cubed.primitive.rechunk")
create_zarr_array = _stage("create_zarr_array", "cubed.core.plan")


def _random(x, numblocks=None, root_seed=None, block_id=None):
    offset = int(np.ravel_multi_index(block_id, numblocks))
    rg = np.random.Generator(np.random.Philox(key=root_seed + offset))
    return rg.random(x.shape)


_random.__module__ = "cubed.random"


def func_with_block_id(func, numblocks):
    def wrap(*a, **kw):
        offset = int(a[-1])
        block_id = tuple(int(i) for i in np.unravel_index(offset, numblocks))
        return func(*a[:-1], block_id=block_id, **kw)

    return wrap


def fuse(op1: PrimitiveOperation, op2: PrimitiveOperation) -> PrimitiveOperation:
    pipeline1, pipeline2 = op1.pipeline, op2.pipeline

    def fused_blockwise_func(out_key):
        return pipeline1.config.block_function(*pipeline2.config.block_function(out_key))

    def fused_func(*args):
        return pipeline2.config.function(pipeline1.config.function(*args))

    spec = BlockwiseSpec(fused_blockwise_func, fused_func, pipeline1.config.function_nargs,
                         pipeline1.config.reads_map, pipeline2.config.write)
    pipe = CubedPipeline(apply_blockwise, "fused_apply_blockwise-001", pipeline2.mappable, spec)
    return PrimitiveOperation(pipe, op2.target_array, max(op1.projected_mem, op2.projected_mem),
                              op2.allowed_mem, op2.reserved_mem, op2.num_tasks, True)


# -- a plan builder ------------------------------------------------------------
def numblocks(shape, chunks):
    return tuple(-(-s // c) for s, c in zip(shape, chunks))


class RefPlan:
    """Builds op and array nodes the way core/plan.py Plan._new does."""

    MEM = 2_000_000_000

    def __init__(self, work_dir):
        self.g = nx.MultiDiGraph()
        self.work_dir = str(work_dir)
        self.n = 0
        self.lazy = []

    def _name(self, kind):
        self.n += 1
        return f"{kind}-{self.n:03}"

    def _array(self, name, target):
        self.g.add_node(name, name=name, type="array", target=target, hidden=False)

    def _op(self, op, out, srcs, num_tasks):
        name = self._name("op")
        self.g.add_node(name, name=name, op_name="blockwise", type="op", hidden=False,
                        primitive_op=op, pipeline=op.pipeline)
        self.g.add_edge(name, out)
        for s in srcs:
            self.g.add_edge(s, name)
        return name

    def lazy_target(self, name, shape, dtype, chunks):
        t = LazyZarrArray(shape, dtype, chunks, f"{self.work_dir}/{name}.zarr")
        self.lazy.append(t)
        self._array(name, t)
        return t

    def blockwise_op(self, func, out_name, shape, dtype, chunks, args):
        """``args``: (array name, target) pairs in call order, each indexed
        like the output's trailing dims (numpy broadcasting)."""
        target = self.lazy_target(out_name, shape, dtype, chunks)
        nd = len(shape)
        reads = {n: CubedArrayProxy(t, t.chunks) for n, t in args}

        def block_function(out_key):
            key = out_key[1:]
            keys = []
            for n, t in args:
                nb = numblocks(t.shape, t.chunks) if t.shape else ()
                tail = key[nd - len(nb):] if nb else ()
                keys.append((n,) + tuple(0 if b == 1 else k for b, k in zip(nb, tail)))
            return keys

        spec = BlockwiseSpec(block_function, func, len(args), reads, CubedArrayProxy(target, chunks))
        ntasks = int(np.prod(numblocks(shape, chunks)))
        keys = [list(k) for k in itertools.product(*[range(b) for b in numblocks(shape, chunks)])]
        op = PrimitiveOperation(CubedPipeline(apply_blockwise, self._name("apply_blockwise"), keys, spec),
                                target, 0, self.MEM, 0, ntasks, True)
        return op, target

    def add(self, op, out_name, srcs):
        return self._op(op, out_name, srcs, op.num_tasks)

    def random(self, shape, chunks, root_seed):
        """map_blocks(_random, dtype=float64, chunks=chunks, numblocks=..., root_seed=...):
        an empty template + an offsets array, the wrapped partial."""
        nb = numblocks(shape, chunks)
        empty_name, off_name = self._name("empty"), self._name("offsets")
        self._array(empty_name, VirtualEmptyArray(shape, np.float64, chunks))
        self._array(off_name, VirtualOffsetsArray(nb))
        fn = functools.partial(func_with_block_id(_random, nb), numblocks=nb, root_seed=root_seed)
        out = self._name("array")
        op, _ = self.blockwise_op(fn, out, shape, np.float64, chunks,
                                  [(empty_name, self.g.nodes[empty_name]["target"]),
                                   (off_name, self.g.nodes[off_name]["target"])])
        return op, out, [empty_name, off_name]

    def scalar(self, value, dtype):
        name = self._name("asarray")
        self._array(name, VirtualInMemoryArray(np.asarray(value, dtype=dtype), ()))
        return name

    def rechunk(self, src_name, chunks):
        src = self.g.nodes[src_name]["target"]
        out = self._name("array")
        target = self.lazy_target(out, src.shape, src.dtype, chunks)
        spec = CubedCopySpec(CubedArrayProxy(src, chunks), CubedArrayProxy(target, chunks))
        ntasks = int(np.prod(numblocks(src.shape, chunks)))
        op = PrimitiveOperation(CubedPipeline(copy_read_to_write, self._name("copy"), [], spec),
                                target, 0, self.MEM, 0, ntasks, False)
        self._op(op, out, [src_name], ntasks)
        return out

    def finalize(self):
        """core/plan.py _create_lazy_zarr_arrays + freeze."""
        g = self.g.copy()
        pipeline_nodes = [n for n, d in g.nodes(data=True) if "primitive_op" in d]
        pipe = CubedPipeline(create_zarr_array, "create_zarr_array", list(self.lazy), None)
        op = PrimitiveOperation(pipe, None, 8, self.MEM, 0, len(self.lazy), False)
        g.add_node("create-arrays", name="create-arrays", op_name="create-arrays", type="op",
                   primitive_op=op, pipeline=pipe)
        g.add_node("arrays", name="arrays", target=None)
        g.add_edge("create-arrays", "arrays")
        for n in pipeline_nodes:
            g.add_edge("arrays", n)
        return nx.freeze(g)


def example_plan(work_dir, root_seed, shape=(40, 60), chunks=(10, 20), rechunk_to=(40, 10)):
    """``c = (astype(random(shape), float32) * 2 + 1).rechunk(rechunk_to)``
    built like the reference under its default optimizer: random fused into
    astype (in-degree 1), the two scalar ops unfused (scalar inputs), one
    rechunk copy (read == write chunking at 2 GB)."""
    p = RefPlan(work_dir)
    rop, rname, rsrcs = p.random(shape, chunks, root_seed)
    aname = p._name("array")
    aop, _ = p.blockwise_op(functools.partial(lambda x, dtype: x.astype(dtype), dtype=np.float32), aname,
                            shape, np.float32, chunks, [(rname, p.g.nodes[rname]["target"])])
    fused = fuse(rop, aop)
    # the random op's output array is fused away: the fused op reads the
    # random op's inputs and writes astype's target
    p.g.remove_node(rname)
    p.lazy = [t for t in p.lazy if t is not rop.target_array]
    p.add(fused, aname, rsrcs)
    two = p.scalar(2, np.float32)
    mname = p._name("array")
    mop, _ = p.blockwise_op(functools.partial(np.multiply), mname, shape, np.float32, chunks,
                            [(aname, p.g.nodes[aname]["target"]), (two, p.g.nodes[two]["target"])])
    p.add(mop, mname, [aname, two])
    one = p.scalar(1, np.float32)
    sname = p._name("array")
    sop, _ = p.blockwise_op(np.add, sname, shape, np.float32, chunks,
                            [(mname, p.g.nodes[mname]["target"]), (one, p.g.nodes[one]["target"])])
    p.add(sop, sname, [mname, one])
    out = p.rechunk(sname, rechunk_to)
    return p.finalize(), out, sname
