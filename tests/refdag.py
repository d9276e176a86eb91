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


# -- reductions (array_api/statistical_functions.py:54-100, core/ops.py:646-903) --
def _ref_fn(name, module):
    def f(*a, **k):
        raise AssertionError("reference chunk functions never run on the MI355X executor")

    f.__name__ = f.__qualname__ = name
    f.__module__ = module
    return f


_mean_func = _ref_fn("_mean_func", "cubed.array_api.statistical_functions")
_mean_combine = _ref_fn("_mean_combine", "cubed.array_api.statistical_functions")
_mean_aggregate = _ref_fn("_mean_aggregate", "cubed.array_api.statistical_functions")
_copy_chunk = _ref_fn("_copy_chunk", "cubed.core.ops")


class RefArray:
    """The side-input ``Array`` map_direct passes as ``arrays=``."""

    def __init__(self, name, target):
        self.name = name
        self.zarray_maybe_lazy = target


def map_direct_wrap(func):
    def wrap(*a, block_id=None, **kw):
        arrays = kw.pop("arrays")
        return func(*(a + arrays), block_id=block_id, **kw)

    return wrap


def mean_plan(work_dir, root_seed, shape=(40, 60), chunks=(10, 20)):
    """``xp.mean(random(shape, chunks), axis=0)`` as the reference plans it at
    2 GB under its default optimizer: random fused into the per-chunk
    ``_mean_func`` (one op, a task per chunk), then ONE op fusing
    merge_chunks (map_direct over the partials), ``_mean_combine``,
    ``_mean_aggregate`` and ``squeeze`` -- the ``merge_chunks -> combine ->
    aggregate -> squeeze`` chain simple_optimize_dag fuses
    (core/optimization.py:11-68)."""
    p = RefPlan(work_dir)
    idt = np.dtype([("n", np.int64), ("total", np.float64)])
    nr = -(-shape[0] // chunks[0])
    rop, rname, rsrcs = p.random(shape, chunks, root_seed)
    # per-chunk reduce
    pname = p._name("array")
    pshape, pchunks = (nr, shape[1]), (1, chunks[1])
    mop, ptarget = p.blockwise_op(functools.partial(_mean_func, axis=(0,), keepdims=True,
                                                    dtype=[("n", np.int64), ("total", np.float64)]),
                                  pname, pshape, idt, pchunks, [(rname, p.g.nodes[rname]["target"])])
    # the partials' block function maps the output key straight to the input key
    a_op = fuse(rop, mop)
    p.g.remove_node(rname)
    p.lazy = [t for t in p.lazy if t is not rop.target_array]
    p.add(a_op, pname, rsrcs)
    # merge_chunks: map_direct(_copy_chunk, partials, target_chunks) -> (nr, c1) chunks
    tchunks = (nr, chunks[1])
    nb = numblocks(pshape, tchunks)
    tnorm = tuple(tuple(min(c, s - i) for i in range(0, s, c)) for s, c in zip(pshape, tchunks))
    empty, offs = p._name("empty"), p._name("offsets")
    p._array(empty, VirtualEmptyArray(pshape, idt, tchunks))
    p._array(offs, VirtualOffsetsArray(nb))
    mfn = functools.partial(func_with_block_id(map_direct_wrap(_copy_chunk), nb),
                            arrays=(RefArray(pname, ptarget),), target_chunks=tnorm)
    gname = p._name("array")
    gop, _ = p.blockwise_op(mfn, gname, pshape, idt, tchunks,
                            [(empty, p.g.nodes[empty]["target"]), (offs, p.g.nodes[offs]["target"])])
    # combine -> (1, shape[1]) chunks (1, c1)
    cname = p._name("array")
    cop, _ = p.blockwise_op(functools.partial(_mean_combine, axis=(0,), keepdims=True,
                                              dtype=[("n", np.int64), ("total", np.float64)]),
                            cname, (1, shape[1]), idt, (1, chunks[1]), [(gname, p.g.nodes[gname]["target"])])
    # aggregate (f64) and squeeze
    aname = p._name("array")
    agg, _ = p.blockwise_op(functools.partial(_mean_aggregate), aname, (1, shape[1]), np.float64,
                            (1, chunks[1]), [(cname, p.g.nodes[cname]["target"])])
    sname = p._name("array")
    sq, starget = p.blockwise_op(functools.partial(np.squeeze, axis=(0,)), sname, (shape[1],), np.float64,
                                 (chunks[1],), [(aname, p.g.nodes[aname]["target"])])
    # squeeze's key function: output block (j,) reads aggregate block (0, j)
    sq_spec = BlockwiseSpec(lambda k: [(aname, 0, k[1])], sq.pipeline.config.function, 1,
                            sq.pipeline.config.reads_map, sq.pipeline.config.write)
    sq = PrimitiveOperation(CubedPipeline(apply_blockwise, "apply_blockwise-sq", sq.pipeline.mappable, sq_spec),
                            starget, 0, p.MEM, 0, sq.num_tasks, True)
    b_op = fuse(fuse(fuse(gop, cop), agg), sq)
    for n in (gname, cname, aname):
        t = p.g.nodes[n]["target"]
        p.g.remove_node(n)
        p.lazy = [x for x in p.lazy if x is not t]
    name = p._op(b_op, sname, [empty, offs, pname], b_op.num_tasks)
    return p.finalize(), sname, pname, name


# -- reduction(..., use_new_impl=True): partial_reduce (core/ops.py:906-1090) --
_partial_reduce = _ref_fn("_partial_reduce", "cubed.core.ops")


def partial_reduce_mean_plan(work_dir, root_seed, shape=(40, 60), chunks=(10, 20)):
    """``reduction_new`` of the mean over axis 0 with split_every 4: ONE
    partial_reduce op whose block function yields an iterator over the 4 row
    blocks of a column block (initial_func ``_mean_func``, reduce_func
    ``_mean_combine``), then ``_mean_aggregate`` + squeeze fused."""
    p = RefPlan(work_dir)
    rop, rname, rsrcs = p.random(shape, chunks, root_seed)
    p.add(rop, rname, rsrcs)
    X = p.g.nodes[rname]["target"]
    idt = np.dtype([("n", np.int64), ("total", np.float64)])
    nb = numblocks(shape, chunks)
    pname = p._name("array")
    pt = p.lazy_target(pname, (1, shape[1]), idt, (1, chunks[1]))

    def block_function(out_key):
        j = out_key[2]
        return (iter([(rname, i, j) for i in range(nb[0])]),)

    fn = functools.partial(_partial_reduce,
                           reduce_func=functools.partial(_mean_combine, dtype=[("n", np.int64), ("total", np.float64)]),
                           # the reference's exact binding (core/ops.py:931-937): axis and
                           # keepdims bound into initial_func, extra_func_kwargs (dtype) into both
                           initial_func=functools.partial(_mean_func, axis=(0,), keepdims=True,
                                                          dtype=[("n", np.int64), ("total", np.float64)]),
                           axis=(0,))
    spec = BlockwiseSpec(block_function, fn, 1, {rname: CubedArrayProxy(X, X.chunks)}, CubedArrayProxy(pt, pt.chunks))
    pop = PrimitiveOperation(CubedPipeline(apply_blockwise, p._name("apply_blockwise"), [], spec), pt,
                             0, p.MEM, 0, nb[1], True)
    p.add(pop, pname, [rname])
    aname = p._name("array")
    agg, _ = p.blockwise_op(functools.partial(_mean_aggregate), aname, (1, shape[1]), np.float64,
                            (1, chunks[1]), [(pname, pt)])
    sname = p._name("array")
    sq, starget = p.blockwise_op(functools.partial(np.squeeze, axis=(0,)), sname, (shape[1],), np.float64,
                                 (chunks[1],), [(aname, p.g.nodes[aname]["target"])])
    sq_spec = BlockwiseSpec(lambda k: [(aname, 0, k[1])], sq.pipeline.config.function, 1,
                            sq.pipeline.config.reads_map, sq.pipeline.config.write)
    sq = PrimitiveOperation(CubedPipeline(apply_blockwise, "apply_blockwise-sq", sq.pipeline.mappable, sq_spec),
                            starget, 0, p.MEM, 0, sq.num_tasks, True)
    b_op = fuse(agg, sq)
    t = p.g.nodes[aname]["target"]
    p.g.remove_node(aname)
    p.lazy = [x for x in p.lazy if x is not t]
    name = p._op(b_op, sname, [pname], b_op.num_tasks)
    return p.finalize(), sname, rname, name


# -- arg reductions (core/ops.py:1093-1153) -------------------------------------
_arg_map_func = _ref_fn("_arg_map_func", "cubed.core.ops")
_arg_func = _ref_fn("_arg_func", "cubed.core.ops")
_arg_combine = _ref_fn("_arg_combine", "cubed.core.ops")
_arg_aggregate = _ref_fn("_arg_aggregate", "cubed.core.ops")


def argreduce_plan(work_dir, root_seed, arg_func=np.argmax, shape=(40, 60), chunks=(10, 20)):
    """``xp.argmax(random(shape, chunks), axis=0)`` as the reference plans it
    (arg_reduction): map_blocks(_arg_map_func) with block_id over the
    materialised input (a task per chunk, {i, v} blocks of one row), fused
    with reduction's pass-through ``_arg_func``; then ONE op fusing
    merge_chunks, ``_arg_combine``, ``_arg_aggregate`` and squeeze."""
    p = RefPlan(work_dir)
    rop, rname, rsrcs = p.random(shape, chunks, root_seed)
    p.add(rop, rname, rsrcs)
    idt = np.dtype([("i", np.int64), ("v", np.float64)])
    nb = numblocks(shape, chunks)
    nr = nb[0]
    offs = p._name("offsets")
    p._array(offs, VirtualOffsetsArray(nb))
    mname = p._name("array")
    pshape, pchunks = (nr, shape[1]), (1, chunks[1])
    fn = functools.partial(func_with_block_id(_arg_map_func, nb), axis=0, arg_func=arg_func, size=chunks[0])
    mop, mt = p.blockwise_op(fn, mname, pshape, idt, pchunks,
                             [(rname, p.g.nodes[rname]["target"]), (offs, p.g.nodes[offs]["target"])])
    fname = p._name("array")
    fop, ft = p.blockwise_op(functools.partial(_arg_func, axis=(0,), keepdims=True), fname, pshape, idt, pchunks,
                             [(mname, mt)])
    a_op = fuse(mop, fop)
    p.g.remove_node(mname)
    p.lazy = [t for t in p.lazy if t is not mt]
    p.add(a_op, fname, [rname, offs])
    tchunks = (nr, chunks[1])
    tnb = numblocks(pshape, tchunks)
    tnorm = tuple(tuple(min(c, s - i) for i in range(0, s, c)) for s, c in zip(pshape, tchunks))
    empty, toffs = p._name("empty"), p._name("offsets")
    p._array(empty, VirtualEmptyArray(pshape, idt, tchunks))
    p._array(toffs, VirtualOffsetsArray(tnb))
    mfn = functools.partial(func_with_block_id(map_direct_wrap(_copy_chunk), tnb),
                            arrays=(RefArray(fname, ft),), target_chunks=tnorm)
    gname = p._name("array")
    gop, _ = p.blockwise_op(mfn, gname, pshape, idt, tchunks,
                            [(empty, p.g.nodes[empty]["target"]), (toffs, p.g.nodes[toffs]["target"])])
    cname = p._name("array")
    cop, _ = p.blockwise_op(functools.partial(_arg_combine, arg_func=arg_func, axis=(0,), keepdims=True),
                            cname, (1, shape[1]), idt, (1, chunks[1]), [(gname, p.g.nodes[gname]["target"])])
    aname = p._name("array")
    agg, _ = p.blockwise_op(functools.partial(_arg_aggregate), aname, (1, shape[1]), np.int64,
                            (1, chunks[1]), [(cname, p.g.nodes[cname]["target"])])
    sname = p._name("array")
    sq, starget = p.blockwise_op(functools.partial(np.squeeze, axis=(0,)), sname, (shape[1],), np.int64,
                                 (chunks[1],), [(aname, p.g.nodes[aname]["target"])])
    sq_spec = BlockwiseSpec(lambda k: [(aname, 0, k[1])], sq.pipeline.config.function, 1,
                            sq.pipeline.config.reads_map, sq.pipeline.config.write)
    sq = PrimitiveOperation(CubedPipeline(apply_blockwise, "apply_blockwise-sq", sq.pipeline.mappable, sq_spec),
                            starget, 0, p.MEM, 0, sq.num_tasks, True)
    b_op = fuse(fuse(fuse(gop, cop), agg), sq)
    for nm in (gname, cname, aname):
        t = p.g.nodes[nm]["target"]
        p.g.remove_node(nm)
        p.lazy = [x for x in p.lazy if x is not t]
    name = p._op(b_op, sname, [empty, toffs, fname], b_op.num_tasks)
    return p.finalize(), sname, rname, name


# -- matmul (array_api/linear_algebra_functions.py:13-78) -----------------------
_matmul = _ref_fn("_matmul", "cubed.array_api.linear_algebra_functions")
_chunk_sum = _ref_fn("_chunk_sum", "cubed.array_api.linear_algebra_functions")


_tensordot = _ref_fn("_tensordot", "cubed.array_api.linear_algebra_functions")


def tensordot_plan(work_dir, seed_a, seed_b, **kw):
    """``xp.tensordot(A, B, axes=1)`` as the reference plans it: blockwise
    ``_tensordot`` (axes ((1,), (0,))) keeping a unit dim per contracted axis,
    then ``sum`` over it (a numpy ``sum`` per chunk, merge_chunks, sum,
    squeeze) -- the matmul plan's shape with the tensordot chunk functions."""
    return matmul_plan(work_dir, seed_a, seed_b, product=functools.partial(_tensordot, axes=((1,), (0,))),
                       ksum=np.sum, **kw)


def matmul_plan(work_dir, seed_a, seed_b, m=60, k=80, n=40, cm=20, ck=20, cn=20, product=None, ksum=None):
    """``xp.matmul(A, B)`` of two random f64 arrays as the reference plans it
    under its default optimizer: the (i, k, j) chunk products ``_matmul``
    fused with the first ``_chunk_sum`` over the unit k dim, then one op
    fusing merge_chunks (map_direct over the k partials), the combining
    ``_chunk_sum`` and ``squeeze``."""
    p = RefPlan(work_dir)
    aop, aname, asrcs = p.random((m, k), (cm, ck), seed_a)
    p.add(aop, aname, asrcs)
    bop, bname, bsrcs = p.random((k, n), (ck, cn), seed_b)
    p.add(bop, bname, bsrcs)
    kb = -(-k // ck)
    pshape, pchunks = (m, kb, n), (cm, 1, cn)
    A, B = p.g.nodes[aname]["target"], p.g.nodes[bname]["target"]
    prod_name = p._name("array")
    prod_t = p.lazy_target(prod_name, pshape, np.float64, pchunks)
    product = product if product is not None else functools.partial(_matmul)
    ksum = ksum if ksum is not None else _chunk_sum
    spec = BlockwiseSpec(lambda key: [(aname, key[1], key[2]), (bname, key[2], key[3])], product,
                         2, {aname: CubedArrayProxy(A, A.chunks), bname: CubedArrayProxy(B, B.chunks)},
                         CubedArrayProxy(prod_t, pchunks))
    ntasks = int(np.prod(numblocks(pshape, pchunks)))
    mm = PrimitiveOperation(CubedPipeline(apply_blockwise, p._name("apply_blockwise"), [], spec), prod_t,
                            0, p.MEM, 0, ntasks, True)
    sname = p._name("array")
    sop, st = p.blockwise_op(functools.partial(ksum, axis=(1,), keepdims=True, dtype=np.float64),
                             sname, pshape, np.float64, pchunks, [(prod_name, prod_t)])
    first = fuse(mm, sop)
    p.g.remove_node(prod_name)
    p.lazy = [t for t in p.lazy if t is not prod_t]
    p.add(first, sname, [aname, bname])
    # merge the kb partials along axis 1, combine, squeeze
    tchunks = (cm, kb, cn)
    nb = numblocks(pshape, tchunks)
    tnorm = tuple(tuple(min(c, s - i) for i in range(0, s, c)) for s, c in zip(pshape, tchunks))
    empty, offs = p._name("empty"), p._name("offsets")
    p._array(empty, VirtualEmptyArray(pshape, np.float64, tchunks))
    p._array(offs, VirtualOffsetsArray(nb))
    mfn = functools.partial(func_with_block_id(map_direct_wrap(_copy_chunk), nb),
                            arrays=(RefArray(sname, st),), target_chunks=tnorm)
    gname = p._name("array")
    gop, _ = p.blockwise_op(mfn, gname, pshape, np.float64, tchunks,
                            [(empty, p.g.nodes[empty]["target"]), (offs, p.g.nodes[offs]["target"])])
    cname = p._name("array")
    cop, _ = p.blockwise_op(functools.partial(ksum, axis=(1,), keepdims=True, dtype=np.float64),
                            cname, (m, 1, n), np.float64, pchunks, [(gname, p.g.nodes[gname]["target"])])
    qname = p._name("array")
    qop, qt = p.blockwise_op(functools.partial(np.squeeze, axis=(1,)), qname, (m, n), np.float64, (cm, cn),
                             [(cname, p.g.nodes[cname]["target"])])
    q_spec = BlockwiseSpec(lambda key: [(cname, key[1], 0, key[2])], qop.pipeline.config.function, 1,
                           qop.pipeline.config.reads_map, qop.pipeline.config.write)
    qop = PrimitiveOperation(CubedPipeline(apply_blockwise, "apply_blockwise-sq", [], q_spec), qt, 0, p.MEM, 0,
                             qop.num_tasks, True)
    second = fuse(fuse(gop, cop), qop)
    for nm in (gname, cname):
        t = p.g.nodes[nm]["target"]
        p.g.remove_node(nm)
        p.lazy = [x for x in p.lazy if x is not t]
    op = p._op(second, qname, [empty, offs, sname], second.num_tasks)
    return p.finalize(), qname, aname, bname, op


# -- index (core/ops.py:374-517) ------------------------------------------------
_read_index_chunk = _ref_fn("_read_index_chunk", "cubed.core.ops")


def index_plan(work_dir, seed, shape=(30, 8), chunks=(10, 8), selection=(slice(1, None, None),)):
    """``-(random(shape)[selection])``: index's map_direct op (target chunks
    = the source chunk lengths along sliced dims, step 1) fused into the
    ``negative`` that consumes it (in-degree 1)."""
    p = RefPlan(work_dir)
    rop, rname, rsrcs = p.random(shape, chunks, seed)
    p.add(rop, rname, rsrcs)
    src = p.g.nodes[rname]["target"]
    sel = tuple(selection) + (slice(None),) * (len(shape) - len(selection))
    out_shape, out_chunks = [], []
    for s, n, c in zip(sel, shape, chunks):
        if isinstance(s, slice):
            a, b, st = s.indices(n)
            out_shape.append(max(0, (b - a + st - 1) // st))
            out_chunks.append(max(c // st, 1))
    out_shape, out_chunks = tuple(out_shape), tuple(out_chunks)
    tnorm = tuple(tuple(min(c, s - i) for i in range(0, s, c)) for s, c in zip(out_shape, out_chunks))
    nb = numblocks(out_shape, out_chunks)
    empty, offs = p._name("empty"), p._name("offsets")
    p._array(empty, VirtualEmptyArray(out_shape, np.float64, out_chunks))
    p._array(offs, VirtualOffsetsArray(nb))
    fn = functools.partial(func_with_block_id(map_direct_wrap(_read_index_chunk), nb),
                           arrays=(RefArray(rname, src),), target_chunks=tnorm, selection=sel)
    iname = p._name("array")
    iop, it = p.blockwise_op(fn, iname, out_shape, np.float64, out_chunks,
                             [(empty, p.g.nodes[empty]["target"]), (offs, p.g.nodes[offs]["target"])])
    nname = p._name("array")
    nop, _ = p.blockwise_op(np.negative, nname, out_shape, np.float64, out_chunks, [(iname, it)])
    fused = fuse(iop, nop)
    p.g.remove_node(iname)
    p.lazy = [t for t in p.lazy if t is not it]
    p._op(fused, nname, [empty, offs, rname], fused.num_tasks)
    return p.finalize(), nname, rname
