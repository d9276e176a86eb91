"""Reference-built DAGs on the MI355X executor (cubed_amd/runtime/
reference_dag.py): the plug-in contract is "any DAG" (cubed/runtime/
types.py:9-14).  The reference cannot be imported here, so the DAGs come from
tests/refdag.py's stand-ins of the reference's classes and chunk-function
wrappers (API-shape fixtures, see its docstring).

CPU: the conversion (array kinds, traced programs through fuse closures and
partial binding, the random chunk function recognised as the Philox leaf,
copy ops) and the launches the dry executor would run; refusals name the op.
GPU: the whole plan executed, the requested array written to its Zarr store
and read back bit-exactly against the oracle (numpy Philox, f32 arithmetic).
"""

import functools
import random

import numpy as np
import pytest

import cubed_amd.lowering as L
from cubed_amd import ir
from cubed_amd.runtime import reference_dag as RD
from cubed_amd.storage import DeviceArray, VirtualEmptyArray, VirtualInMemoryArray, VirtualOffsetsArray

import refdag


def _seed(s):
    random.seed(s)
    return random.getrandbits(128)


def _leaves(e, out):
    """Leaves of an IR expression (Philox / Arg), walking every Expr field."""
    import dataclasses

    if isinstance(e, (ir.Philox, ir.Arg)):
        out.append(e)
        return out
    if dataclasses.is_dataclass(e):
        for f in dataclasses.fields(e):
            v = getattr(e, f.name)
            for c in (v if isinstance(v, (tuple, list)) else (v,)):
                if isinstance(c, ir.Expr):
                    _leaves(c, out)
    return out


def test_reference_dag_is_recognised(tmp_path):
    dag, out, _ = refdag.example_plan(tmp_path, _seed(1))
    assert RD.is_reference_dag(dag)
    import cubed_amd as cubed
    import cubed_amd.array_api as xp

    a = xp.ones((4, 4), chunks=(2, 2), spec=cubed.Spec(allowed_mem="1GB"))
    from cubed_amd.core.plan import arrays_to_plan

    assert not RD.is_reference_dag(arrays_to_plan(a + 1)._finalize_dag())


def test_conversion_keeps_names_counts_and_traces_programs(tmp_path):
    seed = _seed(2)
    dag, out, _ = refdag.example_plan(tmp_path, seed)
    conv = RD.convert_reference_dag(dag)
    g = conv.dag
    assert set(g.nodes) >= set(dag.nodes)
    for n, d in dag.nodes(data=True):
        if "primitive_op" in d:
            assert g.nodes[n]["primitive_op"].num_tasks == d["primitive_op"].num_tasks
        t = d.get("target")
        if isinstance(t, refdag.LazyZarrArray):
            dt = g.nodes[n]["target"]
            assert isinstance(dt, DeviceArray)
            assert (dt.shape, dt.dtype, tuple(dt.chunks)) == (t.shape, t.dtype, t.chunks)
        elif isinstance(t, refdag.VirtualEmptyArray):
            assert isinstance(g.nodes[n]["target"], VirtualEmptyArray)
        elif isinstance(t, refdag.VirtualOffsetsArray):
            assert isinstance(g.nodes[n]["target"], VirtualOffsetsArray)
        elif isinstance(t, refdag.VirtualInMemoryArray):
            assert isinstance(g.nodes[n]["target"], VirtualInMemoryArray)
    progs = {n: d["pipeline"].config.function for n, d in g.nodes(data=True)
             if d.get("pipeline") is not None and isinstance(d["pipeline"].config, RD.BlockwiseSpec)}
    kinds = {n: [type(x).__name__ for x in _leaves(p.outputs, [])] for n, p in progs.items()}
    # the fused random + astype op reads no array: its one leaf is Philox
    fused = [n for n, k in kinds.items() if k == ["Philox"]]
    assert len(fused) == 1
    ph = _leaves(progs[fused[0]].outputs, [])[0]
    assert ph.root_seed == seed and ph.numblocks == (4, 3) and ph.block_arg == 1
    assert progs[fused[0]].outputs.dtype == np.float32
    # the two scalar ops: an array leaf and a 0-d leaf each
    assert sorted(len(k) for k in kinds.values()) == [1, 2, 2]
    # the requested output's Zarr sink is the LazyZarrArray's store
    assert out in conv.sinks


def test_dry_run_launches(tmp_path, built, dry):
    dag, out, _ = refdag.example_plan(tmp_path, _seed(3))
    dry.launched.clear()
    dry.execute_dag(RD.convert_reference_dag(dag).dag, array_names=[out])
    kinds = [type(l).__name__ for l in dry.launched]
    # the executor fuses the elementwise chain into one streaming launch and
    # the rechunk into one copy
    assert kinds.count("CopyLaunch") == 1
    assert 1 <= kinds.count("FusedLaunch") <= 3


def test_unlowerable_reference_op_is_refused(tmp_path):
    p = refdag.RefPlan(tmp_path)
    rop, rname, rsrcs = p.random((8, 8), (4, 4), _seed(4))
    p.add(rop, rname, rsrcs)

    def reduce_like(x):  # a dict of fields, like _mean_func
        return {"n": x.size, "total": np.sum(x)}

    name = p._name("array")
    op, _ = p.blockwise_op(reduce_like, name, (8, 8), np.float64, (4, 4), [(rname, p.g.nodes[rname]["target"])])
    op_name = p.add(op, name, [rname])
    with pytest.raises(L.LoweringError, match=op_name):
        RD.convert_reference_dag(p.finalize())


def test_non_elementwise_index_mapping_is_refused(tmp_path):
    p = refdag.RefPlan(tmp_path)
    rop, rname, rsrcs = p.random((8, 4), (4, 4), _seed(5))
    p.add(rop, rname, rsrcs)
    name = p._name("array")
    op, target = p.blockwise_op(np.negative, name, (4, 8), np.float64, (4, 4),
                                [(rname, p.g.nodes[rname]["target"])])
    # a transpose-like key function: output block (i, j) reads (j, i)
    bf = lambda k: [(rname, k[2], k[1])]  # noqa: E731
    spec = refdag.BlockwiseSpec(bf, np.negative, 1, op.pipeline.config.reads_map, op.pipeline.config.write)
    op = refdag.PrimitiveOperation(refdag.CubedPipeline(refdag.apply_blockwise, "t", [], spec), target,
                                   0, p.MEM, 0, 2, True)
    op_name = p.add(op, name, [rname])
    with pytest.raises(L.LoweringError, match=op_name):
        RD.convert_reference_dag(p.finalize())


@pytest.mark.gpu
def test_reference_plan_runs_on_the_gpu(tmp_path, gpu_executor):
    """The example plan through GpuDagExecutor.execute_dag (recognised as a
    reference DAG), the requested array read back from its Zarr store and
    the intermediate (not requested) left unwritten; values bit-exact vs
    numpy Philox blocks -> f32 -> * 2 + 1 (f32 arithmetic) -> rechunk."""
    from cubed_amd.runtime.types import Callback
    from cubed_amd.zarr_io import ZarrV2Array
    from oracle import cubed_ref as R

    class Rec(Callback):
        def __init__(self):
            self.events = []

        def on_task_end(self, event):
            self.events.append(event)

    seed = _seed(6)
    shape, chunks = (40, 60), (10, 20)
    dag, out, mid = refdag.example_plan(tmp_path, seed, shape, chunks, (40, 10))
    rec = Rec()
    gpu_executor.execute_dag(dag, callbacks=[rec], array_names=[out])
    exp = R.random_array(shape, chunks, seed).astype(np.float32) * np.float32(2) + np.float32(1)
    got = ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...]
    assert got.dtype == np.float32 and got.shape == shape
    np.testing.assert_array_equal(got, exp)
    ops = {n: d["primitive_op"].num_tasks for n, d in dag.nodes(data=True) if "primitive_op" in d}
    got_tasks = {e.array_name: e.num_tasks for e in rec.events}
    for n, k in ops.items():
        if n in got_tasks:
            assert got_tasks[n] == k
    assert not (tmp_path / f"{mid}.zarr").exists()
    # a second execute replays (same DAG, same names)
    gpu_executor.execute_dag(dag, array_names=[out])
    np.testing.assert_array_equal(ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...], exp)


@pytest.mark.gpu
def test_reference_random_unfused_on_the_gpu(tmp_path, gpu_executor):
    """random on its own (the op not fused into a consumer) and a fuse-free
    elementwise consumer reading it from HBM."""
    from cubed_amd.zarr_io import ZarrV2Array
    from oracle import cubed_ref as R

    seed = _seed(7)
    p = refdag.RefPlan(tmp_path)
    rop, rname, rsrcs = p.random((30, 20), (7, 20), seed)
    p.add(rop, rname, rsrcs)
    name = p._name("array")
    op, _ = p.blockwise_op(functools.partial(np.sqrt), name, (30, 20), np.float64, (7, 20),
                           [(rname, p.g.nodes[rname]["target"])])
    p.add(op, name, [rname])
    dag = p.finalize()
    gpu_executor.execute_dag(dag, array_names=[rname, name])
    x = R.random_array((30, 20), (7, 20), seed)
    np.testing.assert_array_equal(ZarrV2Array.open(str(tmp_path / f"{rname}.zarr"))[...], x)
    np.testing.assert_array_equal(ZarrV2Array.open(str(tmp_path / f"{name}.zarr"))[...], np.sqrt(x))


def test_reference_mean_plan_converts_to_one_chain(tmp_path, built, dry):
    """The reference's mean plan (random fused into _mean_func; merge_chunks
    + _mean_combine + _mean_aggregate + squeeze fused into one op): the
    fused closures are taken apart and re-fused, the reduction functions map
    to the IR reductions, and the executor runs the whole chain as fused
    launches (no host code, nothing refused)."""
    dag, out, partials, op = refdag.mean_plan(tmp_path, _seed(8))
    conv = RD.convert_reference_dag(dag)
    prog = conv.dag.nodes[op]["pipeline"].config.function
    assert isinstance(prog, ir.ExprProgram)
    first = [d for n, d in conv.dag.nodes(data=True) if d.get("pipeline") is not None
             and n != op and isinstance(d["pipeline"].config, RD.BlockwiseSpec)]
    assert len(first) == 1 and first[0]["pipeline"].config.function.reduce is not None
    dry.launched.clear()
    dry.execute_dag(conv.dag, array_names=[out])
    assert dry.launched and all(type(l).__name__ in ("FusedLaunch",) for l in dry.launched)


@pytest.mark.gpu
def test_reference_mean_plan_on_the_gpu(tmp_path, gpu_executor):
    """mean(random(40, 60), axis=0) built as the reference builds it: the
    result written to its Zarr store, rtol 1e-12 against the oracle's f64
    column means of the same numpy Philox blocks; TaskEndEvents carry the
    reference's task counts (12 per-chunk tasks, 3 merge tasks)."""
    from cubed_amd.runtime.types import Callback
    from cubed_amd.zarr_io import ZarrV2Array
    from oracle import cubed_ref as R

    class Rec(Callback):
        def __init__(self):
            self.events = []

        def on_task_end(self, event):
            self.events.append(event)

    seed = _seed(9)
    dag, out, partials, op = refdag.mean_plan(tmp_path, seed, (40, 60), (10, 20))
    rec = Rec()
    gpu_executor.execute_dag(dag, callbacks=[rec], array_names=[out])
    x = R.random_array((40, 60), (10, 20), seed)
    got = ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...]
    assert got.shape == (60,) and got.dtype == np.float64
    np.testing.assert_allclose(got, x.mean(axis=0), rtol=1e-12, atol=0)
    counts = {e.array_name: e.num_tasks for e in rec.events}
    assert counts.get(op) == 3


def test_reference_matmul_plan_converts_to_a_gemm_chain(tmp_path, built, dry):
    """The reference matmul plan (_matmul fused with the first _chunk_sum;
    merge_chunks + _chunk_sum + squeeze fused): the product becomes the
    chunk GEMM program and the executor runs one chained GEMM launch (the
    partial-product arrays elided), as for cubed_amd's own matmul."""
    dag, out, a, b, op = refdag.matmul_plan(tmp_path, _seed(10), _seed(11))
    conv = RD.convert_reference_dag(dag)
    progs = [d["pipeline"].config.function for _, d in conv.dag.nodes(data=True)
             if d.get("pipeline") is not None and isinstance(d["pipeline"].config, RD.BlockwiseSpec)]
    assert any(isinstance(p, ir.GemmThenProgram) for p in progs)
    dry.launched.clear()
    dry.execute_dag(conv.dag, array_names=[out])
    kinds = [type(l).__name__ for l in dry.launched]
    assert kinds.count("GemmLaunch") == 1


def test_reference_partial_reduce_plan_converts(tmp_path, built, dry):
    """reduction(..., use_new_impl=True)'s partial_reduce op (a block
    function yielding an iterator of input keys) converts and lowers."""
    dag, out, src, op = refdag.partial_reduce_mean_plan(tmp_path, _seed(22))
    conv = RD.convert_reference_dag(dag)
    dry.launched.clear()
    dry.execute_dag(conv.dag, array_names=[out])
    kinds = {type(l).__name__ for l in dry.launched}
    assert "FusedLaunch" in kinds and kinds <= {"FusedLaunch", "CopyLaunch", "_Alloc"}, kinds


@pytest.mark.gpu
def test_reference_partial_reduce_plan_on_the_gpu(tmp_path, gpu_executor):
    """The partial_reduce mean against the f64 column means of the oracle's
    Philox blocks, rtol 1e-12."""
    from cubed_amd.zarr_io import ZarrV2Array
    from oracle import cubed_ref as R

    seed = _seed(23)
    dag, out, src, op = refdag.partial_reduce_mean_plan(tmp_path, seed)
    gpu_executor.execute_dag(dag, array_names=[out])
    X = R.random_array((40, 60), (10, 20), seed)
    got = ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...]
    np.testing.assert_allclose(got, X.mean(axis=0), rtol=1e-12, atol=0)


def test_reference_argmax_plan_converts(tmp_path, built, dry):
    """The reference arg_reduction plan (map_blocks(_arg_map_func) with
    block_id + _arg_func, merge_chunks + _arg_combine + _arg_aggregate +
    squeeze) converts: the block_id map is a pair reduction with an Iota
    leaf, and the plan lowers to fused launches only."""
    dag, out, src, op = refdag.argreduce_plan(tmp_path, _seed(19))
    conv = RD.convert_reference_dag(dag)
    dry.launched.clear()
    dry.execute_dag(conv.dag, array_names=[out])
    kinds = {type(l).__name__ for l in dry.launched}
    assert kinds <= {"FusedLaunch", "CopyLaunch", "_Alloc"}, kinds


@pytest.mark.gpu
@pytest.mark.parametrize("fn", ["argmax", "argmin"])
def test_reference_argmax_plan_on_the_gpu(tmp_path, gpu_executor, fn):
    """argmax / argmin along axis 0 of a random f64 array, built as the
    reference builds it: bit-exact indices against numpy on the oracle's
    Philox blocks."""
    from cubed_amd.zarr_io import ZarrV2Array
    from oracle import cubed_ref as R

    seed = _seed(20)
    dag, out, src, op = refdag.argreduce_plan(tmp_path, seed, arg_func=getattr(np, fn))
    gpu_executor.execute_dag(dag, array_names=[out])
    X = R.random_array((40, 60), (10, 20), seed)
    got = ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...]
    assert np.array_equal(got, getattr(np, fn)(X, axis=0))


def test_reference_tensordot_plan_converts_to_a_gemm_chain(tmp_path, built, dry):
    """The reference tensordot plan (_tensordot keeping a unit contracted
    dim, then numpy sum over it through merge_chunks) runs as one chained GEMM
    launch, as cubed_amd's own tensordot does."""
    dag, out, a, b, op = refdag.tensordot_plan(tmp_path, _seed(15), _seed(16))
    conv = RD.convert_reference_dag(dag)
    progs = [d["pipeline"].config.function for _, d in conv.dag.nodes(data=True)
             if d.get("pipeline") is not None and isinstance(d["pipeline"].config, RD.BlockwiseSpec)]
    assert any(isinstance(p, ir.GemmThenProgram) for p in progs)
    dry.launched.clear()
    dry.execute_dag(conv.dag, array_names=[out])
    kinds = [type(l).__name__ for l in dry.launched]
    assert kinds.count("GemmLaunch") == 1


@pytest.mark.gpu
def test_reference_tensordot_plan_on_the_gpu(tmp_path, gpu_executor):
    """tensordot(A, B, axes=1) of two random f64 arrays built as the reference
    builds it, against the f64 product of the oracle's Philox blocks."""
    from cubed_amd.zarr_io import ZarrV2Array
    from oracle import cubed_ref as R

    sa, sb = _seed(17), _seed(18)
    dag, out, a, b, op = refdag.tensordot_plan(tmp_path, sa, sb)
    gpu_executor.execute_dag(dag, array_names=[out])
    A = R.random_array((60, 80), (20, 20), sa)
    B = R.random_array((80, 40), (20, 20), sb)
    got = ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...]
    np.testing.assert_allclose(got, A @ B, rtol=1e-12, atol=0)


@pytest.mark.gpu
def test_reference_matmul_plan_on_the_gpu(tmp_path, gpu_executor):
    """matmul of two random f64 arrays built as the reference builds it:
    the result (written to its Zarr store) against the f64 product of the
    oracle's Philox blocks, rtol 1e-12."""
    from cubed_amd.zarr_io import ZarrV2Array
    from oracle import cubed_ref as R

    sa, sb = _seed(12), _seed(13)
    dag, out, a, b, op = refdag.matmul_plan(tmp_path, sa, sb)
    gpu_executor.execute_dag(dag, array_names=[out])
    A = R.random_array((60, 80), (20, 20), sa)
    B = R.random_array((80, 40), (20, 20), sb)
    got = ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...]
    np.testing.assert_allclose(got, A @ B, rtol=1e-12, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("selection", [(slice(1, None, None),), (slice(None, None, None), slice(2, 7, 2)),
                                       (4, slice(None, None, None))])
def test_reference_index_plan_on_the_gpu(tmp_path, gpu_executor, selection):
    """index (map_direct over _read_index_chunk) fused into negative, for
    a shifted slice (vorticity's a[1:]), a strided slice and an integer
    index: bit-exact against numpy indexing of the oracle's Philox blocks."""
    from cubed_amd.zarr_io import ZarrV2Array
    from oracle import cubed_ref as R

    seed = _seed(14)
    dag, out, src = refdag.index_plan(tmp_path, seed, (30, 8), (10, 8), selection)
    gpu_executor.execute_dag(dag, array_names=[out])
    x = R.random_array((30, 8), (10, 8), seed)
    got = ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...]
    np.testing.assert_array_equal(got, -x[selection])


def test_reference_index_plan_converts(tmp_path):
    dag, out, src = refdag.index_plan(tmp_path, _seed(15))
    conv = RD.convert_reference_dag(dag)
    progs = [d["pipeline"].config.function for _, d in conv.dag.nodes(data=True)
             if d.get("pipeline") is not None and isinstance(d["pipeline"].config, RD.BlockwiseSpec)]
    assert any(any(isinstance(l, ir.Region) for l in _leaves_any(p.outputs)) for p in progs)


def _leaves_any(e, out=None):
    import dataclasses

    out = [] if out is None else out
    if isinstance(e, (ir.Philox, ir.Arg, ir.Region)):
        out.append(e)
        return out
    if dataclasses.is_dataclass(e):
        for f in dataclasses.fields(e):
            v = getattr(e, f.name)
            for c in (v if isinstance(v, (tuple, list)) else (v,)):
                if isinstance(c, ir.Expr):
                    _leaves_any(c, out)
    return out


def _kernel_launches(ex):
    sched = ex.last_schedule
    if sched is None:
        return []
    return [type(l).__name__ for step in sched.steps for l in step[1]
            if type(l).__name__ in ("FusedLaunch", "CopyLaunch", "GemmLaunch")]


@pytest.mark.gpu
def test_reference_plan_resumes_from_complete_zarr_sinks(tmp_path, gpu_executor):
    """cubed/runtime/pipeline.py:25-33: with resume, an array whose Zarr
    store holds every chunk counts as computed, whichever process wrote it.
    The same reference plan built twice (fresh DAG objects, same work_dir
    and names -- a second process): once the requested sink is complete the
    resumed run launches no kernel; with only the intermediate complete, the
    rechunk reads it back from its store (uploaded into HBM) and writes the
    same bytes.  The converted arrays' HBM is released after each run."""
    from cubed_amd.zarr_io import ZarrV2Array
    from oracle import cubed_ref as R

    seed = _seed(16)
    shape, chunks = (40, 60), (10, 20)
    exp = R.random_array(shape, chunks, seed).astype(np.float32) * np.float32(2) + np.float32(1)
    dag, out, mid = refdag.example_plan(tmp_path, seed, shape, chunks, (40, 10))
    gpu_executor.execute_dag(dag, array_names=[mid, out])
    assert _kernel_launches(gpu_executor)
    assert not any(d.allocated for d in RD.convert_reference_dag(dag).targets.values())
    np.testing.assert_array_equal(ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...], exp)
    np.testing.assert_array_equal(ZarrV2Array.open(str(tmp_path / f"{mid}.zarr"))[...], exp)

    dag2, out2, mid2 = refdag.example_plan(tmp_path, seed, shape, chunks, (40, 10))
    assert (out2, mid2) == (out, mid) and dag2 is not dag
    gpu_executor.execute_dag(dag2, array_names=[out2], resume=True)
    assert _kernel_launches(gpu_executor) == []

    import shutil

    shutil.rmtree(tmp_path / f"{out}.zarr")
    dag3, out3, _ = refdag.example_plan(tmp_path, seed, shape, chunks, (40, 10))
    gpu_executor.execute_dag(dag3, array_names=[out3], resume=True)
    assert _kernel_launches(gpu_executor) == ["CopyLaunch"]  # only the rechunk
    np.testing.assert_array_equal(ZarrV2Array.open(str(tmp_path / f"{out}.zarr"))[...], exp)


def test_converted_arrays_released_after_write_back(tmp_path, built, dry, monkeypatch):
    """the conversion is cached while the reference keeps its
    finalized DAG alive (an lru_cache of 128 plans, core/plan.py:178); the
    converted targets must not keep HBM after the results reach Zarr (the
    dry run records the write-back instead of copying device memory)."""
    written = []
    monkeypatch.setattr(RD, "write_back", lambda conv, names: written.append(list(names)))
    dags = []
    for s in (17, 18):
        dag, out, _ = refdag.example_plan(tmp_path / str(s), _seed(s))
        RD.execute_reference_dag(dry, dag, array_names=[out])
        dags.append(dag)
        assert written[-1] == [out]
    for dag in dags:
        conv = RD.convert_reference_dag(dag)
        assert conv.targets and not any(d.allocated for d in conv.targets.values())
