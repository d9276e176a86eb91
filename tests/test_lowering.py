"""Lowering decisions of the MI355X executor, checked on CPU (no launches).

``DryExecutor`` (tests/dryrun.py) lowers plans to the exact kernel-argument
tables the GPU path launches; these tests pin the decisions that decide
performance: how many launches a pipeline becomes, whether the streaming
fast path is taken, and that reduction chains are fused into one pass.
"""

import re
import ctypes
import math
import random

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
import cubed_amd.lowering as Lw
from cubed_amd import _native as nat
from cubed_amd import ir
from cubed_amd.core.plan import arrays_to_plan
from cubed_amd.lowering import MODE_STREAM, CopyLaunch, FusedLaunch


def _fused(ex):
    return [l for l in ex.launched if isinstance(l, FusedLaunch)]


def test_quad_means_is_one_streaming_launch(built, dry):
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(1)
    u = xp.astype(crandom.random((200, 16, 32), chunks=(10, 16, 32), spec=spec), xp.float32)
    v = xp.astype(crandom.random((200, 16, 32), chunks=(10, 16, 32), spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=dry, array_names=[u.name, v.name])
    dry.launched.clear()
    m = xp.mean(u * v, axis=0)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    fused = _fused(dry)
    assert len(fused) == 1, [type(l).__name__ for l in dry.launched]
    L = fused[0]
    assert not L.gathers
    P = L.prog
    assert P.mode & MODE_STREAM and P.mode & 4
    assert not P.mode & (32 | 64)  # 512 kept elements: too small a grid for W > 1
    assert (P.ndim, P.nred, P.nleaves, P.nfields) == (2, 1, 2, 2)
    assert L.max_red == 200 and L.max_kept == 16 * 32
    assert P.ninsns == 1  # MUL in place on the first leaf register (its last use)


def test_chain_fusion_can_be_disabled(built, dry):
    dry.fuse_reductions = False
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(1)
    u = xp.astype(crandom.random((200, 16, 32), chunks=(10, 16, 32), spec=spec), xp.float32)
    arrays_to_plan(u).execute(executor=dry, array_names=[u.name])
    dry.launched.clear()
    m = xp.mean(u, axis=0)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    assert len(_fused(dry)) >= 2  # per-chunk reduce + merge/combine/aggregate rounds


def test_elementwise_map_is_streaming(built, dry):
    spec = cubed.Spec(allowed_mem=10**8, executor=dry)
    a = cubed.from_array(np.arange(4096, dtype=np.float64).reshape(64, 64), chunks=(16, 64), spec=spec)
    arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
    dry.launched.clear()
    b = (a + 1) * 2
    arrays_to_plan(b).execute(executor=dry, resume=True, array_names=[b.name])
    fused = _fused(dry)
    assert len(fused) >= 1
    assert fused[-1].prog.nfields == 0


def test_rechunk_lowers_to_one_copy_launch(built, dry):
    spec = cubed.Spec(allowed_mem="288GB", executor=dry)
    x = cubed.from_array(np.arange(64 * 48, dtype=np.float32).reshape(64, 48), chunks=(8, 48), spec=spec)
    arrays_to_plan(x).execute(executor=dry, array_names=[x.name])
    dry.launched.clear()
    y = x.rechunk((64, 8))
    arrays_to_plan(y).execute(executor=dry, resume=True, array_names=[y.name])
    copies = [l for l in dry.launched if isinstance(l, CopyLaunch)]
    assert len(copies) == 1
    # every target element is written exactly once
    boxes = copies[0].boxes
    assert sum(int(np.prod(b.extent)) for b in boxes) == 64 * 48


def test_two_op_rechunk_is_one_direct_copy(built, dry):
    """The reference plans rows -> columns under a small allowed_mem as two
    copy ops through an intermediate (primitive/rechunk.py:144-155; config
    3's 2 GB plan: 625 + 25 tasks).  The executor composes them into ONE
    copy from the source into the target chunks (rewrites.compose_rechunks):
    the intermediate is never allocated, every target element is written
    once, and both ops still report their TaskEndEvents and task counts."""
    from cubed_amd.runtime.types import Callback

    class Count(Callback):
        def __init__(self):
            self.tasks = {}

        def on_task_end(self, e):
            self.tasks[e.array_name] = e.num_tasks

    spec = cubed.Spec(allowed_mem=1_200_000, reserved_mem=0, executor=dry)
    x = cubed.from_array(np.arange(500 * 600, dtype=np.float32).reshape(500, 600), chunks=(10, 600),
                         spec=spec)
    arrays_to_plan(x).execute(executor=dry, array_names=[x.name])
    y = x.rechunk((500, 10))
    plan = arrays_to_plan(y)
    ops = {n: d["primitive_op"].num_tasks for n, d in plan._finalize_dag().nodes(data=True)
           if d.get("op_name") == "rechunk"}
    assert len(ops) == 2  # the reference's two-stage plan
    dry.launched.clear()
    cb = Count()
    plan.execute(executor=dry, resume=True, array_names=[y.name], callbacks=[cb])
    copies = [l for l in dry.launched if isinstance(l, CopyLaunch)]
    assert len(copies) == 1
    boxes = copies[0].boxes
    assert sum(int(np.prod(b.extent)) for b in boxes) == 500 * 600
    # boxes read the SOURCE chunks: no box crosses a 10-row source band
    assert all(b.extent[0] <= 10 for b in boxes)
    for n, t in ops.items():
        assert cb.tasks[n] == t
    ints = [d["target"] for _, d in plan._finalize_dag().nodes(data=True)
            if str(d.get("name", "")).endswith("-int")]
    assert ints and all(not t.allocated for t in ints)


def test_requested_intermediate_keeps_both_copies(built, dry):
    spec = cubed.Spec(allowed_mem=1_200_000, reserved_mem=0, executor=dry)
    x = cubed.from_array(np.arange(500 * 600, dtype=np.float32).reshape(500, 600), chunks=(10, 600),
                         spec=spec)
    arrays_to_plan(x).execute(executor=dry, array_names=[x.name])
    y = x.rechunk((500, 10))
    dag = arrays_to_plan(y)._finalize_dag()
    mid = [n for n in dag.nodes if str(n).endswith("-int")][0]
    dry.launched.clear()
    arrays_to_plan(y).execute(executor=dry, resume=True, array_names=[y.name, mid])
    assert len([l for l in dry.launched if isinstance(l, CopyLaunch)]) == 2


def test_task_table_rows_match_tasks(built, dry):
    spec = cubed.Spec(allowed_mem=10**8, executor=dry)
    a = cubed.from_array(np.ones((30, 40)), chunks=(7, 9), spec=spec)
    arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
    dry.launched.clear()
    s = xp.sum(a, axis=1)
    arrays_to_plan(s).execute(executor=dry, resume=True, array_names=[s.name])
    for L in _fused(dry):
        tab = L.table.numpy().view(nat.TASK_DTYPE)
        assert len(tab) == L.ntasks
        assert (tab["extent"] >= 1).all()


def test_fused_programs_compile_specialised(built, dry):
    """Every fused launch of a mixed plan gets a runtime-specialised gfx950
    kernel (hipRTC; no GPU needed to compile) with the program baked in."""
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(2)
    a = xp.astype(crandom.random((60, 8, 12), chunks=(10, 8, 12), spec=spec), xp.float32)
    b = cubed.from_array(np.arange(60 * 96, dtype=np.int64).reshape(60, 96), chunks=(7, 32), spec=spec)
    outs = [xp.mean(a * a, axis=0), xp.sum(b, axis=1), xp.max(b, axis=0), cubed.nanmean(a, axis=2),
            xp.where(a > 0.5, a, -a), xp.astype(b, xp.float64) / 3]
    arrays_to_plan(*outs).execute(executor=dry, array_names=[o.name for o in outs])
    fused = _fused(dry)
    assert len(fused) >= 6
    for L in fused:
        assert L.handle is not None
        src = nat.program_source(L.handle)
        assert "jit_prologue" in src and "cubed_" in src
        assert nat.lib().cubed_fused_code_bytes(L.handle) > 0


def test_config1_is_one_streaming_launch(built, dry):
    """(a + 1) * 2 -> mean(axis=0) over a 4x4 chunk grid: the add map is fused
    into the mean (executor producer fusion), the reduction rounds into one
    pass, and the chunk index x rows reduction runs on the streaming kernel
    with two reduced dims (the chunks of a column sit 4 slots apart)."""
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(3)
    a = crandom.random((400, 400), chunks=(100, 100), spec=spec)
    arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
    dry.launched.clear()
    m = xp.mean((a + 1) * 2, axis=0)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    fused = _fused(dry)
    assert len(dry.launched) == 1 and len(fused) == 1
    P = fused[0].prog
    assert P.mode & MODE_STREAM
    assert (P.ndim, P.nred, P.nleaves, P.nfields) == (3, 2, 1, 2)
    assert fused[0].ntasks == 4 and fused[0].max_red == 400


def test_producer_fusion_keeps_materialised_inputs(built, dry):
    """A map whose output was already computed (resume) is read, not fused."""
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(3)
    a = crandom.random((400, 400), chunks=(100, 100), spec=spec)
    b = a + 1
    arrays_to_plan(b).execute(executor=dry, array_names=[b.name])
    dry.launched.clear()
    m = xp.mean(b * 2, axis=0)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    fused = _fused(dry)
    assert len(fused) == 1 and fused[0].prog.nleaves == 1
    assert fused[0].prog.leaf_kind[0] == 0  # reads b's chunks (no Philox recompute)


def test_two_random_streams_are_not_fused(built, dry):
    """mean(u * v) over two unmaterialised random arrays: the Philox maps
    are not fused into the mean (a task carries one stream key); they are
    generated as maps and the mean reads them."""
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(42)
    u = xp.astype(crandom.random((50, 37, 40), chunks=(10, 37, 40), spec=spec), xp.float32)
    v = xp.astype(crandom.random((50, 37, 40), chunks=(10, 37, 40), spec=spec), xp.float32)
    m = xp.mean(u * v, axis=0)
    arrays_to_plan(m).execute(executor=dry, array_names=[m.name])
    for L in _fused(dry):
        assert sum(L.prog.leaf_kind[i] == 1 for i in range(L.prog.nleaves)) <= 1


def test_where_producers_fuse_into_one_read(built, dry):
    """where(a > 0.5, a, -a): both maps fuse into the where, and the three
    reads of a's chunk become one leaf (argument dedupe)."""
    x = np.random.default_rng(6).random((40, 30))
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    a = cubed.from_array(x, chunks=(16, 16), spec=spec)
    arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
    dry.launched.clear()
    w = xp.where(a > 0.5, a, -a)
    arrays_to_plan(w).execute(executor=dry, resume=True, array_names=[w.name])
    fused = _fused(dry)
    assert len(fused) == 1 and fused[0].prog.nleaves == 1  # the 0.5 scalar is a constant


def test_vorticity_regions_are_pieces_not_gathers(built, dry):
    """mean(a[1:] * x + b[1:] * y) (config 4 shape): each a[1:] chunk
    straddles two source chunks along the reduced time axis -> two pieces
    per task reading in place, partials combined per task; no scratch."""
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(1)
    a = crandom.random((40, 18, 16), chunks=(10, 9, 8), spec=spec)
    b = crandom.random((40, 18, 16), chunks=(10, 9, 8), spec=spec)
    x = crandom.random((18, 16), chunks=(9, 8), spec=spec)
    y = crandom.random((18, 16), chunks=(9, 8), spec=spec)
    arrays_to_plan(a, b, x, y).execute(executor=dry, array_names=[a.name, b.name, x.name, y.name])
    dry.launched.clear()
    m = xp.mean(a[1:] * x + b[1:] * y)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    fused = _fused(dry)
    first = fused[0]
    assert not first.gathers and first.groups is not None
    assert first.prog.mode & 16  # partials + grouped finish
    assert first.ntasks > first.ngroups


@pytest.mark.parametrize("merge", [False, True])
def test_vorticity_chain_walks_source_chunks(built, dry, monkeypatch, merge):
    """The whole reduction (per-chunk mean + merge/combine rounds + aggregate)
    is ONE launch whose rows are the source chunks: the tail plane of task j
    and the head of task j+1 (both in source chunk j+1) are merged, so no
    single-plane pieces remain and there is one group (the scalar).  With
    row merging (the default) the chunks of one T band, consecutive slots
    of a and of x, become one row with a chunk dim."""
    monkeypatch.setattr(Lw, "MERGE_ROWS", merge)
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(1)
    a = crandom.random((40, 18, 16), chunks=(10, 9, 8), spec=spec)
    b = crandom.random((40, 18, 16), chunks=(10, 9, 8), spec=spec)
    x = crandom.random((18, 16), chunks=(9, 8), spec=spec)
    y = crandom.random((18, 16), chunks=(9, 8), spec=spec)
    arrays_to_plan(a, b, x, y).execute(executor=dry, array_names=[a.name, b.name, x.name, y.name])
    dry.launched.clear()
    m = xp.mean(a[1:] * x + b[1:] * y)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    fused = _fused(dry)
    assert len(fused) == 1
    f = fused[0]
    # every element of a[1:] read exactly once, merged or not
    assert sum(math.prod(r.extent) for r in f.layout.rows) == 39 * 18 * 16
    if not merge:
        assert f.ngroups == 1 and f.ntasks == 4 * 2 * 2  # source chunks x kept blocks
        assert sorted(r.extent[3] for r in f.layout.rows) == [9] * 4 + [10] * 12
    else:
        assert f.ntasks == 4  # one row per source T band
        assert sorted(r.extent[3] for r in f.layout.rows) == [9, 10, 10, 10]


@pytest.mark.parametrize("merge", [False, True])
def test_rechunk_then_mean_reads_the_source(built, dry, monkeypatch, merge):
    """rechunk rows -> columns then mean(axis=0): no copy launch; the mean's
    tasks are cut into per-source-chunk pieces (partials + grouped finish).
    With row merging (the default) the pieces of a column block -- the
    source's stacked row bands, one run of addresses -- are one row, and the
    column blocks -- consecutive columns of the same rows, writing consecutive
    output chunks -- one task of whole rows."""
    monkeypatch.setattr(Lw, "MERGE_ROWS", merge)
    spec = cubed.Spec(allowed_mem="288GB", executor=dry)
    random.seed(1)
    x = xp.astype(crandom.random((500, 500), chunks=(10, 500), spec=spec), xp.float32)
    arrays_to_plan(x).execute(executor=dry, array_names=[x.name])
    dry.launched.clear()
    m = xp.mean(x.rechunk((500, 40)), axis=0)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    assert not [l for l in dry.launched if isinstance(l, CopyLaunch)]
    fused = _fused(dry)
    if not merge:
        assert len(fused) == 1 and fused[0].ntasks == 50 * 13 and fused[0].ngroups == 13
    else:
        f = fused[0]
        assert len(fused) == 1 and f.ntasks == 1 and f.groups is None and f.max_kept == 500
        assert f.layout.rows[0].extent == [500, 500] and f.prog.mode & Lw.MODE_STREAM
    assert not fused[0].gathers


def test_requested_rechunk_is_kept(built, dry):
    spec = cubed.Spec(allowed_mem="288GB", executor=dry)
    x = cubed.from_array(np.ones((60, 50)), chunks=(10, 50), spec=spec)
    arrays_to_plan(x).execute(executor=dry, array_names=[x.name])
    dry.launched.clear()
    y = x.rechunk((60, 10))
    z = y * 2
    arrays_to_plan(y, z).execute(executor=dry, resume=True, array_names=[y.name, z.name])
    assert [l for l in dry.launched if isinstance(l, CopyLaunch)]


def test_full_reduction_is_lifted_to_the_stream_kernel(built, dry):
    """mean over all axes: the inner dims are walked as kept dims by the
    streaming kernel (partials), then folded per task + epilogue."""
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(2)
    a = crandom.random((400, 64, 64), chunks=(100, 64, 64), spec=spec)
    arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
    dry.launched.clear()
    m = xp.mean(a * 2)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    first = _fused(dry)[0]
    assert first.fold is not None and first.prog.mode & MODE_STREAM
    assert first.max_kept == 64 * 64 and first.max_red == 4 * 100  # inner dims lifted; chunks x rows reduced


def test_concat_is_one_copy_launch(built, dry):
    """A concat whose middle output chunk straddles three inputs is one box
    copy launch (no scratch gather, no per-input launches)."""
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    a = xp.asarray(np.ones((4, 5)), chunks=(3, 2), spec=spec)
    b = xp.asarray(np.ones((1, 5)), chunks=(3, 2), spec=spec)
    c = xp.asarray(np.ones((3, 5)), chunks=(3, 2), spec=spec)
    d = xp.concat([a, b, c], axis=0)
    arrays_to_plan(a, b, c).execute(executor=dry, array_names=[a.name, b.name, c.name])
    dry.launched.clear()
    arrays_to_plan(d).execute(executor=dry, resume=True, array_names=[d.name])
    copies = [l for l in dry.launched if isinstance(l, CopyLaunch)]
    assert len(dry.launched) == 1 and len(copies) == 1
    # middle row of output blocks: 3 column blocks x 3 source pieces
    assert copies[0].nboxes == 3 * 1 + 3 * 3 + 3 * 1


def test_stack_and_reshape_lower(built, dry):
    from cubed_amd.array_api.manipulation_functions import reshape_rechunk

    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    s = xp.stack([xp.ones((4, 6), chunks=(2, 3), spec=spec) for _ in range(3)], axis=1)
    assert s.shape == (4, 3, 6) and s.chunks == ((2, 2), (1, 1, 1), (3, 3))
    arrays_to_plan(s).execute(executor=dry, array_names=[s.name])
    r = xp.reshape(xp.arange(12, chunks=4, spec=spec), (3, 4))
    assert r.chunks == ((1, 1, 1), (4,))
    # dask's reshape_rechunk examples (vendor/dask/array/reshape.py)
    assert reshape_rechunk((6, 5, 4), (3, 2, 5, 4), ((3, 3), (5,), (2, 2))) == \
        (((2, 4), (5,), (2, 2)), ((1, 2), (2,), (5,), (2, 2)))
    assert reshape_rechunk((6, 5, 4), (30, 4), ((2, 2, 2), (2, 3), (4,))) == \
        (((1,) * 6, (5,), (4,)), ((5,) * 6, (4,)))
    with pytest.raises(NotImplementedError):
        reshape_rechunk((6, 5, 4), (4, 5, 6), ((6,), (5,), (4,)))


def test_int_indexed_copy_box_strides(built, dry):
    """a[1, 2:4]: the int-indexed leading dim has no destination dim; the
    box's destination stride is the kept dim's (regression: it took the int
    dim's 0 and wrote both elements to one place)."""
    spec = cubed.Spec(None, allowed_mem=100000, executor=dry)
    a = xp.asarray(np.arange(16).reshape(4, 4), chunks=(2, 2), spec=spec)
    b = a[1, 2:4]
    arrays_to_plan(b).execute(executor=dry, array_names=[b.name])
    copies = [l for l in dry.launched if isinstance(l, CopyLaunch)]
    assert copies and all(bx.dstride[-1] == 1 and bx.extent[-1] == 2 for bx in copies[-1].boxes)


def test_block_id_functions_trace_per_block(built, dry):
    """map_blocks with a ``block_id`` function (test_core.py:184-209):
    traced once per output block, blocks with equal programs share a launch
    (sum(block_id) = 0..4 over 5 blocks: 5 programs; with ``% 2``: 2)."""
    spec = cubed.Spec(None, allowed_mem=100000, executor=dry)
    a = xp.arange(10, dtype="int64", chunks=(2,), spec=spec)

    def f(block, block_id=None, c=0):
        return np.ones_like(block) * int(sum(block_id)) + c

    def g(block, block_id=None):
        return block * (block_id[0] % 2)

    for func, n in ((f, 5), (g, 2)):
        dry.launched.clear()
        b = cubed.map_blocks(func, a, dtype="int64")
        arrays_to_plan(b).execute(executor=dry, array_names=[b.name])
        assert len(_fused(dry)) == n + 1  # + the arange launch


def test_numpy_reduction_in_map_blocks_lowers(built, dry):
    spec = cubed.Spec(None, allowed_mem=100000, executor=dry)
    a = xp.asarray(np.arange(10), chunks=5, spec=spec)
    b = cubed.map_blocks(np.max, a, axis=0, keepdims=True, dtype=a.dtype, chunks=(1,))
    arrays_to_plan(b).execute(executor=dry, array_names=[b.name])
    assert _fused(dry)[-1].prog.nfields == 1


def test_copy_launch_picks_flat_path_for_packed_destinations(monkeypatch):
    # rechunk piece: 30 rows of 250 f64 out of 4000-wide source rows into a
    # packed (., 250) destination chunk -> CUBED_COPY_FLAT, work = 16-B words
    from cubed_amd.lowering import Box

    packed = Box(1 << 20, 1 << 30, [30, 250], [4000, 1], [250, 1])
    cl = CopyLaunch([packed], 8, "cpu")
    assert (cl.path, cl.lane, cl.work) == (nat.COPY_FLAT, 16, 30 * 250 * 8 // 16)
    # destination rows not packed (dst stride 400): per-row kernel
    strided = Box(1 << 20, 1 << 30, [30, 250], [4000, 1], [400, 1])
    assert CopyLaunch([strided], 8, "cpu").path == nat.COPY_ROWS
    import cubed_amd.lowering as Lw

    monkeypatch.setattr(Lw, "COPY_FLAT", False)
    assert CopyLaunch([packed], 8, "cpu").path == nat.COPY_ROWS


def test_matmul_and_k_sum_are_one_chained_gemm(built, dry):
    """xp.matmul's (i, k, j) chunk products and its sum over k lower to ONE
    cubed_gemm_chain launch: a task per output chunk whose segments are the
    (A_ik, B_kj) pairs in k order; the (M, nk, N) partials are never
    allocated (gemm_chains.py)."""
    from cubed_amd.lowering import GemmLaunch

    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(3)
    A = xp.astype(crandom.random((400, 1024), chunks=(100, 256), spec=spec), xp.bfloat16)
    B = xp.astype(crandom.random((1024, 312), chunks=(256, 104), spec=spec), xp.bfloat16)
    arrays_to_plan(A, B).execute(executor=dry, array_names=[A.name, B.name])
    dry.launched.clear()
    m = xp.matmul(A, B)
    assert m.dtype == xp.bfloat16
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    assert [type(l).__name__ for l in dry.launched] == ["GemmLaunch"]
    g = dry.launched[0]
    assert g.n == 4 * 3 and all(int(t["nseg"]) == 4 and int(t["ktot"]) == 1024 for t in g.tasks)
    assert (g.in_code, g.out_code) == (12, 12)
    assert g.kernel_path() == nat.GEMM_MFMA
    # segments of task (i, j) walk k in order over A's row i and B's column j
    t0 = g.tasks[0]
    seg = g.segs[int(t0["seg0"]):int(t0["seg0"]) + 4]
    assert [int(s["k"]) for s in seg] == [256] * 4
    assert len({int(s["a"]) for s in seg}) == 4 and len({int(s["b"]) for s in seg}) == 4


@pytest.mark.parametrize("dt", ["bf16", "f32"])
def test_matmul_of_a_regular_grid_is_packed(built, dry, dt, monkeypatch):
    """One GPU, a regular chunk grid of one product (chunks >= 256 wide):
    the GemmLaunch takes the packed-operand path with its workspace from
    the executor's scratch -- (3 + 3 panels) x k blocks (bf16 16 tiles of
    32 KiB, f32 64 steps of 16 KiB); when the workspace does not fit beside
    the plan's arrays it stays on the unpacked kernels."""
    import cubed_amd.runtime.executors.gpu as G

    def plan():
        spec = cubed.Spec(allowed_mem="2GB", executor=dry)
        a = cubed.from_array(np.ones((600, 1024), np.float32), chunks=(300, 256), spec=spec)
        b = cubed.from_array(np.ones((1024, 520), np.float32), chunks=(256, 264), spec=spec)
        if dt == "bf16":
            a, b = xp.astype(a, xp.bfloat16), xp.astype(b, xp.bfloat16)
        dry.launched.clear()
        arrays_to_plan(xp.matmul(a, b)).execute(executor=dry)
        return [l for l in dry.launched if type(l).__name__ == "GemmLaunch"][0]

    g = plan()
    assert g.grid == (2, 2) and g.packed is not None
    assert g.packed[1] == (3 + 3) * (16 * 32768 if dt == "bf16" else 64 * 16384) + 8 * 128  # + round counters
    # the executor's decision: a workspace only when it fits beside the plan
    dry.check_memory = True
    used = dry._resident_bytes + dry.owned_bytes()
    monkeypatch.setattr(G, "HBM_BYTES_PER_GPU", used + 4096)
    assert dry._gemm_workspace(8192) is None and dry._gemm_workspace(1024) is not None
    # and a launch given no workspace keeps the unpacked kernels
    g2 = type(g)(g.tasks, g.segs, g.in_code, g.out_code, "cpu", 0, grid=(2, 2), scratch=lambda n: None)
    assert g2.packed is None


def test_matmul_without_k_sum_fusion_is_per_chunk(built, dry):
    dry.fuse_gemm_sums = False
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    a = cubed.from_array(np.ones((64, 96), np.float32), chunks=(32, 32), spec=spec)
    b = cubed.from_array(np.ones((96, 64), np.float32), chunks=(32, 32), spec=spec)
    m = xp.matmul(a, b)
    arrays_to_plan(m).execute(executor=dry, array_names=[m.name])
    kinds = [type(l).__name__ for l in dry.launched]
    assert kinds[0] == "GemmLaunch" and "FusedLaunch" in kinds
    g = dry.launched[0]
    assert g.n == 2 * 3 * 2 and all(int(t["nseg"]) == 1 for t in g.tasks)


def test_raw_void_arrays_are_refused():
    """A 2-byte void array is not taken for bf16 data: only the
    tagged carrier enters; its tag survives numpy views and copies."""
    from cubed_amd import ir

    raw = np.zeros((4, 4), dtype="V2")
    with pytest.raises(TypeError, match="raw void"):
        cubed.from_array(raw, chunks=2)
    with pytest.raises(TypeError, match="raw void"):
        xp.asarray(raw)
    ok = ir.numpy_to_bf16(np.ones((4, 4), np.float32))
    assert ir.is_bf16(ok.dtype) and ok[1:].copy().dtype.metadata == {"cubed_bf16": True}
    assert cubed.from_array(ok, chunks=2).dtype == xp.bfloat16


def test_bfloat16_promotion():
    assert xp.result_type(xp.bfloat16, xp.bfloat16) == xp.bfloat16
    assert xp.result_type(xp.bfloat16, xp.float32) == xp.float32
    assert xp.result_type(xp.float64, xp.bfloat16) == xp.float64
    with pytest.raises(TypeError):
        xp.result_type(xp.bfloat16, xp.int32)


def test_five_input_map_splits_into_two_fused_launches(built, dry):
    """A chunk function reading 5 arrays (more than one fused program's 4
    leaves) runs as a part program into an HBM temporary + the remainder,
    instead of raising (cubed_amd/split.py)."""
    spec = cubed.Spec(allowed_mem=10**8, executor=dry)
    arrs = [cubed.from_array(np.full((64, 48), i + 1.0), chunks=(32, 24), spec=spec) for i in range(5)]
    m = cubed.map_blocks(lambda a, b, c, d, e: a * b + c * d + e, *arrs, dtype=np.float64)
    arrays_to_plan(m).execute(executor=dry, array_names=[m.name])
    fused = _fused(dry)
    assert len(fused) == 2
    assert fused[0].prog.nleaves <= 4 and fused[1].prog.nleaves <= 4
    # the 4 chunk tasks read and write consecutive slots: one streaming task
    assert fused[0].ntasks == fused[1].ntasks == 1


def test_split_program_keeps_every_input():
    from cubed_amd import ir
    from cubed_amd.lowering import collect_leaves, program_fits
    from cubed_amd.split import split_program

    f8 = np.dtype(np.float64)
    a = [ir.Arg(i, f8, (0, 1)) for i in range(6)]
    e = ir.apply_op("add", [ir.apply_op("multiply", [a[0], a[1]], f8),
                            ir.apply_op("multiply", [a[2], a[3]], f8)], f8)
    e = ir.apply_op("add", [e, ir.apply_op("subtract", [a[4], a[5]], f8)], f8)
    p = ir.ExprProgram(ndim=2, nargs=6, outputs=e, out_axes=(0, 1), name="six")
    assert not program_fits(p)
    parts, rest = split_program(p)
    assert parts and program_fits(rest) and all(program_fits(s) for s, _ in parts)
    used = {l.index for s, _ in parts for l in collect_leaves([s.outputs])}
    used |= {l.index for l in collect_leaves([rest.outputs]) if l.index < 6}
    assert used == set(range(6))


def test_complex_programs_lower_to_real_slabs(built, dry):
    """Complex arithmetic is rewritten into real expressions over the
    real/imaginary slabs (cubed_amd/complex.py): a complex product reads
    four part leaves and writes two part outputs; a complex sum is two
    reduced fields per level; a complex rechunk copies both slabs."""
    import numpy as np

    from cubed_amd.lowering import CopyLaunch

    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    Z = (np.arange(48.0) + 1j * np.arange(48.0)[::-1]).reshape(6, 8)
    z = cubed.from_array(Z, chunks=(3, 4), spec=spec)
    w = cubed.from_array(Z + 1, chunks=(3, 4), spec=spec)
    arrays_to_plan(z, w).execute(executor=dry, array_names=[z.name, w.name])
    dry.launched.clear()
    p = z * w
    arrays_to_plan(p).execute(executor=dry, resume=True, array_names=[p.name])
    f = _fused(dry)
    # 4 part leaves + 2 live parts in the VM's 6 registers: the leaf registers
    # are computed in place at their last use (Codegen.gen), one launch
    assert len(f) == 1 and f[0].prog.nleaves == 4 and f[0].prog.nouts == 2
    dry.launched.clear()
    s = xp.sum(z * w, axis=0)
    arrays_to_plan(s).execute(executor=dry, resume=True, array_names=[s.name])
    f = _fused(dry)
    assert any(l.prog.nfields == 2 for l in f) and all(l.prog.nfields in (0, 2) for l in f)
    dry.launched.clear()
    r = z.rechunk((6, 2))
    arrays_to_plan(r).execute(executor=dry, resume=True, array_names=[r.name])
    copies = [l for l in dry.launched if isinstance(l, CopyLaunch)]
    assert copies and sum(len(c.boxes) for c in copies) == 2 * 4 * 2  # 2 slabs x 4 targets x 2 pieces


def test_stream_groups_per_thread_choice(monkeypatch):
    """W (kept groups per thread of the streaming JIT kernel, mode bits):
    ~256 B of loads in flight per lane, and only when the W-wide grid fills
    the CUs without a time split (profiles/r02_stream_ab.log)."""
    from types import SimpleNamespace

    from cubed_amd import lowering as Lw

    def bits(vtype, nleaves, ntasks, max_kept):
        return Lw._stream_groups_mode(SimpleNamespace(vtype=vtype, nleaves=nleaves), ntasks, max_kept)

    # config 2 quad-means: 2 f32 leaves, 1 task of 720*1440 kept -> W = 4 (254
    # workgroups; the JIT kernel then keeps one row per lane in flight)
    assert bits(Lw.V_F32, 2, 1, 720 * 1440) == Lw.MODE_STREAM_W4
    # ... W = 1 where the wide grid would not fill the CUs unsplit
    assert bits(Lw.V_F32, 2, 1, 400000) == 0
    # config 1: 1 f64 leaf, 20000 kept -> the W = 2 grid (10 workgroups) would split: W = 1
    assert bits(Lw.V_F64, 1, 1, 20000) == 0
    # the elided rechunk+mean: 2500 source-chunk pieces of 1000 kept -> W = 1
    # (a W = 2 workgroup would cover 2048 elements: half its waves idle)
    assert bits(Lw.V_F32, 1, 2500, 1000) == 0
    # 4-leaf f64 programs (vorticity) already hold 256 B per lane -> W = 1
    assert bits(Lw.V_F64, 4, 100, 720000) == 0
    # a 1-leaf f32 mean over a wide kept dim -> W = 2
    assert bits(Lw.V_F32, 1, 1, 4 << 20) == Lw.MODE_STREAM_W2
    monkeypatch.setattr(Lw, "FORCE_STREAM_W", 4)
    assert bits(Lw.V_F64, 1, 1, 20000) == Lw.MODE_STREAM_W4


def test_two_random_streams_split(built, dry):
    """The reference's quad_means test under fuse_all_optimize_dag
    (test_core.py:540-570): one op draws from two unmaterialised random
    arrays; the VM carries one Philox key per task, so the executor
    materialises one stream into an HBM temporary (cubed_amd/split.py) and
    the per-chunk reduce reads it next to the other stream."""
    from cubed_amd.core.optimization import fuse_all_optimize_dag

    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(42)
    u = crandom.random((50, 1, 98, 192), chunks=(10, 1, -1, -1), spec=spec)
    v = crandom.random((50, 1, 98, 192), chunks=(10, 1, -1, -1), spec=spec)
    m = xp.mean(u * v, axis=0)
    dry.launched.clear()
    arrays_to_plan(m).execute(executor=dry, array_names=[m.name], optimize_function=fuse_all_optimize_dag)
    fused = _fused(dry)
    kinds = [list(l.prog.leaf_kind)[:l.prog.nleaves] for l in fused]
    philox = 1  # include/cubed_amd.h CUBED_LEAF_PHILOX
    # every launch draws from at most one random stream
    assert all(k.count(philox) <= 1 for k in kinds), kinds
    # a map launch whose only leaf is a random stream (the materialised part)
    assert any(l.prog.nfields == 0 and k == [philox] for l, k in zip(fused, kinds))


def test_complex_matmul_is_two_real_chains_per_output_chunk(built, dry):
    """complex64 matmul: one negation launch (-B.imag) and ONE chained GEMM
    launch whose tasks are (real, imag) pairs per output chunk, each a K loop
    over 2 nk segments on the f32 part slabs (gemm_chains.complex_chain_tables)."""
    from cubed_amd.lowering import GemmLaunch

    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    x = (np.arange(64 * 48).reshape(64, 48) % 7 + 1j).astype(np.complex64)
    a = cubed.from_array(x, chunks=(32, 16), spec=spec)
    b = cubed.from_array(x.T.copy(), chunks=(16, 32), spec=spec)
    arrays_to_plan(a, b).execute(executor=dry, array_names=[a.name, b.name])
    m = xp.matmul(a, b)
    dry.launched.clear()
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    fused = _fused(dry)
    gl = [l for l in dry.launched if isinstance(l, GemmLaunch)]
    assert len(gl) == 1 and len(fused) == 1
    assert fused[0].prog.nfields == 0  # the -B.imag map
    L = gl[0]
    assert L.in_code == L.out_code == 9  # f32 parts
    M = m.zarray
    assert L.n == 2 * M.nchunks
    A, B = a.zarray, b.zarray
    nk = A.numblocks[1]
    for t in range(M.nchunks):
        re, im = L.tasks[2 * t], L.tasks[2 * t + 1]
        assert re["nseg"] == im["nseg"] == 2 * nk and re["ktot"] == im["ktot"] == 2 * 48
        key = (t // M.numblocks[1], t % M.numblocks[1])
        assert re["c"] == M.chunk_addr(key, "real") and im["c"] == M.chunk_addr(key, "imag")
        sr = L.segs[re["seg0"]:re["seg0"] + 2 * nk]
        si = L.segs[im["seg0"]:im["seg0"] + 2 * nk]
        for k in range(nk):
            assert sr[k]["a"] == A.chunk_addr((key[0], k), "real") == si[k]["a"]
            assert sr[k]["b"] == B.chunk_addr((k, key[1]), "real")
            assert si[k]["b"] == B.chunk_addr((k, key[1]), "imag")
            assert sr[nk + k]["a"] == A.chunk_addr((key[0], k), "imag") == si[nk + k]["a"]
            assert si[nk + k]["b"] == B.chunk_addr((k, key[1]), "real")
            assert sr[nk + k]["b"] not in (B.chunk_addr((k, key[1]), "real"), B.chunk_addr((k, key[1]), "imag"))


@pytest.mark.parametrize("dtype", [np.float64, np.int64, np.uint64, np.float32])
def test_argmax_is_one_pair_reduction(built, dry, dtype):
    """argmax over every dtype: ONE fused reduce launch whose program holds
    the pair {v: argmax, i: pair_index} over x and the global index (Iota
    leaves), value accumulator f64 for floats, i64 for ints."""
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    a = cubed.from_array(np.arange(60, dtype=dtype).reshape(6, 10), chunks=(2, 10), spec=spec)
    arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
    r = xp.argmax(a, axis=0)
    dry.launched.clear()
    arrays_to_plan(r).execute(executor=dry, resume=True, array_names=[r.name])
    fused = _fused(dry)
    assert len(fused) == 1
    P = fused[0].prog
    assert P.nfields == 2
    assert (P.field_rop[0], P.field_rop[1]) == (ir.ROPS["argmax"], ir.ROPS["pair_index"])
    assert P.field_acc[1] == 1 and P.field_acc[0] == (0 if np.dtype(dtype).kind == "f" else 1)


def test_complex_prod_is_one_pair_reduction(built, dry):
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    z = cubed.from_array((np.arange(40) + 1j).astype(np.complex64).reshape(4, 10), chunks=(2, 5), spec=spec)
    arrays_to_plan(z).execute(executor=dry, array_names=[z.name])
    r = xp.prod(z, axis=0)
    dry.launched.clear()
    arrays_to_plan(r).execute(executor=dry, resume=True, array_names=[r.name])
    fused = _fused(dry)
    assert len(fused) == 1
    P = fused[0].prog
    assert P.nfields == 2
    assert (P.field_rop[0], P.field_rop[1]) == (ir.ROPS["cprod"], ir.ROPS["pair_imag"])
    assert P.field_acc[0] == P.field_acc[1] == 0


def test_var_is_one_fused_triple_pass(built, dry):
    """var(axis=0) over merge rounds: the per-chunk {n, mu, M2} program and
    every varc combine round compose into ONE streaming pass of the var
    triple (fields n / mu / M2 with the var / var_mean / var_m2 ops), the
    aggregate M2 / max(n - correction, 0) in its epilogue."""
    spec = cubed.Spec(allowed_mem=120_000, reserved_mem=0, executor=dry)
    a = cubed.from_array(np.zeros((400, 64)), chunks=(5, 64), spec=spec)
    arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
    dry.launched.clear()
    v = xp.var(a, axis=0, correction=1.0)
    plan = arrays_to_plan(v)
    nops = sum(1 for _, d in plan._finalize_dag().nodes(data=True) if d.get("op_name") == "blockwise")
    assert nops >= 3  # per-chunk + combine rounds + aggregate
    plan.execute(executor=dry, resume=True, array_names=[v.name])
    fused = _fused(dry)
    assert len(dry.launched) == 1 and len(fused) == 1
    P = fused[0].prog
    assert P.mode & MODE_STREAM
    assert P.nfields == 3
    assert [P.field_rop[i] for i in range(3)] == [ir.ROPS["var"], ir.ROPS["var_mean"], ir.ROPS["var_m2"]]
    assert [P.field_acc[i] for i in range(3)] == [1, 0, 0]
    assert P.nepi > 0


def test_var_triple_rejected_when_malformed(built):
    """The library's program check refuses a var lead without its partners."""
    P = nat.Program()
    P.vtype, P.ndim, P.nred, P.mode, P.nleaves, P.nfields, P.nouts = 1, 2, 1, 4, 1, 2, 1
    P.field_rop[0], P.field_acc[0] = ir.ROPS["var"], 1
    P.field_rop[1] = ir.ROPS["var_mean"]
    P.nepi = -1
    h = ctypes.c_void_p()
    rc = nat.lib().cubed_fused_compile(ctypes.byref(P), nat.INCLUDE_DIRS.encode(), ctypes.byref(h))
    assert rc != 0 and b"triple" in nat.lib().cubed_last_error()


def _balanced_runs(G, blocks, nru):
    """stream_body's balanced split (kernels.h), restated: per workgroup g the
    (column block c, rows [lo, hi), slot, contributors) segments of its run."""
    Ut = blocks * nru

    def owner(u):
        return ((u + 1) * G - 1) // Ut
    out = []
    for g in range(G):
        S0, S1 = g * Ut // G, (g + 1) * Ut // G
        u = S0
        while u < S1:
            c = u // nru
            lo = u - c * nru
            hi = min(S1 - c * nru, nru)
            first, last = owner(c * nru), owner((c + 1) * nru - 1)
            out.append((g, c, lo, hi, g - first, last - first + 1))
            u = c * nru + hi
    return out


@pytest.mark.parametrize("G,blocks,nru", [(256, 49, 7000), (256, 49, 50000), (256, 20, 20000),
                                          (256, 3, 1000), (248, 7, 777), (8, 1, 513)])
def test_balanced_split_partition(G, blocks, nru):
    """Every (block, row) unit is covered once; each block's contributors take
    slots 0..nsp-1 in row order, all agreeing on nsp, and nsp never exceeds
    the host's slot count (fused.hip plan_launch); runs differ by <= 1 row."""
    segs = _balanced_runs(G, blocks, nru)
    minlen = blocks * nru // G
    K = (nru + minlen - 1) // minlen + 1
    per_block = {}
    for g, c, lo, hi, slot, nsp in segs:
        assert 0 <= lo < hi <= nru and 0 <= slot < nsp <= K
        per_block.setdefault(c, []).append((lo, hi, slot, nsp))
    assert sorted(per_block) == list(range(blocks))
    for c, lst in per_block.items():
        lst.sort()
        assert lst[0][0] == 0 and lst[-1][1] == nru
        assert all(a[1] == b[0] for a, b in zip(lst, lst[1:]))
        assert [x[2] for x in lst] == list(range(len(lst)))
        assert {x[3] for x in lst} == {len(lst)}
    run = {}
    for g, c, lo, hi, *_ in segs:
        run[g] = run.get(g, 0) + hi - lo
    assert max(run.values()) - min(run.values()) <= 1 and len(run) == G


def test_even_streams_mark_uniform_tasks(built, dry, monkeypatch):
    """With the balanced split enabled (lowering.STREAM_EVEN, off by default)
    tasks of one reduced extent carry CUBED_MODE_STREAM_EVEN, and the library
    sizes a balanced split's workspace for its slot count."""
    from cubed_amd import _native as nat

    monkeypatch.setattr(Lw, "STREAM_EVEN", True)

    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(1)
    u = xp.astype(crandom.random((200, 16, 32), chunks=(10, 16, 32), spec=spec), xp.float32)
    v = xp.astype(crandom.random((200, 16, 32), chunks=(10, 16, 32), spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=dry, array_names=[u.name, v.name])
    dry.launched.clear()
    m = xp.mean(u * v, axis=0)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    (L,) = _fused(dry)
    P = L.prog
    assert P.mode & Lw.MODE_STREAM_EVEN
    # the per-rank share of config 3: one task, 50000 kept, 7000 rows
    P.mode &= ~(Lw.MODE_STREAM_W2 | Lw.MODE_STREAM_W4)
    lib = nat.lib()
    nf, ntasks, kept, red = P.nfields, 1, 50000, 7000
    bpt = -(-(-(-kept // 256) * 64) // 256)  # column blocks: 64 lanes x 4 elements x 4 waves
    even = lib.cubed_fused_workspace_bytes(P, ntasks, kept, red)
    P.mode &= ~Lw.MODE_STREAM_EVEN
    plain = lib.cubed_fused_workspace_bytes(P, ntasks, kept, red)
    minlen = ntasks * bpt * red // 256
    K = -(-red // minlen) + 1
    assert even == K * ntasks * kept * nf * 8 + ntasks * bpt * 4
    assert plain == 5 * ntasks * kept * nf * 8 + ntasks * bpt * 4  # uniform split: 49 x 5 workgroups


def test_partials_programs_compile_a_specialised_finish(built, dry):
    """A partials-mode program's JIT module carries the SoA finish
    (cubed_fused_finish_compiled) next to its main / split kernels; other
    programs do not."""
    import ctypes as C

    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(1)
    u = xp.astype(crandom.random((200, 16, 32), chunks=(10, 16, 32), spec=spec), xp.float32)
    v = xp.astype(crandom.random((200, 16, 32), chunks=(10, 16, 32), spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=dry, array_names=[u.name, v.name])
    dry.launched.clear()
    m = xp.mean(u * v, axis=0)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    (L,) = _fused(dry)
    assert "finish_soa_body" not in nat.program_source(L.handle)
    P = nat.Program()
    C.memmove(C.addressof(P), C.addressof(L.prog), C.sizeof(P))
    P.mode |= Lw.MODE_PARTIALS
    src = nat.program_source(nat.compile_program(P))
    # kernel names: <main>_partials_p<program digest>_finish / _fold
    assert re.search(r"_partials_p[0-9a-f]{8}_finish\(", src) and "cubed::finish_soa_body(JP," in src
    # ... and the lifted fold with the program's own epilogue
    assert re.search(r"_partials_p[0-9a-f]{8}_fold\(", src) and "cubed::fold_groups_split_body<true>(JP," in src
    assert {"cubed_fused_finish_compiled", "cubed_fold_groups_compiled"} <= set(nat.EXPORTED_SYMBOLS)
