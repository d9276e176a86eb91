"""Rank rehearsal on one GPU (``-m gpu``): every rank of an 8-rank job run in
ONE process through ``runtime.comm.LoopbackComm`` -- each rank allocates
only its block-cyclic share, lowers its own pieces (DistPiecesLaunch) and
launches them for real; its collectives are local copies, and the reduce
inputs it would hand to RCCL are recorded.  Folding the 8 recorded partials
in rank order (the RCCL sum) and running the aggregate must give the
single-GPU result: the rehearsed launch list is the one the 8-GPU bench runs
(bench.py ``rechunk_mean_rehearsal``), so its timing rests on a correct path.

Reference: the reduction rounds this distributes, cubed/core/ops.py:849-892;
mean's combine/aggregate, cubed/array_api/statistical_functions.py:61-100.
"""

import random

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _plan(ex, shape, chunks, cols):
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    spec = cubed.Spec(allowed_mem="288GB", executor=ex)
    random.seed(2000)
    x = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
    m = xp.mean(x.rechunk((shape[0], cols)), axis=0)
    return x, m


@pytest.mark.parametrize("shape,cols", [((4000, 3000), 100),    # uniform groups: merged kept runs
                                        ((4050, 3050), 100)])   # ragged edge chunks: combine_groups
def test_eight_rehearsed_ranks_fold_to_one_gpu_result(gpu_executor, shape, cols):
    import torch

    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.comm import LoopbackComm
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor
    from cubed_amd.runtime.executors.dist import DistPiecesLaunch

    chunks = (100, shape[1])
    x1, m1 = _plan(gpu_executor, shape, chunks, cols)
    want = m1.compute(resume=True)
    host = x1.compute(resume=True).astype(np.float64)
    np.testing.assert_allclose(want, host.mean(axis=0).astype(np.float32), rtol=1e-6)

    world = 8
    scat, direct = [], []
    for r in range(world):
        comm = LoopbackComm(r, world, record=True)
        ex = GpuDagExecutor("cuda:0", comm=comm)
        x, m = _plan(ex, shape, chunks, cols)
        assert x.zarray.world == world and x.zarray.rank == r
        arrays_to_plan(m).execute(executor=ex, array_names=[m.name], resume=True)
        torch.cuda.synchronize()
        launches = [l for v in ex._cache.values() for l in v[1] if isinstance(l, DistPiecesLaunch)]
        assert len(launches) == 1
        dp = launches[0]
        direct.append(dp.soa_direct)
        # several owners of the output blocks: ONE reduce-scatter of the f64
        # totals in owner-major order; the counts never cross the ranks
        kinds = [kind for kind, _ in comm.records]
        assert kinds == ["reduce_scatter_sum"], kinds
        assert dp.scatter is not None and dp.scatter.mine == [g for g in range(dp.ngroups) if g % world == r]
        scat.append((dp.scatter, comm.records[0][1]))
        del x, m, ex
    # uniform groups stream as merged kept runs (no combine_groups pass)
    assert all(direct) == (shape[0] % chunks[0] == 0 and shape[1] % cols == 0)
    total = scat[0][1].clone()
    for r in range(1, world):  # the RCCL sum, in rank order
        total += scat[r][1]
    ngroups = -(-shape[1] // cols)
    tot = scat[0][0].unpermute(total)[0].cpu().numpy()
    assert tot.shape == (ngroups, cols)
    got = (tot / shape[0]).reshape(-1)[:shape[1]].astype(np.float32)
    np.testing.assert_allclose(got, want, rtol=1e-6)
    # every rank finished exactly its own blocks: their counts are the global ones
    for sc, _ in scat:
        cnt = sc.fin.view(torch.int64)[:sc.L * sc.mko].view(sc.L, sc.mko)[:len(sc.mine), 0]
        assert (cnt == shape[0]).all()


def _targets_unwritten(plan, keep):
    from cubed_amd.storage import DeviceArray

    keep_ids = keep if isinstance(keep, set) else {id(keep)}
    for _, d in plan._finalize_dag().nodes(data=True):
        t = d.get("target")
        if isinstance(t, DeviceArray) and id(t) not in keep_ids:
            t.written = False


@pytest.mark.parametrize("shape,rows,cols", [((4000, 3000), 100, 100),    # config 3's shape, reduced
                                             ((4050, 3050), 100, 90),     # ragged edge chunks both ways
                                             ((1200, 1000), 150, 1000)])  # one target chunk per rank row
def test_eight_rehearsed_ranks_rechunk_bit_exact(gpu_executor, shape, rows, cols):
    """Config 3's MATERIALISED rechunk (rows -> columns) on 8 rehearsed
    ranks: each rank packs, copies its local pieces and writes the pieces it
    receives into its target slots (RechunkLaunch); the LoopbackMesh hands
    every receive the bytes its peer sent, matched by pair and order.  The
    target assembled from the 8 ranks' slots equals the 1-GPU rechunk bit
    for bit.  Reference: cubed/primitive/rechunk.py:23-98,187-192."""
    import torch

    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.comm import LoopbackComm, LoopbackMesh
    from cubed_amd.runtime.executors.dist import RechunkLaunch
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    def build(ex):
        spec = cubed.Spec(allowed_mem="288GB", executor=ex)
        random.seed(2002)
        x = xp.astype(crandom.random(shape, chunks=(rows, shape[1]), spec=spec), xp.float32)
        arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
        y = x.rechunk((shape[0], cols))
        return x, y, arrays_to_plan(y)

    x1, y1, _ = build(gpu_executor)
    want = y1.compute()
    assert np.array_equal(want.view(np.uint32), x1.compute().view(np.uint32))

    world = 8
    mesh = LoopbackMesh(world)
    ranks = []
    for r in range(world):
        ex = GpuDagExecutor("cuda:0", comm=LoopbackComm(r, world, mesh=mesh))
        x, y, plan = build(ex)
        plan.execute(executor=ex, array_names=[y.name], resume=True)  # record phase
        ranks.append((ex, x, y, plan))
    torch.cuda.synchronize()
    mesh.phase = "replay"
    planned = 0
    for ex, x, y, plan in ranks:
        _targets_unwritten(plan, x.zarray)
        plan.execute(executor=ex, array_names=[y.name], resume=True)
        rl = [l for v in ex._cache.values() for l in v[1] if isinstance(l, RechunkLaunch)]
        assert len(rl) == 1
        planned += rl[0].plan.send_bytes
        assert ex.comm.recv_bytes == 2 * rl[0].plan.recv_bytes  # record + replay
    torch.cuda.synchronize()
    assert planned == sum(n for _, _, n in mesh.log)
    Y = ranks[0][2].zarray
    got = np.empty(shape, np.float32)
    import itertools

    for tc in itertools.product(*[range(n) for n in Y.numblocks]):
        owner = Y.chunk_offset(tc) % world
        Yo = ranks[owner][2].zarray
        assert Yo.rank == owner
        st, ext = Yo.chunk_start(tc), Yo.chunk_extent(tc)
        got[st[0]:st[0] + ext[0], st[1]:st[1] + ext[1]] = Yo.read_chunk(tc)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def _mesh_rehearsal(world, build, passes=2):
    """Run ``build(ex) -> (inputs, out, plan)`` on every rank of a rehearsed
    ``world`` whose collectives and transfers go through ONE LoopbackMesh:
    a record pass, then ``passes`` replay passes (each combines every rank's
    inputs of the same collective).  Returns the ranks' (executor, out)."""
    import torch

    from cubed_amd.runtime.comm import LoopbackComm, LoopbackMesh
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    mesh = LoopbackMesh(world)
    ranks = []
    for r in range(world):
        ex = GpuDagExecutor("cuda:0", comm=LoopbackComm(r, world, mesh=mesh))
        ins, out, plan = build(ex)
        plan.execute(executor=ex, array_names=[out.name], resume=True)
        ranks.append((ex, ins, out, plan))
    torch.cuda.synchronize()
    mesh.phase = "replay"
    for _ in range(passes):
        for ex, ins, out, plan in ranks:
            _targets_unwritten(plan, set(id(a.zarray) for a in ins))
            plan.execute(executor=ex, array_names=[out.name], resume=True)
        torch.cuda.synchronize()
    return ranks


def _assemble(ranks, world):
    """The array each rank holds a block-cyclic share of, from the owners."""
    import itertools

    Y = ranks[0][2].zarray
    got = np.empty(Y.shape, Y.dtype)
    for tc in itertools.product(*[range(n) for n in Y.numblocks]):
        owner = Y.chunk_offset(tc) % world
        Yo = ranks[owner][2].zarray
        st, ext = Yo.chunk_start(tc), Yo.chunk_extent(tc)
        got[tuple(slice(s, s + e) for s, e in zip(st, ext))] = Yo.read_chunk(tc)
    return got


@pytest.mark.parametrize("world", [4, 8])
def test_rehearsed_mean_when_pieces_cut_kept_dims(gpu_executor, world):
    """mean(x.rechunk(cols), axis=0) whose source chunks (40, 70) cut every
    100-wide target column block: each output block has several groups.  All
    ranks rehearsed through one mesh (reduce-scatter combining every rank's
    partials), the output assembled from its owners' slots equals the 1-GPU
    result (rtol 1e-6, the f32 output of f64 sums in another association).
    Reference: cubed/core/ops.py:849-892, primitive/rechunk.py:23-98."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.executors.dist import DistPiecesLaunch

    shape = (800, 1000)

    def build(ex):
        spec = cubed.Spec(allowed_mem="288GB", executor=ex)
        random.seed(2010)
        x = xp.astype(crandom.random(shape, chunks=(40, 70), spec=spec), xp.float32)
        arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
        m = xp.mean(x.rechunk((shape[0], 100)), axis=0)
        return [x], m, arrays_to_plan(m)

    _, m1, p1 = build(gpu_executor)
    want = m1.compute(resume=True)
    ranks = _mesh_rehearsal(world, build)
    for ex, _, _, _ in ranks:
        dps = [l for v in ex._cache.values() for l in v[1] if isinstance(l, DistPiecesLaunch)]
        assert len(dps) == 1 and dps[0].ngroups > 10 and dps[0].scatter is not None
    got = _assemble(ranks, world)
    np.testing.assert_allclose(got, want, rtol=1e-6)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_rehearsed_matmul_bit_identical_to_one_gpu(gpu_executor, world, dtype):
    """Config 5's matmul, reduced (8 x 8 chunk grid, ragged last chunk row and
    column, 200-wide k chunks so every chunk edge falls inside a k block):
    all ranks rehearsed through one mesh -- halo transfers, each rank's A
    blocks packed into the k-major image and sent to every peer, B packed
    locally, the packed GEMM over the rank's C columns.  C assembled from
    its owners equals the 1-GPU result bit for bit: the image is the 1-GPU
    packed A, so every element is the same f32 chain over K.
    Reference: cubed/array_api/linear_algebra_functions.py:35-78."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.executors.dist import DistGemmLaunch

    dt = xp.bfloat16 if dtype == "bfloat16" else xp.float32

    def build(ex):
        spec = cubed.Spec(allowed_mem="288GB", executor=ex)
        random.seed(2020)
        A = xp.astype(crandom.random((700, 1600), chunks=(300, 200), spec=spec), dt)
        B = xp.astype(crandom.random((1600, 2048), chunks=(200, 264), spec=spec), dt)
        arrays_to_plan(A, B).execute(executor=ex, array_names=[A.name, B.name])
        C = xp.matmul(A, B)
        return [A, B], C, arrays_to_plan(C)

    _, C1, p1 = build(gpu_executor)
    p1.execute(executor=gpu_executor, array_names=[C1.name], resume=True)
    want = C1.compute(resume=True)
    ranks = _mesh_rehearsal(world, build)
    for ex, _, _, _ in ranks:
        assert [l for v in ex._cache.values() for l in v[1] if isinstance(l, DistGemmLaunch)]
    got = _assemble(ranks, world)
    if dtype == "bfloat16":  # compute() widens bf16 exactly to f32
        got = (got.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
    assert got.dtype == want.dtype == np.float32
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
