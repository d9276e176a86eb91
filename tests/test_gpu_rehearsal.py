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

    for _, d in plan._finalize_dag().nodes(data=True):
        t = d.get("target")
        if isinstance(t, DeviceArray) and t is not keep:
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
