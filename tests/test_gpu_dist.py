"""Multi-GPU executor parity (``-m gpu``): the distributed executor run by 2
and 3 ranks that share one MI355X, against the oracle.

Each rank is a process with its own GpuDagExecutor(comm=...) over a gloo
process group (the Comm layer stages device buffers through the host for
gloo; with RCCL on a multi-GPU node the same launches run with device
buffers).  Every HIP launch of the distributed path runs for real: chunk
ownership (block-cyclic), whole-chunk fetches, rechunk pack/exchange/unpack,
partials-mode reductions with the cross-rank combine (sum -> reduce, max ->
all-gather + cubed_combine_partials) and cubed_fused_finish.  Results are
assembled on every rank (gather_distributed) and compared here with the same
tolerances as the single-GPU parity tests.
"""

import random

import numpy as np
import pytest

from distutil import run_ranks
from oracle import cubed_ref as R

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]


def _seeds(seed, n):
    random.seed(seed)
    return [random.getrandbits(128) for _ in range(n)]


def _cases(rank, world, zdir):
    import os

    import torch

    torch.cuda.set_device(0)
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.comm import Comm
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    ex = GpuDagExecutor("cuda:0", comm=Comm())
    assert ex.world == world
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)
    out = {}

    def note(what):
        print(f"[rank {rank}/{world}] {what}", flush=True)

    # quad-means (bench workload, small): chain in partials mode, SUM fields
    random.seed(4)
    shape, chunks = (60, 24, 40), (10, 24, 40)
    u = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    v = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=ex, array_names=[u.name, v.name])
    out["quad"] = xp.mean(u * v, axis=0).compute(resume=True)
    note("quad")

    # config 1 shape of work on a 4x4 chunk grid
    random.seed(7)
    a = crandom.random((200, 200), chunks=(50, 50), spec=spec)
    out["config1"] = xp.mean((a + 1) * 2, axis=0).compute()
    note("config1")

    # non-SUM fields: all-gather + combine in rank order
    x = np.random.default_rng(8).random((33, 500)) + 0.5
    b = cubed.from_array(x, chunks=(10, 128), spec=spec)
    out["max0"] = xp.max(b, axis=0).compute()
    out["min_all"] = xp.min(b).compute()
    out["sum1"] = xp.sum(b, axis=1).compute()
    note("sum1")

    # var / std: {n, mu, M2} triples are not an RCCL sum -- all-gathered and
    # folded in rank order with Chan's update
    out["var0"] = xp.var(b, axis=0).compute()
    out["std_all"] = xp.std(b, correction=1.0).compute()
    out["var_rechunk"] = xp.var(b.rechunk((33, 100)), axis=0).compute()
    note("var")

    # rechunk: rows -> columns, and misaligned
    y = np.random.default_rng(9).random((60, 50)).astype(np.float32)
    c = cubed.from_array(y, chunks=(10, 50), spec=spec)
    out["rechunk_cols"] = c.rechunk((60, 10)).compute()
    out["rechunk_mis"] = cubed.from_array(y, chunks=(7, 9), spec=spec).rechunk((13, 4)).compute()
    note("rechunk_mis")

    # elementwise across different chunk grids (whole-chunk fetches)
    p = cubed.from_array(y, chunks=(10, 50), spec=spec)
    q = cubed.from_array(y * 2, chunks=(20, 25), spec=spec)
    out["add_misaligned"] = (p + q).compute()
    note("add_misaligned")

    # matmul (operand panels fetched, k-reduction)
    r = np.random.default_rng(2)
    m1 = r.random((96, 80)).astype(np.float32)
    m2 = r.random((80, 64)).astype(np.float32)
    A = cubed.from_array(m1, chunks=(32, 40), spec=spec)
    B = cubed.from_array(m2, chunks=(40, 32), spec=spec)
    out["matmul"] = xp.matmul(A, B).compute()
    note("matmul")

    # index + broadcast + full mean (config 4 shape of work)
    rng = np.random.default_rng(11)
    AA, BB = rng.random((30, 9, 8)), rng.random((30, 9, 8))
    X, Y = rng.random((9, 8)), rng.random((9, 8))
    a3 = cubed.from_array(AA, chunks=(10, 3, 4), spec=spec)
    b3 = cubed.from_array(BB, chunks=(10, 3, 4), spec=spec)
    x3 = cubed.from_array(X, chunks=(3, 4), spec=spec)
    y3 = cubed.from_array(Y, chunks=(3, 4), spec=spec)
    out["vort"] = xp.mean(a3[1:] * x3 + b3[1:] * y3).compute()
    note("vort")

    # rechunk read through by a reduction: pieces run where their chunks live
    z = np.random.default_rng(15).random((60, 50))
    zc = cubed.from_array(z, chunks=(7, 50), spec=spec)
    out["rechunk_mean"] = xp.mean(zc.rechunk((60, 9)), axis=0).compute()
    out["rechunk_max"] = xp.max(zc.rechunk((60, 9)), axis=0).compute()
    note("rechunk_mean")

    # concat / stack / reshape: sources on other ranks are fetched
    c1 = cubed.from_array(np.arange(70.0).reshape(7, 10), chunks=(3, 4), spec=spec)
    c2 = cubed.from_array(np.arange(100.0, 120.0).reshape(2, 10), chunks=(3, 4), spec=spec)
    out["concat"] = xp.concat([c1, c2, c1], axis=0).compute()
    out["stack"] = xp.stack([c1, c1 * 2], axis=1).compute()
    out["reshape"] = xp.reshape(cubed.from_array(np.arange(24.0), chunks=4, spec=spec), (4, 6)).compute()
    note("manipulation")

    # independent pipelines in parallel (compute_arrays_in_parallel): local
    # kernel ops fork onto side streams, ops with collectives stay on the
    # executor's stream in one order on every rank
    pa = zc * 2 + 1
    pb = xp.astype(zc, xp.float32) - 3
    from cubed_amd.core.plan import arrays_to_plan as a2p
    forks = getattr(ex, "parallel_forks", 0)
    a2p(pa, pb).execute(executor=ex, array_names=[pa.name, pb.name], compute_arrays_in_parallel=True)
    pm, ps = xp.mean(pa, axis=0), xp.sum(pb, axis=1)
    a2p(pm, ps).execute(executor=ex, array_names=[pm.name, ps.name], resume=True,
                        compute_arrays_in_parallel=True)
    out["par_mean"] = pm.compute(resume=True)
    out["par_sum"] = ps.compute(resume=True)
    out["par_forked"] = np.array([getattr(ex, "parallel_forks", 0) > forks])
    note("parallel")

    # a chunk function over FIVE inputs (more than one fused program holds):
    # split into HBM temporaries that follow the block-cyclic ownership, then
    # reduced over several chunks per output block
    random.seed(21)
    five = [crandom.random((60, 40), chunks=(10, 20), spec=spec) for _ in range(5)]
    arrays_to_plan(*five).execute(executor=ex, array_names=[a.name for a in five])
    y5 = cubed.map_blocks(lambda a, b, c, d, e: a * b + c * d - e, *five, dtype=np.float64)
    out["five_map"] = y5.compute(resume=True)
    out["five_mean0"] = xp.mean(y5, axis=0).compute(resume=True)
    out["five_sum"] = xp.sum(y5).compute(resume=True)
    note("five")

    # matmul whose chunk grid divides by the world (6 x 6 at 2 and 3 ranks):
    # A's packed image assembled by point-to-point transfers (DistGemmLaunch)
    from cubed_amd.runtime.executors.dist import DistGemmLaunch

    for name, dt in (("bf16", xp.bfloat16), ("f32", xp.float32)):
        random.seed(31)
        A6 = xp.astype(crandom.random((700, 1200), chunks=(300, 200), spec=spec), dt)
        B6 = xp.astype(crandom.random((1200, 1584), chunks=(200, 264), spec=spec), dt)
        arrays_to_plan(A6, B6).execute(executor=ex, array_names=[A6.name, B6.name])
        out[f"mm6_{name}"] = xp.matmul(A6, B6).compute(resume=True)
        out[f"mm6_{name}_dist"] = np.array([any(isinstance(l, DistGemmLaunch)
                                               for v in ex._cache.values() for l in v[1])])
    note("mm6")

    # Zarr sink written by every rank (its own chunks), read back as a source
    zpath = os.path.join(zdir, "w.zarr")
    cubed.to_zarr(zc * 3, zpath)
    out["zarr"] = cubed.from_zarr(zpath, spec=spec).compute()
    note("zarr")
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_executor_matches_oracle(world, tmp_path):
    res = run_ranks(_cases, world, str(tmp_path), timeout=300)
    # every rank assembles the same results
    for r in range(1, world):
        for k in res[0]:
            assert np.array_equal(res[0][k], res[r][k], equal_nan=True), k
    got = res[0]

    s1, s2 = _seeds(4, 2)
    shape, chunks = (60, 24, 40), (10, 24, 40)
    U = R.random_array(shape, chunks, s1).astype(np.float32)
    V = R.random_array(shape, chunks, s2).astype(np.float32)
    exp = R.mean(U * V, chunks, 0, allowed_mem=2_000_000_000, reserved_mem=100_000_000)
    assert got["quad"].dtype == np.float32
    assert np.allclose(got["quad"], exp, rtol=1e-6, atol=0)

    (s,) = _seeds(7, 1)
    xa = R.random_array((200, 200), (50, 50), s)
    assert np.allclose(got["config1"], R.mean((xa + 1) * 2, (50, 50), 0, allowed_mem=2_000_000_000),
                       rtol=1e-12, atol=0)

    x = np.random.default_rng(8).random((33, 500)) + 0.5
    assert np.array_equal(got["max0"], x.max(axis=0))
    assert got["min_all"] == x.min()
    assert np.allclose(got["sum1"], x.sum(axis=1), rtol=1e-12, atol=0)
    assert np.allclose(got["var0"], x.var(axis=0), rtol=1e-12, atol=0)
    assert np.isclose(got["std_all"], x.std(ddof=1), rtol=1e-12, atol=0)
    assert np.allclose(got["var_rechunk"], x.var(axis=0), rtol=1e-12, atol=0)

    z = np.random.default_rng(15).random((60, 50))
    assert np.allclose(got["par_mean"], (z * 2 + 1).mean(axis=0), rtol=1e-12, atol=0)
    assert np.allclose(got["par_sum"], (z.astype(np.float32) - np.float32(3)).astype(np.float64).sum(axis=1),
                       rtol=1e-6, atol=0)
    assert got["par_forked"].all()

    y = np.random.default_rng(9).random((60, 50)).astype(np.float32)
    assert np.array_equal(got["rechunk_cols"], y)
    assert np.array_equal(got["rechunk_mis"], y)
    assert np.array_equal(got["add_misaligned"], y + y * 2)

    r = np.random.default_rng(2)
    m1 = r.random((96, 80)).astype(np.float32)
    m2 = r.random((80, 64)).astype(np.float32)
    assert np.allclose(got["matmul"], (m1.astype(np.float64) @ m2).astype(np.float32), rtol=1e-5, atol=1e-5)

    rng = np.random.default_rng(11)
    AA, BB = rng.random((30, 9, 8)), rng.random((30, 9, 8))
    X, Y = rng.random((9, 8)), rng.random((9, 8))
    assert np.isclose(got["vort"], np.mean(AA[1:] * X + BB[1:] * Y), rtol=1e-12, atol=0)

    z = np.random.default_rng(15).random((60, 50))
    assert np.allclose(got["rechunk_mean"], z.mean(axis=0), rtol=1e-12, atol=0)
    assert np.array_equal(got["rechunk_max"], z.max(axis=0))

    a70 = np.arange(70.0).reshape(7, 10)
    assert np.array_equal(got["concat"], np.concatenate([a70, np.arange(100.0, 120.0).reshape(2, 10), a70]))
    assert np.array_equal(got["stack"], np.stack([a70, a70 * 2], axis=1))
    assert np.array_equal(got["reshape"], np.arange(24.0).reshape(4, 6))
    assert np.array_equal(got["zarr"], z * 3)

    # the multi-GPU matmul is bit-identical to the 1-GPU chained GEMM
    import torch

    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    ex1 = GpuDagExecutor("cuda:0", comm=None)
    spec1 = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex1)
    for name, dt in (("bf16", xp.bfloat16), ("f32", xp.float32)):
        random.seed(31)
        A6 = xp.astype(crandom.random((700, 1200), chunks=(300, 200), spec=spec1), dt)
        B6 = xp.astype(crandom.random((1200, 1584), chunks=(200, 264), spec=spec1), dt)
        arrays_to_plan(A6, B6).execute(executor=ex1, array_names=[A6.name, B6.name])
        want = xp.matmul(A6, B6).compute(resume=True)
        assert got[f"mm6_{name}_dist"].all(), name
        assert np.array_equal(got[f"mm6_{name}"].view(np.uint32), want.view(np.uint32)), name
    torch.cuda.synchronize()

    F = [R.random_array((60, 40), (10, 20), sd) for sd in _seeds(21, 5)]
    y5 = F[0] * F[1] + F[2] * F[3] - F[4]
    assert np.array_equal(got["five_map"], y5)  # one IEEE op per node, stored at f64: bit-exact
    assert np.allclose(got["five_mean0"], y5.mean(axis=0), rtol=1e-12, atol=0)
    assert np.isclose(got["five_sum"], y5.sum(), rtol=1e-12, atol=0)
