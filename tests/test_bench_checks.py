"""bench.py's value checks at world size > 1 (CPU, gloo, no GPU).

The N-GPU bench must not publish numbers its checks never saw: every check
sums each rank's share of the expected values with one f64 all-reduce and
every rank compares the same numbers (bench.py ``sampled_check``).  Here two
gloo ranks hold block-cyclic shares of CPU-resident DeviceArrays; one test
is the honest run, the others corrupt ONE rank's input chunk or output chunk
and must make every rank's verdict fail and ``finish`` return exit status 1.
"""

import os
import sys
import types

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distutil import run_ranks  # noqa: E402


def _arrays(rank, world, corrupt):
    from cubed_amd.storage import DeviceArray

    rng = np.random.default_rng(3)
    u = rng.random((20, 6, 8)).astype(np.float32)
    v = rng.random((20, 6, 8)).astype(np.float32)
    m = np.mean((u * v).astype(np.float64), axis=0).astype(np.float32)
    if corrupt == "input" and rank == 1:
        u = u.copy()
        u[:, :, :] += 0.25  # rank 1's chunks of u differ from what the output was computed from
    if corrupt == "output" and rank == 1:
        m = m.copy() * 1.001
    arrs = []
    for val, chunks in ((u, (5, 3, 8)), (v, (5, 3, 8)), (m, (3, 8))):
        d = DeviceArray(val.shape, val.dtype, chunks, name=f"a{len(arrs)}")
        d.allocate("cpu", rank, world)
        d.from_numpy(val)
        arrs.append(types.SimpleNamespace(zarray=d, shape=d.shape))
    return arrs


def _rank(rank, world, corrupt):
    import bench

    bench.CHECKS.clear()
    U, V, M = _arrays(rank, world, corrupt)
    chk = bench.column_mean_check([U, V], M, lambda a, b: a * b, 1e-6, "test")
    bench.CHECKS.append(("quad-means sampled", chk))
    line = {}
    import io
    import contextlib

    with contextlib.redirect_stdout(io.StringIO()):
        rc = bench.finish(line, bench.CHECKS, rank, world)
    return chk["pass"], chk["world"], chk["entries"], rc, line["checks_failed"]


def test_two_ranks_pass_together():
    res = run_ranks(_rank, 2, None)
    for ok, world, entries, rc, failed in res:
        assert ok and world == 2 and entries == 48 and rc == 0 and failed == []


@pytest.mark.parametrize("corrupt", ["input", "output"])
def test_one_corrupt_rank_fails_every_rank(corrupt):
    res = run_ranks(_rank, 2, corrupt)
    for ok, world, entries, rc, failed in res:
        assert not ok and rc == 1 and failed == ["quad-means sampled"]


def _agree(rank, world):
    import bench

    # a failure seen on one rank only still fails the run on every rank
    checks = [("x", {"pass": rank != 1})]
    line = {}
    import io
    import contextlib

    with contextlib.redirect_stdout(io.StringIO()):
        rc = bench.finish(line, checks, rank, world)
    return rc, line["checks_failed"]


def test_failure_on_one_rank_is_agreed():
    (rc0, f0), (rc1, f1) = run_ranks(_agree, 2)
    assert rc0 == rc1 == 1
    assert f0 == ["(another rank)"] and f1 == ["x"]


def test_single_rank_check_without_process_group():
    import bench

    U, V, M = _arrays(0, 1, None)
    chk = bench.column_mean_check([U, V], M, lambda a, b: a * b, 1e-6, "test")
    assert chk["pass"] and chk["world"] == 1 and chk["max_rel_err"] < 1e-7
    M.zarray.slabs[None][:8].zero_()  # clobber one output element
    assert not bench.column_mean_check([U, V], M, lambda a, b: a * b, 1e-6, "test")["pass"]
