"""The oracle pinned against the golden vectors (CPU only).

The oracle (oracle/cubed_ref.py, oracle/philox.c) is the checker every GPU
parity test trusts, so it is itself checked here against fixtures produced by
numpy's own Philox and by the reference's own rechunk planner
(tests/golden/make_golden.py).
"""

import ctypes
import json
import os

import numpy as np
import pytest

from oracle import cubed_ref as R

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_root_seed_after_42():
    g = load("philox_blocks.json")
    assert R.root_seed_after(42) == int(g["root_seed_after_seed_42"], 16)


@pytest.mark.parametrize("case", load("philox_blocks.json")["cases"], ids=lambda c: f"{c['offset']}-{c['shape']}")
def test_random_block_golden(case):
    seed = int(case["root_seed"])
    got = R.random_block(seed, case["offset"], tuple(case["shape"]))
    if "values" in case:
        exp = np.array([float.fromhex(v) for v in case["values"]]).reshape(case["shape"])
        assert np.array_equal(got, exp)
    else:
        assert float.hex(float(got.reshape(-1)[0])) == case["first"]
        assert float.hex(float(got.reshape(-1)[-1])) == case["last"]
        assert float.hex(float(np.sum(got))) == case["sum"]


def _c_oracle():
    path = os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "liboracle.so")
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.oracle_philox_uniform.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_void_p]
    return lib


@pytest.mark.parametrize("case", load("philox_blocks.json")["cases"], ids=lambda c: f"{c['offset']}-{c['shape']}")
def test_c_philox_golden(built, case):
    lib = _c_oracle()
    key = int(case["root_seed"]) + case["offset"]
    n = int(np.prod(case["shape"]))
    out = np.empty(n)
    lib.oracle_philox_uniform(key & (2**64 - 1), (key >> 64) & (2**64 - 1), 0, n, out.ctypes.data)
    if "values" in case:
        assert [float.hex(float(v)) for v in out] == case["values"]
    else:
        assert float.hex(float(out[0])) == case["first"]
        assert float.hex(float(out[-1])) == case["last"]
        assert float.hex(float(np.sum(out))) == case["sum"]


def test_c_philox_random_access(built):
    """Any start offset (the GPU kernel generates elements independently)."""
    lib = _c_oracle()
    seed = R.root_seed_after(5)
    full = R.random_block(seed, 3, (1001,))
    for start in (0, 1, 3, 4, 5, 997):
        out = np.empty(1001 - start)
        lib.oracle_philox_uniform(((seed + 3) & (2**64 - 1)), (seed + 3) >> 64, start, len(out), out.ctypes.data)
        assert np.array_equal(out, full[start:])


@pytest.mark.parametrize("case", load("rechunk_plans.json"), ids=lambda c: f"{c['shape']}-{c['source_chunks']}-{c['max_mem']}")
def test_rechunk_plan_golden(case):
    args = (tuple(case["shape"]), tuple(case["source_chunks"]), tuple(case["target_chunks"]),
            case["itemsize"], case["max_mem"])
    if "error" in case:
        with pytest.raises(ValueError, match=r"exceeds max_mem"):
            R.rechunking_plan(*args)
        return
    r, i, w = R.rechunking_plan(*args)
    assert list(r) == case["read"] and list(i) == case["int"] and list(w) == case["write"]


@pytest.mark.parametrize("case", load("rechunk_plans.json"), ids=lambda c: f"{c['shape']}-{c['source_chunks']}-{c['max_mem']}")
def test_product_rechunk_plan_golden(case):
    """The product's own planner (cubed_amd/primitive/rechunk.py) agrees too."""
    from cubed_amd.primitive.rechunk import rechunking_plan

    args = (tuple(case["shape"]), tuple(case["source_chunks"]), tuple(case["target_chunks"]),
            case["itemsize"], case["max_mem"])
    if "error" in case:
        with pytest.raises(ValueError, match=r"exceeds max_mem"):
            rechunking_plan(*args)
        return
    r, i, w = rechunking_plan(*args)
    assert list(r) == case["read"] and list(i) == case["int"] and list(w) == case["write"]


def test_random_array_blocks_use_offsets():
    seed = R.root_seed_after(7)
    a = R.random_array((7, 5), (3, 2), seed)
    # block (1, 2) has C-order offset 1*3+2 = 5
    assert np.array_equal(a[3:6, 4:5], R.random_block(seed, 5, (3, 1)))


def test_mean_rounds_match_numpy():
    rng = np.random.default_rng(0)
    x = rng.random((100, 7, 9))
    got = R.mean(x, (1, 7, 9), 0, allowed_mem=20_000)  # forces several merge rounds
    assert np.allclose(got, x.mean(axis=0), rtol=1e-12, atol=0)
    f = x.astype(np.float32)
    got32 = R.mean(f, (10, 7, 9), 0, allowed_mem=2_000_000_000)
    assert got32.dtype == np.float32
    assert np.allclose(got32, f.astype(np.float64).mean(axis=0), rtol=1e-6, atol=0)


@pytest.mark.parametrize("axis", [0, 1, (0, 1), None])
@pytest.mark.parametrize("correction", [0.0, 1.0])
def test_var_restatement_matches_numpy(axis, correction):
    """The oracle's var (parity unpinned: no reference var) against numpy's
    f64 var over merge rounds (small allowed_mem) and one round; std = sqrt."""
    rng = np.random.default_rng(3)
    x = rng.random((90, 70)) * 5 + 1e3  # offset mean: cancellation-sensitive
    want = x.var(axis=axis, ddof=correction)
    for mem in (30_000, 2_000_000_000):
        got = R.var(x, (7, 9), axis, allowed_mem=mem, correction=correction)
        assert np.allclose(got, want, rtol=1e-12, atol=0)
    s = R.var(x, (7, 9), axis, allowed_mem=30_000, correction=correction, sqrt=True)
    assert np.allclose(s, x.std(axis=axis, ddof=correction), rtol=1e-12, atol=0)


def test_var_restatement_edge_cases():
    x = np.arange(12.0).reshape(3, 4)
    x[1, 2] = np.nan
    got = R.var(x, (2, 2), 0, allowed_mem=10**9)
    want = x.var(axis=0)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert np.allclose(got[~np.isnan(got)], want[~np.isnan(want)], rtol=1e-12)
    # reduced extent <= correction: numpy's rcount clamp gives inf / nan
    y = np.array([[2.0, 3.0]])
    with np.errstate(invalid="ignore", divide="ignore"):
        assert np.array_equal(R.var(y, (1, 1), 0, 10**9, correction=1.0), y.var(axis=0, ddof=1), equal_nan=True)
    f = x[[0, 2]].astype(np.float32)
    g = R.var(f, (1, 3), 0, allowed_mem=10**9)
    assert g.dtype == np.float32
    assert np.allclose(g, f.astype(np.float64).var(axis=0), rtol=1e-6)


def test_reference_cases_through_oracle():
    c = load("reference_cases.json")
    a = np.array(c["mean_axis_0"]["a"])
    assert np.array_equal(R.mean(a, tuple(c["mean_axis_0"]["chunks"]), 0, 10**9), c["mean_axis_0"]["expected"])
    x = np.array(c["nanmean_all"]["a"])
    got = R.nanmean(x, (2, 2), (0, 1), 10**9)
    assert np.isclose(got, c["nanmean_all"]["expected"], rtol=1e-15)
    y = np.ones((100, 10), dtype=np.uint8)
    s = R.chunked_reduce(y, (1, 10), 0, "sum", allowed_mem=1000)
    assert np.array_equal(s.reshape(-1), c["reduction_multiple_rounds_uint8"]["expected"])


def test_rechunk_values_unchanged():
    x = np.arange(60 * 50, dtype=np.float32).reshape(60, 50)
    out, plan, ntasks = R.rechunk(x, (10, 50), (60, 10), allowed_mem=100_000)
    assert np.array_equal(out, x)
    assert len(ntasks) in (1, 2)


def test_matmul_restatement_pinned_by_reference_case():
    """The reference's own matmul case (test_array_api.py: a 4x4 int array in
    2x2 chunks times itself) through the restated blockwise products +
    _sum_wo_cat rounds."""
    c = load("reference_cases.json")["matmul"]
    a = np.asarray(c["a"])
    got = R.matmul(a, a, tuple(c["chunks"]), tuple(c["chunks"]))
    assert np.array_equal(got, np.asarray(c["expected"]))


def test_matmul_restatement_rounds():
    """f32 operands with several k chunks: the result is the f32 sum of f32
    chunk products in k order (one combine round at 2 GB), equal to numpy's
    own chunked computation, and within the f32 bound of an f64 product."""
    r = np.random.default_rng(4)
    x = r.random((70, 90)).astype(np.float32)
    y = r.random((90, 50)).astype(np.float32)
    got = R.matmul(x, y, (32, 30), (30, 20))
    parts = [np.matmul(x[:, k:k + 30], y[k:k + 30]) for k in range(0, 90, 30)]
    exp = (parts[0] + parts[1]) + parts[2]
    assert got.dtype == np.float32 and np.array_equal(got, exp)
    ex64 = x.astype(np.float64) @ y.astype(np.float64)
    assert np.all(np.abs(got - ex64) <= 90 * 2.0 ** -24 * (np.abs(x).astype(np.float64) @ np.abs(y)))

