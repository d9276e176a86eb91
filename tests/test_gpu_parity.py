"""Parity of the HIP path with the oracle (needs an MI355X; ``-m gpu``).

Every case builds a plan through the drop-in API, runs it on the
GpuDagExecutor (libcubed_amd.so kernels through the C ABI) and compares with
the oracle (oracle/cubed_ref.py) on the same seeded inputs.  Tolerances
(DESIGN.md "Parity"): bit-exact for Philox, copies/rechunk, integer work and
outer-axis f32/f64 means (sequential accumulation in numpy's order); rtol
1e-12 for f64 reductions whose summation order differs from numpy's
pairwise inner-axis sums; rtol 1e-6 for f32 results of such reductions.
"""

import json
import os
import random

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
import cubed_amd.lowering as L
from cubed_amd.core.ops import merge_chunks, partial_reduce, reduction
from cubed_amd.core.plan import arrays_to_plan
from oracle import cubed_ref as R

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ex(gpu_executor):
    return gpu_executor


def mkspec(ex, mem="2GB", reserved="100MB"):
    return cubed.Spec(allowed_mem=mem, reserved_mem=reserved, executor=ex)


def seeds(seed, n):
    random.seed(seed)
    return [random.getrandbits(128) for _ in range(n)]


# ----------------------------------------------------------------- Philox (H1)


@pytest.mark.parametrize("shape, chunks", [((100, 60), (30, 25)), ((7,), (3,)), ((5, 6, 7), (2, 3, 4)), ((1001,), (1001,))])
def test_random_bit_exact(ex, shape, chunks):
    spec = mkspec(ex)
    random.seed(42)
    a = crandom.random(shape, chunks=chunks, spec=spec)
    (s,) = seeds(42, 1)
    assert np.array_equal(a.compute(), R.random_array(shape, chunks, s))


def test_random_golden_first_values(ex):
    g = json.load(open(os.path.join(GOLDEN, "philox_blocks.json")))
    spec = mkspec(ex)
    random.seed(42)
    a = crandom.random((8,), chunks=(8,), spec=spec).compute()
    exp = [float.fromhex(v) for v in g["cases"][0]["values"]]
    assert [float(x) for x in a] == exp


# ------------------------------------------------------- elementwise (H2, H12)


def test_reference_cases(ex):
    c = json.load(open(os.path.join(GOLDEN, "reference_cases.json")))
    spec = mkspec(ex, mem=100000, reserved=0)
    a = xp.asarray(c["add"]["a"], chunks=(2, 2), spec=spec)
    b = xp.asarray(c["add"]["b"], chunks=(2, 2), spec=spec)
    assert np.array_equal(xp.add(a, b).compute(), c["add"]["expected"])
    m = xp.asarray(c["mean_axis_0"]["a"], chunks=(2, 2), spec=spec)
    assert np.array_equal(xp.mean(m, axis=0).compute(), c["mean_axis_0"]["expected"])
    s = xp.asarray(c["sum"]["a"], chunks=(2, 2), spec=spec)
    assert xp.sum(s).compute() == c["sum"]["expected"]
    assert np.array_equal(xp.sum(s, axis=0).compute(), c["sum_axis_0"]["expected"])
    mm = xp.asarray(c["matmul"]["a"], chunks=(2, 2), spec=spec)
    assert np.array_equal(xp.matmul(mm, mm).compute(), c["matmul"]["expected"])
    assert np.array_equal(xp.astype(s, xp.int32).compute(), c["astype_int32"]["expected"])
    assert np.array_equal(xp.negative(s).compute(), c["negative"]["expected"])
    n = xp.asarray(c["nanmean_all"]["a"], chunks=(2, 2), spec=spec)
    assert np.isclose(cubed.nanmean(n).compute(), c["nanmean_all"]["expected"], rtol=1e-15)
    ns = xp.asarray(c["nansum_axis_0"]["a"], chunks=(2, 2), spec=spec)
    assert np.array_equal(cubed.nansum(ns, axis=0).compute(), c["nansum_axis_0"]["expected"])


def test_reduction_multiple_rounds_uint8(ex):
    spec = cubed.Spec(allowed_mem=1000, executor=ex)
    a = xp.ones((100, 10), dtype=np.uint8, chunks=(1, 10), spec=spec)
    b = xp.sum(a, axis=0, dtype=np.uint8)
    assert np.array_equal(b.compute(), np.ones((100, 10)).sum(axis=0))


def test_partial_reduce(ex):
    spec = mkspec(ex, mem=100000, reserved=0)
    a = xp.asarray(np.arange(242).reshape((11, 22)), chunks=(3, 4), spec=spec)
    b = partial_reduce(a, np.sum, split_every={0: 8})
    assert np.array_equal(b.compute(), np.arange(242).reshape((11, 22)).sum(axis=0, keepdims=True))


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.int64, np.int32])
def test_elementwise_chain(ex, dtype):
    rng = np.random.default_rng(5)
    x = (rng.random((37, 53)) * 100).astype(dtype)
    y = (rng.random((37, 53)) * 100 + 1).astype(dtype)
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=(10, 16), spec=spec)
    b = cubed.from_array(y, chunks=(10, 16), spec=spec)
    got = ((a + 1) * 2 - b).compute()
    exp = (x + dtype(1)) * dtype(2) - y
    assert got.dtype == exp.dtype
    assert np.array_equal(got, exp)


def test_where_and_comparisons(ex):
    rng = np.random.default_rng(6)
    x = rng.random((40, 30))
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=(16, 16), spec=spec)
    got = xp.where(a > 0.5, a, -a).compute()
    assert np.array_equal(got, np.where(x > 0.5, x, -x))


# ---------------------------------------------------------- reductions (H8-H11)


@pytest.mark.parametrize("T, chunk_t, mem", [(50, 10, "2GB"), (100, 10, "2GB"), (100, 1, 20_000_000), (37, 5, "2GB")])
def test_quad_means_f64(ex, T, chunk_t, mem):
    spec = mkspec(ex, mem=mem, reserved=0)
    random.seed(3)
    shape, chunks = (T, 1, 37, 40), (chunk_t, 1, -1, -1)
    u = crandom.random(shape, chunks=chunks, spec=spec)
    v = crandom.random(shape, chunks=chunks, spec=spec)
    s1, s2 = seeds(3, 2)
    U = R.random_array(shape, chunks, s1)
    V = R.random_array(shape, chunks, s2)
    got = xp.mean(u * v, axis=0).compute()
    exp = R.mean(U * V, (chunk_t, 1, 37, 40), 0, allowed_mem=spec.allowed_mem)
    assert np.allclose(got, exp, rtol=1e-12, atol=0)


@pytest.mark.parametrize("T", [40, 103, 1000])
def test_quad_means_f32_stream(ex, T):
    """The bench workload's kernel (streaming fast path, one fused pass over
    the time axis) vs the oracle's chunked rounds: f64 accumulation, result
    rounded to f32, rtol 1e-6."""
    spec = mkspec(ex)
    random.seed(4)
    shape, chunks = (T, 72, 144), (10, 72, 144)
    u = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    v = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=ex, array_names=[u.name, v.name])
    s1, s2 = seeds(4, 2)
    U = R.random_array(shape, chunks, s1).astype(np.float32)
    V = R.random_array(shape, chunks, s2).astype(np.float32)
    m = xp.mean(u * v, axis=0)
    got = m.compute(resume=True)
    exp = R.mean(U * V, chunks, 0, allowed_mem=2_000_000_000, reserved_mem=100_000_000)
    assert got.dtype == np.float32
    assert np.allclose(got, exp, rtol=1e-6, atol=0)


def _fused_launches(e):
    return [l for lst in e._cache.values() for l in lst[1] if isinstance(l, L.FusedLaunch)]


@pytest.mark.parametrize("w", [1, 2, 4])
def test_stream_groups_per_thread(gpu_executor, monkeypatch, w):
    """The streaming kernel with W kept groups per thread (forced by
    CUBED_AMD_STREAM_W; by default only grids that fill the CUs unsplit take
    W > 1): f32 quad-means over 72 x 144 kept elements (40.5 wave blocks of
    256: a partial last block) and an f64 map-reduce over 1000 kept elements
    (3 lane-interleaved 256-element runs + a 232-element run on the dk = 2
    fallback), both against the oracle."""
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    monkeypatch.setattr(L, "FORCE_STREAM_W", w)
    e = GpuDagExecutor("cuda:0")
    spec = mkspec(e)
    random.seed(4)
    shape, chunks = (103, 72, 144), (10, 72, 144)
    u = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    v = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=e, array_names=[u.name, v.name])
    s1, s2 = seeds(4, 2)
    U = R.random_array(shape, chunks, s1).astype(np.float32)
    V = R.random_array(shape, chunks, s2).astype(np.float32)
    seen = []
    keep = [xp.mean(u * v, axis=0)]  # alive: the cache entries die with their plans
    got = keep[-1].compute(resume=True)
    seen += _fused_launches(e)
    exp = R.mean(U * V, chunks, 0, allowed_mem=2_000_000_000, reserved_mem=100_000_000)
    assert np.allclose(got, exp, rtol=1e-6, atol=0)

    random.seed(8)
    a = crandom.random((200, 1000), chunks=(50, 1000), spec=spec)
    arrays_to_plan(a).execute(executor=e, array_names=[a.name])  # an array leaf, not a Philox leaf
    (s,) = seeds(8, 1)
    x = R.random_array((200, 1000), (50, 1000), s)
    keep.append(xp.mean((a + 1) * 2, axis=0))
    got = keep[-1].compute(resume=True)
    seen += _fused_launches(e)
    exp = R.mean((x + 1) * 2, (50, 1000), 0, allowed_mem=2_000_000_000)
    assert np.allclose(got, exp, rtol=1e-12, atol=0)
    # the streaming map branch (no reduction): one IEEE op per element, bit-exact
    keep.append((a + 1) * 2)
    np.testing.assert_array_equal(keep[-1].compute(resume=True), (x + 1) * 2)
    seen += _fused_launches(e)
    # a full reduction runs "lifted" in partials mode (per-element SoA
    # partials, then a fold): the W-group partial writes
    random.seed(9)
    b = crandom.random((200, 20000), chunks=(50, 20000), spec=spec)
    arrays_to_plan(b).execute(executor=e, array_names=[b.name])
    (sb,) = seeds(9, 1)
    y = R.random_array((200, 20000), (50, 20000), sb)
    keep.append(xp.mean(b * 3))
    got = keep[-1].compute(resume=True)
    assert np.allclose(got, np.mean(y * 3), rtol=1e-12, atol=0)
    seen += _fused_launches(e)
    assert any(l.prog.mode & L.MODE_PARTIALS and l.prog.mode & L.MODE_STREAM for l in seen)

    bits = {1: 0, 2: L.MODE_STREAM_W2, 4: L.MODE_STREAM_W4}[int(w)]
    streams = list({id(l): l for l in seen if l.prog.mode & L.MODE_STREAM}.values())
    assert len(streams) >= 2
    assert all(l.prog.mode & (L.MODE_STREAM_W2 | L.MODE_STREAM_W4) == bits for l in streams)


def test_config1_small(ex):
    spec = mkspec(ex)
    random.seed(7)
    a = crandom.random((200, 200), chunks=(50, 50), spec=spec)
    (s,) = seeds(7, 1)
    x = R.random_array((200, 200), (50, 50), s)
    got = xp.mean((a + 1) * 2, axis=0).compute()
    exp = R.mean((x + 1) * 2, (50, 50), 0, allowed_mem=2_000_000_000)
    assert np.allclose(got, exp, rtol=1e-12, atol=0)


@pytest.mark.parametrize("even", [True, False])
def test_balanced_split_streams(gpu_executor, monkeypatch, even):
    """Split streaming reductions with the balanced split (every task the same
    reduced extent: CUBED_MODE_STREAM_EVEN, equal row runs per workgroup that
    cross column blocks) and with the uniform split (bit cleared): int64 sums
    bit-exact, f64 means rtol 1e-12 and f32 means rtol 1e-6 against numpy,
    ragged last column chunk included."""
    from cubed_amd import _native as nat
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    monkeypatch.setattr(L, "STREAM_EVEN", even)
    e = GpuDagExecutor("cuda:0")
    spec = mkspec(e)
    rng = np.random.default_rng(11)
    xi = rng.integers(-2**40, 2**40, size=(1500, 19000), dtype=np.int64)
    xf = rng.random((1500, 19000)) + 7.0
    keep = []
    a = cubed.from_array(xi, chunks=(500, 5000), spec=spec)
    keep.append(xp.sum(a, axis=0))
    np.testing.assert_array_equal(keep[-1].compute(), xi.sum(axis=0))
    b = cubed.from_array(xf, chunks=(500, 5000), spec=spec)
    keep.append(xp.mean(b, axis=0))
    np.testing.assert_allclose(keep[-1].compute(), xf.mean(axis=0), rtol=1e-12, atol=0)
    c = xp.astype(b, xp.float32)
    keep.append(xp.mean(c, axis=0))
    want32 = xf.astype(np.float32).astype(np.float64).mean(axis=0).astype(np.float32)
    np.testing.assert_allclose(keep[-1].compute(), want32, rtol=1e-6, atol=0)
    streams = [l for l in _fused_launches(e) if l.prog.mode & L.MODE_STREAM and l.prog.nfields]
    assert streams
    lib = nat.lib()
    for l in streams:
        assert bool(l.prog.mode & 256) == even
        # the launch split (a workspace) -- balanced or not
        assert lib.cubed_fused_workspace_bytes(l.prog, l.ntasks, l.max_kept, l.max_red) > 0


def test_mean_of_unmaterialised_random(ex):
    """random -> elementwise -> mean with nothing materialised: the Philox
    map is fused into the reduction's first pass (one stream key per
    chunk), the chain over chunks must not reuse one key."""
    spec = mkspec(ex)
    random.seed(17)
    a = crandom.random((200, 120), chunks=(50, 40), spec=spec)
    (s,) = seeds(17, 1)
    x = R.random_array((200, 120), (50, 40), s)
    got = xp.mean(a * 3 - 1, axis=0).compute()
    exp = R.mean(x * 3 - 1, (50, 40), 0, allowed_mem=2_000_000_000)
    assert np.allclose(got, exp, rtol=1e-12, atol=0)
    got1 = xp.sum(a, axis=1).compute()
    assert np.allclose(got1, x.sum(axis=1), rtol=1e-12, atol=0)


@pytest.mark.parametrize("fn, npfn", [(xp.sum, np.sum), (xp.max, np.max), (xp.min, np.min), (xp.prod, np.prod)])
@pytest.mark.parametrize("axis", [0, 1, None])
def test_reductions_f64(ex, fn, npfn, axis):
    rng = np.random.default_rng(8)
    x = rng.random((33, 500)) + 0.5
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=(10, 128), spec=spec)
    got = fn(a, axis=axis).compute()
    assert np.allclose(got, npfn(x, axis=axis), rtol=1e-12, atol=0)


@pytest.mark.parametrize("axis", [0, 1])
def test_sum_int64_exact(ex, axis):
    x = np.arange(30 * 40, dtype=np.int64).reshape(30, 40) - 600
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=(7, 9), spec=spec)
    assert np.array_equal(xp.sum(a, axis=axis).compute(), x.sum(axis=axis))


def test_nanmean_rows(ex):
    x = np.random.default_rng(1).random((20, 30))
    x[x < 0.3] = np.nan
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=(6, 7), spec=spec)
    assert np.allclose(cubed.nanmean(a, axis=1).compute(), np.nanmean(x, axis=1), rtol=1e-12)


def test_any_all(ex):
    x = np.zeros((20, 30), dtype=bool)
    x[3, 4] = True
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=(6, 7), spec=spec)
    assert bool(xp.any(a).compute()) is True
    assert bool(xp.all(a).compute()) is False
    assert np.array_equal(xp.any(a, axis=0).compute(), x.any(axis=0))


def test_custom_reduction(ex):
    # core/ops.py reduction() with user func/combine (test_core.py:335-347 style)
    spec = cubed.Spec(allowed_mem=1000, executor=ex)
    a = xp.ones((100, 10), dtype=np.uint8, chunks=(1, 10), spec=spec)
    b = reduction(a, np.sum, axis=0, dtype=np.uint64)
    assert np.array_equal(b.compute(), np.full((1, 10), 100) if b.ndim == 2 else np.full(10, 100))


# ------------------------------------------------------------- rechunk (H15)


@pytest.mark.parametrize("shape, source, target, mem", [
    ((60, 50), (10, 50), (60, 10), 100_000),
    ((60, 50), (10, 50), (60, 10), 10**9),
    ((33, 47), (5, 47), (33, 4), 40_000),
    ((10, 10), (2, 3), (5, 5), 100_000),
    ((3, 3), (2, 1), (1, 2), 100_000),
])
def test_rechunk_bit_exact(ex, shape, source, target, mem):
    x = np.random.default_rng(9).random(shape).astype(np.float32)
    spec = cubed.Spec(allowed_mem=mem, executor=ex)
    a = cubed.from_array(x, chunks=source, spec=spec)
    b = a.rechunk(target)
    assert b.chunksize == tuple(target)
    assert np.array_equal(b.compute(), x)


def test_rechunk_int_dtypes(ex):
    x = np.arange(64 * 48, dtype=np.int16).reshape(64, 48)
    spec = cubed.Spec(allowed_mem=10**8, executor=ex)
    b = cubed.from_array(x, chunks=(8, 48), spec=spec).rechunk((64, 8))
    assert np.array_equal(b.compute(), x)


@pytest.mark.parametrize("flat", [True, False])
@pytest.mark.parametrize("dtype, shape, source, target", [
    (np.float64, (300, 4000), (30, 4000), (300, 250)),   # 2000-B rows: 16-B lanes
    (np.int32, (512, 1000), (64, 1000), (512, 250)),     # 1000-B rows: 8-B lanes
    (np.int16, (400, 1000), (50, 1000), (400, 250)),     # 500-B rows: 4-B lanes
    (np.uint8, (1000, 999), (100, 999), (1000, 37)),     # 37-B rows: 1-B lanes
])
def test_rechunk_copy_paths_bit_exact(ex, monkeypatch, flat, dtype, shape, source, target):
    # packed-destination pieces take k_copy_flat (CUBED_COPY_FLAT) unless
    # lowering.COPY_FLAT = False selects the per-row kernel; boxes span
    # several workgroups so segment and row boundaries fall mid-wave
    monkeypatch.setattr(L, "COPY_FLAT", flat)
    x = np.random.default_rng(5).integers(0, 2**31, size=shape).astype(dtype)
    spec = cubed.Spec(allowed_mem=10**9, executor=ex)
    b = cubed.from_array(x, chunks=source, spec=spec).rechunk(target)
    assert b.chunksize == tuple(target)
    assert np.array_equal(b.compute(), x)


def test_merge_chunks_values(ex):
    x = np.arange(100, dtype=np.float64).reshape(10, 10)
    spec = cubed.Spec(allowed_mem=100000, executor=ex)
    a = cubed.from_array(x, chunks=(2, 2), spec=spec)
    assert np.array_equal(merge_chunks(a, (4, 6)).compute(), x)


# ------------------------------------------------------------- matmul (H13)


def test_matmul_f32(ex):
    r = np.random.default_rng(2)
    x = r.random((96, 80)).astype(np.float32)
    y = r.random((80, 64)).astype(np.float32)
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=(32, 40), spec=spec)
    b = cubed.from_array(y, chunks=(40, 32), spec=spec)
    got = xp.matmul(a, b).compute()
    exp = (x.astype(np.float64) @ y.astype(np.float64)).astype(np.float32)
    assert np.allclose(got, exp, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("shape_a, shape_b, ca, cb", [
    ((300, 256), (256, 190), (150, 128), (128, 95)),    # float4 rows, M/N tails
    ((300, 257), (257, 190), (150, 129), (129, 95)),    # odd K: scalar operand path
    ((520, 1040), (1040, 260), (260, 520), (520, 260)), # several 128-tiles and K tiles
])
def test_matmul_f32_tiles(ex, shape_a, shape_b, ca, cb):
    """The 128x128x32 MFMA tile kernel against an f64 product (error bound
    of an f32 fma chain + f32 k-chunk sums: rtol 1e-5 at these K)."""
    r = np.random.default_rng(12)
    x = r.random(shape_a).astype(np.float32) - 0.5
    y = r.random(shape_b).astype(np.float32) - 0.5
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=ca, spec=spec)
    b = cubed.from_array(y, chunks=cb, spec=spec)
    got = xp.matmul(a, b).compute()
    exp = x.astype(np.float64) @ y.astype(np.float64)
    scale = np.abs(x).astype(np.float64) @ np.abs(y).astype(np.float64)
    assert got.dtype == np.float32
    assert np.all(np.abs(got - exp) <= 1e-6 * scale + 1e-30)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_matmul_ragged_chunks(ex, dtype):
    """f32/f64 chunk products on the hand-written kernels, ragged chunks
    (several shapes per launch), against an f64 product; bound = the f32 (or
    f64) rounding of a length-K dot product plus the k-chunk sums."""
    r = np.random.default_rng(21)
    x = (r.random((150, 130)) - 0.5).astype(dtype)
    y = (r.random((130, 170)) - 0.5).astype(dtype)
    spec = mkspec(ex)
    got = xp.matmul(cubed.from_array(x, chunks=(64, 50), spec=spec),
                    cubed.from_array(y, chunks=(50, 80), spec=spec)).compute()
    exp = x.astype(np.float64) @ y.astype(np.float64)
    scale = np.abs(x).astype(np.float64) @ np.abs(y).astype(np.float64)
    eps = 1e-6 if dtype == np.float32 else 1e-14
    assert got.dtype == dtype
    assert np.all(np.abs(got - exp) <= eps * scale + 1e-300)


def test_tensordot_golden(ex):
    c = json.load(open(os.path.join(GOLDEN, "reference_cases.json")))["tensordot_axes_1"]
    spec = mkspec(ex)
    x = xp.asarray(np.arange(400, dtype=np.float64).reshape(20, 20), chunks=(5, 4), spec=spec)
    y = xp.asarray(np.arange(200, dtype=np.float64).reshape(20, 10), chunks=(4, 5), spec=spec)
    assert np.array_equal(xp.tensordot(x, y, axes=1).compute(), c["expected"])


# ----------------------------------------------------------- index (H14)


def test_index_slice_and_mean(ex):
    """config 4 shape of work: mean(a[1:] * x + b[1:] * y)"""
    rng = np.random.default_rng(11)
    A = rng.random((30, 9, 8))
    B = rng.random((30, 9, 8))
    X = rng.random((9, 8))
    Y = rng.random((9, 8))
    spec = mkspec(ex)
    a = cubed.from_array(A, chunks=(10, 3, 4), spec=spec)
    b = cubed.from_array(B, chunks=(10, 3, 4), spec=spec)
    x = cubed.from_array(X, chunks=(3, 4), spec=spec)
    y = cubed.from_array(Y, chunks=(3, 4), spec=spec)
    got = xp.mean(a[1:] * x + b[1:] * y).compute()
    exp = np.mean(A[1:] * X + B[1:] * Y)
    assert np.isclose(got, exp, rtol=1e-12, atol=0)


@pytest.mark.parametrize("expr", ["mean0", "nanmean_all", "max_all", "argmax0_f32", "sum02"])
def test_region_chains_walk_source_chunks(ex, expr):
    """Reductions over straddling index regions as one chain launch over
    merged source-chunk pieces (chains.chain_piece_rows): the straddled axis
    is reduced, kept dims are whole blocks."""
    rng = np.random.default_rng(29)
    A = rng.random((47, 10, 12))
    A[5, 3, 4] = np.nan
    spec = mkspec(ex)
    a = cubed.from_array(A, chunks=(10, 4, 5), spec=spec)
    sa, SA = a[1:], A[1:]
    if expr == "mean0":
        got, exp = xp.mean(sa * 2, axis=0).compute(), np.mean(SA * 2, axis=0)
    elif expr == "nanmean_all":
        got, exp = cubed.nanmean(sa).compute(), np.nanmean(SA)
    elif expr == "max_all":
        got, exp = xp.max(a[3:]).compute(), np.max(A[3:])
        assert np.isnan(got) and np.isnan(exp)
        return
    elif expr == "argmax0_f32":
        s32 = xp.astype(a, xp.float32)[2:]
        got, exp = xp.argmax(s32, axis=0).compute(), np.argmax(A.astype(np.float32)[2:], axis=0)
        assert np.array_equal(got, exp)
        return
    else:
        got, exp = xp.sum(sa, axis=(0, 2)).compute(), np.sum(SA, axis=(0, 2))
    assert np.allclose(got, exp, rtol=1e-12, atol=0, equal_nan=True)


@pytest.mark.parametrize("expr", ["map", "sum0", "sum1", "mean_all", "max0"])
def test_straddling_regions_as_pieces(ex, expr):
    """index regions that straddle source chunks run as per-chunk pieces
    (no scratch gather): maps write disjoint sub-boxes; reductions across a
    cut combine the pieces' partials in order (grouped finish)."""
    rng = np.random.default_rng(13)
    A = rng.random((23, 17, 9))
    B = rng.random((23, 17, 9))
    spec = mkspec(ex)
    a = cubed.from_array(A, chunks=(5, 6, 9), spec=spec)
    b = cubed.from_array(B, chunks=(5, 6, 9), spec=spec)
    sa, sb = a[2:, 1:], b[:-2, :-1]
    SA, SB = A[2:, 1:], B[:-2, :-1]
    if expr == "map":
        got, exp = (sa * 2 + sb).compute(), SA * 2 + SB
        assert np.array_equal(got, exp)
        return
    if expr == "sum0":
        got, exp = xp.sum(sa * sb, axis=0).compute(), (SA * SB).sum(axis=0)
    elif expr == "sum1":
        got, exp = xp.sum(sa - sb, axis=1).compute(), (SA - SB).sum(axis=1)
    elif expr == "mean_all":
        got, exp = xp.mean(sa + sb).compute(), np.mean(SA + SB)
    else:
        got, exp = xp.max(sa * sb, axis=0).compute(), (SA * SB).max(axis=0)
        assert np.array_equal(got, exp)
        return
    assert np.allclose(got, exp, rtol=1e-12, atol=0)


@pytest.mark.parametrize("mem", [10**9, 60_000])
@pytest.mark.parametrize("op", ["mean0", "sum1", "map", "both"])
def test_rechunk_read_through(ex, mem, op):
    """A rechunk consumed by one op is read through (rewrites.elide_rechunks):
    the consumer reads the source's chunks in place, values unchanged (maps
    bit-exact, reductions rtol 1e-12).  mem=60 kB forces the reference's
    two-op rechunk through an intermediate."""
    x = np.random.default_rng(14).random((60, 50))
    spec = cubed.Spec(allowed_mem=mem, executor=ex)
    a = cubed.from_array(x, chunks=(10, 50), spec=spec)
    b = a.rechunk((60, 10))
    if op == "mean0":
        assert np.allclose(xp.mean(b, axis=0).compute(), x.mean(axis=0), rtol=1e-12, atol=0)
    elif op == "sum1":
        assert np.allclose(xp.sum(b, axis=1).compute(), x.sum(axis=1), rtol=1e-12, atol=0)
    elif op == "map":
        assert np.array_equal((b * 3 + 1).compute(), x * 3 + 1)
    else:  # the rechunked array is also requested: not elided
        c = b * 2
        got_b, got_c = cubed.compute(b, c) if hasattr(cubed, "compute") else (b.compute(), c.compute())
        assert np.array_equal(got_b, x) and np.array_equal(got_c, x * 2)


ARG_A = [[11, 12, 13], [11, 11, 14], [10, 13, 11]]


@pytest.mark.parametrize("fn, axis", [("argmax", None), ("argmax", 0), ("argmin", 0),
                                      ("argmax", 1), ("argmin", None)])
def test_arg_reductions_reference_cases(ex, fn, axis):
    """test_array_api.py:524-548: argmax/argmin of a 3x3 int array in 2x2 chunks."""
    spec = mkspec(ex)
    a = xp.asarray(ARG_A, chunks=(2, 2), spec=spec)
    got = getattr(xp, fn)(a, axis=axis).compute()
    exp = getattr(np.array(ARG_A), fn)(axis=axis)
    assert np.array_equal(got, exp) and np.asarray(got).dtype == np.int64


@pytest.mark.parametrize("fn", ["argmax", "argmin"])
def test_arg_reductions_ties_and_nans(ex, fn):
    """First index on ties; the first NaN wins (numpy's rule), across chunks."""
    x = np.round(np.random.default_rng(16).random((41, 37)) * 4) / 4  # many ties
    x[5, 3] = np.nan
    x[20, 3] = np.nan
    x[7, 30] = np.nan
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=(6, 8), spec=spec)
    for axis in (0, 1, None):
        got = getattr(xp, fn)(a, axis=axis).compute()
        assert np.array_equal(got, getattr(x, fn)(axis=axis)), axis


@pytest.mark.parametrize("dtype", ["float64", "float32", "float16", "int64", "uint64", "int32", "int16",
                                   "uint32", "uint8", "bool"])
@pytest.mark.parametrize("fn", ["argmax", "argmin"])
def test_arg_reductions_pairs(ex, fn, dtype):
    """One-pass argmax/argmin over {value, index} pairs for every dtype
    (64-bit values included): bit-exact indexes vs numpy, ties -> first
    index, NaN -> first NaN, -0 == +0, +-inf and the dtype's extreme values,
    over axis 0, 1, None and keepdims."""
    rng = np.random.default_rng(23)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        x = (np.round(rng.standard_normal((45, 39)) * 2) / 2).astype(dt)  # ties
        x[3, 4] = -0.0
        x[9, 4] = 0.0
        x[2, 10], x[30, 10] = np.inf, -np.inf
        x[11, 20], x[12, 21] = np.finfo(dt).max, np.finfo(dt).min
        x[40, 5] = x[17, 5] = np.nan
        x[:, 33] = np.nan
    elif dt.kind == "b":
        x = rng.random((45, 39)) < 0.5
        x[:, 7] = False
        x[:, 8] = True
    else:
        info = np.iinfo(dt)
        x = rng.integers(max(info.min, -5), min(info.max, 5) + 1, (45, 39)).astype(dt)
        x[1, 2], x[44, 2] = info.max, info.min
        x[6, 9] = x[8, 9] = info.max
        x[10, 12] = x[20, 12] = info.min
        if dt.itemsize == 8:  # values that no f64 holds exactly
            x[30, 14], x[31, 14] = info.max - 1, info.max
            x[32, 15], x[33, 15] = info.min + 1, info.min
    spec = mkspec(ex)
    a = cubed.from_array(x, chunks=(7, 10), spec=spec)
    for axis in (0, 1, None):
        for keepdims in (False, True):
            got = np.asarray(getattr(xp, fn)(a, axis=axis, keepdims=keepdims).compute())
            exp = getattr(np, fn)(x, axis=axis, keepdims=keepdims)
            assert got.dtype == np.int64 and np.array_equal(got, exp), (axis, keepdims)


@pytest.mark.parametrize("fn", ["argmax", "argmin"])
def test_arg_reductions_merge_rounds_and_0d(ex, fn):
    """Many chunks along the reduced axis under a small allowed_mem: the
    pairs go through several merge + combine rounds (core/ops.py:849-889);
    a 0-d array gives index 0; an empty axis raises as numpy does."""
    rng = np.random.default_rng(5)
    x = np.round(rng.standard_normal((400, 6)) * 3)
    x[123, 2] = x[301, 2] = np.nan
    spec = cubed.Spec(allowed_mem=20000, executor=ex)
    a = cubed.from_array(x, chunks=(3, 6), spec=spec)
    for axis in (0, None):
        assert np.array_equal(getattr(xp, fn)(a, axis=axis).compute(), getattr(np, fn)(x, axis=axis))
    z = xp.asarray(np.float64(4.0), spec=mkspec(ex))
    assert int(getattr(xp, fn)(z).compute()) == 0
    with pytest.raises(ValueError):
        getattr(xp, fn)(xp.asarray(np.zeros((0, 3)), spec=mkspec(ex)), axis=0)


# ----------------------------------------------------------- callbacks / resume


def test_task_end_events_and_resume(ex):
    class Counter(cubed.Callback):
        def __init__(self):
            self.value = 0

        def on_task_end(self, event):
            self.value += event.num_tasks

    spec = mkspec(ex, mem=100000, reserved=0)
    a = xp.asarray([[1, 2, 3], [4, 5, 6], [7, 8, 9]], chunks=(2, 2), spec=spec)
    d = xp.negative(xp.astype(xp.negative(a), np.float32))
    c = Counter()
    res = d.compute(callbacks=[c])
    assert c.value == d.plan.num_tasks()
    assert np.array_equal(res, np.array([[1, 2, 3], [4, 5, 6], [7, 8, 9]], dtype=np.float32))
    c2 = Counter()
    d.compute(callbacks=[c2], resume=True)
    assert c2.value == 0 or c2.value < c.value


class TaskCounter(cubed.Callback):
    """cubed/tests/utils.py TaskCounter: sums TaskEndEvent.num_tasks."""

    def __init__(self):
        self.value = 0

    def on_task_end(self, event):
        self.value += event.num_tasks


def test_callbacks_exact_counts(ex):
    """cubed/tests/test_executor_features.py:51-63 (test_callbacks): an
    add of two 3x3 arrays in 2x2 chunks is 4 tasks plus one created array."""
    spec = mkspec(ex, mem=100000, reserved=0)
    a = xp.asarray([[1, 2, 3], [4, 5, 6], [7, 8, 9]], chunks=(2, 2), spec=spec)
    b = xp.asarray([[1, 1, 1], [1, 1, 1], [1, 1, 1]], chunks=(2, 2), spec=spec)
    c = xp.add(a, b)
    tc = TaskCounter()
    assert np.array_equal(c.compute(callbacks=[tc]), np.array([[2, 3, 4], [5, 6, 7], [8, 9, 10]]))
    num_created_arrays = 1
    assert tc.value == num_created_arrays + 4


def test_resume_exact_counts(ex):
    """cubed/tests/test_executor_features.py:121-150 (test_resume), restated
    with its exact task counts: c computed, then d = -c with resume runs only
    d's 4 tasks (the create-arrays task runs again, for both arrays)."""
    spec = mkspec(ex, mem=100000, reserved=0)
    a = xp.asarray([[1, 2, 3], [4, 5, 6], [7, 8, 9]], chunks=(2, 2), spec=spec)
    b = xp.asarray([[1, 1, 1], [1, 1, 1], [1, 1, 1]], chunks=(2, 2), spec=spec)
    c = xp.add(a, b)
    d = xp.negative(c)
    num_created_arrays = 2  # c, d
    assert d.plan.num_tasks(optimize_graph=False) == num_created_arrays + 8
    tc = TaskCounter()
    c.compute(callbacks=[tc], optimize_graph=False)
    num_created_arrays = 1  # c
    assert tc.value == num_created_arrays + 4
    tc = TaskCounter()
    got = d.compute(callbacks=[tc], optimize_graph=False, resume=True)
    num_created_arrays = 2  # c, d
    assert tc.value == num_created_arrays + 4
    assert np.array_equal(got, -np.array([[2, 3, 4], [5, 6, 7], [8, 9, 10]]))


# ----------------------------------------------------- full-size properties


def test_bench_size_quad_means_properties(ex):
    """BASELINE config 2 at full size (1000, 720, 1440) f32: checked through
    size-independent properties -- against a direct f64 column sum on the GPU
    for a sample of columns, and mean(u*u) of U[0,1) ~ 1/3."""
    import torch

    spec = mkspec(ex)
    random.seed(12)
    shape, chunks = (1000, 720, 1440), (10, 720, 1440)
    u = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    arrays_to_plan(u).execute(executor=ex, array_names=[u.name])
    m = xp.mean(u * u, axis=0)
    got = m.compute(resume=True)
    assert got.shape == (720, 1440)
    assert abs(float(got.mean()) - 1 / 3) < 1e-3
    # exact check of 64 sampled columns: gather them from the chunk slabs
    rng = np.random.default_rng(0)
    cols = rng.integers(0, 720 * 1440, 64)
    t = torch.empty((1000, 64), dtype=torch.float32, device=ex.device)
    za = u.zarray
    for c in range(100):
        raw, _ = za._slab_view(None, za.local_slot((c, 0, 0)), (10, 720, 1440))
        blk = raw.view(torch.float32).view(10, 720 * 1440)
        t[c * 10:(c + 1) * 10] = blk[:, torch.as_tensor(cols, device=ex.device)]
    col = t.cpu().numpy().astype(np.float64)
    exp = ((col * col).sum(axis=0) / 1000).astype(np.float32)
    assert np.allclose(got.reshape(-1)[cols], exp, rtol=1e-6, atol=0)
    del u, m
    torch.cuda.empty_cache()


def test_bench_size_rechunk_roundtrip(ex):
    """config 3 shape at reduced size (10000^2 f32): rechunk rows->columns
    ->rows is the identity (bit-exact), checked by a checksum of checksums."""
    import torch

    spec = cubed.Spec(allowed_mem="288GB", executor=ex)
    random.seed(13)
    N = 10000
    x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
    arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
    y = x.rechunk((N, 1000))
    z = y.rechunk((1000, N))
    arrays_to_plan(z).execute(executor=ex, resume=True, array_names=[z.name])
    torch.cuda.synchronize()
    xs = x.zarray.slabs[None][: x.nbytes].view(torch.int32).to(torch.int64)
    zs = z.zarray.slabs[None][: z.nbytes].view(torch.int32).to(torch.int64)
    assert int(xs.sum()) == int(zs.sum())
    assert torch.equal(x.zarray.slabs[None][: x.nbytes], z.zarray.slabs[None][: z.nbytes])


# ------------------------------------------- specialised vs interpreted kernels


@pytest.mark.parametrize("case", ["quad", "where", "nanmean", "int_sum_rows", "cast_chain"])
def test_specialised_kernels_match_interpreter(monkeypatch, case):
    """The runtime-specialised kernels (default) and the ahead-of-time
    interpreter kernels (CUBED_AMD_JIT=0) compute bit-identical results."""
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    def run():
        ex = GpuDagExecutor("cuda:0")
        spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)
        rng = np.random.default_rng(21)
        x = rng.random((64, 40, 24))
        x[x < 0.1] = np.nan
        a = cubed.from_array(x, chunks=(16, 40, 24), spec=spec)
        b = cubed.from_array((x * 100).astype(np.float32), chunks=(16, 40, 24), spec=spec)
        if case == "quad":
            out = xp.mean(b * b, axis=0)
        elif case == "where":
            out = xp.where(a > 0.5, a * 2, -a)
        elif case == "nanmean":
            out = cubed.nanmean(a, axis=2)
        elif case == "int_sum_rows":
            out = xp.sum(xp.astype(b, xp.int64), axis=2)
        else:
            out = xp.astype(xp.astype(b, xp.int32) * 3 + 1, xp.float64) / 7
        return out.compute()

    monkeypatch.setenv("CUBED_AMD_JIT", "1")
    got = run()
    monkeypatch.setenv("CUBED_AMD_JIT", "0")
    exp = run()
    assert got.dtype == exp.dtype
    assert np.array_equal(got, exp, equal_nan=True)


@pytest.mark.parametrize("merge", [True, False])
def test_row_merging_values(ex, monkeypatch, merge):
    """Task-row merging (lowering._merge_group_rows / _merge_kept_runs) on
    stream-eligible geometries -- a read-through rechunk + mean / int64 sum
    (one task of whole rows when merged, 6 x 8 pieces + grouped finish when
    not) and the vorticity chain mean(a[1:] * x + b[1:] * y) (one row per T
    band with a chunk dim) -- against numpy: int64 exact, f32 means of f64
    sums rtol 1e-6, f64 rtol 1e-12."""
    from cubed_amd import lowering as L

    monkeypatch.setattr(L, "MERGE_ROWS", merge)
    rng = np.random.default_rng(21)
    X = rng.random((600, 2048)).astype(np.float32)
    I = rng.integers(-1000, 1000, (600, 2048))
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    x = cubed.from_array(X, chunks=(100, 2048), spec=spec)
    i = cubed.from_array(I, chunks=(100, 2048), spec=spec)
    got = xp.mean(x.rechunk((600, 256)), axis=0).compute()
    np.testing.assert_allclose(got, X.astype(np.float64).mean(axis=0).astype(np.float32), rtol=1e-6, atol=0)
    assert np.array_equal(xp.sum(i.rechunk((600, 256)), axis=0).compute(), I.sum(axis=0))
    A, B = rng.random((41, 24, 32)), rng.random((41, 24, 32))
    XX, YY = rng.random((24, 32)), rng.random((24, 32))
    a = cubed.from_array(A, chunks=(10, 8, 8), spec=spec)
    b = cubed.from_array(B, chunks=(10, 8, 8), spec=spec)
    xx = cubed.from_array(XX, chunks=(8, 8), spec=spec)
    yy = cubed.from_array(YY, chunks=(8, 8), spec=spec)
    got = xp.mean(a[1:] * xx + b[1:] * yy).compute()
    np.testing.assert_allclose(got, (A[1:] * XX + B[1:] * YY).mean(), rtol=1e-12, atol=0)
