"""var / std on the MI355X executor (``-m gpu``): the {n, mu, M2} triple
reduction (Welford per element, Chan's update across splits, merge rounds,
partial_reduce rounds and GPUs) against numpy's f64 ``var(ddof=correction)``
and the oracle's chunked restatement (oracle/cubed_ref.py ``var``).

Parity is UNPINNED against the reference: cubed v0.12.0 has no var / std
(api_status.md:72,74); the semantics are numpy's, computed in f64 as the
reference computes mean (statistical_functions.py:28-100 is the pattern).
Tolerances: rtol 1e-12 for f64 results, 1e-6 for f32 results.

Rounding note (round 5): in the vectorised streaming kernel the Welford
update of a 4-element group multiplies by one shared 1/n (vm.h
``var_add_inv``) instead of dividing every element by n -- the group's
elements fold the same rows, so n is common -- which moves var / std by a
few ulp against the per-element division (the scalar path and earlier
builds).  The tolerances above cover it; no test compares var bit for bit
across builds.
"""

import random

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
from cubed_amd.core.plan import arrays_to_plan
from oracle import cubed_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ex(gpu_executor):
    return gpu_executor


def _arr(ex, x, chunks, mem="2GB"):
    spec = cubed.Spec(allowed_mem=mem, reserved_mem=0, executor=ex)
    return cubed.from_array(x, chunks=chunks, spec=spec)


def _close(got, exp, rtol):
    got, exp = np.asarray(got, np.float64), np.asarray(exp, np.float64)
    assert got.shape == exp.shape
    assert np.array_equal(np.isnan(got), np.isnan(exp))
    m = ~np.isnan(exp)
    np.testing.assert_allclose(got[m], exp[m], rtol=rtol, atol=0)


@pytest.mark.parametrize("axis", [0, 1, (0, 1), None])
@pytest.mark.parametrize("correction", [0.0, 1.0])
def test_var_f64_matches_numpy(ex, axis, correction):
    rng = np.random.default_rng(11)
    x = rng.random((180, 150)) * 7 + 40  # offset mean: a two-pass-accurate var is needed
    a = _arr(ex, x, (32, 40))
    got = xp.var(a, axis=axis, correction=correction).compute()
    _close(got, np.var(x, axis=axis, ddof=correction), 1e-12)
    _close(got, R.var(x, (32, 40), axis, 2_000_000_000, correction=correction), 1e-12)
    got = xp.std(a, axis=axis, correction=correction, keepdims=True).compute()
    _close(got, np.std(x, axis=axis, ddof=correction, keepdims=True), 1e-12)


@pytest.mark.parametrize("mem", [2_000_000_000, 120_000])
def test_var_merge_rounds(ex, mem):
    """A small allowed_mem forces several merge + combine rounds (the varc
    programs); the chain fusion folds them into one pass."""
    rng = np.random.default_rng(12)
    x = rng.standard_normal((400, 64))
    a = _arr(ex, x, (5, 64), mem=mem)
    got = xp.var(a, axis=0).compute()
    _close(got, np.var(x, axis=0), 1e-12)
    _close(got, R.var(x, (5, 64), 0, mem), 1e-12)


@pytest.mark.parametrize("rows", [300, 301])  # 301: an edge chunk along the reduced axis
def test_var_unfused_combine_rounds(ex, rows):
    """Chain fusion off (or not applicable: a ragged reduced axis): the
    per-chunk var program writes {n, mu, M2} (three output slabs) and every
    varc combine round runs as its own launch (Chan's update on partial
    triples)."""
    ex2 = type(ex)("cuda:0")
    ex2.fuse_reductions = rows % 7 == 0
    rng = np.random.default_rng(13)
    x = rng.random((rows, 50)) + 3
    a = _arr(ex2, x, (7, 50), mem=150_000)
    got = xp.var(a, axis=0).compute()
    _close(got, np.var(x, axis=0), 1e-12)
    _close(got, R.var(x, (7, 50), 0, 150_000), 1e-12)


def test_var_new_impl(ex):
    """reduction(use_new_impl=True): partial_reduce + tree_reduce rounds."""
    rng = np.random.default_rng(14)
    x = rng.random((120, 90))
    a = _arr(ex, x, (10, 30))
    got = xp.var(a, axis=0, use_new_impl=True).compute()
    _close(got, np.var(x, axis=0), 1e-12)
    got = xp.std(a, axis=None, use_new_impl=True).compute()
    _close(got, np.std(x), 1e-12)


def test_var_nan_propagates(ex):
    rng = np.random.default_rng(15)
    x = rng.random((60, 40))
    x[17, 5] = np.nan
    x[3, 33] = np.inf
    a = _arr(ex, x, (16, 16))
    with np.errstate(invalid="ignore"):
        exp = np.var(x, axis=0)
    got = xp.var(a, axis=0).compute()
    assert np.isnan(got[5]) and np.isnan(got[33])
    _close(got, exp, 1e-12)


def test_var_degrees_of_freedom(ex):
    """n <= correction: numpy's clamp gives NaN (0 / 0) for one element."""
    x = np.arange(12.0).reshape(1, 12)
    a = _arr(ex, x, (1, 5))
    got = xp.var(a, axis=0, correction=1.0).compute()
    assert np.all(np.isnan(got))
    got = xp.var(a, axis=0).compute()
    assert np.array_equal(got, np.zeros(12))


def test_var_f32_stream(ex):
    """f32 input on the streaming kernel (quad-means layout), f64 triples,
    f32 output within rtol 1e-6 of numpy's f64 var."""
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)
    random.seed(21)
    shape, chunks = (230, 36, 64), (10, 36, 64)
    u = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    arrays_to_plan(u).execute(executor=ex, array_names=[u.name])
    U = u.compute(resume=True)
    got = xp.var(u, axis=0).compute(resume=True)
    assert got.dtype == np.float32
    _close(got, np.var(U.astype(np.float64), axis=0), 1e-6)
    got = xp.std(u * u, axis=0).compute(resume=True)
    _close(got, np.std(U.astype(np.float64) * U, axis=0), 1e-6)


def test_var_rejects_integers(ex):
    a = _arr(ex, np.arange(10), (5,))
    with pytest.raises(TypeError):
        xp.var(a)
