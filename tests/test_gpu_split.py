"""Oversized chunk programs split into several fused launches (needs an
MI355X; ``-m gpu``).  A chunk function over more inputs than one fused
program holds (CUBED_MAX_LEAVES = 4) runs as part programs into HBM
temporaries + the remainder (cubed_amd/split.py); values must equal the
single-program semantics: bit-exact for maps (every node rounded to its
dtype either way), and for reductions the same per-chunk sums."""

import numpy as np
import pytest

import cubed_amd as cubed
from cubed_amd.core.plan import arrays_to_plan
from cubed_amd.lowering import FusedLaunch

pytestmark = pytest.mark.gpu


@pytest.fixture()
def ex(gpu_executor):
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    return GpuDagExecutor("cuda:0")


def _inputs(n, shape, seed, dtype=np.float64):
    r = np.random.default_rng(seed)
    return [(r.random(shape) - 0.5).astype(dtype) for _ in range(n)]


def _fused(ex):
    return [l for v in ex._cache.values() for l in v[1] if isinstance(l, FusedLaunch)]


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_five_input_map_bit_exact(ex, dtype):
    xs = _inputs(5, (130, 70), 1, dtype)
    spec = cubed.Spec(allowed_mem=10**8, executor=ex)
    arrs = [cubed.from_array(x, chunks=(40, 30), spec=spec) for x in xs]
    m = cubed.map_blocks(lambda a, b, c, d, e: a * b + c * d + e, *arrs, dtype=dtype)
    got = m.compute()
    a, b, c, d, e = xs
    exp = a * b + c * d + e
    assert got.dtype == dtype
    assert np.array_equal(got, exp)
    assert len(_fused(ex)) == 2


def test_six_input_map_with_where(ex):
    xs = _inputs(6, (64, 64), 2)
    spec = cubed.Spec(allowed_mem=10**8, executor=ex)
    arrs = [cubed.from_array(x, chunks=(32, 16), spec=spec) for x in xs]
    m = cubed.map_blocks(lambda a, b, c, d, e, f: np.where(a > 0, b * c, d - e) + f, *arrs,
                         dtype=np.float64)
    a, b, c, d, e, f = xs
    assert np.array_equal(m.compute(), np.where(a > 0, b * c, d - e) + f)


def test_split_map_feeds_a_reduction(ex):
    """The split map's output (not fusable into the sum: it does not fit one
    program) is materialised and reduced: mean over axis 0 as numpy's f64
    sums within 1e-12."""
    import cubed_amd.array_api as xp

    xs = _inputs(5, (120, 48), 3)
    spec = cubed.Spec(allowed_mem=10**8, executor=ex)
    arrs = [cubed.from_array(x, chunks=(40, 24), spec=spec) for x in xs]
    m = cubed.map_blocks(lambda a, b, c, d, e: a * b + c * d + e, *arrs, dtype=np.float64)
    got = xp.mean(m, axis=0).compute()
    a, b, c, d, e = xs
    assert np.allclose(got, (a * b + c * d + e).mean(axis=0), rtol=1e-12, atol=0)
