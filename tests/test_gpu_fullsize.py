"""BASELINE configs 1, 3, 4 and 5 at FULL size on the MI355X (``-m gpu``),
checked through size-independent properties (the full oracle would take
minutes on the host):

* config 3: rechunk 50000^2 f32 rows -> columns on the reference's 2 GB
  plan -- every target chunk bit-exact against the resident source, one
  source chunk bit-exact against the oracle's Philox;
* config 1: (a + 1) * 2 -> mean(axis=0), random((20000, 20000), (5000,
  5000)) f64 -- 64 sampled columns summed in f64 from the resident chunks
  (rtol 1e-12) and the grand mean of U[0,1) data ~ 3;
* config 4 (pangeo vorticity): mean(a[1:] * x + b[1:] * y), a, b (1000, 900,
  800), x, y (900, 800) f64, chunks 100 -- a chunked f64 sum on the GPU over
  the resident inputs (rtol 1e-12);
* config 5: matmul of two 40000^2 arrays in (5000, 5000) chunks, f32 and
  bf16 -- 64 sampled entries against f64 dot products of the resident
  (rounded) operands within 8 sqrt(K) 2^-24 sum|a||b| (+ 2^-8 |C| for a
  bf16 output), the bound of tests/test_gpu_matmul.py.

The same workloads (and checks) run in bench.py's extras; here they are
tests.  Reference anchors: random.py:13-36, statistical_functions.py:28-100,
core/ops.py:374-486 (index), linear_algebra_functions.py:35-78 (matmul).
"""

import random

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
from cubed_amd.core.plan import arrays_to_plan

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]


@pytest.fixture(scope="module")
def ex(gpu_executor):
    return gpu_executor


def _chunk(arr, coords):
    """torch view (on the device) of one resident chunk, in its dtype."""
    import torch

    tdt = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}
    ext = arr.chunk_extent(coords)
    raw, _ = arr._slab_view(None, arr.local_slot(coords), ext)
    return raw.view(tdt.get(np.dtype(arr.dtype), torch.bfloat16)).reshape(ext)


def _free():
    import gc

    import torch

    gc.collect()
    torch.cuda.empty_cache()


def test_rechunk_full_size(ex):
    """config 3: rechunk 50000^2 f32 rows -> columns with the reference's own
    2 GB plan (two rechunk ops, composed into one copy): EVERY target chunk
    bit-exact against the resident source chunks, and one source row chunk
    bit-exact against the oracle's Philox (random.py:31-36), so the whole
    chain is pinned at full size."""
    import torch

    from oracle import cubed_ref as R

    N = 50000
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    random.seed(2000)
    x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
    arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
    y = x.rechunk((N, 1000))
    plan = arrays_to_plan(y)
    ops = [d for _, d in plan._finalize_dag().nodes(data=True) if d.get("op_name") == "rechunk"]
    assert len(ops) == 2  # the reference's read / write stages at 2 GB
    plan.execute(executor=ex, resume=True, array_names=[y.name])
    X, Y = x.zarray, y.zarray
    assert Y.numblocks == (1, 50)
    for j in range(50):
        got = _chunk(Y, (0, j)).view(torch.int32)
        for i in range(50):
            src = _chunk(X, (i, 0))[:, j * 1000:(j + 1) * 1000].view(torch.int32)
            assert torch.equal(got[i * 1000:(i + 1) * 1000], src), (i, j)
    b = 17  # a source row chunk against the oracle (block offset = its index)
    exp = R.random_block(R.root_seed_after(2000), b, (1000, N)).astype(np.float32)
    assert np.array_equal(_chunk(X, (b, 0)).cpu().numpy().view(np.int32), exp.view(np.int32))
    del x, y, plan, X, Y
    _free()


def test_config1_full_size(ex):
    import torch

    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    random.seed(3000)
    a = crandom.random((20000, 20000), chunks=(5000, 5000), spec=spec)
    arrays_to_plan(a).execute(executor=ex, array_names=[a.name])
    m = xp.mean((a + 1) * 2, axis=0)
    got = m.compute(resume=True)
    assert got.shape == (20000,) and got.dtype == np.float64
    assert abs(float(got.mean()) - 3.0) < 1e-3
    cols = np.sort(np.random.default_rng(1).choice(20000, 64, replace=False))
    A = a.zarray
    acc = torch.zeros(64, dtype=torch.float64, device=ex.device)
    for c in range(64):
        j, jj = divmod(int(cols[c]), 5000)
        for i in range(4):
            acc[c] += torch.sum((_chunk(A, (i, j))[:, jj] + 1) * 2)
    exp = acc.cpu().numpy() / 20000
    np.testing.assert_allclose(got[cols], exp, rtol=1e-12, atol=0)
    del a, m, A
    _free()


def test_vorticity_full_size(ex):
    import itertools

    import torch

    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    random.seed(5000)
    T = 1000
    a = crandom.random((T, 900, 800), chunks=100, spec=spec)
    b = crandom.random((T, 900, 800), chunks=100, spec=spec)
    x = crandom.random((900, 800), chunks=100, spec=spec)
    y = crandom.random((900, 800), chunks=100, spec=spec)
    arrays_to_plan(a, b, x, y).execute(executor=ex, array_names=[a.name, b.name, x.name, y.name])
    got = xp.mean(a[1:] * x + b[1:] * y).compute(resume=True)
    A, B, X, Y = a.zarray, b.zarray, x.zarray, y.zarray
    total = torch.zeros((), dtype=torch.float64, device=ex.device)
    for c in itertools.product(*[range(n) for n in A.numblocks]):
        ca, cb = _chunk(A, c), _chunk(B, c)
        if c[0] == 0:  # a[1:]: the first time row is not read
            ca, cb = ca[1:], cb[1:]
        total += torch.sum(ca * _chunk(X, c[1:]) + cb * _chunk(Y, c[1:]))
    exp = float(total) / ((T - 1) * 900 * 800)
    assert abs(float(got) - 0.5) < 1e-3  # E[a x + b y] = 2 * 1/4
    np.testing.assert_allclose(float(got), exp, rtol=1e-12, atol=0)
    del a, b, x, y, A, B, X, Y
    _free()


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_matmul_full_size(ex, dt):
    import torch

    n, c = 40000, 5000
    spec = cubed.Spec(allowed_mem="288GB", executor=ex)
    random.seed(4000)
    xdt = xp.bfloat16 if dt == "bf16" else xp.float32
    A = xp.astype(crandom.random((n, n), chunks=(c, c), spec=spec), xdt)
    B = xp.astype(crandom.random((n, n), chunks=(c, c), spec=spec), xdt)
    arrays_to_plan(A, B).execute(executor=ex, array_names=[A.name, B.name])
    m = xp.matmul(A, B)
    arrays_to_plan(m).execute(executor=ex, resume=True, array_names=[m.name])
    torch.cuda.synchronize()
    rng = np.random.default_rng(5)
    rows = np.sort(rng.choice(n, 8, replace=False))
    cols = np.sort(rng.choice(n, 8, replace=False))
    nk = n // c
    Az, Bz, Cz = A.zarray, B.zarray, m.zarray
    Ar = torch.stack([torch.cat([_chunk(Az, (i // c, kk))[i % c] for kk in range(nk)])
                      for i in rows]).double().cpu().numpy()
    Bc = torch.stack([torch.cat([_chunk(Bz, (kk, j // c))[:, j % c] for kk in range(nk)])
                      for j in cols], dim=1).double().cpu().numpy()
    got = np.array([[float(_chunk(Cz, (i // c, j // c))[i % c, j % c].double()) for j in cols]
                    for i in rows])
    exp = Ar @ Bc
    bound = 8.0 * np.sqrt(n) * 2.0 ** -24 * (np.abs(Ar) @ np.abs(Bc))
    if dt == "bf16":
        bound = bound + 2.0 ** -8 * np.abs(exp)
    err = np.abs(got - exp)
    assert np.all(err <= bound), float(np.max(err / bound))
    assert abs(float(np.mean(got)) / n - 0.25) < 0.01  # E[a b] = 1/4 per term
    del A, B, m, Az, Bz, Cz
    _free()
