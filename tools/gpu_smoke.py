"""Quick GPU smoke: build small plans, execute on the MI355X executor, compare with numpy."""
import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import random, sys, traceback
import numpy as np
import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
from cubed_amd.runtime.executors.gpu import GpuDagExecutor

ex = GpuDagExecutor()
spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)
fails = 0

def philox_array(shape, chunks, seed):
    from numpy.random import Generator, Philox
    import itertools
    from cubed_amd.utils import normalize_chunks, chunk_starts
    nc = normalize_chunks(chunks, shape, dtype=np.float64)
    nb = tuple(len(c) for c in nc)
    out = np.empty(shape)
    for bid in itertools.product(*[range(n) for n in nb]):
        off = int(np.ravel_multi_index(bid, nb))
        sl = tuple(slice(chunk_starts(nc[d])[b], chunk_starts(nc[d])[b+1]) for d, b in enumerate(bid))
        out[sl] = Generator(Philox(key=seed + off)).random(tuple(s.stop - s.start for s in sl))
    return out

def check(name, fn):
    global fails
    try:
        got, exp, exact = fn()
        if exact:
            ok = np.array_equal(got, exp)
        else:
            ok = np.allclose(got, exp, rtol=(1e-5 if np.asarray(got).dtype == np.float32 else 1e-12), atol=0)
        print(f"{'PASS' if ok else 'FAIL'} {name}", "" if ok else f"max abs err {np.max(np.abs(np.asarray(got, float) - np.asarray(exp, float)))}", flush=True)
        if not ok:
            fails += 1
    except Exception:
        fails += 1
        print(f"ERROR {name}"); traceback.print_exc()

def t_asarray_add():
    a = xp.asarray([[1, 2, 3], [4, 5, 6], [7, 8, 9]], chunks=(2, 2), spec=spec)
    b = xp.asarray([[1, 1, 1], [1, 1, 1], [1, 1, 1]], chunks=(2, 2), spec=spec)
    return xp.add(a, b).compute(), np.array([[2, 3, 4], [5, 6, 7], [8, 9, 10]]), True

def t_mean0():
    x = np.array([[1.0, 2.0, 3.0], [4.0, 5.0, 6.0], [7.0, 8.0, 9.0]])
    a = xp.asarray(x, chunks=(2, 2), spec=spec)
    return xp.mean(a, axis=0).compute(), x.mean(axis=0), True

def t_random():
    random.seed(42)
    a = crandom.random((100, 60), chunks=(30, 25), spec=spec)
    random.seed(42); seed = random.getrandbits(128)
    return a.compute(), philox_array((100, 60), (30, 25), seed), True

def t_config1_small():
    random.seed(7)
    a = crandom.random((200, 200), chunks=(50, 50), spec=spec)
    random.seed(7); seed = random.getrandbits(128)
    x = philox_array((200, 200), (50, 50), seed)
    m = xp.mean((a + 1) * 2, axis=0)
    return m.compute(), ((x + 1) * 2).mean(axis=0), False

def t_quad():
    random.seed(3)
    u = crandom.random((50, 1, 37, 40), chunks=(10, 1, -1, -1), spec=spec)
    v = crandom.random((50, 1, 37, 40), chunks=(10, 1, -1, -1), spec=spec)
    random.seed(3); s1 = random.getrandbits(128); s2 = random.getrandbits(128)
    U = philox_array(u.shape, (10, 1, 37, 40), s1); V = philox_array(v.shape, (10, 1, 37, 40), s2)
    return xp.mean(u * v, axis=0).compute(), (U * V).mean(axis=0), False

def t_quad_f32():
    random.seed(4)
    u = xp.astype(crandom.random((40, 30, 20), chunks=(10, 30, 20), spec=spec), xp.float32)
    v = xp.astype(crandom.random((40, 30, 20), chunks=(10, 30, 20), spec=spec), xp.float32)
    random.seed(4); s1 = random.getrandbits(128); s2 = random.getrandbits(128)
    U = philox_array(u.shape, (10, 30, 20), s1).astype(np.float32); V = philox_array(v.shape, (10, 30, 20), s2).astype(np.float32)
    got = xp.mean(u * v, axis=0).compute()
    exp = (U * V).astype(np.float64).mean(axis=0).astype(np.float32)
    return got, exp, True

def t_rechunk():
    x = np.arange(60 * 50, dtype=np.float32).reshape(60, 50)
    a = cubed.from_array(x, chunks=(10, 50), spec=spec)
    return a.rechunk((60, 10)).compute(), x, True

def t_sum_all():
    x = np.arange(30 * 40, dtype=np.int64).reshape(30, 40)
    a = cubed.from_array(x, chunks=(7, 9), spec=spec)
    return xp.sum(a).compute(), x.sum(), True

def t_sum_axis1():
    x = np.random.default_rng(0).random((33, 500))
    a = cubed.from_array(x, chunks=(10, 128), spec=spec)
    return xp.sum(a, axis=1).compute(), x.sum(axis=1), False

def t_where_nan():
    x = np.random.default_rng(1).random((20, 30)); x[x < 0.3] = np.nan
    a = cubed.from_array(x, chunks=(6, 7), spec=spec)
    return cubed.nanmean(a, axis=1).compute(), np.nanmean(x, axis=1), False

def t_matmul():
    x = np.arange(16, dtype=np.float64).reshape(4, 4)
    a = xp.asarray(x, chunks=(2, 2), spec=spec)
    return xp.matmul(a, a).compute(), x @ x, True

def t_matmul_f32():
    r = np.random.default_rng(2)
    x = r.random((96, 80)).astype(np.float32); y = r.random((80, 64)).astype(np.float32)
    a = cubed.from_array(x, chunks=(32, 40), spec=spec); b = cubed.from_array(y, chunks=(40, 32), spec=spec)
    got = xp.matmul(a, b).compute()
    return got, (x.astype(np.float64) @ y.astype(np.float64)).astype(np.float32), False

for name, fn in list(globals().items()):
    if name.startswith("t_"):
        check(name, fn)
print("FAILS", fails)
sys.exit(1 if fails else 0)
