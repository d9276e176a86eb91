"""Chained chunk GEMMs (matmul / tensordot, BASELINE config 5) on the MI355X.

``xp.matmul`` keeps the reference's plan -- (i, k, j) chunk products then a
sum over k (cubed/array_api/linear_algebra_functions.py:13-78) -- and the
executor runs it as ONE ``cubed_gemm_chain`` launch per matmul (the k-sum
fused into the K loop, cubed_amd/gemm_chains.py).  These tests check that
launch, its kernels (the bf16 16x16x32 and f32 32x32x2 MFMA tiles, the
element-wise fallback) and the unfused per-chunk form against an f64 product
of the SAME (dtype-rounded) inputs.

Parity: numpy's f32 matmul (BLAS) and the reference's k-chunk f32 sums have
their own summation order, so f32 results are compared with an error bound,
not bit for bit.  bf16 has no reference dtype (cubed/array_api/dtypes.py
:14-37): "parity unpinned" -- the check is the bound alone.

Bounds (written per test): an f32 accumulation of K products of magnitude
sum |a||b| = S has error <= K * 2^-24 * S (gamma_K); in practice the error
grows like sqrt(K), so the tests use the tighter 8 * sqrt(K) * 2^-24 * S
(checked to hold with a wide margin at K = 40000) plus, for bf16 outputs, the
final rounding of the result to bf16 (2^-9 relative).
"""

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.lowering as L
from cubed_amd import _native as nat
from cubed_amd import ir

pytestmark = pytest.mark.gpu

U = 2.0 ** -24


@pytest.fixture()
def ex(gpu_executor):
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor, LaunchTimer

    e = GpuDagExecutor("cuda:0")
    e.timing = LaunchTimer()
    return e


def _launches(ex, cls=L.GemmLaunch):
    out = []
    for lst in ex._cache.values():
        for l in lst[1]:
            if isinstance(l, cls):
                out.append(l)
    return out


def _bf16_round(x):
    return ir.bf16_to_numpy(ir.numpy_to_bf16(x))


def _operands(shape_a, shape_b, seed, signed=True):
    r = np.random.default_rng(seed)
    x = r.random(shape_a, dtype=np.float64)
    y = r.random(shape_b, dtype=np.float64)
    if signed:
        x, y = x - 0.5, y - 0.5
    return x.astype(np.float32), y.astype(np.float32)


def _check_bound(got, x64, y64, K, out_bf16=False, factor=8.0):
    exp = x64 @ y64
    scale = np.abs(x64) @ np.abs(y64)
    bound = factor * np.sqrt(K) * U * scale
    if out_bf16:
        bound = bound + 2.0 ** -8 * np.abs(exp)
    err = np.abs(got.astype(np.float64) - exp)
    worst = float(np.max(err / np.maximum(bound, 1e-300)))
    assert np.all(err <= bound), f"max err / bound = {worst}"
    return worst


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_chained_matmul_k40000(ex, dt):
    """K = 40000 in 8 chunks of 5000 (config 5's K and chunking; 5000 is not
    a multiple of the 64-deep K tile, so segment boundaries fall inside
    tiles), ragged M/N edge chunks and tiles; one launch, MFMA path."""
    x, y = _operands((296, 40000), (40000, 264), 7)
    spec = cubed.Spec(allowed_mem="20GB", executor=ex)
    a = cubed.from_array(x, chunks=(150, 5000), spec=spec)
    b = cubed.from_array(y, chunks=(5000, 136), spec=spec)
    if dt == "bf16":
        a, b = xp.astype(a, xp.bfloat16), xp.astype(b, xp.bfloat16)
        x64, y64 = _bf16_round(x).astype(np.float64), _bf16_round(y).astype(np.float64)
    else:
        x64, y64 = x.astype(np.float64), y.astype(np.float64)
    m = xp.matmul(a, b)
    assert m.dtype == (ir.bfloat16 if dt == "bf16" else np.float32)
    got = m.compute()
    assert got.dtype == np.float32  # bf16 results come back widened exactly to f32
    gl = _launches(ex)
    assert len(gl) == 1 and gl[0].kernel_path() == nat.GEMM_MFMA
    assert all(int(t["nseg"]) == 8 and int(t["ktot"]) == 40000 for t in gl[0].tasks)
    _check_bound(got, x64, y64, 40000, out_bf16=(dt == "bf16"))


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_mfma_path_equals_element_path_bound(ex, dt, monkeypatch):
    """The same chain through the element-wise kernel (forced): both within
    the bound; for bf16 inputs every product is exact in f32, so the two
    kernels differ only by summation order."""
    x, y = _operands((200, 640), (640, 136), 3)
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    res = {}
    for path in (nat.GEMM_MFMA, nat.GEMM_ANY):
        monkeypatch.setattr(L.GemmLaunch, "__init__", _forced_path_init(path))
        from cubed_amd.runtime.executors.gpu import GpuDagExecutor

        e = GpuDagExecutor("cuda:0")
        spec = cubed.Spec(allowed_mem="2GB", executor=e)
        a = cubed.from_array(x, chunks=(100, 128), spec=spec)
        b = cubed.from_array(y, chunks=(128, 136), spec=spec)
        if dt == "bf16":
            a, b = xp.astype(a, xp.bfloat16), xp.astype(b, xp.bfloat16)
        res[path] = xp.matmul(a, b).compute()
        assert _launches(e)[0].kernel_path() == path
    rnd = _bf16_round if dt == "bf16" else (lambda v: v)
    for got in res.values():
        _check_bound(got, rnd(x).astype(np.float64), rnd(y).astype(np.float64), 640,
                     out_bf16=(dt == "bf16"))


_orig_init = L.GemmLaunch.__init__


def _forced_path_init(path):
    def init(self, tasks, segs, in_code, out_code, device, zero_ptr, path_=None, grid=None, scratch=None):
        _orig_init(self, tasks, segs, in_code, out_code, device, zero_ptr, path=path)
    return init


def test_ragged_k_takes_element_path(ex):
    """A last k chunk shorter than the 64-deep K tile: the element kernel
    (auto-selected), still exact to the bound."""
    x, y = _operands((130, 300), (300, 72), 5)
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    a = xp.astype(cubed.from_array(x, chunks=(64, 130), spec=spec), xp.bfloat16)
    b = xp.astype(cubed.from_array(y, chunks=(130, 72), spec=spec), xp.bfloat16)
    got = xp.matmul(a, b).compute()
    assert _launches(ex)[0].kernel_path() == nat.GEMM_ANY
    _check_bound(got, _bf16_round(x).astype(np.float64), _bf16_round(y).astype(np.float64), 300,
                 out_bf16=True)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_unfused_per_chunk_products(ex, dt):
    """With the k-sum fusion off, every (i, k, j) task is a one-segment chain
    writing its partial product, then the reference's sum reduction runs:
    the reference's own plan, same bound (+ the bf16 rounding of each
    partial for bf16)."""
    ex.fuse_gemm_sums = False
    x, y = _operands((256, 512), (512, 128), 9)
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    a = cubed.from_array(x, chunks=(128, 128), spec=spec)
    b = cubed.from_array(y, chunks=(128, 128), spec=spec)
    if dt == "bf16":
        a, b = xp.astype(a, xp.bfloat16), xp.astype(b, xp.bfloat16)
        x64, y64 = _bf16_round(x).astype(np.float64), _bf16_round(y).astype(np.float64)
    else:
        x64, y64 = x.astype(np.float64), y.astype(np.float64)
    got = xp.matmul(a, b).compute()
    gl = _launches(ex)
    assert len(gl) == 1 and all(int(t["nseg"]) == 1 for t in gl[0].tasks) and gl[0].n == 2 * 4 * 1
    if dt == "bf16":
        exp = x64 @ y64
        scale = np.abs(x64) @ np.abs(y64)
        # 4 partials each rounded to bf16 (2^-9 relative of the partial's scale) + the final rounding
        assert np.all(np.abs(got - exp) <= 5 * 2.0 ** -8 * scale)
    else:
        _check_bound(got, x64, y64, 512)


def test_matmul_int64_exact(ex):
    r = np.random.default_rng(4)
    x = r.integers(-50, 50, (90, 130)).astype(np.int64)
    y = r.integers(-50, 50, (130, 70)).astype(np.int64)
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    got = xp.matmul(cubed.from_array(x, chunks=(40, 60), spec=spec),
                    cubed.from_array(y, chunks=(60, 30), spec=spec)).compute()
    assert got.dtype == np.int64 and np.array_equal(got, x @ y)


def test_matmul_f64_bound(ex):
    r = np.random.default_rng(6)
    x = r.random((100, 700)) - 0.5
    y = r.random((700, 90)) - 0.5
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    got = xp.matmul(cubed.from_array(x, chunks=(64, 200), spec=spec),
                    cubed.from_array(y, chunks=(200, 64), spec=spec)).compute()
    exp = x @ y
    scale = np.abs(x) @ np.abs(y)
    assert got.dtype == np.float64
    assert np.all(np.abs(got - exp) <= 700 * 2.0 ** -53 * scale)


def test_bf16_astype_round_trip(ex):
    """astype to bf16 rounds to nearest even (ties, inf, overflow, subnormals
    as torch does; NaN stays NaN); back to f32 it is exact."""
    import torch

    v = np.array([1.0, 1.00390625, 1.01171875, -3.14159, 2.5e-3, np.nan, np.inf, -np.inf, 3.4e38,
                  1e-40, 0.0, -0.0] * 11, dtype=np.float32)
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    a = cubed.from_array(v, chunks=(50,), spec=spec)
    got = xp.astype(xp.astype(a, xp.bfloat16), xp.float32).compute()
    exp = torch.from_numpy(v).to(torch.bfloat16).float().numpy()
    nan = np.isnan(exp)
    assert np.array_equal(np.isnan(got), nan)  # NaN payloads differ (torch: 0xFFFF), NaN-ness not
    assert np.array_equal(got[~nan].view(np.uint32), exp[~nan].view(np.uint32))


@pytest.mark.parametrize("shapes", [((600, 1200), (1200, 704), (300, 400), (400, 352)),    # 2 x 2 regular grid
                                    ((700, 1304), (1304, 1000), (300, 400), (400, 352))])  # ragged last row / column
@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_grid_tiling_bit_identical(gpu_executor, shapes, dt, monkeypatch):
    """f32 chains over a regular chunk grid run as ONE grid-tiled launch
    (cubed_gemm_chain_grid: 256 x 256 tiles over the whole matrix, tiles
    straddling chunk boundaries) -- bit-identical to the per-chunk tiling
    (each output element is the same f32 chain over K), and within the
    bound of the f64 product (K = 1304: four k chunks of 400 / 104)."""
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    sa, sb, ca, cb = shapes
    x, y = _operands(sa, sb, 21)
    res = {}
    monkeypatch.setattr(L.GemmLaunch, "GRID_INPUTS", {ir.dtype_code(np.float32), ir.dtype_code(ir.bfloat16)})
    # packed operands (the default), the unpacked grid kernels, per-chunk tiles
    for variant, grid, packed in (("packed", True, True), ("grid", True, False), ("chunk", False, False)):
        monkeypatch.setattr(L.GemmLaunch, "GRID", grid)
        monkeypatch.setattr(L.GemmLaunch, "PACKED", packed)
        e = GpuDagExecutor("cuda:0")
        spec = cubed.Spec(allowed_mem="2GB", executor=e)
        a = cubed.from_array(x, chunks=ca, spec=spec)
        b = cubed.from_array(y, chunks=cb, spec=spec)
        if dt == "bf16":
            a, b = xp.astype(a, xp.bfloat16), xp.astype(b, xp.bfloat16)
        res[variant] = xp.matmul(a, b).compute()
        gl = _launches(e)
        assert len(gl) == 1 and (gl[0].grid is not None) == grid and (gl[0].packed is not None) == packed
        if grid:
            assert gl[0].grid == (-(-sa[0] // ca[0]), -(-sb[1] // cb[1]))
    for variant in ("grid", "chunk"):
        assert np.array_equal(res["packed"].view(np.uint32), res[variant].view(np.uint32)), variant
    res[True] = res["packed"]
    if dt == "bf16":
        x64, y64 = _bf16_round(x).astype(np.float64), _bf16_round(y).astype(np.float64)
    else:
        x64, y64 = x.astype(np.float64), y.astype(np.float64)
    _check_bound(res[True], x64, y64, sa[1], out_bf16=(dt == "bf16"))


def test_grid_check_refuses_irregular_tables(built):
    """The host check: chunks narrower than a tile, bf16, or a task table
    that is not a chunk grid stay on the per-chunk launch."""
    tasks = np.zeros(4, dtype=nat.CHAIN_DTYPE)
    segs = np.zeros(4, dtype=nat.SEG_DTYPE)
    for t in range(4):
        segs[t] = (4096 * (t + 1), 8192 * (t + 1), 64, 64, 128, 0)
        tasks[t] = (65536 * (t + 1), 128, 128, 128, t, 1, 64, 0)
    L_ = nat.lib()
    args = (tasks.ctypes.data, 2, 2, segs.ctypes.data, 4)
    assert L_.cubed_gemm_grid_check(*args, ir.dtype_code(np.float32), ir.dtype_code(np.float32)) != 0  # 128 < 256
    tasks["m"], tasks["n"], tasks["ldc"] = 256, 256, 256
    segs["ldb"] = 256
    assert L_.cubed_gemm_grid_check(*args, ir.dtype_code(np.float32), ir.dtype_code(np.float32)) == 0
    assert L_.cubed_gemm_grid_check(*args, ir.dtype_code(ir.bfloat16), ir.dtype_code(np.float32)) == 0
    assert L_.cubed_gemm_grid_check(*args, ir.dtype_code(np.float64), ir.dtype_code(np.float64)) != 0
    tasks["ktot"][3] = 128
    assert L_.cubed_gemm_grid_check(*args, ir.dtype_code(np.float32), ir.dtype_code(np.float32)) != 0


@pytest.mark.parametrize("shapes", [((700, 1144), (1144, 392), (300, 520), (520, 256)),  # ragged M, N; K edge mid-tile
                                    ((512, 2048), (2048, 512), (256, 512), (512, 256))])  # whole tiles
def test_packed_bf16_bit_identical(gpu_executor, shapes, monkeypatch):
    """bf16 chains over a regular chunk grid of one product run packed
    (cubed_gemm_chain_packed: A and B^T rewritten into the GEMM's LDS image,
    then whole-matrix tiles) -- bit-identical to the per-chunk one-wave
    kernel (each element the same f32 chain over K in the same order), and
    within the bound of the f64 product."""
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    sa, sb, ca, cb = shapes
    x, y = _operands(sa, sb, 23)
    res = {}
    for packed in (True, False):
        monkeypatch.setattr(L.GemmLaunch, "PACKED", packed)
        e = GpuDagExecutor("cuda:0")
        spec = cubed.Spec(allowed_mem="2GB", executor=e)
        a = xp.astype(cubed.from_array(x, chunks=ca, spec=spec), xp.bfloat16)
        b = xp.astype(cubed.from_array(y, chunks=cb, spec=spec), xp.bfloat16)
        res[packed] = xp.matmul(a, b).compute()
        gl = _launches(e)
        assert len(gl) == 1 and (gl[0].packed is not None) == packed
    assert np.array_equal(res[True].view(np.uint32), res[False].view(np.uint32))
    _check_bound(res[True], _bf16_round(x).astype(np.float64), _bf16_round(y).astype(np.float64), sa[1],
                 out_bf16=True)


@pytest.mark.parametrize("in_dt,out_dt", [("bf16", "f32"), ("f32", "f32"), ("bf16", "bf16")])
def test_packed_abi_accumulate(gpu_executor, in_dt, out_dt):
    """The C ABI directly: accumulate = 1 (C += A @ B), chunk tables of one
    product (3 x 2 chunks, ragged last row / column, K segments 520 / 520 /
    104): cubed_gemm_chain_packed equals cubed_gemm_chain bit for bit (bf16
    output: the paired-column stores of the packed epilogue); a short
    workspace is refused."""
    import torch

    cast = (lambda t: t.bfloat16()) if in_dt == "bf16" else (lambda t: t)
    ocast = (lambda t: t.bfloat16()) if out_dt == "bf16" else (lambda t: t)

    ti, tj, cm, cn, ks = 3, 2, 300, 256, [520, 520, 104]
    ms = [cm, cm, 100]
    ns = [cn, 136]
    r = np.random.default_rng(31)
    dev = "cuda:0"
    Ach = {(I, s): cast(torch.from_numpy(r.random((ms[I], k), dtype=np.float32) - 0.5).to(dev))
           for I in range(ti) for s, k in enumerate(ks)}
    Bch = {(s, J): cast(torch.from_numpy(r.random((k, ns[J]), dtype=np.float32) - 0.5).to(dev))
           for J in range(tj) for s, k in enumerate(ks)}
    C0 = {(I, J): ocast(torch.from_numpy(r.random((ms[I], ns[J]), dtype=np.float32)).to(dev))
          for I in range(ti) for J in range(tj)}
    outs = []
    for _ in range(2):
        C = {key: v.clone() for key, v in C0.items()}
        tasks = np.zeros(ti * tj, dtype=nat.CHAIN_DTYPE)
        segs = np.zeros(ti * tj * len(ks), dtype=nat.SEG_DTYPE)
        for I in range(ti):
            for J in range(tj):
                t = I * tj + J
                tasks[t] = (C[I, J].data_ptr(), ms[I], ns[J], ns[J], t * len(ks), len(ks), sum(ks), 1)
                for s, k in enumerate(ks):
                    segs[t * len(ks) + s] = (Ach[I, s].data_ptr(), Bch[s, J].data_ptr(), k, k, ns[J], 0)
        outs.append((C, tasks, segs))
    Lb = nat.lib()
    bf = ir.dtype_code(ir.bfloat16) if in_dt == "bf16" else ir.dtype_code(np.float32)  # (the input code)
    f32 = ir.dtype_code(ir.bfloat16) if out_dt == "bf16" else ir.dtype_code(np.float32)  # (the output code)
    zero = torch.zeros(64, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    C, tasks, segs = outs[0]
    d_t = torch.from_numpy(tasks.view(np.uint8).copy()).to(dev)
    d_s = torch.from_numpy(segs.view(np.uint8).copy()).to(dev)
    nat.check(Lb.cubed_gemm_chain(tasks.ctypes.data, d_t.data_ptr(), len(tasks), segs.ctypes.data, d_s.data_ptr(),
                                  len(segs), bf, f32, zero.data_ptr(), nat.GEMM_AUTO, stream), "cubed_gemm_chain")
    C, tasks, segs = outs[1]
    d_t2 = torch.from_numpy(tasks.view(np.uint8).copy()).to(dev)
    d_s2 = torch.from_numpy(segs.view(np.uint8).copy()).to(dev)
    nbytes = Lb.cubed_gemm_pack_bytes(tasks.ctypes.data, ti, tj, segs.ctypes.data, len(segs), bf, f32)
    assert nbytes == ((3 + 2) * 18 * 32768 if in_dt == "bf16" else (3 + 2) * 72 * 16384) + 8 * 128  # + round counters
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    assert ws.data_ptr() % 256 == 0
    rc = Lb.cubed_gemm_chain_packed(tasks.ctypes.data, d_t2.data_ptr(), ti, tj, segs.ctypes.data, d_s2.data_ptr(),
                                    len(segs), bf, f32, ws.data_ptr(), nbytes - 32768, stream)
    assert rc == -4 and b"workspace" in Lb.cubed_last_error()
    nat.check(Lb.cubed_gemm_chain_packed(tasks.ctypes.data, d_t2.data_ptr(), ti, tj, segs.ctypes.data,
                                         d_s2.data_ptr(), len(segs), bf, f32, ws.data_ptr(), nbytes, stream),
              "cubed_gemm_chain_packed")
    torch.cuda.synchronize()
    for key in C0:
        a, b = outs[0][0][key].float().cpu().numpy(), outs[1][0][key].float().cpu().numpy()
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), key
    # and the product itself: C0 + A @ B within the f32 bound
    A = torch.cat([torch.cat([Ach[I, s] for s in range(len(ks))], 1) for I in range(ti)], 0).double().cpu().numpy()
    B = torch.cat([torch.cat([Bch[s, J] for J in range(tj)], 1) for s in range(len(ks))], 0).double().cpu().numpy()
    Cin = torch.cat([torch.cat([C0[I, J] for J in range(tj)], 1) for I in range(ti)], 0).double().cpu().numpy()
    got = torch.cat([torch.cat([outs[1][0][I, J] for J in range(tj)], 1) for I in range(ti)], 0).double().cpu().numpy()
    exp = Cin + A @ B
    bound = 8 * np.sqrt(sum(ks)) * U * (np.abs(Cin) + np.abs(A) @ np.abs(B))
    if out_dt == "bf16":
        bound = bound + 2.0 ** -8 * np.abs(exp)
    assert np.all(np.abs(got - exp) <= bound)


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("shapes", [
    ((300, 32), (32, 264), (256, 32), (32, 256)),          # K = one 32-deep step, one segment
    ((520, 200), (200, 520), (260, 40), (40, 264)),         # five 40-deep segments, K % 64 != 0
    ((256, 1000), (1000, 256), (256, 1000), (1000, 256)),   # one output chunk (ti = tj = 1)
    ((777, 3000), (3000, 600), (259, 600), (600, 296)),     # ragged everywhere, tiles straddle chunks
    # 47 x 20 tiles: xcd_lockstep's lockstep groups, its round-robin 32-tile runs and contiguous rest
    ((12000, 256), (256, 5120), (3000, 128), (128, 2560)),
])
def test_packed_matches_unpacked_edge_shapes(gpu_executor, dt, shapes, monkeypatch):
    """Packed vs unpacked kernels on edge geometries (a single K step,
    short segments, a single chunk, ragged rows / columns / k): bit for bit."""
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    sa, sb, ca, cb = shapes
    x, y = _operands(sa, sb, 41)
    res = {}
    for packed in (True, False):
        monkeypatch.setattr(L.GemmLaunch, "PACKED", packed)
        e = GpuDagExecutor("cuda:0")
        spec = cubed.Spec(allowed_mem="2GB", executor=e)
        a = cubed.from_array(x, chunks=ca, spec=spec)
        b = cubed.from_array(y, chunks=cb, spec=spec)
        if dt == "bf16":
            a, b = xp.astype(a, xp.bfloat16), xp.astype(b, xp.bfloat16)
        res[packed] = xp.matmul(a, b).compute()
        gl = _launches(e)
        n_tasks = (-(-sa[0] // ca[0])) * (-(-sb[1] // cb[1]))
        if packed and n_tasks > 1 and sa[1] > ca[1]:  # (one k chunk: the per-chunk product lowering)
            assert gl[0].packed is not None
    assert np.array_equal(res[True].view(np.uint32), res[False].view(np.uint32))
    rnd = _bf16_round if dt == "bf16" else (lambda v: v)
    _check_bound(res[True], rnd(x).astype(np.float64), rnd(y).astype(np.float64), sa[1], out_bf16=(dt == "bf16"))


@pytest.mark.parametrize("packed", [True, False])
def test_matmul_against_the_reference_algorithm(gpu_executor, packed, monkeypatch):
    """f32 (the reference's dtype) on the packed and the unpacked GEMM against
    the oracle's restatement of linear_algebra_functions.py:13-78 (f32 chunk
    products, then the f32 k-chunk sum rounds of _sum_wo_cat).  The two sum
    the same products in different orders, so each is within 8 sqrt(K)
    2^-24 sum|a||b| of the exact product and they are within twice that of
    each other."""
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor
    from oracle import cubed_ref as R

    r = np.random.default_rng(77)
    x = (r.random((1024, 2048)) - 0.5).astype(np.float32)
    y = (r.random((2048, 768)) - 0.5).astype(np.float32)
    ca, cb = (512, 512), (512, 384)
    monkeypatch.setattr(L.GemmLaunch, "PACKED", packed)
    e = GpuDagExecutor("cuda:0")
    spec = cubed.Spec(allowed_mem="2GB", executor=e)
    got = xp.matmul(cubed.from_array(x, chunks=ca, spec=spec), cubed.from_array(y, chunks=cb, spec=spec)).compute()
    gl = _launches(e)
    assert (gl[0].packed is not None) == packed
    ref = R.matmul(x, y, ca, cb)
    scale = np.abs(x).astype(np.float64) @ np.abs(y).astype(np.float64)
    bound = 8 * np.sqrt(2048) * 2.0 ** -24 * scale
    assert got.dtype == ref.dtype == np.float32
    assert np.all(np.abs(got.astype(np.float64) - ref) <= 2 * bound)
    exact = x.astype(np.float64) @ y.astype(np.float64)
    assert np.all(np.abs(got - exact) <= bound) and np.all(np.abs(ref - exact) <= bound)

