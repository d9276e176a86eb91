"""Complex dtypes on the MI355X executor (cubed_amd/complex.py): complex64 /
complex128 arrays stored as real + imaginary slabs, complex arithmetic
lowered to real expressions.  Checked against numpy on the same inputs:
exact for layout copies, parts, conjugation, negation, add/subtract,
comparisons and NaN/inf tests; multiply / divide / abs / sqrt / exp / log
within a few ulp of the magnitudes that enter each part (|z||w|, |z|/|w|,
|result|: a part may cancel, and numpy's SIMD loops may contract
multiply-adds where the kernels are built with -ffp-contract=off); sums
(complex64 -> complex128 as statistical_functions.py:137-147) within 1e-12.
Reference anchors: array_api/elementwise_functions.py abs/conj/real/imag,
array_object.py __abs__/__complex__, statistical_functions.py sum,
nan_functions.py nansum."""

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ex(gpu_executor):
    return gpu_executor


def mkspec(ex):
    return cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)


def cdata(shape, dtype, seed, specials=True):
    rng = np.random.default_rng(seed)
    z = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(dtype)
    if specials:
        f = z.reshape(-1)
        f[0] = 0
        f[1] = complex(np.inf, 1)
        f[2] = complex(1, np.nan)
        f[3] = complex(-0.0, 2.5)
        f[4] = complex(3, 0)
        f[5] = complex(-2, -0.0)
    return z


def close(got, exp, dtype, ulps=4, scale=None):
    """Each part within ulps x eps x scale (default: the modulus of the
    expected complex value -- the error of a part is bounded relative to
    the magnitudes that enter it, not to the part, which may cancel)."""
    got, exp = np.asarray(got), np.asarray(exp)
    assert got.dtype == exp.dtype, (got.dtype, exp.dtype)
    eps = np.finfo(np.dtype(dtype)).eps
    if scale is None:
        scale = np.abs(exp)
    scale = np.maximum(np.where(np.isfinite(scale), scale, 0), np.finfo(np.dtype(dtype)).tiny)
    for part in ((lambda a: a.real), (lambda a: a.imag)) if got.dtype.kind == "c" else ((lambda a: a),):
        g, e = part(got), part(exp)
        both_nan = np.isnan(g) & np.isnan(e)
        same = (g == e) | both_nan
        ok = same | (np.abs(g - e) <= ulps * eps * scale)
        assert ok.all(), (g[~ok][:5], e[~ok][:5])


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_roundtrip_parts_and_exact_ops(ex, dtype):
    Z = cdata((13, 11), dtype, 1)
    W = cdata((13, 11), dtype, 2, specials=False)
    spec = mkspec(ex)
    z = cubed.from_array(Z, chunks=(5, 4), spec=spec)
    w = cubed.from_array(W, chunks=(5, 4), spec=spec)
    got = z.compute()
    assert got.dtype == Z.dtype and np.array_equal(got, Z, equal_nan=True)
    for fn, ref in [(xp.real, np.real), (xp.imag, np.imag), (xp.conj, np.conj),
                    (xp.negative, np.negative), (xp.isnan, np.isnan), (xp.isinf, np.isinf),
                    (xp.isfinite, np.isfinite)]:
        r = fn(z).compute()
        e = ref(Z)
        assert r.dtype == e.dtype and np.array_equal(r, e, equal_nan=True), fn.__name__
    for op, ref in [("add", np.add), ("subtract", np.subtract), ("equal", np.equal),
                    ("not_equal", np.not_equal)]:
        r = getattr(xp, op)(z, w).compute()
        e = ref(Z, W)
        assert r.dtype == e.dtype and np.array_equal(r, e, equal_nan=True), op
    # mixed with a real array and a python scalar
    X = np.random.default_rng(3).random((13, 11)).astype("f4" if dtype == "complex64" else "f8")
    x = cubed.from_array(X, chunks=(5, 4), spec=spec)
    r = (x + z - 2).compute()
    assert np.array_equal(r, X + Z - np.asarray(2, dtype=Z.dtype), equal_nan=True)


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_multiply_divide_abs_and_functions(ex, dtype):
    Z = cdata((9, 17), dtype, 4)
    W = cdata((9, 17), dtype, 5, specials=False)
    W.reshape(-1)[7] = 0  # 0 divisor: numpy's inf/nan results
    spec = mkspec(ex)
    z = cubed.from_array(Z, chunks=(4, 8), spec=spec)
    w = cubed.from_array(W, chunks=(4, 8), spec=spec)
    with np.errstate(all="ignore"):
        close((z * w).compute(), Z * W, dtype, scale=np.abs(Z) * np.abs(W))
        close((z / w).compute(), Z / W, dtype, scale=np.abs(Z) / np.abs(W))
        close(abs(z).compute(), np.abs(Z), dtype)
        close(xp.square(w).compute(), np.square(W), dtype)
        close(xp.sqrt(w).compute(), np.sqrt(W), dtype, ulps=8)
        close(xp.exp(w).compute(), np.exp(W), dtype, ulps=16)
        close(xp.log(w).compute(), np.log(W), dtype, ulps=16)


def test_astype_where_and_layout(ex):
    Z = cdata((20, 12), "complex128", 6, specials=False)
    spec = mkspec(ex)
    z = cubed.from_array(Z, chunks=(6, 5), spec=spec)
    r = xp.astype(z, xp.complex64).compute()
    assert r.dtype == np.complex64 and np.array_equal(r, Z.astype(np.complex64))
    X = np.arange(240.0).reshape(20, 12)
    x = cubed.from_array(X, chunks=(6, 5), spec=spec)
    r = xp.astype(x, xp.complex128).compute()
    assert np.array_equal(r, X.astype(np.complex128))
    c = xp.where(x > 100, z, xp.conj(z)).compute()
    assert np.array_equal(c, np.where(X > 100, Z, np.conj(Z)))
    # rechunk / index / concat move both slabs bit-exactly
    assert np.array_equal(z.rechunk((20, 3)).compute(), Z)
    assert np.array_equal(z[3:17, 1:].compute(), Z[3:17, 1:])
    assert np.array_equal(xp.concat([z, z[:4]], axis=0).compute(), np.concatenate([Z, Z[:4]]))
    assert complex(z[2, 3]) == complex(Z[2, 3])


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_sum_and_nansum(ex, dtype):
    Z = cdata((40, 30), dtype, 7, specials=False)
    Z[3, 4] = complex(np.nan, 1)
    Z[10, 2] = complex(2, np.nan)
    spec = mkspec(ex)
    z = cubed.from_array(Z, chunks=(7, 9), spec=spec)
    for axis in (0, 1, None):
        got = xp.sum(z, axis=axis).compute()
        exp = np.sum(Z, axis=axis, dtype=np.complex128)
        assert got.dtype == np.complex128
        assert np.allclose(got, exp, rtol=1e-12, atol=0, equal_nan=True), axis
        got = cubed.nansum(z, axis=axis).compute()
        exp = np.nansum(Z, axis=axis, dtype=np.complex128)
        assert np.allclose(got, exp, rtol=1e-12, atol=0, equal_nan=True), axis
    # sum of a complex expression fused into the reduction
    got = xp.sum(z * xp.conj(z), axis=0).compute()
    exp = np.sum(Z * np.conj(Z), axis=0, dtype=np.complex128)
    assert np.allclose(got, exp, rtol=1e-6 if dtype == "complex64" else 1e-12, equal_nan=True)


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_prod_and_nanprod(ex, dtype):
    """prod / nanprod of complex chunks: one pair reduction whose {re, im}
    accumulators multiply as complex numbers (cubed_rop CPROD), through the
    merge + combine rounds, against numpy's complex128 product.  np.nanprod
    through core ``reduction`` treats an element with a NaN part as 1
    (numpy's _replace_nan)."""
    from cubed_amd.core.ops import reduction

    rng = np.random.default_rng(31)
    Z = (rng.uniform(0.9, 1.1, (40, 30)) * np.exp(1j * rng.uniform(-np.pi, np.pi, (40, 30)))).astype(dtype)
    Z[3, 4] = complex(np.nan, 1)
    Z[10, 2] = complex(2, np.nan)
    spec = mkspec(ex)
    z = cubed.from_array(Z, chunks=(7, 9), spec=spec)
    for axis in (0, 1, None):
        got = xp.prod(z, axis=axis).compute()
        exp = np.prod(Z, axis=axis, dtype=np.complex128)
        assert got.dtype == np.complex128
        assert np.allclose(got, exp, rtol=1e-12, atol=0, equal_nan=True), axis
        got = reduction(z, np.nanprod, axis=axis, dtype=np.complex128,
                        extra_func_kwargs=dict(dtype=np.complex128)).compute()
        exp = np.nanprod(Z, axis=axis, dtype=np.complex128)
        assert np.allclose(got, exp, rtol=1e-12, atol=0, equal_nan=True), axis
    # many merge + combine rounds of the pair accumulators
    small = cubed.Spec(allowed_mem=20000, executor=ex)
    W = Z[:, :3].copy()
    W[np.isnan(W)] = 1
    got = xp.prod(cubed.from_array(W, chunks=(2, 3), spec=small), axis=0).compute()
    assert np.allclose(got, np.prod(W, axis=0, dtype=np.complex128), rtol=1e-12, atol=0)


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_complex_matmul(ex, dtype):
    """Complex matmul as chained real GEMMs over the part slabs
    (gemm_chains.complex_chain_tables; complex64 on the f32 MFMA kernel,
    complex128 on the f64 element kernel), ragged chunks, against numpy's
    complex128 product; bound 8 sqrt(2K) eps sum|x||y| per part."""
    X = cdata((150, 128), dtype, 9, specials=False)
    Y = cdata((128, 172), dtype, 10, specials=False)
    spec = mkspec(ex)
    got = xp.matmul(cubed.from_array(X, chunks=(64, 48), spec=spec),
                    cubed.from_array(Y, chunks=(48, 80), spec=spec)).compute()
    assert got.dtype == np.dtype(dtype)
    exp = X.astype(np.complex128) @ Y.astype(np.complex128)
    scale = np.abs(X).astype(np.float64) @ np.abs(Y).astype(np.float64)
    bound = 8 * np.sqrt(2 * 128) * np.finfo(np.dtype(dtype)).eps * scale
    assert np.all(np.abs(got.real - exp.real) <= bound)
    assert np.all(np.abs(got.imag - exp.imag) <= bound)


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_trigonometric_hyperbolic_and_pow(ex, dtype):
    """sin/cos/tan/sinh/cosh/tanh of complex values (npymath's finite-value
    formulas) and complex powers (exp(w log z)) against numpy, finite
    inputs incl. a zero imaginary part and |re| > 22 for tanh; bound: 64 ulps
    of the modulus of the inputs' magnitudes (pow: of |z ** w|)."""
    Z = cdata((6, 7), dtype, 11, specials=False) * 2
    Z.reshape(-1)[0] = complex(1.5, 0)
    Z.reshape(-1)[1] = complex(-30, 0.7)
    Z.reshape(-1)[2] = complex(25, -1.2)
    W = cdata((6, 7), dtype, 12, specials=False) * 0.5
    W.reshape(-1)[3] = 0
    spec = mkspec(ex)
    z = cubed.from_array(Z, chunks=(3, 4), spec=spec)
    w = cubed.from_array(W, chunks=(3, 4), spec=spec)
    with np.errstate(all="ignore"):
        for name in ("sin", "cos", "tan", "sinh", "cosh", "tanh"):
            got = getattr(xp, name)(z).compute()
            exp = getattr(np, name)(Z)
            close(got, exp, dtype, ulps=64, scale=np.maximum(np.abs(exp), 1.0))
        got = xp.pow(z, w).compute()
        exp = np.power(Z, W)
        close(got, exp, dtype, ulps=64, scale=np.maximum(np.abs(exp), 1e-30))


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_inverse_trigonometric_hyperbolic_and_logs(ex, dtype):
    """asin/acos/atan/asinh/acosh/atanh of complex values (Kahan's branch-cut
    formulas, the principal branches of numpy's C99 casin & co.) and
    log1p/expm1/log2/log10 against numpy, finite inputs incl. points on the
    real and imaginary axes (|x| > 1 on the cuts, with a +0 / -0 imaginary
    part); bound: 64 ulps of max(|result|, 1) (atan / atanh: 256, their
    real part ~ log1p of a ratio near the unit circle)."""
    Z = cdata((6, 7), dtype, 13, specials=False) * 2
    f = Z.reshape(-1)
    f[0], f[1], f[2], f[3] = complex(2, 0), complex(-3, -0.0), complex(0, 0.5), complex(0.3, 0)
    f[4], f[5] = complex(1e-3, -2e-3), complex(-0.0, 1.5)
    spec = mkspec(ex)
    z = cubed.from_array(Z, chunks=(3, 4), spec=spec)
    names = {"asin": "arcsin", "acos": "arccos", "atan": "arctan", "asinh": "arcsinh",
             "acosh": "arccosh", "atanh": "arctanh", "log1p": "log1p", "expm1": "expm1",
             "log2": "log2", "log10": "log10"}
    with np.errstate(all="ignore"):
        for name, npname in names.items():
            got = getattr(xp, name)(z).compute()
            exp = getattr(np, npname)(Z)
            close(got, exp, dtype, ulps=256 if name in ("atan", "atanh") else 64,
                  scale=np.maximum(np.abs(exp), 1.0))


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_integer_powers_bit_exact(ex, dtype):
    """npy_cpow multiplies out a constant integral exponent
    (|n| < 100): z**2 == z*z exactly, (1j)**2 == -1 + 0j with a ZERO
    imaginary part, (-2)**2 == 4 + 0j, z**-3 == 1 / z**3 (Smith's division),
    0**n == 0 (n > 0) / nan (n < 0).  The executor takes the same branch,
    so the results are bit-identical to numpy, signed zeros included."""
    Z = cdata((5, 8), dtype, 13, specials=False)
    f = Z.reshape(-1)
    f[0], f[1], f[2], f[3], f[4] = 1j, -2, 0, complex(-0.0, 1.5), complex(3.0, -0.0)
    spec = mkspec(ex)
    z = cubed.from_array(Z, chunks=(3, 4), spec=spec)
    pw = np.dtype(dtype).type
    for n in (1, 2, 3, 5, 7, -1, -2, -3, 10, 99, 0):
        with np.errstate(all="ignore"):
            exp = np.power(Z, pw(n))
        got = (z ** n).compute()
        assert got.dtype == exp.dtype
        for part in ("real", "imag"):
            g, e = getattr(got, part), getattr(exp, part)
            both_nan = np.isnan(g) & np.isnan(e)
            bits = g.view(np.uint32 if dtype == "complex64" else np.uint64) == \
                e.view(np.uint32 if dtype == "complex64" else np.uint64)
            assert (bits | both_nan).all(), (n, part, g[~(bits | both_nan)][:4], e[~(bits | both_nan)][:4])
    assert (z ** 2).compute().reshape(-1)[0].imag == 0.0
