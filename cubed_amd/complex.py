"""Complex dtypes (complex64 / complex128) on the MI355X path.

The reference computes complex chunks with numpy (array_api/dtypes.py
complex64/complex128; elementwise_functions.py real/imag/conj/abs and the
arithmetic operators; statistical_functions.py sum/prod promoting complex64
to complex128; nan_functions.py nansum).  Here a complex array is stored
as two HBM slabs per chunk -- the ``real`` and ``imag`` parts, each a real
array of the part dtype (f32 / f64), the same SoA layout as the structured
reduction intermediates (storage.DeviceArray) -- and every chunk program
that touches complex values is rewritten, before lowering, into a program
over real expressions (``split_program``): a complex leaf becomes its two
part leaves, complex arithmetic becomes the real formulas numpy evaluates
(npymath's nc_sum/nc_diff/nc_prod and Smith's division, hypot for abs), a
complex output becomes the structured output {real, imag}, and a complex
reduction field becomes one field per part (a sum: two independent sums; a
product: the pair reduction cprod, whose {re, im} accumulators multiply as
complex numbers).  Layout copies (rechunk, index, concat) move each part slab.

Powers (exp(w log z)), sin / cos / tan and their hyperbolic forms (the
FreeBSD / npymath formulas numpy uses for finite values) are rewritten too.
Ops with no real-pair form here (inverse trigonometric functions, ordering
comparisons) raise LoweringError.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, Optional, Tuple, Union

import numpy as np

from . import ir

PARTS = ("real", "imag")


def is_complex(dt) -> bool:
    return np.dtype(dt).kind == "c"


def part_dtype(dt) -> np.dtype:
    """complex64 -> float32, complex128 -> float64."""
    dt = np.dtype(dt)
    return np.dtype(f"f{dt.itemsize // 2}")


def complex_dtype(part) -> np.dtype:
    return np.dtype(f"c{np.dtype(part).itemsize * 2}")


class ComplexLoweringError(Exception):
    pass


def _err(msg):
    from .lowering import LoweringError

    return LoweringError(msg)


# a decomposed value: ("r", expr) or ("c", re, im)
Val = Union[Tuple[str, ir.Expr], Tuple[str, ir.Expr, ir.Expr]]


def _bin(op, a, b, dt):
    return ir.Binary(op, a, b, np.dtype(dt))


def _un(op, a, dt):
    return ir.Unary(op, a, np.dtype(dt))


def _const(v, dt):
    return ir.Const(np.array(v, dtype=dt).item(), np.dtype(dt))


def _const_value(e, const_args):
    """The value of a constant expression (a Const, or an argument reading a
    constant, possibly cast), else None."""
    while isinstance(e, ir.Cast):
        e = e.x
    if isinstance(e, ir.Const):
        return e.value
    if isinstance(e, ir.Arg) and e.index in const_args:
        v = const_args[e.index]
        if e.field == "real":
            return np.real(v)
        if e.field == "imag":
            return np.imag(v)
        return None if e.field is not None else v
    return None


def _integral_exponent(br, bi, const_args):
    """n when the exponent is the constant n + 0i with n integral and
    |n| < 100 (npy_cpow's ``(n = (npy_intp)br) == br`` test), else None."""
    r, i = _const_value(br, const_args), _const_value(bi, const_args)
    if r is None or i is None:
        return None
    try:
        r, i = float(np.real(r)), float(np.real(i))
    except (TypeError, ValueError):
        return None
    if i != 0.0 or not np.isfinite(r) or r != int(r) or not -100 < int(r) < 100:
        return None
    return int(r)


class _Splitter:
    def __init__(self):
        self.memo: Dict[int, Val] = {}

    def pair(self, e: ir.Expr, part) -> Tuple[ir.Expr, ir.Expr]:
        """(re, im) of e as values of dtype ``part`` (a real e gets im = 0)."""
        v = self.split(e)
        if v[0] == "c":
            return ir.cast(v[1], part), ir.cast(v[2], part)
        return ir.cast(v[1], part), _const(0, part)

    def split(self, e: ir.Expr) -> Val:
        key = id(e)
        if key in self.memo:
            return self.memo[key]
        out = self._split(e)
        self.memo[key] = out
        return out

    def _split(self, e: ir.Expr) -> Val:
        dt = np.dtype(e.dtype)
        if isinstance(e, ir.Const):
            if is_complex(dt):
                v = complex(e.value)
                p = part_dtype(dt)
                return ("c", _const(v.real, p), _const(v.imag, p))
            return ("r", e)
        if isinstance(e, ir.Field):
            if is_complex(dt):
                p = part_dtype(dt)
                return ("c", ir.Field(e.name + "#re", p), ir.Field(e.name + "#im", p))
            return ("r", e)
        if isinstance(e, (ir.Arg, ir.Region)):  # incl. ReshapeArg, Concat
            if is_complex(dt):
                if e.field is not None:
                    raise _err("complex fields of structured arrays are not lowered")
                p = part_dtype(dt)
                return ("c", dataclasses.replace(e, dtype=p, field="real"),
                        dataclasses.replace(e, dtype=p, field="imag"))
            return ("r", e)
        if isinstance(e, ir.LEAF_TYPES):
            return ("r", e)
        if isinstance(e, ir.Cast):
            return self._cast(e)
        if isinstance(e, ir.Where):
            c = self.split(e.c)
            if c[0] == "c":
                raise _err("a complex where() condition")
            if is_complex(dt):
                p = part_dtype(dt)
                ar, ai = self.pair(e.a, p)
                br, bi = self.pair(e.b, p)
                return ("c", ir.Where(c[1], ar, br, p), ir.Where(c[1], ai, bi, p))
            return ("r", ir.Where(c[1], self.real(e.a), self.real(e.b), dt))
        if isinstance(e, ir.Unary):
            return self._unary(e)
        if isinstance(e, ir.Binary):
            return self._binary(e)
        raise _err(f"complex rewrite: unknown node {type(e).__name__}")

    def real(self, e):
        v = self.split(e)
        if v[0] == "c":
            raise _err("a complex value where a real one is required")
        return v[1]

    def _cast(self, e: ir.Cast) -> Val:
        dt = np.dtype(e.dtype)
        v = self.split(e.x)
        if is_complex(dt):
            p = part_dtype(dt)
            re, im = self.pair(e.x, p)
            return ("c", re, im)
        if v[0] == "r":
            return ("r", ir.cast(v[1], dt))
        # complex -> real (numpy discards the imaginary part); -> bool: z != 0
        if dt.kind == "b":
            p = np.dtype(v[1].dtype)
            z = _const(0, p)
            return ("r", _bin("logical_or", _bin("not_equal", v[1], z, np.bool_),
                              _bin("not_equal", v[2], z, np.bool_), np.bool_))
        return ("r", ir.cast(v[1], dt))

    def _unary(self, e: ir.Unary) -> Val:
        v = self.split(e.x)
        if v[0] == "r":
            if e.op == "conj":
                return ("r", e.x if np.dtype(e.x.dtype) == np.dtype(e.dtype) else ir.cast(e.x, e.dtype))
            if e.op in ("real",):
                return ("r", ir.cast(e.x, e.dtype))
            if e.op == "imag":
                return ("r", _const(0, e.dtype))
            return ("r", e)
        _, re, im = v
        p = np.dtype(re.dtype)
        op = e.op
        if op in ("negative",):
            return ("c", _un("negative", re, p), _un("negative", im, p))
        if op in ("positive",):
            return ("c", re, im)
        if op == "conj":
            return ("c", re, _un("negative", im, p))
        if op == "real":
            return ("r", re)
        if op == "imag":
            return ("r", im)
        if op == "abs":
            return ("r", _bin("hypot", re, im, p))
        if op == "isnan":
            return ("r", _bin("logical_or", _un("isnan", re, np.bool_), _un("isnan", im, np.bool_), np.bool_))
        if op == "isinf":
            return ("r", _bin("logical_or", _un("isinf", re, np.bool_), _un("isinf", im, np.bool_), np.bool_))
        if op == "isfinite":
            return ("r", _bin("logical_and", _un("isfinite", re, np.bool_), _un("isfinite", im, np.bool_),
                              np.bool_))
        if op == "square":
            return self._mul(re, im, re, im, p)
        if op == "reciprocal":
            return self._div(_const(1, p), _const(0, p), re, im, p)
        if op == "exp":
            # npy_cexp for finite values: exp(re) * (cos im, sin im); a zero
            # imaginary part stays exact (exp(inf + 0j) = inf + 0j)
            r = _un("exp", re, p)
            cr = _bin("multiply", r, _un("cos", im, p), p)
            ci = _bin("multiply", r, _un("sin", im, p), p)
            zero = _bin("equal", im, _const(0, p), np.bool_)
            return ("c", ir.Where(zero, r, cr, p), ir.Where(zero, im, ci, p))
        if op == "log":
            return ("c", _un("log", _bin("hypot", re, im, p), p), _bin("atan2", im, re, p))
        if op in ("log2", "log10"):
            # numpy: log(z) / log(base), part by part
            k = _const(1.0 / np.log(2.0 if op == "log2" else 10.0), p)
            return ("c", _bin("multiply", _un("log", _bin("hypot", re, im, p), p), k, p),
                    _bin("multiply", _bin("atan2", im, re, p), k, p))
        if op == "log1p":
            # log|1 + z| = log1p(2x + x^2 + y^2) / 2 (no cancellation for small z), arg = atan2(y, 1 + x)
            one = _const(1, p)
            t = _bin("add", _bin("multiply", re, _bin("add", _const(2, p), re, p), p), _bin("multiply", im, im, p), p)
            return ("c", _bin("multiply", _un("log1p", t, p), _const(0.5, p), p),
                    _bin("atan2", im, _bin("add", one, re, p), p))
        if op == "expm1":
            # numpy nc_expm1: (expm1(x) cos y - 2 sin^2(y/2), exp(x) sin y)
            s2 = _un("sin", _bin("multiply", im, _const(0.5, p), p), p)
            r = _bin("subtract", _bin("multiply", _un("expm1", re, p), _un("cos", im, p), p),
                     _bin("multiply", _const(2, p), _bin("multiply", s2, s2, p), p), p)
            return ("c", r, _bin("multiply", _un("exp", re, p), _un("sin", im, p), p))
        if op == "sqrt":
            return self._sqrt(re, im, p)
        if op in ("sinh", "cosh", "sin", "cos"):
            return self._hyp(op, re, im, p)
        if op in ("tanh", "tan"):
            if op == "tanh":
                return self._tanh(re, im, p)
            # tan z = -i tanh(i z), i z = (-im, re)
            _, a, b = self._tanh(_un("negative", im, p), re, p)
            return ("c", b, _un("negative", a, p))
        if op in ("asin", "acos", "asinh", "acosh", "atan", "atanh"):
            return self._inverse(op, re, im, p)
        if op == "sign":
            # numpy 2: z / |z|, 0 at 0
            a = _bin("hypot", re, im, p)
            z = _bin("equal", a, _const(0, p), np.bool_)
            return ("c", ir.Where(z, _const(0, p), _bin("divide", re, a, p), p),
                    ir.Where(z, _const(0, p), _bin("divide", im, a, p), p))
        raise _err(f"complex {op} is not lowered on the MI355X executor")

    def _hyp(self, op, re, im, p) -> Val:
        # npy_csinh / npy_ccosh for finite values (FreeBSD s_csinh.c):
        #   sinh z = (sinh x cos y, cosh x sin y), cosh z = (cosh x cos y, sinh x sin y),
        # y = 0 exact: sinh(x + 0i) = (sinh x, y), cosh(x + 0i) = (cosh x, x y);
        # sin z = -i sinh(i z) = (sin x cosh y, cos x sinh y),
        # cos z = cosh(i z) = (cos x cosh y, -sin x sinh y)
        if op in ("sin", "cos"):
            x, y = _un("negative", im, p), re  # i z
        else:
            x, y = re, im
        shx, chx = _un("sinh", x, p), _un("cosh", x, p)
        cy, sy = _un("cos", y, p), _un("sin", y, p)
        zero = _bin("equal", y, _const(0, p), np.bool_)
        if op in ("sinh", "sin"):
            a = ir.Where(zero, shx, _bin("multiply", shx, cy, p), p)
            b = ir.Where(zero, y, _bin("multiply", chx, sy, p), p)
        else:
            a = ir.Where(zero, chx, _bin("multiply", chx, cy, p), p)
            b = ir.Where(zero, _bin("multiply", x, y, p), _bin("multiply", shx, sy, p), p)
        if op == "sin":   # -i (a + i b) = (b, -a)
            return ("c", b, _un("negative", a, p))
        return ("c", a, b)

    def _inverse(self, op, re, im, p) -> Val:
        """Inverse trigonometric / hyperbolic functions on the principal
        branches numpy uses (C99 casin & co., branch cuts on the axes), from
        Kahan's acos ("Branch cuts for complex elementary functions", 1987),
        which avoids the cancellation of 1 - z^2:
            A = sqrt(1 - z), B = sqrt(1 + z):
            acos z = (2 atan2(re A, re B), asinh(im(conj(B) A)))
            asin z = pi/2 - acos z,  acosh z = +-i acos z (re >= 0)
            atanh z = (log1p(4x / ((1 - x)^2 + y^2)) / 4,
                       atan2(2y, (1 - x)(1 + x) - y^2) / 2)
            asinh z = -i asin(i z), atan z = -i atanh(i z).
        Finite inputs; |z| near the overflow threshold of the part type is
        not rescaled."""
        one = _const(1, p)
        if op in ("asinh", "atan"):
            # -i f(i z), i z = (-y, x); -i (a + i b) = (b, -a)
            _, a, b = self._inverse("asin" if op == "asinh" else "atanh", _un("negative", im, p), re, p)
            return ("c", b, _un("negative", a, p))
        if op == "atanh":
            x, y = re, im
            omx = _bin("subtract", one, x, p)
            d = _bin("add", _bin("multiply", omx, omx, p), _bin("multiply", y, y, p), p)
            r = _bin("multiply", _un("log1p", _bin("divide", _bin("multiply", _const(4, p), x, p), d, p), p),
                     _const(0.25, p), p)
            den = _bin("subtract", _bin("multiply", omx, _bin("add", one, x, p), p), _bin("multiply", y, y, p), p)
            i = _bin("multiply", _bin("atan2", _bin("multiply", _const(2, p), y, p), den, p), _const(0.5, p), p)
            return ("c", r, i)
        # acos (Kahan): A = sqrt(1 - z), B = sqrt(1 + z)
        _, ar, ai = self._sqrt(_bin("subtract", one, re, p), _un("negative", im, p), p)
        _, br, bi = self._sqrt(_bin("add", one, re, p), im, p)
        a = _bin("multiply", _const(2, p), _bin("atan2", ar, br, p), p)
        b = _un("asinh", _bin("subtract", _bin("multiply", br, ai, p), _bin("multiply", bi, ar, p), p), p)
        if op == "acos":
            return ("c", a, b)
        if op == "asin":
            # asin z = pi/2 - acos z (Kahan's asin part im(conj(A) B) is exactly
            # -im(conj(B) A)); the real part carries an absolute error of an ulp
            # of pi/2 rather than a relative one -- one fused program (the VM's
            # 6 registers do not hold both of Kahan's products)
            return ("c", _bin("subtract", _const(np.pi / 2, p), a, p), _un("negative", b, p))
        # acosh z = +-i acos z, the sign that makes the real part >= 0:
        # (|b|, copysign(a, -b)) -- im(acos z) carries the opposite sign of
        # im z, signed zeros included, so z need not stay live
        return ("c", _un("abs", b, p), _bin("copysign", a, _un("negative", b, p), p))

    def _tanh(self, re, im, p) -> Val:
        # npy_ctanh (FreeBSD s_ctanh.c, Kahan's algorithm) for finite values:
        #   |x| >= 22: (copysign(1, x), 4 sin y cos y exp(-2|x|))
        #   else t = tan y, beta = 1 + t^2, s = sinh x, rho = sqrt(1 + s^2),
        #        denom = 1 + beta s^2: (beta rho s / denom, t / denom)
        x, y = re, im
        one = _const(1, p)
        t = _un("tan", y, p)
        beta = _bin("add", one, _bin("multiply", t, t, p), p)
        sx = _un("sinh", x, p)
        s2 = _bin("multiply", sx, sx, p)
        rho = _un("sqrt", _bin("add", one, s2, p), p)
        denom = _bin("add", one, _bin("multiply", beta, s2, p), p)
        a = _bin("divide", _bin("multiply", _bin("multiply", beta, rho, p), sx, p), denom, p)
        b = _bin("divide", t, denom, p)
        big = _bin("greater_equal", _un("abs", x, p), _const(22, p), np.bool_)
        e = _un("exp", _bin("multiply", _const(-2, p), _un("abs", x, p), p), p)
        bb = _bin("multiply", _bin("multiply", _const(4, p), _bin("multiply", _un("sin", y, p),
                                                                  _un("cos", y, p), p), p), e, p)
        return ("c", ir.Where(big, _bin("copysign", one, x, p), a, p), ir.Where(big, bb, b, p))

    def _ipow(self, ar, ai, n, p) -> Val:
        """npy_cpow's integer branch (numpy npymath npy_math_complex.c.src):
        w = n + 0i with |n| < 100 multiplied out -- n = 1, 2, 3 directly,
        otherwise binary exponentiation from 1 + 0i, and 1 / z^|n| (Smith's
        division) for n < 0; z = 0 gives 0 + 0i for n > 0, nan + nan i for
        n < 0.  The same IEEE operations in the same order, so x**2 of a
        complex x is bit-identical to numpy (signed zeros included)."""
        zero = _const(0, p)
        if n == 0:
            return ("c", _const(1, p), zero)
        if n == 1:
            res = ("c", ar, ai)
        elif n == 2:
            res = self._mul(ar, ai, ar, ai, p)
        elif n == 3:
            _, sr, si = self._mul(ar, ai, ar, ai, p)
            res = self._mul(ar, ai, sr, si, p)
        else:
            m, mask = abs(n), 1
            aa = (_const(1, p), zero)
            pw = (ar, ai)
            while True:
                if m & mask:
                    aa = self._mul(aa[0], aa[1], pw[0], pw[1], p)[1:]
                mask <<= 1
                if m < mask:
                    break
                pw = self._mul(pw[0], pw[1], pw[0], pw[1], p)[1:]
            res = ("c",) + tuple(aa)
            if n < 0:
                res = self._div(_const(1, p), zero, res[1], res[2], p)
        zero_z = _bin("logical_and", _bin("equal", ar, zero, np.bool_), _bin("equal", ai, zero, np.bool_),
                      np.bool_)
        zval = zero if n > 0 else _const(np.nan, p)
        return ("c", ir.Where(zero_z, zval, res[1], p), ir.Where(zero_z, zval, res[2], p))

    def _pow(self, ar, ai, br, bi, p) -> Val:
        # z ** w = exp(w log z) (npy_cpow's general branch); w = 0 -> 1 + 0i,
        # z = 0 with real w > 0 -> 0 + 0i.  A constant integral w with |w| <
        # 100 takes numpy's multiplied-out branch (_ipow)
        n = _integral_exponent(br, bi, getattr(self, "const_args", {}))
        if n is not None:
            return self._ipow(ar, ai, n, p)
        lr = _un("log", _bin("hypot", ar, ai, p), p)
        li = _bin("atan2", ai, ar, p)
        _, er, ei = self._mul(br, bi, lr, li, p)
        r = _un("exp", er, p)
        cr = _bin("multiply", r, _un("cos", ei, p), p)
        ci = _bin("multiply", r, _un("sin", ei, p), p)
        zero_w = _bin("logical_and", _bin("equal", br, _const(0, p), np.bool_),
                      _bin("equal", bi, _const(0, p), np.bool_), np.bool_)
        zero_z = _bin("logical_and",
                      _bin("logical_and", _bin("equal", ar, _const(0, p), np.bool_),
                           _bin("equal", ai, _const(0, p), np.bool_), np.bool_),
                      _bin("logical_and", _bin("greater", br, _const(0, p), np.bool_),
                           _bin("equal", bi, _const(0, p), np.bool_), np.bool_), np.bool_)
        re = ir.Where(zero_w, _const(1, p), ir.Where(zero_z, _const(0, p), cr, p), p)
        im = ir.Where(zero_w, _const(0, p), ir.Where(zero_z, _const(0, p), ci, p), p)
        return ("c", re, im)

    def _sqrt(self, re, im, p) -> Val:
        # npy_csqrt (principal branch): t = sqrt((|re| + |z|) / 2);
        # re >= 0: (t, im / 2t); re < 0: (|im| / 2t, copysign(t, im)); z = 0: (0, im)
        a = _bin("hypot", re, im, p)
        t = _un("sqrt", _bin("multiply", _bin("add", _un("abs", re, p), a, p), _const(0.5, p), p), p)
        t2 = _bin("multiply", t, _const(2, p), p)
        pos = _bin("greater_equal", re, _const(0, p), np.bool_)
        zero = _bin("equal", a, _const(0, p), np.bool_)
        r_pos, i_pos = t, _bin("divide", im, t2, p)
        r_neg, i_neg = _bin("divide", _un("abs", im, p), t2, p), _bin("copysign", t, im, p)
        rr = ir.Where(zero, _const(0, p), ir.Where(pos, r_pos, r_neg, p), p)
        ii = ir.Where(zero, im, ir.Where(pos, i_pos, i_neg, p), p)
        return ("c", rr, ii)

    def _mul(self, ar, ai, br, bi, p) -> Val:
        # nc_prod: (ar*br - ai*bi, ar*bi + ai*br)
        return ("c", _bin("subtract", _bin("multiply", ar, br, p), _bin("multiply", ai, bi, p), p),
                _bin("add", _bin("multiply", ar, bi, p), _bin("multiply", ai, br, p), p))

    def _div(self, ar, ai, br, bi, p) -> Val:
        # numpy's complex division (Smith's algorithm, loops.c.src):
        # |br| >= |bi|: rat = bi/br, scl = 1/(br + bi*rat),
        #               ((ar + ai*rat)*scl, (ai - ar*rat)*scl)   [br = bi = 0: (ar/|br|, ai/|bi|)]
        # else:         rat = br/bi, scl = 1/(bi + br*rat),
        #               ((ar*rat + ai)*scl, (ai*rat - ar)*scl)
        abr, abi = _un("abs", br, p), _un("abs", bi, p)
        first = _bin("greater_equal", abr, abi, np.bool_)
        one = _const(1, p)
        rat1 = _bin("divide", bi, br, p)
        scl1 = _bin("divide", one, _bin("add", br, _bin("multiply", bi, rat1, p), p), p)
        r1 = _bin("multiply", _bin("add", ar, _bin("multiply", ai, rat1, p), p), scl1, p)
        i1 = _bin("multiply", _bin("subtract", ai, _bin("multiply", ar, rat1, p), p), scl1, p)
        rat2 = _bin("divide", br, bi, p)
        scl2 = _bin("divide", one, _bin("add", bi, _bin("multiply", br, rat2, p), p), p)
        r2 = _bin("multiply", _bin("add", _bin("multiply", ar, rat2, p), ai, p), scl2, p)
        i2 = _bin("multiply", _bin("subtract", _bin("multiply", ai, rat2, p), ar, p), scl2, p)
        both0 = _bin("logical_and", _bin("equal", abr, _const(0, p), np.bool_),
                     _bin("equal", abi, _const(0, p), np.bool_), np.bool_)
        r0, i0 = _bin("divide", ar, abr, p), _bin("divide", ai, abi, p)
        re = ir.Where(both0, r0, ir.Where(first, r1, r2, p), p)
        im = ir.Where(both0, i0, ir.Where(first, i1, i2, p), p)
        return ("c", re, im)

    def _binary(self, e: ir.Binary) -> Val:
        va, vb = self.split(e.a), self.split(e.b)
        if va[0] == "r" and vb[0] == "r":
            return ("r", e)
        dt = np.dtype(e.dtype)
        ct = dt if is_complex(dt) else np.result_type(
            *[x.dtype for x in (e.a, e.b)])
        if not is_complex(ct):
            raise _err(f"complex operand of {e.op} with a real result")
        p = part_dtype(ct)
        ar, ai = self.pair(e.a, p)
        br, bi = self.pair(e.b, p)
        op = e.op
        if op in ("add", "subtract"):
            return ("c", _bin(op, ar, br, p), _bin(op, ai, bi, p))
        if op == "multiply":
            return self._mul(ar, ai, br, bi, p)
        if op == "divide":
            return self._div(ar, ai, br, bi, p)
        if op == "pow":
            return self._pow(ar, ai, br, bi, p)
        if op == "equal":
            return ("r", _bin("logical_and", _bin("equal", ar, br, np.bool_), _bin("equal", ai, bi, np.bool_),
                              np.bool_))
        if op == "not_equal":
            return ("r", _bin("logical_or", _bin("not_equal", ar, br, np.bool_),
                              _bin("not_equal", ai, bi, np.bool_), np.bool_))
        raise _err(f"complex {op} is not lowered on the MI355X executor")


def program_has_complex(p) -> bool:
    if not isinstance(p, ir.ExprProgram):
        return False
    seen = set()

    def walk(e):
        if id(e) in seen:
            return False
        seen.add(id(e))
        if is_complex(e.dtype):
            return True
        return any(walk(c) for c in e.children())

    if any(walk(e) for e in p.all_exprs()):
        return True
    return p.reduce is not None and any(is_complex(f.dtype) for f in p.reduce.fields)


def split_program(p: ir.ExprProgram, const_args=None) -> ir.ExprProgram:
    """The program over real expressions that computes ``p``'s complex values
    part by part (unchanged when ``p`` has no complex value).
    ``const_args``: {argument index: value} of arguments that read a
    constant (a promoted scalar), so numpy's constant-exponent branches of
    ``pow`` can be taken."""
    if not program_has_complex(p):
        return p
    s = _Splitter()
    s.const_args = dict(const_args or {})
    reduce = p.reduce
    if reduce is not None:
        fields = []
        for f in reduce.fields:
            v = s.split(f.expr)
            if not is_complex(f.dtype):
                if v[0] == "c":
                    raise _err(f"a complex value reduced into the real field {f.name}")
                fields.append(dataclasses.replace(f, expr=v[1]))
                continue
            if f.rop not in ("sum", "nansum", "prod", "nanprod"):
                raise _err(f"{f.rop} of complex values is not lowered (sum/nansum/prod/nanprod are)")
            pt = part_dtype(f.dtype)
            re, im = s.pair(f.expr, pt)
            rop = f.rop
            if rop in ("nansum", "nanprod"):
                # numpy's nan-reductions replace an element whose real OR
                # imaginary part is NaN by the identity (0 / 1 + 0j)
                nan = _bin("logical_or", _un("isnan", re, np.bool_), _un("isnan", im, np.bool_), np.bool_)
                one = 0 if rop == "nansum" else 1
                re, im = ir.Where(nan, _const(one, pt), re, pt), ir.Where(nan, _const(0, pt), im, pt)
                rop = "sum" if rop == "nansum" else "prod"
            if rop == "prod":
                # one pair reduction: the {re, im} accumulators multiply as
                # complex numbers (cubed_rop CPROD / PAIR_IMAG)
                if len(reduce.fields) != 1:
                    raise _err("a complex product shares its reduction with another field")
                fields.append(ir.ReduceField(f.name + "#re", "cprod", re, pt))
                fields.append(ir.ReduceField(f.name + "#im", "pair_imag", im, pt))
                continue
            fields.append(ir.ReduceField(f.name + "#re", rop, re, pt))
            fields.append(ir.ReduceField(f.name + "#im", rop, im, pt))
        reduce = dataclasses.replace(reduce, fields=tuple(fields))
    if p.structured:
        items = []
        for name, e in p.outputs:
            v = s.split(e)
            if v[0] == "c":
                raise _err("complex fields of structured outputs are not lowered")
            items.append((name, v[1]))
        outputs = tuple(items)
    else:
        v = s.split(p.outputs)
        outputs = (("real", v[1]), ("imag", v[2])) if v[0] == "c" else v[1]
    return dataclasses.replace(p, outputs=outputs, reduce=reduce)
