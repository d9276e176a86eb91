"""Elementwise functions (cubed/array_api/elementwise_functions.py).

Same dtype checks and result dtypes as the reference; each builds an
``elemwise`` op whose program is one IR node, so chains fuse into a single
kernel.  Functions are generated from a table: (name, dtype category, result
rule, op)."""

import numpy as np

from ..core import elemwise
from .data_type_functions import result_type
from .dtypes import (
    _boolean_dtypes,
    _floating_dtypes,
    _integer_dtypes,
    _integer_or_boolean_dtypes,
    _numeric_dtypes,
    _real_floating_dtypes,
    _real_numeric_dtypes,
)

_CATS = {
    "numeric": (_numeric_dtypes, "numeric"),
    "floating": (_floating_dtypes, "floating-point"),
    "real_floating": (_real_floating_dtypes, "real floating-point"),
    "real_numeric": (_real_numeric_dtypes, "real numeric"),
    "int_or_bool": (_integer_or_boolean_dtypes, "integer or boolean"),
    "integer": (_integer_dtypes, "integer"),
    "boolean": (_boolean_dtypes, "boolean"),
    "all": (None, None),
}


def _check(name, cat, *xs):
    allowed, label = _CATS[cat]
    if allowed is None:
        return
    for x in xs:
        if x.dtype not in allowed:
            raise TypeError(f"Only {label} dtypes are allowed in {name}")


def _unary(name, cat, rule="same", op=None, int_identity=False):
    op = op or name

    def f(x, /):
        _check(name, cat, x)
        if int_identity and x.dtype in _integer_dtypes:
            return x
        dtype = np.bool_ if rule == "bool" else x.dtype
        return elemwise(op, x, dtype=dtype)

    f.__name__ = name
    f.__doc__ = f"Elementwise ``{name}`` (numpy semantics) as one fused-program node."
    return f


def _binary(name, cat, rule="promote", op=None):
    op = op or name

    def f(x1, x2, /):
        _check(name, cat, x1, x2)
        dtype = np.bool_ if rule == "bool" else result_type(x1, x2)
        return elemwise(op, x1, x2, dtype=dtype)

    f.__name__ = name
    f.__doc__ = f"Elementwise ``{name}`` (numpy semantics) as one fused-program node."
    return f


_complex_cat = ((np.dtype("complex64"), np.dtype("complex128")), "complex floating-point")


def _part_dtype(dt):
    return np.dtype(f"f{np.dtype(dt).itemsize // 2}")


def abs(x, /):
    """|x|; complex arrays give their part dtype (elementwise_functions.py:22-31)."""
    _check("abs", "numeric", x)
    dtype = _part_dtype(x.dtype) if x.dtype.kind == "c" else x.dtype
    return elemwise("abs", x, dtype=dtype)


def _complex_only(name, part_result):
    def f(x, /):
        if x.dtype not in _complex_cat[0]:
            raise TypeError(f"Only complex floating-point dtypes are allowed in {name}")
        return elemwise(name, x, dtype=_part_dtype(x.dtype) if part_result else x.dtype)

    f.__name__ = name
    f.__doc__ = (f"Elementwise ``{name}`` of a complex array (elementwise_functions.py); "
                 "computed on its real/imaginary slabs (cubed_amd/complex.py).")
    return f


conj = _complex_only("conj", False)
real = _complex_only("real", True)
imag = _complex_only("imag", True)
acos = _unary("acos", "floating")
acosh = _unary("acosh", "floating")
asin = _unary("asin", "floating")
asinh = _unary("asinh", "floating")
atan = _unary("atan", "floating")
atanh = _unary("atanh", "floating")
bitwise_invert = _unary("bitwise_invert", "int_or_bool")
ceil = _unary("ceil", "real_numeric", int_identity=True)
cos = _unary("cos", "floating")
cosh = _unary("cosh", "floating")
exp = _unary("exp", "floating")
expm1 = _unary("expm1", "floating")
floor = _unary("floor", "real_numeric", int_identity=True)
isfinite = _unary("isfinite", "numeric", "bool")
isinf = _unary("isinf", "numeric", "bool")
isnan = _unary("isnan", "numeric", "bool")
log = _unary("log", "floating")
log1p = _unary("log1p", "floating")
log2 = _unary("log2", "floating")
log10 = _unary("log10", "floating")
logical_not = _unary("logical_not", "boolean", "bool")
negative = _unary("negative", "numeric")
positive = _unary("positive", "numeric")
round = _unary("round", "numeric")
sign = _unary("sign", "numeric")
sin = _unary("sin", "floating")
sinh = _unary("sinh", "floating")
sqrt = _unary("sqrt", "floating")
square = _unary("square", "numeric")
tan = _unary("tan", "floating")
tanh = _unary("tanh", "floating")
trunc = _unary("trunc", "real_numeric", int_identity=True)

add = _binary("add", "numeric")
atan2 = _binary("atan2", "real_floating")
bitwise_and = _binary("bitwise_and", "int_or_bool")
bitwise_left_shift = _binary("bitwise_left_shift", "integer")
bitwise_or = _binary("bitwise_or", "int_or_bool")
bitwise_right_shift = _binary("bitwise_right_shift", "integer")
bitwise_xor = _binary("bitwise_xor", "int_or_bool")
divide = _binary("divide", "floating")
equal = _binary("equal", "all", "bool")
floor_divide = _binary("floor_divide", "real_numeric")
greater = _binary("greater", "all", "bool")
greater_equal = _binary("greater_equal", "all", "bool")
less = _binary("less", "all", "bool")
less_equal = _binary("less_equal", "all", "bool")
logaddexp = _binary("logaddexp", "real_floating")
logical_and = _binary("logical_and", "boolean", "bool")
logical_or = _binary("logical_or", "boolean", "bool")
logical_xor = _binary("logical_xor", "boolean", "bool")
multiply = _binary("multiply", "numeric")
not_equal = _binary("not_equal", "all", "bool")
pow = _binary("pow", "numeric")
remainder = _binary("remainder", "real_numeric")
subtract = _binary("subtract", "numeric")
maximum = _binary("maximum", "real_numeric")
minimum = _binary("minimum", "real_numeric")
hypot = _binary("hypot", "real_floating")
copysign = _binary("copysign", "real_floating")
