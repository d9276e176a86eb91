"""The Array object (cubed/array_api/array_object.py).

Operators build ``elemwise`` ops exactly as the reference (:121-348); a Python
scalar operand becomes a 0-d ``asarray`` of the array's dtype (weak scalar
rule, :401-446), which the executor folds into a kernel constant."""

import math

import numpy as np

from ..core.array import CoreArray
from ..core.ops import elemwise
from ..utils import memory_repr
from .creation_functions import asarray
from .data_type_functions import result_type
from .dtypes import (
    _boolean_dtypes,
    _complex_floating_dtypes,
    _dtype_categories,
    _floating_dtypes,
    _integer_dtypes,
    _numeric_dtypes,
)
from .linear_algebra_functions import matmul


def _binop(opname, category, reflected=False, bool_result=False, matmul_op=False):
    def method(self, other, /):
        other = self._check_allowed_dtypes(other, category, opname)
        if other is NotImplemented:
            return other
        if matmul_op:
            return matmul(other, self) if reflected else matmul(self, other)
        dtype = np.bool_ if bool_result else result_type(self, other)
        a, b = (other, self) if reflected else (self, other)
        return elemwise(opname, a, b, dtype=dtype)

    return method


class Array(CoreArray):
    """Chunked array (HBM-resident when computed) conforming to the Python
    Array API standard."""

    def __init__(self, name, zarray, spec, plan):
        super().__init__(name, zarray, spec, plan)

    def __array__(self, dtype=None, copy=None) -> np.ndarray:
        x = self.compute()
        if dtype and x.dtype != dtype:
            x = x.astype(dtype)
        if not isinstance(x, np.ndarray):
            x = np.array(x)
        return x

    def __repr__(self):
        return f"cubed.Array<{self.name}, shape={self.shape}, dtype={self.dtype}, chunks={self.chunks}>"

    def _repr_inline_(self, max_width):
        return f"cubed.Array<chunksize={self.chunksize}>"

    @property
    def device(self):
        return "cpu"

    @property
    def mT(self):
        from .linear_algebra_functions import matrix_transpose

        return matrix_transpose(self)

    @property
    def T(self):
        if self.ndim != 2:
            raise ValueError("x.T requires x to have 2 dimensions.")
        from .linear_algebra_functions import matrix_transpose

        return matrix_transpose(self)

    # unary operators
    def __neg__(self, /):
        if self.dtype not in _numeric_dtypes:
            raise TypeError("Only numeric dtypes are allowed in __neg__")
        return elemwise("negative", self, dtype=self.dtype)

    def __pos__(self, /):
        if self.dtype not in _numeric_dtypes:
            raise TypeError("Only numeric dtypes are allowed in __pos__")
        return elemwise("positive", self, dtype=self.dtype)

    def __abs__(self, /):
        if self.dtype not in _numeric_dtypes:
            raise TypeError("Only numeric dtypes are allowed in __abs__")
        dtype = np.dtype(f"f{self.dtype.itemsize // 2}") if self.dtype.kind == "c" else self.dtype
        return elemwise("abs", self, dtype=dtype)

    def __complex__(self, /):
        if self.ndim != 0:
            raise TypeError("complex is only allowed on arrays with 0 dimensions")
        return complex(self.compute())

    def __invert__(self, /):
        if self.dtype not in _dtype_categories["integer or boolean"]:
            raise TypeError("Only integer or boolean dtypes are allowed in __invert__")
        return elemwise("bitwise_invert", self, dtype=self.dtype)

    def __float__(self, /):
        if self.ndim != 0:
            raise TypeError("float is only allowed on arrays with 0 dimensions")
        if self.dtype.kind == "c":
            raise TypeError("float is not allowed on complex floating-point arrays")
        return float(self.compute())

    def __int__(self, /):
        if self.ndim != 0:
            raise TypeError("int is only allowed on arrays with 0 dimensions")
        return int(self.compute())

    def __bool__(self, /):
        if self.ndim != 0:
            raise TypeError("bool is only allowed on arrays with 0 dimensions")
        return bool(self.compute())

    def __index__(self, /):
        if self.ndim != 0:
            raise TypeError("index is only allowed on arrays with 0 dimensions")
        import operator

        return operator.index(self.compute())

    __add__ = _binop("add", "numeric")
    __sub__ = _binop("subtract", "numeric")
    __mul__ = _binop("multiply", "numeric")
    __truediv__ = _binop("divide", "floating-point")
    __floordiv__ = _binop("floor_divide", "real numeric")
    __mod__ = _binop("remainder", "real numeric")
    __pow__ = _binop("pow", "numeric")
    __matmul__ = _binop("matmul", "numeric", matmul_op=True)
    __and__ = _binop("bitwise_and", "integer or boolean")
    __or__ = _binop("bitwise_or", "integer or boolean")
    __xor__ = _binop("bitwise_xor", "integer or boolean")
    __lshift__ = _binop("bitwise_left_shift", "integer")
    __rshift__ = _binop("bitwise_right_shift", "integer")
    __eq__ = _binop("equal", "all", bool_result=True)
    __ne__ = _binop("not_equal", "all", bool_result=True)
    __ge__ = _binop("greater_equal", "all", bool_result=True)
    __gt__ = _binop("greater", "all", bool_result=True)
    __le__ = _binop("less_equal", "all", bool_result=True)
    __lt__ = _binop("less", "all", bool_result=True)
    __radd__ = _binop("add", "numeric", reflected=True)
    __rsub__ = _binop("subtract", "numeric", reflected=True)
    __rmul__ = _binop("multiply", "numeric", reflected=True)
    __rtruediv__ = _binop("divide", "floating-point", reflected=True)
    __rfloordiv__ = _binop("floor_divide", "numeric", reflected=True)
    __rmod__ = _binop("remainder", "numeric", reflected=True)
    __rpow__ = _binop("pow", "numeric", reflected=True)
    __rmatmul__ = _binop("matmul", "numeric", reflected=True, matmul_op=True)
    __rand__ = _binop("bitwise_and", "integer or boolean", reflected=True)
    __ror__ = _binop("bitwise_or", "integer or boolean", reflected=True)
    __rxor__ = _binop("bitwise_xor", "integer or boolean", reflected=True)
    __rlshift__ = _binop("bitwise_left_shift", "integer", reflected=True)
    __rrshift__ = _binop("bitwise_right_shift", "integer", reflected=True)

    def __hash__(self):
        return id(self)

    # helpers
    def _check_allowed_dtypes(self, other, dtype_category, op):
        if self.dtype not in _dtype_categories[dtype_category]:
            raise TypeError(f"Only {dtype_category} dtypes are allowed in {op}")
        if isinstance(other, (int, complex, float, bool)):
            other = self._promote_scalar(other)
        elif isinstance(other, CoreArray):
            if other.dtype not in _dtype_categories[dtype_category]:
                raise TypeError(f"Only {dtype_category} dtypes are allowed in {op}")
        else:
            return NotImplemented
        return other

    def _promote_scalar(self, scalar):
        if isinstance(scalar, bool):
            if self.dtype not in _boolean_dtypes:
                raise TypeError("Python bool scalars can only be promoted with bool arrays")
        elif isinstance(scalar, int):
            if self.dtype in _boolean_dtypes:
                raise TypeError("Python int scalars cannot be promoted with bool arrays")
            if self.dtype in _integer_dtypes:
                info = np.iinfo(self.dtype)
                if not (info.min <= scalar <= info.max):
                    raise OverflowError(
                        "Python int scalars must be within the bounds of the dtype for integer arrays")
        elif isinstance(scalar, float):
            if self.dtype not in _floating_dtypes:
                raise TypeError("Python float scalars can only be promoted with floating-point arrays.")
        elif isinstance(scalar, complex):
            if self.dtype not in _complex_floating_dtypes:
                raise TypeError(
                    "Python complex scalars can only be promoted with complex floating-point arrays.")
        else:
            raise TypeError("'scalar' must be a Python scalar")
        return asarray(scalar, dtype=self.dtype, spec=self.spec)
