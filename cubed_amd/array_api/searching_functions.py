from ..core.ops import arg_reduction, elemwise
from .data_type_functions import result_type


def argmax(x, /, *, axis=None, keepdims=False):
    return arg_reduction(x, "argmax", axis=axis, keepdims=keepdims)


def argmin(x, /, *, axis=None, keepdims=False):
    return arg_reduction(x, "argmin", axis=axis, keepdims=keepdims)


def where(condition, x1, x2, /):
    """elemwise(where, condition, x1, x2) (searching_functions.py:30-32)."""
    dtype = result_type(x1, x2)
    return elemwise("where", condition, x1, x2, dtype=dtype)
