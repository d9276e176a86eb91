from ..chunkfuncs import NumpyReduction
from ..core import reduction
from .creation_functions import asarray

_np_all = NumpyReduction("all", "all")
_np_any = NumpyReduction("any", "any")


def all(x, /, *, axis=None, keepdims=False):
    if x.size == 0:
        return asarray(True, dtype=x.dtype)
    return reduction(x, _np_all, axis=axis, dtype=bool, keepdims=keepdims)


def any(x, /, *, axis=None, keepdims=False):
    if x.size == 0:
        return asarray(False, dtype=x.dtype)
    return reduction(x, _np_any, axis=axis, dtype=bool, keepdims=keepdims)
