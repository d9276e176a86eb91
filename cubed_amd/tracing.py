"""Lowering of user chunk functions by symbolic tracing.

``map_blocks(lambda a: (a + 1) * 2, x)`` and friends: the function is called
once at plan time on proxy objects that record numpy ufunc calls and Python
operators into IR.  Functions that do anything else (indexing, shape changes,
non-numpy calls) are not traceable and stay opaque -- the executor then
refuses the plan with a clear error rather than running host code.
"""

from __future__ import annotations

import numpy as np

from . import ir


class _Proxy:
    __array_priority__ = 1000

    def __init__(self, expr: ir.Expr, ndim: int):
        self.expr = expr
        self.ndim = ndim
        self.dtype = expr.dtype

    @property
    def shape(self):
        raise _Untraceable("shape is not known while tracing")

    # numpy protocol
    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        if method != "__call__" or kwargs.get("out") is not None:
            return NotImplemented
        name = ir.NUMPY_ELEMENTWISE.get(ufunc)
        if name is None:
            raise _Untraceable(f"ufunc {ufunc.__name__}")
        dtype = kwargs.get("dtype")
        xs = [_lift(i) for i in inputs]
        out_dtype = np.result_type(*[_np_like(i) for i in inputs]) if dtype is None else np.dtype(dtype)
        if name in ir.COMPARISONS or name in ir.UNARY_BOOL_RESULT:
            out_dtype = np.dtype(np.bool_)
        elif name == "divide" and out_dtype.kind in "biu":
            out_dtype = np.dtype(np.float64)
        return _Proxy(ir.apply_op(name, [x.expr for x in xs], out_dtype),
                      max(x.ndim for x in xs))

    def __array_function__(self, func, types, args, kwargs):
        fill = {np.ones_like: 1, np.zeros_like: 0}.get(func)
        if func is np.full_like and len(args) >= 2:
            fill = args[1]
        if fill is not None and set(kwargs) <= {"dtype"} and len(args) <= 2:
            # a constant of the chunk's shape (the task's extents come from its
            # output block, so the operand is not read at all)
            x = _lift(args[0])
            dt = np.dtype(kwargs["dtype"]) if kwargs.get("dtype") is not None else x.dtype
            return _Proxy(ir.Const(np.array(fill).astype(dt).item(), dt), x.ndim)
        if func is getattr(np, "astype", None) and len(args) >= 2 and set(kwargs) <= {"copy"}:
            return _lift(args[0]).astype(args[1])
        if func is np.where and not kwargs:
            c, a, b = (_lift(x) for x in args)
            dt = np.result_type(_np_like(args[1]), _np_like(args[2]))
            return _Proxy(ir.apply_op("where", [c.expr, a.expr, b.expr], dt),
                          max(c.ndim, a.ndim, b.ndim))
        raise _Untraceable(f"function {getattr(func, '__name__', func)}")

    def astype(self, dtype, copy=True):
        return _Proxy(ir.cast(self.expr, dtype), self.ndim)

    def _bin(self, other, name, reflected=False):
        a, b = (_lift(other), self) if reflected else (self, _lift(other))
        ufunc = getattr(np, {"pow": "power"}.get(name, name))
        return self.__array_ufunc__(ufunc, "__call__", a, b)

    def __add__(self, o): return self._bin(o, "add")
    def __radd__(self, o): return self._bin(o, "add", True)
    def __sub__(self, o): return self._bin(o, "subtract")
    def __rsub__(self, o): return self._bin(o, "subtract", True)
    def __mul__(self, o): return self._bin(o, "multiply")
    def __rmul__(self, o): return self._bin(o, "multiply", True)
    def __truediv__(self, o): return self._bin(o, "divide")
    def __rtruediv__(self, o): return self._bin(o, "divide", True)
    def __pow__(self, o): return self._bin(o, "pow")
    def __neg__(self): return self.__array_ufunc__(np.negative, "__call__", self)
    def __abs__(self): return self.__array_ufunc__(np.absolute, "__call__", self)
    def __lt__(self, o): return self._bin(o, "less")
    def __le__(self, o): return self._bin(o, "less_equal")
    def __gt__(self, o): return self._bin(o, "greater")
    def __ge__(self, o): return self._bin(o, "greater_equal")


class _Untraceable(Exception):
    pass


class _Unusable:
    """Stand-in for an argument the traced function must not touch."""

    def __getattr__(self, name):
        raise _Untraceable("argument without output dims")

    def _fail(self, *a, **k):
        raise _Untraceable("argument without output dims")

    __array_ufunc__ = __array_function__ = None
    __add__ = __radd__ = __sub__ = __rsub__ = __mul__ = __rmul__ = __truediv__ = _fail
    __rtruediv__ = __pow__ = __neg__ = __abs__ = __lt__ = __le__ = __gt__ = __ge__ = _fail
    __array__ = _fail


def _np_like(x):
    if isinstance(x, _Proxy):
        return np.empty((), dtype=x.dtype)
    # Python scalars follow NEP 50 weak promotion against the array dtype
    return x


def _lift(x):
    if isinstance(x, _Proxy):
        return x
    if isinstance(x, (bool, int, float, np.generic)):
        dt = np.result_type(x) if isinstance(x, np.generic) else None
        if dt is None:
            dt = np.dtype(np.bool_) if isinstance(x, bool) else (
                np.dtype(np.int64) if isinstance(x, int) else np.dtype(np.float64))
        return _Proxy(ir.Const(x, dt), 0)
    raise _Untraceable(f"operand of type {type(x).__name__}")


def trace_callable(func, arrays, inds, out_ind, dtype, kwargs):
    """IR program for ``func(*chunks, **kwargs)`` or None if untraceable."""
    if not callable(func):
        return None
    space = len(out_ind)
    pos = {idx: i for i, idx in enumerate(out_ind)}
    proxies = []
    for i, (a, ind) in enumerate(zip(arrays, inds)):
        axes = [pos.get(idx) for idx in ind] if ind is not None else None
        if axes is not None and None in axes and len(axes) == space:
            # map_blocks(drop_axis=d, new_axis=d) relabels an axis: a dropped
            # dim of a full-rank argument lands on the output dim at its position
            used = {x for x in axes if x is not None}
            axes = [d if x is None and d not in used else x for d, x in enumerate(axes)]
        if axes is None or None in axes:
            # an argument whose dims are not output dims can only be passed
            # through unused (e.g. ``lambda x, y: x`` with y's dim dropped)
            proxies.append(_Unusable())
            continue
        proxies.append(_Proxy(ir.Arg(i, a.dtype, tuple(axes)), a.ndim))
    try:
        with np.errstate(all="ignore"):
            out = func(*proxies, **kwargs)
    except _Untraceable:
        return None
    except Exception:
        return None
    if not isinstance(out, _Proxy):
        return None
    e = ir.cast(out.expr, dtype) if dtype is not None else out.expr
    return ir.ExprProgram(ndim=space, nargs=len(arrays), outputs=e, out_axes=tuple(range(space)),
                          name=getattr(func, "__name__", "traced"))
