"""Chunk functions of the reductions, as program builders.

The reference passes numpy callables to ``reduction``/``partial_reduce``:
``_mean_func``/``_mean_combine``/``_mean_aggregate``/``_numel``
(array_api/statistical_functions.py:54-100), the nan variants
(nan_functions.py:37-59), ``nxp.sum``/``max``/``min``/``prod`` with a
``dtype`` kwarg (statistical_functions.py:22-156) and ``_chunk_sum``
(linear_algebra_functions.py:77-78).  Each object below has the same name and
meaning but, instead of running on a numpy chunk, builds the IR program that
the fused reduction kernels execute (sequential fp64/int64 accumulation,
structured ``{n, total}`` fields stored SoA).
"""

from __future__ import annotations

import functools
from typing import Any, Dict, Optional, Sequence

import numpy as np

from . import ir


class ChunkReduction:
    """A reduction applied to one (possibly merged) chunk with keepdims.

    ``fields(in_dtype, kwargs)`` -> list of (name, rop, out dtype, field of
    the input or None).  ``structured`` -> result is a dict of fields."""

    name = "reduction"
    structured = False

    def fields(self, in_dtype, kwargs):  # pragma: no cover - abstract
        raise NotImplementedError

    def __call__(self, *args, **kwargs):
        raise TypeError(f"{self.name} is a MI355X chunk reduction; it has no host implementation")

    def program(self, ndim: int, in_dtype, axis: Sequence[int], keepdims: bool = True,
                **kwargs) -> ir.ExprProgram:
        axis = tuple(sorted(axis))
        fs = self.fields(np.dtype(in_dtype), kwargs)
        rfs = []
        for name, rop, dt, src_field in fs:
            src_dt = np.dtype(in_dtype)[src_field] if src_field is not None else np.dtype(in_dtype)
            x = ir.Arg(0, src_dt, tuple(range(ndim)), field=src_field)
            rfs.append(ir.ReduceField(name, rop, x, np.dtype(dt)))
        stage = ir.ReduceStage(axis, tuple(rfs))
        if self.structured:
            outputs = tuple((f.name, ir.Field(f.name, f.dtype)) for f in rfs)
        else:
            outputs = ir.Field(rfs[0].name, rfs[0].dtype)
        out_axes = tuple(range(ndim)) if keepdims else tuple(d for d in range(ndim) if d not in axis)
        return ir.ExprProgram(ndim=ndim, nargs=1, outputs=outputs, out_axes=out_axes,
                              reduce=stage, name=self.name)


class NumpyReduction(ChunkReduction):
    """``np.sum``/``np.max``/... applied with ``axis``, ``keepdims`` and an
    optional ``dtype`` (numpy's reduction dtype rules)."""

    def __init__(self, rop: str, name: Optional[str] = None):
        self.rop = rop
        self.name = name or rop

    def fields(self, in_dtype, kwargs):
        requested = kwargs.get("dtype")
        if isinstance(requested, (list, tuple)) or (requested is not None and np.dtype(requested).names):
            raise TypeError("structured dtype passed to a plain reduction")
        out = ir.reduction_result_dtype(self.rop, in_dtype, requested)
        return [("value", self.rop, out, None)]


class _MeanFunc(ChunkReduction):
    name = "_mean_func"
    structured = True

    def fields(self, in_dtype, kwargs):
        dt = dict(kwargs["dtype"])
        return [("n", "count", dt["n"], None), ("total", "sum", dt["total"], None)]


class _MeanCombine(ChunkReduction):
    name = "_mean_combine"
    structured = True

    def fields(self, in_dtype, kwargs):
        dt = dict(kwargs["dtype"])
        return [("n", "sum", dt["n"], "n"), ("total", "sum", dt["total"], "total")]


class _NanMeanFunc(ChunkReduction):
    name = "_nanmean_func"
    structured = True

    def fields(self, in_dtype, kwargs):
        return [("n", "count_nonnan", np.int64, None),
                ("total", "nansum", ir.reduction_result_dtype("nansum", in_dtype), None)]


class _NanMeanCombine(ChunkReduction):
    name = "_nanmean_combine"
    structured = True

    def fields(self, in_dtype, kwargs):
        return [("n", "nansum", in_dtype["n"], "n"), ("total", "nansum", in_dtype["total"], "total")]


class _VarFunc(ChunkReduction):
    """Per-chunk ``{n, mu, M2}`` of var/std: count, mean and sum of squared
    deviations, folded element by element with Welford's update (the triple
    reduction ``var``).  The reference v0.12.0 has no var (api_status.md:72,74);
    the intermediate follows later cubed's structured {n, mu, M2} with Chan's
    pairwise combine, computed in f64 like mean's total."""

    name = "_var_func"
    structured = True

    def fields(self, in_dtype, kwargs):
        return [("n", "var", np.int64, None), ("mu", "var_mean", np.float64, None),
                ("M2", "var_m2", np.float64, None)]


class _VarCombine(ChunkReduction):
    """Combine round of var/std: folds the {n, mu, M2} partials of a merged
    chunk with Chan's update (``varc``)."""

    name = "_var_combine"
    structured = True

    def fields(self, in_dtype, kwargs):
        return [("n", "varc", np.int64, "n"), ("mu", "var_mean", np.float64, "mu"),
                ("M2", "var_m2", np.float64, "M2")]


_mean_func = _MeanFunc()
_mean_combine = _MeanCombine()
_nanmean_func = _NanMeanFunc()
_nanmean_combine = _NanMeanCombine()
_chunk_sum = NumpyReduction("sum", "_chunk_sum")


class ChunkMap:
    """An elementwise chunk function built per call site (aggregates)."""

    name = "map"

    def program(self, ndim: int, in_dtype, out_dtype) -> ir.ExprProgram:  # pragma: no cover
        raise NotImplementedError

    def __call__(self, *args, **kwargs):
        raise TypeError(f"{self.name} is a MI355X chunk function; it has no host implementation")


class _MeanAggregate(ChunkMap):
    name = "_mean_aggregate"

    def program(self, ndim, in_dtype, out_dtype=None):
        axes = tuple(range(ndim))
        total = ir.Arg(0, np.dtype(in_dtype)["total"], axes, field="total")
        n = ir.Arg(0, np.dtype(in_dtype)["n"], axes, field="n")
        res = ir.Binary("divide", ir.cast(total, np.float64), ir.cast(n, np.float64),
                        np.dtype(np.float64))
        return ir.ExprProgram(ndim=ndim, nargs=1, outputs=res, out_axes=axes, name=self.name)


class _VarAggregate(ChunkMap):
    """var = M2 / max(n - correction, 0) (numpy's ``rcount`` clamp, so n <=
    correction gives NaN / inf as numpy does); std = its square root."""

    def __init__(self, correction=0.0, sqrt=False):
        self.correction = float(correction)
        self.sqrt = bool(sqrt)
        self.name = "_std_aggregate" if sqrt else "_var_aggregate"

    def program(self, ndim, in_dtype, out_dtype=None):
        axes = tuple(range(ndim))
        f8 = np.dtype(np.float64)
        m2 = ir.Arg(0, np.dtype(in_dtype)["M2"], axes, field="M2")
        n = ir.Arg(0, np.dtype(in_dtype)["n"], axes, field="n")
        rcount = ir.Binary("maximum", ir.Binary("subtract", ir.cast(n, np.float64), ir.Const(self.correction, f8), f8),
                           ir.Const(0.0, f8), f8)
        res = ir.Binary("divide", ir.cast(m2, np.float64), rcount, f8)
        if self.sqrt:
            res = ir.Unary("sqrt", res, f8)
        return ir.ExprProgram(ndim=ndim, nargs=1, outputs=res, out_axes=axes, name=self.name)


_var_func = _VarFunc()
_var_combine = _VarCombine()
_mean_aggregate = _MeanAggregate()
_nanmean_aggregate = _MeanAggregate()


class ArgReduction(ChunkReduction):
    """``_arg_func`` + ``_arg_combine`` (core/ops.py:1124-1145): the reference
    keeps {i, v} per block and picks, with argmax/argmin, the pair whose value
    wins.  Here the {v, i} pairs are reduced by the pair op ``argmax`` /
    ``argmin`` (first NaN, else the larger / smaller value, ties to the
    smaller index -- numpy's choice, independent of the combine order), so the
    per-chunk pass and every combine round are the same program."""

    structured = True

    def __init__(self, arg_func: str):
        self.rop = arg_func
        self.name = f"_arg_combine[{arg_func}]"

    def fields(self, in_dtype, kwargs):
        return [("v", self.rop, in_dtype["v"], "v"), ("i", "pair_index", np.dtype(np.int64), "i")]


class _ArgAggregate(ChunkMap):
    name = "_arg_aggregate"

    def program(self, ndim, in_dtype, out_dtype=None):
        axes = tuple(range(ndim))
        return ir.ExprProgram(ndim=ndim, nargs=1, outputs=ir.Arg(0, np.dtype(np.int64), axes, field="i"),
                              out_axes=axes, name=self.name)


_arg_aggregate = _ArgAggregate()


def as_chunk_reduction(func) -> Optional[ChunkReduction]:
    """Map a user-supplied reduction callable to a ChunkReduction."""
    if isinstance(func, functools.partial):
        inner = as_chunk_reduction(func.func)
        if inner is None:
            return None
        return _BoundReduction(inner, dict(func.keywords))
    if isinstance(func, ChunkReduction):
        return func
    rop = ir.NUMPY_REDUCTIONS.get(func)
    if rop is not None:
        return NumpyReduction(rop, getattr(func, "__name__", rop))
    return None


class _BoundReduction(ChunkReduction):
    """``functools.partial(reduction, **kw)`` (reduction_new's initial_func /
    reduce_func, core/ops.py:931-945)."""

    def __init__(self, inner: ChunkReduction, kw: Dict[str, Any]):
        self.inner = inner
        self.kw = kw
        self.name = inner.name
        self.structured = inner.structured

    def fields(self, in_dtype, kwargs):
        merged = {k: v for k, v in self.kw.items() if k not in ("axis", "keepdims")}
        merged.update({k: v for k, v in kwargs.items() if k not in ("axis", "keepdims")})
        return self.inner.fields(in_dtype, merged)

    @property
    def bound_axis(self):
        return self.kw.get("axis")
