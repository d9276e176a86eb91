"""Chunk-function IR: what a Cubed task computes, in a form the MI355X
kernels can run.

In the reference a task's function is an opaque Python closure over numpy
calls (``BlockwiseSpec.function``, primitive/blockwise.py:34-58, composed by
``fuse``/``fuse_multiple`` :368-508).  Here every op the API builds carries a
``Program`` instead: a small expression tree over the task's input chunks
(``Arg`` leaves), an optional reduction stage with named fields (the
structured ``{n, total}`` intermediates of statistical_functions.py:38), and
output expressions.  Fusion composes programs (``fuse_programs``) exactly
where the reference composes closures, so the GPU executor runs one kernel per
fused pipeline.  A ``Program`` is deliberately not callable on numpy arrays:
there is no CPU path in the product.

Shapes: a program iterates over a ``space`` of rank ``ndim``.  Each leaf maps
its own dims to space dims (``axes``; ``None`` for a unit dim that has no
space dim).  A leaf dim of extent 1 under a space dim of larger extent
broadcasts.  Outputs map output dims to space dims (``out_axes``); reduced
space dims are kept as unit output dims (keepdims) or dropped (squeeze).
"""

from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

# ----------------------------------------------------------------- dtypes

# numpy has no bfloat16: it is carried as a 2-byte void dtype tagged with
# metadata (its bit pattern = the top half of an IEEE f32).  The kernels
# load/store it as CUBED_BF16; host readback widens it exactly to float32
# (bf16_to_numpy).  numpy keeps the tag through views, copies and slices;
# an UNtagged 2-byte void array handed to from_array / asarray is refused
# (check_input_dtype) instead of being read as bf16.
bfloat16 = np.dtype("V2", metadata={"cubed_bf16": True})


def check_input_dtype(dt):
    """Refuse raw void dtypes at the API boundary: only the tagged bfloat16
    carrier (and structured dtypes) may enter as 'V'."""
    dt = np.dtype(dt)
    if dt.kind == "V" and not dt.names and not (dt.metadata or {}).get("cubed_bf16"):
        raise TypeError(f"raw void dtype {dt} is not an array dtype here (bfloat16 data: "
                        "use cubed_amd.array_api.bfloat16 / ir.numpy_to_bf16)")
    return dt

DTYPE_CODES = {
    bfloat16: 12,
    np.dtype("bool"): 0, np.dtype("int8"): 1, np.dtype("int16"): 2,
    np.dtype("int32"): 3, np.dtype("int64"): 4, np.dtype("uint8"): 5,
    np.dtype("uint16"): 6, np.dtype("uint32"): 7, np.dtype("uint64"): 8,
    np.dtype("float32"): 9, np.dtype("float64"): 10, np.dtype("float16"): 11,
}
CODE_DTYPES = {v: k for k, v in DTYPE_CODES.items()}


def dtype_code(dt) -> int:
    dt = np.dtype(dt)
    if dt not in DTYPE_CODES:
        raise NotImplementedError(f"dtype {dt} is not supported by the MI355X kernels")
    return DTYPE_CODES[dt]


def is_float(dt) -> bool:
    dt = np.dtype(dt)
    return dt.kind == "f" or dt == bfloat16


def is_bf16(dt) -> bool:
    return np.dtype(dt) == bfloat16


def bf16_to_numpy(a: np.ndarray) -> np.ndarray:
    """bfloat16 bits (the V2 carrier dtype) -> the same values as float32."""
    return (np.ascontiguousarray(a).view(np.uint16).astype(np.uint32) << 16).view(np.float32)


def numpy_to_bf16(a: np.ndarray) -> np.ndarray:
    """float values -> bfloat16 bits (round to nearest even through f32, NaN
    kept quiet), as the V2 carrier dtype."""
    u = np.ascontiguousarray(np.asarray(a, dtype=np.float32)).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r = np.where(nan, ((u >> 16) | 0x40).astype(np.uint16), r)
    return r.view(bfloat16)


def is_int(dt) -> bool:
    return np.dtype(dt).kind in "iu"


def is_bool(dt) -> bool:
    return np.dtype(dt).kind == "b"


# ----------------------------------------------------------------- op tables
# name -> opcode of include/cubed_amd.h
UNARY_OPS = {
    "negative": 16, "abs": 17, "sqrt": 18, "exp": 19, "log": 20, "sin": 21,
    "cos": 22, "tan": 23, "tanh": 24, "floor": 25, "ceil": 26, "trunc": 27,
    "round": 28, "isnan": 29, "isinf": 30, "isfinite": 31, "logical_not": 32,
    "bitwise_invert": 33, "sign": 34, "square": 35, "reciprocal": 36,
    "log1p": 37, "expm1": 38, "log2": 39, "log10": 40, "sinh": 41, "cosh": 42,
    "asin": 43, "acos": 44, "atan": 45, "asinh": 46, "acosh": 47, "atanh": 48,
    "exp2": 49, "signbit": 50, "positive": None,
}
BINARY_OPS = {
    "add": 64, "subtract": 65, "multiply": 66, "divide": 67, "floor_divide": 68,
    "remainder": 69, "pow": 70, "maximum": 71, "minimum": 72, "equal": 73,
    "not_equal": 74, "less": 75, "less_equal": 76, "greater": 77,
    "greater_equal": 78, "logical_and": 79, "logical_or": 80, "logical_xor": 81,
    "bitwise_and": 82, "bitwise_or": 83, "bitwise_xor": 84,
    "bitwise_left_shift": 85, "bitwise_right_shift": 86, "atan2": 87,
    "hypot": 88, "logaddexp": 89, "copysign": 90, "fmax": 91, "fmin": 92,
    "logaddexp2": 93,
}
COMPARISONS = {"equal", "not_equal", "less", "less_equal", "greater", "greater_equal",
               "logical_and", "logical_or", "logical_xor"}
UNARY_BOOL_RESULT = {"isnan", "isinf", "isfinite", "logical_not", "signbit"}
# complex-only elementwise functions (no VM opcode: rewritten by complex.py)
COMPLEX_PARTS_OPS = {"conj", "real", "imag"}

# reduction ops (enum cubed_rop)
ROPS = {"sum": 1, "nansum": 2, "count": 3, "count_nonnan": 4, "max": 5, "min": 6,
        "prod": 7, "nanmax": 8, "nanmin": 9, "any": 10, "all": 11, "nanprod": 12,
        # pair reductions: field 0 = the lead, field 1 = its partner
        # (include/cubed_amd.h cubed_rop)
        "argmax": 13, "argmin": 14, "cprod": 15, "pair_index": 16, "pair_imag": 17,
        # var triples: field 0 = n (var: folds values, varc: folds {n, mu, M2}
        # partials), field 1 = mu, field 2 = M2 (Chan's pairwise update)
        "var": 18, "varc": 19, "var_mean": 20, "var_m2": 21}
PAIR_PARTNER = {"argmax": "pair_index", "argmin": "pair_index", "cprod": "pair_imag"}
TRIPLE_ROPS = ("var", "varc")


# ----------------------------------------------------------------- expressions


class Expr:
    dtype: np.dtype

    def children(self) -> Tuple["Expr", ...]:
        return ()

    def with_children(self, ch: Sequence["Expr"]) -> "Expr":
        return self


@dataclass(frozen=True, eq=False)
class Arg(Expr):
    """Input chunk ``index`` of the task (optionally one structured field).
    ``axes[d]`` is the space dim of leaf dim d (None: unit dim, no space dim)."""
    index: int
    dtype: np.dtype
    axes: Tuple[Optional[int], ...]
    field: Optional[str] = None


@dataclass(frozen=True, eq=False)
class Region(Expr):
    """A side-input region read by a map_direct function (merge_chunks'
    _copy_chunk core/ops.py:784, index's _read_index_chunk core/ops.py:481).
    ``region(block_id)`` gives the global slices for the task's output block;
    ``block_arg`` is the offsets-array argument that carries the block id."""
    array_name: str
    dtype: np.dtype
    axes: Tuple[Optional[int], ...]
    region: Callable[[Tuple[int, ...]], Tuple[slice, ...]]
    block_arg: int
    field: Optional[str] = None
    target: Any = None  # the side input's target (DeviceArray / virtual array)


@dataclass(frozen=True, eq=False)
class ReshapeArg(Arg):
    """Input chunk ``index`` read as a chunk of the reshaped array
    (reshape_chunks' ``_reshape_chunk``, array_api/manipulation_functions.py
    :249-275): C-order chunk bytes are unchanged, only the extents change.
    The task's input block (``in_numblocks`` grid) maps to the output block
    of the same linear offset in the ``out_chunks`` grid; ``axes`` index the
    output chunk's dims."""
    in_numblocks: Tuple[int, ...] = ()
    out_chunks: Tuple[Tuple[int, ...], ...] = ()


@dataclass(frozen=True, eq=False)
class Concat(Region):
    """concat's ``_read_concat_chunk`` (array_api/manipulation_functions.py
    :107-121): the output block is assembled along ``axis`` from regions of
    several side inputs.  ``region(block_id)`` returns a list of
    (source index, region of that source, offset along ``axis`` inside the
    output block); ``sources`` are the side inputs' targets."""
    sources: Tuple[Any, ...] = ()
    axis: int = 0


@dataclass(frozen=True, eq=False)
class Philox(Expr):
    """numpy ``Generator(Philox(key=root_seed + block_offset)).random()``
    stream over one block of the random array in C order
    (cubed/random.py:31-36).  ``chunks`` is the random array's normalized
    chunking (the block's extents give the C-order strides of the stream);
    ``axes`` maps its dims to space dims like ``Arg.axes``."""
    root_seed: int
    numblocks: Tuple[int, ...]
    block_arg: int
    axes: Tuple[Optional[int], ...]
    chunks: Tuple[Tuple[int, ...], ...]
    dtype: np.dtype = np.dtype("float64")


@dataclass(frozen=True, eq=False)
class BlockOffset(Expr):
    block_arg: int
    numblocks: Tuple[int, ...]
    dtype: np.dtype = np.dtype("int64")


@dataclass(frozen=True, eq=False)
class Iota(Expr):
    """Global index along dim ``dim`` of the array whose block is arg ``arg``
    (chunk start + local coordinate): arange / linspace / eye / tril masks.
    ``axes``/``chunks`` as for Philox."""
    dim: int
    arg: int
    axes: Tuple[Optional[int], ...]
    chunks: Tuple[Tuple[int, ...], ...]
    dtype: np.dtype = np.dtype("int64")


@dataclass(frozen=True, eq=False)
class Const(Expr):
    value: Any
    dtype: np.dtype


@dataclass(frozen=True, eq=False)
class Field(Expr):
    """A reduced field, usable after the reduction stage (epilogue)."""
    name: str
    dtype: np.dtype


@dataclass(frozen=True, eq=False)
class Unary(Expr):
    op: str
    x: Expr
    dtype: np.dtype

    def children(self):
        return (self.x,)

    def with_children(self, ch):
        return replace(self, x=ch[0])


@dataclass(frozen=True, eq=False)
class Binary(Expr):
    op: str
    a: Expr
    b: Expr
    dtype: np.dtype

    def children(self):
        return (self.a, self.b)

    def with_children(self, ch):
        return replace(self, a=ch[0], b=ch[1])


@dataclass(frozen=True, eq=False)
class Where(Expr):
    c: Expr
    a: Expr
    b: Expr
    dtype: np.dtype

    def children(self):
        return (self.c, self.a, self.b)

    def with_children(self, ch):
        return replace(self, c=ch[0], a=ch[1], b=ch[2])


@dataclass(frozen=True, eq=False)
class Cast(Expr):
    x: Expr
    dtype: np.dtype

    def children(self):
        return (self.x,)

    def with_children(self, ch):
        return replace(self, x=ch[0])


LEAF_TYPES = (Arg, Region, Philox, BlockOffset, Const, Field, Iota)


def cast(x: Expr, dtype) -> Expr:
    dtype = np.dtype(dtype)
    if x.dtype == dtype:
        return x
    if isinstance(x, Const):
        return Const(np.array(x.value).astype(dtype).item(), dtype)
    return Cast(x, dtype)


def transform(e: Expr, fn: Callable[[Expr], Optional[Expr]], memo=None) -> Expr:
    """Bottom-up rewrite; ``fn`` returns a replacement for leaves (or None)."""
    if memo is None:
        memo = {}
    key = id(e)
    if key in memo:
        return memo[key]
    if isinstance(e, LEAF_TYPES):
        r = fn(e)
        out = e if r is None else r
    else:
        ch = tuple(transform(c, fn, memo) for c in e.children())
        out = e.with_children(ch) if any(a is not b for a, b in zip(ch, e.children())) else e
    memo[key] = out
    return out


def leaves(e: Expr, out=None) -> List[Expr]:
    if out is None:
        out = []
    seen = set()

    def walk(x):
        if id(x) in seen:
            return
        seen.add(id(x))
        if isinstance(x, LEAF_TYPES):
            out.append(x)
        for c in x.children():
            walk(c)

    walk(e)
    return out


# ----------------------------------------------------------------- programs


@dataclass(frozen=True)
class ReduceField:
    name: str
    rop: str
    expr: Expr
    dtype: np.dtype  # dtype of the reduced field as stored / seen by Field()


@dataclass(frozen=True)
class ReduceStage:
    axes: Tuple[int, ...]  # reduced space dims
    fields: Tuple[ReduceField, ...]


class Program:
    """Base class of chunk programs.  Calling one on numpy data is an error:
    programs only run through the MI355X executor."""

    nargs: int

    def __call__(self, *args, **kwargs):
        raise TypeError(
            f"{type(self).__name__} is a MI355X chunk program and has no host "
            "implementation; execute the plan with cubed_amd's GPU executor"
        )


@dataclass(frozen=True, eq=False)
class ExprProgram(Program):
    """Elementwise expression (+ optional reduction) over the task's chunks."""
    ndim: int
    nargs: int
    outputs: Union[Expr, Tuple[Tuple[str, Expr], ...]]
    out_axes: Tuple[Optional[int], ...]
    reduce: Optional[ReduceStage] = None
    name: str = "expr"

    @property
    def structured(self) -> bool:
        return isinstance(self.outputs, tuple)

    def output_items(self) -> List[Tuple[Optional[str], Expr]]:
        if self.structured:
            return list(self.outputs)
        return [(None, self.outputs)]

    def all_exprs(self) -> List[Expr]:
        ex = [e for _, e in self.output_items()]
        if self.reduce is not None:
            ex += [f.expr for f in self.reduce.fields]
        return ex


@dataclass(frozen=True, eq=False)
class MatmulProgram(Program):
    """Per task: C = A @ B of two chunks, with a unit dim inserted at
    ``k_axis`` of the output (the blockwise contraction of
    linear_algebra_functions.py:35-64)."""
    nargs: int = 2
    name: str = "matmul"
    out_dtype: np.dtype = np.dtype("float64")


@dataclass(frozen=True, eq=False)
class TensordotProgram(Program):
    axes: Tuple[Tuple[int, ...], Tuple[int, ...]] = ((), ())
    nargs: int = 2
    name: str = "tensordot"
    out_dtype: np.dtype = np.dtype("float64")


@dataclass(frozen=True, eq=False)
class GemmThenProgram(Program):
    """A chunk GEMM fused (by the DAG optimizer) with the program that
    consumes its output chunk: the executor runs the GEMM into the GEMM op's
    own target geometry (``gemm_target``) and then ``then`` over it."""
    gemm: Any = None
    gemm_block_function: Any = None
    gemm_reads: Any = None
    gemm_target: Any = None
    then: Any = None
    then_block_function: Any = None
    nargs: int = 2
    name: str = "gemm+"


@dataclass(frozen=True, eq=False)
class PerBlockProgram(Program):
    """A user chunk function that takes ``block_id`` (map_blocks,
    core/ops.py:520-643): traced once per output block with the block id
    bound, so block-dependent constants (``int(sum(block_id))``) become IR
    constants.  The executor groups blocks whose traced programs are equal
    and launches each group (``trace(block_id)`` raises when untraceable)."""
    func: Any = None
    kwargs: Any = None
    args_meta: Tuple[Tuple[Any, int], ...] = ()  # (dtype, ndim) of the array args (no offsets)
    inds: Tuple[Any, ...] = ()
    out_ind: Tuple[Any, ...] = ()
    dtype: Any = None
    nargs: int = 1
    name: str = "per-block"

    def trace(self, block_id):
        import functools
        from types import SimpleNamespace

        from .tracing import trace_callable

        arrays = [SimpleNamespace(dtype=np.dtype(dt), ndim=nd) for dt, nd in self.args_meta]
        f = functools.partial(self.func, block_id=tuple(int(b) for b in block_id), **(self.kwargs or {}))
        prog = trace_callable(f, arrays, list(self.inds), self.out_ind, self.dtype, {})
        if prog is None:
            raise FusionError(f"{getattr(self.func, '__name__', self.func)!r} is not traceable for block "
                              f"{tuple(block_id)}")
        return replace(prog, nargs=self.nargs, name=getattr(self.func, "__name__", "per-block"))


@dataclass(frozen=True, eq=False)
class OpaqueProgram(Program):
    """A user function the IR could not express.  Plans containing one can be
    built (like the reference) but the GPU executor refuses to run them."""
    func: Any = None
    nargs: int = 1
    name: str = "opaque"

    def __call__(self, *args, **kwargs):
        raise NotImplementedError(
            f"function {getattr(self.func, '__name__', self.func)!r} cannot be lowered to "
            "MI355X kernels (only numpy ufuncs/reductions and cubed_amd's own chunk "
            "functions are supported)"
        )


# ----------------------------------------------------------------- builders


def right_aligned_axes(ndim_arg: int, ndim_space: int) -> Tuple[int, ...]:
    return tuple(range(ndim_space - ndim_arg, ndim_space))


def elementwise_program(op: str, arg_dtypes: Sequence[np.dtype], arg_ndims: Sequence[int],
                        out_dtype, compute_dtype=None) -> ExprProgram:
    """numpy ufunc ``op`` applied to broadcast chunks (core/ops.py:359-371)."""
    n = max(arg_ndims) if arg_ndims else 0
    out_dtype = np.dtype(out_dtype)
    args = [Arg(i, np.dtype(dt), right_aligned_axes(nd, n)) for i, (dt, nd) in
            enumerate(zip(arg_dtypes, arg_ndims))]
    e = apply_op(op, args, out_dtype, compute_dtype)
    return ExprProgram(ndim=n, nargs=len(args), outputs=e, out_axes=tuple(range(n)), name=op)


def apply_op(op: str, xs: Sequence[Expr], out_dtype, compute_dtype=None) -> Expr:
    out_dtype = np.dtype(out_dtype)
    if op == "where":
        c, a, b = xs
        ct = np.dtype(compute_dtype) if compute_dtype is not None else out_dtype
        return Where(cast(c, np.bool_), cast(a, ct), cast(b, ct), ct)
    if op == "astype":
        return cast(xs[0], out_dtype)
    if op in COMPLEX_PARTS_OPS:
        # complex -> part / conjugate: computed on the complex value itself
        # (cubed_amd/complex.py rewrites it into real expressions)
        return Unary(op, xs[0], out_dtype)
    if op in UNARY_OPS:
        x = xs[0]
        if op == "positive":
            return cast(x, out_dtype)
        if op == "abs" and np.dtype(x.dtype).kind == "c":
            return Unary(op, x, out_dtype)  # |z|, a real result
        if op in UNARY_BOOL_RESULT:
            return Unary(op, x, np.dtype(np.bool_))
        ct = np.dtype(compute_dtype) if compute_dtype is not None else out_dtype
        if op == "bitwise_invert" and is_bool(ct):
            return Unary("logical_not", cast(x, ct), ct)
        return cast(Unary(op, cast(x, ct), ct), out_dtype)
    if op in BINARY_OPS:
        a, b = xs
        if compute_dtype is not None:
            ct = np.dtype(compute_dtype)
        elif op in COMPARISONS:
            ct = np.result_type(a.dtype, b.dtype)
        else:
            ct = out_dtype
        if op in ("logical_and", "logical_or", "logical_xor"):
            ct = np.dtype(np.bool_)
        if is_bool(ct) and op in ("add", "maximum"):
            op = "logical_or"
        elif is_bool(ct) and op in ("multiply", "minimum"):
            op = "logical_and"
        e = Binary(op, cast(a, ct), cast(b, ct), np.dtype(np.bool_) if op in COMPARISONS else ct)
        return cast(e, out_dtype)
    raise NotImplementedError(f"elementwise op {op!r} has no MI355X lowering")


def reduce_program(ndim: int, arg_dtype, axes: Sequence[int], fields: Sequence[Tuple[str, str, Any]],
                   structured: bool, keepdims: bool = True, value: Optional[Expr] = None) -> ExprProgram:
    """Per-chunk reduction over ``axes`` (keepdims) of one input chunk.
    ``fields`` = (name, rop, dtype)."""
    x = value if value is not None else Arg(0, np.dtype(arg_dtype), tuple(range(ndim)))
    rfs = tuple(ReduceField(name, rop, x, np.dtype(dt)) for name, rop, dt in fields)
    stage = ReduceStage(tuple(sorted(axes)), rfs)
    if structured:
        outputs = tuple((f.name, Field(f.name, f.dtype)) for f in rfs)
    else:
        outputs = Field(rfs[0].name, rfs[0].dtype)
    if keepdims:
        out_axes = tuple(range(ndim))
    else:
        out_axes = tuple(d for d in range(ndim) if d not in axes)
    return ExprProgram(ndim=ndim, nargs=1, outputs=outputs, out_axes=out_axes, reduce=stage,
                       name="reduce")


# ----------------------------------------------------------------- fusion


class FusionError(Exception):
    pass


def _output_map(p: ExprProgram) -> Dict[Optional[str], Expr]:
    return {name: e for name, e in p.output_items()}


def _remap_leaf_axes(axes, mapping):
    """Compose leaf->space(p1) axes with space(p1)->space(p2) ``mapping``."""
    return tuple(None if a is None else mapping.get(a) for a in axes)


def _remap_expr(e: Expr, mapping: Dict[int, Optional[int]], arg_offset: int) -> Expr:
    def fn(leaf):
        if isinstance(leaf, Arg):
            return replace(leaf, index=leaf.index + arg_offset, axes=_remap_leaf_axes(leaf.axes, mapping))
        if isinstance(leaf, Region):
            return replace(leaf, block_arg=leaf.block_arg + arg_offset,
                           axes=_remap_leaf_axes(leaf.axes, mapping))
        if isinstance(leaf, Philox):
            return replace(leaf, block_arg=leaf.block_arg + arg_offset,
                           axes=_remap_leaf_axes(leaf.axes, mapping))
        if isinstance(leaf, BlockOffset):
            return replace(leaf, block_arg=leaf.block_arg + arg_offset)
        if isinstance(leaf, Iota):
            return replace(leaf, arg=leaf.arg + arg_offset, axes=_remap_leaf_axes(leaf.axes, mapping))
        return None
    return transform(e, fn)


def fuse_programs(consumer: Program, producers: Sequence[Optional[Program]],
                  producer_nargs: Sequence[int]) -> Program:
    """Program of ``consumer(producer_0(...), producer_1(...), ...)``.

    ``producers[i]`` computes consumer arg i (None: arg i stays an input and
    takes one slot).  The fused program's args are the producers' args in
    order -- the same grouping as primitive/blockwise.py fuse_multiple :420-508
    (and fuse :368-417 for a single producer)."""
    if isinstance(consumer, OpaqueProgram) or any(isinstance(p, OpaqueProgram) for p in producers if p):
        return OpaqueProgram(func=("fused", consumer, tuple(producers)), nargs=sum(producer_nargs))
    if not isinstance(consumer, ExprProgram) or not all(
            p is None or isinstance(p, ExprProgram) for p in producers):
        raise FusionError("only expression programs fuse")
    reduced_producers = [p for p in producers if p is not None and p.reduce is not None]
    if reduced_producers and consumer.reduce is not None:
        raise FusionError("two reduction stages in one pipeline")
    if len(reduced_producers) > 1:
        raise FusionError("two reducing producers feed one consumer")

    offsets = []
    acc = 0
    for n in producer_nargs:
        offsets.append(acc)
        acc += n
    nargs = acc

    if reduced_producers:
        # consumer becomes the epilogue of the producer's reduction
        pi = next(i for i, p in enumerate(producers) if p is not None and p.reduce is not None)
        prod = producers[pi]
        # every consumer arg must be that producer's output (or a constant)
        outs = _output_map(prod)
        # consumer space dim -> producer space dim, through the consumer's leaf
        # axes of arg pi and the producer's out_axes
        def sub(leaf):
            if isinstance(leaf, ReshapeArg):
                raise FusionError("reshape of a reduction result")
            if isinstance(leaf, Arg):
                if leaf.index != pi:
                    raise FusionError("epilogue reads an array other than the reduction result")
                src = outs.get(leaf.field) if leaf.field is not None else outs.get(None)
                if src is None:
                    raise FusionError(f"field {leaf.field} not produced")
                return _remap_expr(src, {}, offsets[pi])
            if isinstance(leaf, (Region, Philox, BlockOffset, Iota)):
                raise FusionError("epilogue with a side input")
            return None
        # output axes: consumer out dim -> consumer space dim -> leaf dim of
        # arg pi -> producer out dim -> producer space dim
        arg_leaves = [l for e in consumer.all_exprs() for l in leaves(e) if isinstance(l, Arg)]
        cons_axes = arg_leaves[0].axes if arg_leaves else tuple(range(consumer.ndim))
        space_to_leafdim = {a: d for d, a in enumerate(cons_axes) if a is not None}
        new_out_axes = []
        for a in consumer.out_axes:
            if a is None:
                new_out_axes.append(None)
                continue
            d = space_to_leafdim.get(a)
            new_out_axes.append(None if d is None else prod.out_axes[d])
        outputs = consumer.outputs
        if isinstance(outputs, tuple):
            outputs = tuple((n, transform(e, sub)) for n, e in outputs)
        else:
            outputs = transform(outputs, sub)
        reduce = ReduceStage(
            prod.reduce.axes,
            tuple(replace(f, expr=_remap_expr(f.expr, {a: a for a in range(prod.ndim)}, offsets[pi]))
                  for f in prod.reduce.fields))
        return ExprProgram(ndim=prod.ndim, nargs=nargs, outputs=outputs,
                           out_axes=tuple(new_out_axes), reduce=reduce,
                           name=f"{prod.name}+{consumer.name}")

    # no reducing producer: substitute producer outputs into the consumer
    # (which may itself reduce)
    def sub(leaf):
        if isinstance(leaf, Arg):
            p = producers[leaf.index]
            if p is None:
                return replace(leaf, index=offsets[leaf.index])
            if isinstance(leaf, ReshapeArg):
                # the producer's space is the input chunk's shape, not the
                # reshaped one: keep its output materialised
                raise FusionError("producer fused into a chunk reshape")
            outs = _output_map(p)
            src = outs.get(leaf.field) if leaf.field is not None else outs.get(None)
            if src is None and leaf.field is not None and isinstance(outs.get(None), (Arg, Region)) \
                    and outs[None].dtype.names and leaf.field in outs[None].dtype.names:
                # a copy of a structured array (merge_chunks, squeeze): project the field
                whole = outs[None]
                src = replace(whole, field=leaf.field, dtype=whole.dtype[leaf.field])
            if src is None:
                if leaf.field is not None and None in outs:
                    raise FusionError("structured field of an unstructured producer")
                raise FusionError("producer output missing")
            # producer space dim -> consumer space dim: via producer out dim d
            mapping = {}
            for d, pa in enumerate(p.out_axes):
                if pa is not None and d < len(leaf.axes):
                    mapping[pa] = leaf.axes[d]
            return _remap_expr(src, mapping, offsets[leaf.index])
        if isinstance(leaf, (Region, Philox, BlockOffset, Iota)):
            # the consumer's own block-id / template args are renumbered like
            # its other args (they are never produced by a fused predecessor)
            idx = leaf.arg if isinstance(leaf, Iota) else leaf.block_arg
            if producers[idx] is not None:
                raise FusionError("block-id argument produced by a fused op")
            ident = {a: a for a in range(consumer.ndim)}
            return _remap_expr(leaf, ident, offsets[idx] - idx)
        return None

    outputs = consumer.outputs
    if isinstance(outputs, tuple):
        outputs = tuple((n, transform(e, sub)) for n, e in outputs)
    else:
        outputs = transform(outputs, sub)
    reduce = None
    if consumer.reduce is not None:
        reduce = ReduceStage(consumer.reduce.axes,
                             tuple(replace(f, expr=transform(f.expr, sub)) for f in consumer.reduce.fields))
    names = "+".join(p.name for p in producers if p is not None)
    return ExprProgram(ndim=consumer.ndim, nargs=nargs, outputs=outputs, out_axes=consumer.out_axes,
                       reduce=reduce, name=f"{names}+{consumer.name}" if names else consumer.name)


# ----------------------------------------------------------------- numpy registry
# numpy / array-API callables that user code passes to blockwise / map_blocks
# / reduction, mapped to IR.  Anything else becomes an OpaqueProgram.

def _np_name_map():
    m = {}
    for name in list(UNARY_OPS) + list(BINARY_OPS):
        alias = {"pow": "power", "bitwise_invert": "invert", "asin": "arcsin",
                 "acos": "arccos", "atan": "arctan", "asinh": "arcsinh",
                 "acosh": "arccosh", "atanh": "arctanh", "atan2": "arctan2",
                 "bitwise_left_shift": "left_shift", "bitwise_right_shift": "right_shift",
                 "round": "rint"}.get(name, name)
        f = getattr(np, alias, None)
        if f is not None:
            m[f] = name
    m[np.round] = "round"
    m[np.true_divide] = "divide"
    m[np.absolute] = "abs"
    m[np.conj] = m[np.conjugate] = "conj"
    m[np.real] = "real"
    m[np.imag] = "imag"
    return m


NUMPY_ELEMENTWISE = _np_name_map()
NUMPY_REDUCTIONS = {
    np.sum: "sum", np.nansum: "nansum", np.prod: "prod", np.nanprod: "nanprod",
    np.max: "max", np.min: "min", np.amax: "max", np.amin: "min",
    np.nanmax: "nanmax", np.nanmin: "nanmin", np.any: "any", np.all: "all",
}


def reduction_result_dtype(rop: str, dtype, requested=None) -> np.dtype:
    """numpy's result dtype of ``np.<rop>(chunk, dtype=requested)``."""
    dtype = np.dtype(dtype)
    if requested is not None:
        return np.dtype(requested)
    if rop in ("any", "all"):
        return np.dtype(np.bool_)
    if rop in ("sum", "nansum", "prod", "nanprod"):
        if dtype.kind == "b":
            return np.dtype(np.int64)
        if dtype.kind == "i" and dtype.itemsize < 8:
            return np.dtype(np.int64)
        if dtype.kind == "u" and dtype.itemsize < 8:
            return np.dtype(np.uint64)
    return dtype


def acc_is_int(rop: str, dtype) -> bool:
    dtype = np.dtype(dtype)
    if rop in ("count", "count_nonnan", "any", "all", "pair_index", "var", "varc"):
        return True
    if rop in ("cprod", "pair_imag", "var_mean", "var_m2"):
        return False
    return dtype.kind in "iub"


def leaves_of_program(p) -> List[Expr]:
    """Every leaf of an ExprProgram's outputs and reduced fields."""
    out: List[Expr] = []
    for e in p.all_exprs():
        leaves(e, out)
    return out
