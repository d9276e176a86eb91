"""Plans built by the reference cubed, run on the MI355X executor.

The reference's executor plug-in contract is "any DAG" (``DagExecutor.
execute_dag``, cubed/runtime/types.py:9-14): op nodes carry a
``CubedPipeline(function, name, mappable, config)`` whose stage function is
``apply_blockwise`` (config ``BlockwiseSpec(block_function, function,
function_nargs, reads_map, write)``, primitive/blockwise.py:34-103),
``copy_read_to_write`` (config ``CubedCopySpec(read, write)``,
primitive/rechunk.py:187-192) or ``create_zarr_array`` (core/plan.py:430-
456); array nodes carry ``target`` = a ``LazyZarrArray`` (intermediates,
storage/zarr.py:8-103), a ``zarr.Array`` (sources) or a virtual array
(storage/virtual.py:14-182).  ``GpuDagExecutor.execute_dag`` recognises such
a DAG (stage functions from the ``cubed`` package) and hands it here:

* every target becomes an HBM ``DeviceArray`` with the same shape, dtype and
  chunks (virtual arrays their ``cubed_amd.storage`` counterparts, Zarr
  sources an upload op reading the store with ``cubed_amd.zarr_io``);
* a pipeline the reference optimizer fused is taken apart into the
  pipelines its ``fuse``/``fuse_multiple`` closure holds, each converted and
  fused again with this package's ``fuse``/``fuse_multiple`` (IR programs
  compose);
* the reference's own chunk functions map to their IR counterparts: the
  reduction functions (``_mean_func``/``_mean_combine``/``_mean_aggregate``,
  the nan variants, ``nxp.sum``/``max``/... with ``axis``/``keepdims``/
  ``dtype``), ``squeeze``, merge_chunks' ``_copy_chunk`` under map_direct (a
  ``Region`` leaf), ``index``'s ``_read_index_chunk`` (a Region leaf with the
  selection), matmul's ``_matmul`` chunk product and ``_chunk_sum``
  (linear_algebra_functions.py:13-78: the executor runs the product and its
  k-sum rounds as one chained GEMM), tensordot's ``_tensordot`` (:96-153,
  with the ``sum`` over the contracted dims), ``arg_reduction``'s
  ``_arg_map_func`` (a block_id map: a pair reduction with an Iota leaf) /
  ``_arg_func`` / ``_arg_combine`` / ``_arg_aggregate``, and ``random`` (``map_blocks(_random,
  ...)`` under ``func_with_block_id``, cubed/random.py:13-36) the bit-exact
  Philox leaf;
* any other chunk function is lowered by tracing it on proxies
  (``cubed_amd.tracing``): elementwise numpy / ``array_api_compat`` calls,
  Python operators, ``astype``, ``where``, with ``functools.partial``
  keyword binding;
* rechunk copies keep their read / write chunking and become copy launches.

The converted DAG keeps the reference's op names, task counts and array
names, so callbacks see the same TaskEndEvents and ``resume`` works.  After
the run, the requested arrays are written into their Zarr stores (the
paths of their ``LazyZarrArray``s, Zarr v2 via ``cubed_amd.zarr_io``) where
the reference's ``compute()`` reads them back.

What is not lowered raises ``LoweringError`` naming the op: user chunk
functions that are not elementwise, nested block keys other than
``partial_reduce``'s, and functions taking ``block_id`` other than
``random`` and ``_arg_map_func``.  The reference cannot be imported in
this image, so the tests build DAGs of the reference's shape from stand-ins
with the same class names and attributes (tests/test_reference_dag.py).
"""

from __future__ import annotations

import functools
import os
import weakref
from typing import Dict

import networkx as nx
import numpy as np

from .. import ir, tracing
from ..core.ops import UploadSpec, upload_stage
from ..core.plan import create_arrays_op
from ..lowering import LoweringError
from ..primitive.blockwise import BlockwiseSpec, apply_blockwise
from ..primitive.rechunk import copy_read_to_write
from ..primitive.types import CubedArrayProxy, CubedCopySpec, PrimitiveOperation
from ..storage import (
    DeviceArray,
    VirtualEmptyArray,
    VirtualFullArray,
    VirtualInMemoryArray,
    VirtualOffsetsArray,
)
from ..utils import normalize_chunks
from .types import CubedPipeline


def _module_of(f) -> str:
    return getattr(f, "__module__", "") or ""


def is_reference_dag(dag) -> bool:
    """True when the DAG's stage functions come from the reference package
    (``cubed.*``), not from this one."""
    for _, d in dag.nodes(data=True):
        p = d.get("pipeline")
        if p is not None:
            mod = _module_of(p.function)
            return mod == "cubed" or mod.startswith("cubed.")
    return False


class ConvertedDag:
    """The executor-side DAG of a reference DAG and where its outputs go."""

    def __init__(self, dag, targets: Dict[str, DeviceArray], sinks: Dict[str, object]):
        self.dag = dag
        self.targets = targets  # array name -> DeviceArray
        self.sinks = sinks      # array name -> reference target (LazyZarrArray / zarr.Array)


def _store_path(t):
    """Filesystem path of a reference Zarr target (a LazyZarrArray's store is
    the path string new_temp_path made; a zarr.Array's a DirectoryStore)."""
    store = getattr(t, "store", None)
    if isinstance(store, str):
        base = store
    elif store is not None and isinstance(getattr(store, "path", None), str):
        base = store.path
    else:
        raise LoweringError(f"Zarr target {t!r}: only local directory stores are supported")
    sub = getattr(t, "path", "") if type(t).__name__ != "LazyZarrArray" else ""
    return os.path.join(base, sub) if sub else base


class _Converter:
    def __init__(self, dag):
        self.ref = dag
        self.arrays: Dict[int, object] = {}
        self.sources = []  # (node name, ZarrV2Array, DeviceArray): uploads to add

    # -- arrays ----------------------------------------------------------------
    def array(self, t, name):
        key = id(t)
        if key in self.arrays:
            return self.arrays[key]
        kind = type(t).__name__
        if kind == "LazyZarrArray":
            out = DeviceArray(t.shape, t.dtype, t.chunks, name=name)
        elif kind == "VirtualEmptyArray":
            out = VirtualEmptyArray(t.shape, t.dtype, t.chunks)
        elif kind == "VirtualFullArray":
            out = VirtualFullArray(t.shape, t.dtype, t.chunks, fill_value=t.fill_value)
        elif kind == "VirtualOffsetsArray":
            out = VirtualOffsetsArray(t.shape)
        elif kind == "VirtualInMemoryArray":
            out = VirtualInMemoryArray(np.asarray(t.array), t.chunks)
        elif kind == "Array" and hasattr(t, "store"):
            # an existing Zarr array (from_zarr / a computed intermediate)
            from ..zarr_io import ZarrV2Array

            src = ZarrV2Array.open(_store_path(t))
            out = DeviceArray(src.shape, src.dtype, src.chunks, name=name)
            self.sources.append((name, src, out))
        elif isinstance(t, (DeviceArray, VirtualEmptyArray, VirtualFullArray, VirtualOffsetsArray,
                            VirtualInMemoryArray)):
            out = t
        else:
            raise LoweringError(f"array {name}: reference target {kind} is not supported")
        self.arrays[key] = out
        return out

    def proxy(self, p, name):
        return CubedArrayProxy(self.array(p.array, name), p.chunks)

    # -- chunk functions -------------------------------------------------------
    def program(self, op, cfg, reads, write):
        """IR program of the reference chunk function ``cfg.function``."""
        out = write.array
        nd = out.ndim
        first = tuple(0 for _ in range(nd))
        try:
            args = list(cfg.block_function(("out",) + first))
        except Exception as e:  # noqa: BLE001 -- a key function that fails is not lowerable
            raise LoweringError(f"op {op}: block function failed on {first}: {e}") from None
        names = []
        for nci in args:
            if not (isinstance(nci, tuple) and nci and isinstance(nci[0], str)):
                raise LoweringError(f"op {op}: nested block keys (contractions / partial reductions) "
                                    "of reference chunk functions are not lowered")
            names.append(nci[0])
        arrays = [reads[n].array for n in names]
        self._check_alignment(op, cfg, arrays, out)
        inds = [tuple(range(nd - a.ndim, nd)) for a in arrays]
        fn = cfg.function
        if _is_reference_random(fn):  # the random op itself (not fused)
            fn = _random_leaf(fn, write.chunks, out.shape, out.dtype)
        prog = tracing.trace_callable(fn, arrays, inds, tuple(range(nd)), out.dtype, {})
        if prog is None:
            raise LoweringError(
                f"op {op}: chunk function {cfg.function!r} is not traceable to a fused chunk program "
                "(elementwise numpy calls and operators are; reductions, side-input reads and "
                "block_id functions other than random are not)")
        return prog

    def blockwise(self, name, p, meta):
        """Our PrimitiveOperation for a reference blockwise pipeline.  A
        pipeline the reference optimizer fused (``fuse`` / ``fuse_multiple``
        closures, primitive/blockwise.py:368-508) is taken apart into the
        pipelines it closes over, each converted, and fused again with this
        package's ``fuse`` / ``fuse_multiple`` (which compose IR programs)."""
        parts = _fused_parts(p.config.function)
        if parts is not None:
            from ..primitive.blockwise import fuse, fuse_multiple

            kind, data = parts
            if kind == "fuse":
                p1, p2 = data
                return fuse(self.blockwise(_written_name(p1, [p2], name), p1, meta), self.blockwise(name, p2, meta))
            consumer, preds = data
            return fuse_multiple(self.blockwise(name, consumer, meta),
                                 *[self.blockwise(_written_name(pp, [consumer], name), pp, meta)
                                   if pp is not None else None for pp in preds])
        cfg = p.config
        reads = {n: self.proxy(px, n) for n, px in cfg.reads_map.items()}
        write = self.proxy(cfg.write, name)
        prog = self.known_program(name, cfg, reads, write)
        if prog is None:
            prog = self.program(name, cfg, reads, write)
        spec = BlockwiseSpec(cfg.block_function, prog, cfg.function_nargs, reads, write)
        pipe = CubedPipeline(apply_blockwise, p.name, p.mappable, spec)
        return PrimitiveOperation(pipeline=pipe, target_array=write.array, **meta)

    def known_program(self, op, cfg, reads, write):
        """IR for the reference's own chunk functions, which are not
        elementwise and so not traceable: the reduction functions
        (statistical_functions.py:54-100, nan_functions.py:21-77, ``nxp.sum``
        / ``max`` / ... with ``axis``/``keepdims``/``dtype``), ``squeeze``
        (core/ops.py:1156-1169) and merge_chunks' ``_copy_chunk`` under
        map_direct (core/ops.py:646-787).  None: not one of them."""
        base, kw, wrappers = _unwrap(cfg.function)
        bname = getattr(base, "__name__", "")
        bmod = _module_of(base)
        out = write.array
        first = tuple(0 for _ in range(out.ndim))
        keys = list(cfg.block_function(("out",) + first))
        if bname == "_copy_chunk" and bmod.startswith("cubed"):
            src_arr = kw.get("arrays", (None,))[0]
            tgt = getattr(src_arr, "zarray_maybe_lazy", None)
            if tgt is None or "target_chunks" not in kw:
                raise LoweringError(f"op {op}: merge_chunks without its side input / target chunks")
            src = self.array(tgt, src_arr.name)
            names = [k[0] for k in keys]
            block_arg = next((i for i, n in enumerate(names)
                              if isinstance(reads[n].array, VirtualOffsetsArray)), None)
            if block_arg is None:
                raise LoweringError(f"op {op}: map_direct without its block offsets argument")
            from ..core.ops import _merged_region

            leaf = ir.Region(src_arr.name, src.dtype, tuple(range(src.ndim)),
                             _merged_region(tuple(tuple(c) for c in kw["target_chunks"])), block_arg, target=src)
            return ir.ExprProgram(ndim=out.ndim, nargs=len(keys), outputs=leaf,
                                  out_axes=tuple(range(out.ndim)), name="map_direct")
        if bname == "_read_index_chunk" and bmod.startswith("cubed"):
            return self._index_program(op, kw, keys, reads, out)
        if bmod.startswith("cubed") and bname in ("_arg_map_func", "_arg_func", "_arg_combine", "_arg_aggregate"):
            return self._arg_program(op, bname, kw, keys, reads, out)
        if bname == "_partial_reduce" and bmod.startswith("cubed"):
            return self._partial_reduce_program(op, cfg, kw, reads, first)
        if wrappers:
            return None  # other block_id / map_direct functions: traced (random) or refused
        if bname == "_matmul" and bmod.startswith("cubed") and len(keys) == 2:
            # per (i, k, j) task: A_ik @ B_kj with a unit k dim (linear_algebra_functions.py:62-64)
            return ir.MatmulProgram(out_dtype=np.dtype(out.dtype))
        if bname == "_tensordot" and bmod.startswith("cubed") and len(keys) == 2 and "axes" in kw:
            # tensordot's chunk contraction with a unit dim per contracted axis
            # (linear_algebra_functions.py:96-153); its sum over those dims follows
            axes = tuple(tuple(int(a) for a in ((ax,) if isinstance(ax, int) else ax)) for ax in kw["axes"])
            return ir.TensordotProgram(axes=axes, out_dtype=np.dtype(out.dtype))
        if len(keys) != 1 or not isinstance(keys[0], tuple):
            return None
        x = reads[keys[0][0]].array
        from .. import chunkfuncs as CF

        reductions = {"_mean_func": CF._mean_func, "_mean_combine": CF._mean_combine,
                      "_nanmean_func": CF._nanmean_func, "_nanmean_combine": CF._nanmean_combine,
                      "_chunk_sum": CF._chunk_sum}
        red = None
        if bmod.startswith("cubed") and bname in reductions:
            red = reductions[bname]
        elif bname in _NUMPY_REDUCTION_NAMES and "axis" in kw and (
                bmod.startswith("numpy") or bmod.startswith("array_api_compat") or bmod.startswith("cubed")):
            red = CF.as_chunk_reduction(getattr(np, bname))
        if red is not None:
            axis = kw["axis"]
            axis = (axis,) if isinstance(axis, int) else tuple(axis)
            extra = {k: v for k, v in kw.items() if k not in ("axis", "keepdims")}
            return red.program(x.ndim, x.dtype, axis, keepdims=bool(kw.get("keepdims", True)), **extra)
        if bmod.startswith("cubed") and bname in ("_mean_aggregate", "_nanmean_aggregate"):
            return CF._mean_aggregate.program(x.ndim, x.dtype)
        if bname == "squeeze" and "axis" in kw:
            axis = kw["axis"]
            axis = (axis,) if isinstance(axis, int) else tuple(axis)
            axes = tuple(range(x.ndim))
            outputs = ir.Arg(0, x.dtype, axes) if not x.dtype.names else \
                tuple((f, ir.Arg(0, x.dtype[f], axes, field=f)) for f in x.dtype.names)
            return ir.ExprProgram(ndim=x.ndim, nargs=1, outputs=outputs,
                                  out_axes=tuple(d for d in axes if d not in axis), name="squeeze")
        return None

    def _arg_program(self, op, bname, kw, keys, reads, out):
        """``arg_reduction``'s chunk functions (core/ops.py:1093-1153): the
        block_id map ``_arg_map_func`` -- per block {i, v} with i the GLOBAL
        index (block offset + local argmax) -- is one pair reduction over the
        block with an Iota leaf for i; ``_arg_combine`` is this package's pair
        reduction over {v, i} (chunkfuncs.ArgReduction: first NaN, else the
        larger / smaller value, ties to the smaller index -- numpy's
        argmax/argmin, so the combine order does not change the result);
        ``_arg_func`` passes the pairs through and ``_arg_aggregate`` keeps i."""
        from .. import chunkfuncs as CF

        x = reads[keys[0][0]].array
        dt = np.dtype(x.dtype)
        n = x.ndim
        axes = tuple(range(n))
        if bname in ("_arg_map_func", "_arg_combine"):
            name = getattr(kw.get("arg_func"), "__name__", "")
            if name not in ("argmax", "argmin"):
                raise LoweringError(f"op {op}: arg reduction with {kw.get('arg_func')!r}")
        if bname == "_arg_map_func":
            if dt.names or dt.kind not in "fiub":
                raise LoweringError(f"op {op}: arg reduction of {dt}")
            axis = int(kw["axis"])
            chunks = tuple(tuple(c) for c in normalize_chunks(x.chunks, x.shape, dt))
            idx = ir.Iota(axis, 0, axes, chunks)
            fields = (ir.ReduceField("v", name, ir.Arg(0, dt, axes), dt),
                      ir.ReduceField("i", "pair_index", idx, np.dtype(np.int64)))
            return ir.ExprProgram(ndim=n, nargs=len(keys),
                                  outputs=tuple((f, ir.Field(f, fd.dtype)) for f, fd in
                                                (("i", fields[1]), ("v", fields[0]))),
                                  out_axes=axes, reduce=ir.ReduceStage((axis,), fields), name="_arg_map_func")
        if bname == "_arg_func":
            return ir.ExprProgram(ndim=n, nargs=1,
                                  outputs=tuple((f, ir.Arg(0, dt[f], axes, field=f)) for f in ("i", "v")),
                                  out_axes=axes, name="_arg_func")
        if bname == "_arg_combine":
            axis = kw["axis"]
            axis = (axis,) if isinstance(axis, int) else tuple(axis)
            return CF.ArgReduction(name).program(n, dt, axis, keepdims=True)
        return CF._arg_aggregate.program(n, dt)

    def _partial_reduce_program(self, op, cfg, kw, reads, first):
        """``partial_reduce``'s ``_partial_reduce`` (core/ops.py:1008-1090,
        reduction(..., use_new_impl=True) and tree_reduce): the block
        function yields an ITERATOR of input keys (a group of blocks), which
        this package's partial_reduce lowers the same way -- one task
        reduces the merged view of its group with the initial function's
        fields (reduce_func's when there is none), e.g. mean's {n, total}."""
        group = cfg.block_function(("out",) + first)[0]
        k0 = next(iter(group))
        x = reads[k0[0]].array
        f = kw.get("initial_func") or kw.get("reduce_func")
        r = self._chunk_reduction(op, f)
        axis = kw["axis"]
        axis = (axis,) if isinstance(axis, int) else tuple(axis)
        return r.program(x.ndim, x.dtype, axis, keepdims=True)

    def _chunk_reduction(self, op, f):
        """This package's ChunkReduction for a reference reduction callable
        (a partial of ``_mean_func`` & co. or of a numpy reduction)."""
        from .. import chunkfuncs as CF

        base, kw, _ = _unwrap(f)
        name, mod = getattr(base, "__name__", ""), _module_of(base)
        named = {"_mean_func": CF._mean_func, "_mean_combine": CF._mean_combine,
                 "_nanmean_func": CF._nanmean_func, "_nanmean_combine": CF._nanmean_combine,
                 "_chunk_sum": CF._chunk_sum}
        inner = None
        if mod.startswith("cubed") and name in named:
            inner = named[name]
        elif name in _NUMPY_REDUCTION_NAMES:
            inner = CF.as_chunk_reduction(getattr(np, name))
        if inner is None:
            raise LoweringError(f"op {op}: partial_reduce with {f!r} is not lowered")
        kw = {k: v for k, v in kw.items() if k not in ("axis", "keepdims")}
        return CF._BoundReduction(inner, kw) if kw else inner

    def _index_program(self, op, kw, keys, reads, out):
        """``index``'s map_direct function (core/ops.py:374-517): output block
        b reads ``x.oindex[_target_chunk_selection(target_chunks, b,
        selection)]`` -- a Region leaf over the side input with this package's
        ``_read_index_region`` (same selection arithmetic)."""
        from ..core.ops import _read_index_region

        src_arr = kw.get("arrays", (None,))[0]
        tgt = getattr(src_arr, "zarray_maybe_lazy", None)
        if tgt is None or "selection" not in kw or "target_chunks" not in kw:
            raise LoweringError(f"op {op}: index without its side input / selection")
        src = self.array(tgt, src_arr.name)
        norm, axes, k = [], [], 0
        for d, sel in enumerate(kw["selection"]):
            n = src.shape[d]
            if isinstance(sel, slice):
                start, stop, step = sel.indices(n)
                norm.append(slice(start, stop, step))
                axes.append(k)
                k += 1
            elif isinstance(sel, (list, tuple)):
                norm.append([int(v) + n if int(v) < 0 else int(v) for v in sel])
                axes.append(k)
                k += 1
            else:
                v = int(sel)
                norm.append(v + n if v < 0 else v)
                axes.append(None)
        names = [kk[0] for kk in keys]
        block_arg = next((i for i, nm in enumerate(names) if isinstance(reads[nm].array, VirtualOffsetsArray)), None)
        if block_arg is None:
            raise LoweringError(f"op {op}: map_direct without its block offsets argument")
        region = _read_index_region(tuple(norm), tuple(tuple(c) for c in kw["target_chunks"]))
        leaf = ir.Region(src_arr.name, src.dtype, tuple(axes), region, block_arg, target=src)
        return ir.ExprProgram(ndim=out.ndim, nargs=len(keys), outputs=leaf, out_axes=tuple(range(out.ndim)),
                              name="map_direct")

    def _check_alignment(self, op, cfg, arrays, out):
        """The trailing-dims (numpy broadcasting) index mapping the traced
        program assumes: arg block coordinates equal the output's trailing
        coordinates, or 0 along dims where the arg has one block."""
        if out.ndim == 0:
            return
        probes = {tuple(0 for _ in out.numblocks), tuple(n - 1 for n in out.numblocks)}
        for key in probes:
            for nci, a in zip(cfg.block_function(("out",) + key), arrays):
                coords = tuple(nci[1:])
                nb = getattr(a, "numblocks", None)
                if nb is None:
                    nb = tuple(len(c) for c in normalize_chunks(a.chunks, a.shape, a.dtype))
                tail = key[len(key) - len(coords):] if coords else ()
                want = tuple(0 if n == 1 else k for n, k in zip(nb, tail))
                if coords != want:
                    raise LoweringError(f"op {op}: block index mapping {key} -> {coords} is not "
                                        "elementwise (broadcast over trailing dims)")

    # -- ops -------------------------------------------------------------------
    def convert(self):
        ref = self.ref
        g = nx.MultiDiGraph()
        nodes = dict(ref.nodes(data=True))
        targets: Dict[str, DeviceArray] = {}
        sinks: Dict[str, object] = {}
        # arrays first: every op's reads / write resolve to the same objects
        for name, d in nodes.items():
            if "target" in d and d.get("target") is not None:
                conv = self.array(d["target"], name)
                if isinstance(conv, DeviceArray):
                    targets[name] = conv
                    if type(d["target"]).__name__ == "LazyZarrArray":
                        sinks[name] = d["target"]
        for name, d in nodes.items():
            attrs = {k: v for k, v in d.items() if k not in ("pipeline", "primitive_op", "target")}
            if "target" in d:
                t = d["target"]
                attrs["target"] = None if t is None else self.array(t, name)
            p = d.get("pipeline")
            if p is not None:
                op = self.op(name, p, d.get("primitive_op"), targets)
                if op is not None:
                    attrs.update(primitive_op=op, pipeline=op.pipeline)
            g.add_node(name, **attrs)
        for u, v, k in ref.edges(keys=True):
            g.add_edge(u, v, key=k)
        # Zarr sources without a producing op: an upload op each
        for i, (name, src, tgt) in enumerate(self.sources):
            if any("pipeline" in nodes.get(u, {}) for u in ref.predecessors(name)):
                continue
            up = f"upload-{name}"
            pipe = CubedPipeline(upload_stage, up, [], UploadSpec(src, tgt))
            op = PrimitiveOperation(pipeline=pipe, target_array=tgt, projected_mem=0, allowed_mem=0,
                                    reserved_mem=0, num_tasks=tgt.nchunks, fusable=False)
            g.add_node(up, name=up, op_name="upload", type="op", primitive_op=op, pipeline=pipe)
            g.add_edge(up, name)
        return ConvertedDag(nx.freeze(g), targets, sinks)

    def op(self, name, p, pop, targets):
        fname = getattr(p.function, "__name__", "")
        cfg = p.config
        meta = dict(projected_mem=getattr(pop, "projected_mem", 0), allowed_mem=getattr(pop, "allowed_mem", 0),
                    reserved_mem=getattr(pop, "reserved_mem", 0),
                    num_tasks=getattr(pop, "num_tasks", 1), fusable=getattr(pop, "fusable", False))
        if fname == "create_zarr_array":
            devs = [self.array(t, getattr(t, "name", None) or "array") for t in p.mappable]
            devs = [t for t in devs if isinstance(t, DeviceArray)]
            op = create_arrays_op(devs, meta["allowed_mem"], meta["reserved_mem"])
            return PrimitiveOperation(pipeline=op.pipeline, target_array=None, **meta)
        if fname == "apply_blockwise":
            return self.blockwise(name, p, meta)
        if fname == "copy_read_to_write":
            spec = CubedCopySpec(self.proxy(cfg.read, name + "-read"), self.proxy(cfg.write, name))
            pipe = CubedPipeline(copy_read_to_write, p.name, p.mappable, spec)
            return PrimitiveOperation(pipeline=pipe, target_array=spec.write.array, **meta)
        raise LoweringError(f"op {name}: reference stage function {fname or p.function!r} is not supported")


def _written_name(producer, consumers, default):
    """The array name a fused-away producer pipeline writes: the key its
    consumer's ``reads_map`` holds for that target (the DAG no longer has a
    node for it)."""
    t = producer.config.write.array
    for c in consumers:
        for k, px in getattr(c.config, "reads_map", {}).items():
            if px.array is t:
                return k
        inner = _fused_parts(c.config.function)
        if inner is not None:
            kind, data = inner
            subs = list(data) if kind == "fuse" else [data[0]] + [q for q in data[1] if q is not None]
            found = _written_name(producer, subs, None)
            if found is not None:
                return found
    return default


# ------------------------------------------------------------------ function anatomy
_NUMPY_REDUCTION_NAMES = {"sum", "prod", "max", "min", "nansum", "nanmax", "nanmin", "all", "any"}


def _cells(fn):
    code = getattr(fn, "__code__", None)
    if code is None or not fn.__closure__:
        return {}
    out = {}
    for n, c in zip(code.co_freevars, fn.__closure__):
        try:
            out[n] = c.cell_contents
        except ValueError:
            pass
    return out


def _fused_parts(fn):
    """("fuse", (pipeline1, pipeline2)) / ("fuse_multiple", (pipeline,
    predecessor pipelines)) for the reference's fused chunk functions, else
    None."""
    if getattr(fn, "__name__", "") != "fused_func":
        return None
    cells = _cells(fn)
    if "pipeline1" in cells and "pipeline2" in cells:
        return "fuse", (cells["pipeline1"], cells["pipeline2"])
    if "pipeline" in cells and "predecessor_pipelines" in cells:
        return "fuse_multiple", (cells["pipeline"], list(cells["predecessor_pipelines"]))
    return None


def _unwrap(fn):
    """(base function, merged partial keywords, wrappers): through
    ``functools.partial`` layers and map_blocks' / map_direct's ``wrap``
    closures (core/ops.py:531-560, 680-697) down to the chunk function."""
    kw = {}
    wrappers = []
    for _ in range(16):
        if isinstance(fn, functools.partial):
            kw = {**(fn.keywords or {}), **kw}
            fn = fn.func
            continue
        if getattr(fn, "__name__", "") == "wrap" and "func" in _cells(fn):
            wrappers.append(fn)
            fn = _cells(fn)["func"]
            continue
        break
    return fn, kw, wrappers


# ------------------------------------------------------------------ random
def _is_reference_random(f) -> bool:
    """``partial(wrap, numblocks=..., root_seed=...)`` where ``wrap`` is
    map_blocks' ``func_with_block_id`` closure over ``cubed.random._random``."""
    if not isinstance(f, functools.partial):
        return False
    inner = f.func
    if getattr(inner, "__name__", "") != "wrap" or not inner.__closure__:
        return False
    kw = f.keywords or {}
    if "root_seed" not in kw or "numblocks" not in kw:
        return False
    for cell in inner.__closure__:
        try:
            v = cell.cell_contents
        except ValueError:
            continue
        if getattr(v, "__name__", "") == "_random" and _module_of(v).endswith("random"):
            return True
    return False


def _random_leaf(f, out_chunks, shape, dtype):
    """A traceable stand-in for the reference random chunk function: the
    Philox leaf reading the block offset from the offsets argument."""
    kw = f.keywords
    nd = len(shape)
    chunks = normalize_chunks(out_chunks, shape, dtype)

    def standin(*args):
        off = args[-1]
        if not isinstance(off, tracing._Proxy) or not isinstance(off.expr, ir.Arg):
            raise tracing._Untraceable("random without its offsets argument")
        leaf = ir.Philox(root_seed=int(kw["root_seed"]), numblocks=tuple(kw["numblocks"]),
                         block_arg=off.expr.index, axes=tuple(range(nd)), chunks=chunks)
        return tracing._Proxy(leaf, nd)

    return standin


# ------------------------------------------------------------------ run
_CACHE: Dict[int, tuple] = {}


def _drop(key):
    _CACHE.pop(key, None)


def convert_reference_dag(dag) -> ConvertedDag:
    """The executor-side DAG of a reference DAG, cached while it lives."""
    key = id(dag)
    hit = _CACHE.get(key)
    if hit is not None and hit[0]() is dag:
        return hit[1]
    conv = _Converter(dag).convert()
    _CACHE[key] = (weakref.ref(dag), conv)
    weakref.finalize(dag, _drop, key)
    return conv


def execute_reference_dag(executor, dag, callbacks=None, array_names=None, resume=None, spec=None,
                          **kwargs):
    """Run a reference-built DAG on ``executor`` and write the requested
    arrays to their Zarr stores.  With ``resume``, an array whose Zarr store
    already holds every chunk counts as computed (cubed/runtime/pipeline.py
    :25-33, whatever process wrote it); one that an op still to run reads is
    uploaded from its store first.  Afterwards the converted arrays' HBM is
    released: the results live in their Zarr stores, which is where the
    reference reads them from (and the reference keeps finalized DAGs -- so
    this conversion -- alive in an lru_cache, core/plan.py:178)."""
    conv = convert_reference_dag(dag)
    _mark_zarr_complete(executor, conv, resume)
    try:
        executor.execute_dag(conv.dag, callbacks=callbacks, array_names=array_names, resume=resume,
                             spec=spec, **kwargs)
        write_back(conv, array_names)
    finally:
        for d in conv.targets.values():
            d.zarr_complete = False
            if d.allocated:
                d.release()
    return conv


def _mark_zarr_complete(executor, conv: ConvertedDag, resume):
    """resume: flag the arrays whose Zarr sink is complete on disk (the
    pipeline walk skips their ops), and upload those an op still to run
    reads."""
    from ..zarr_io import ZarrV2Array, upload_zarr, zarr_complete
    from .pipeline import already_computed

    for name, d in conv.targets.items():
        t = conv.sinks.get(name)
        d.zarr_complete = bool(resume) and t is not None and not d.written and zarr_complete(_store_path(t))
    if not resume:
        return
    dag = conv.dag
    nodes = dict(dag.nodes(data=True))
    for n, nd in nodes.items():
        if "pipeline" not in nd or already_computed(n, dag, nodes, resume=True):
            continue
        for a in dag.predecessors(n):
            d = nodes[a].get("target")
            if isinstance(d, DeviceArray) and getattr(d, "zarr_complete", False) and not d.written:
                executor.allocate(d)
                upload_zarr(ZarrV2Array.open(_store_path(conv.sinks[a])), d)
                d.written = True


def write_back(conv: ConvertedDag, array_names):
    """The requested arrays, device -> their reference Zarr stores (created
    here with the LazyZarrArray's shape, dtype, chunks and fill value);
    arrays found complete on disk by a resume are not rewritten."""
    from ..zarr_io import ZarrV2Array, write_device_array

    for name in array_names or ():
        t = conv.sinks.get(name)
        d = conv.targets.get(name)
        if t is None or d is None or getattr(d, "zarr_complete", False):
            continue
        dst = ZarrV2Array.create(_store_path(t), d.shape, d.dtype, d.chunks,
                                 fill_value=getattr(t, "fill_value", None), mode="a")
        write_device_array(d, dst)


__all__ = ["is_reference_dag", "convert_reference_dag", "execute_reference_dag", "ConvertedDag"]
