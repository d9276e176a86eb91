"""Lowering of fused Cubed pipelines to libcubed_amd launches.

For one pipeline (an op node of the finalized DAG) this builds, once, every
device-side table its launch needs:

* ``FusedLaunch``: an IR ``ExprProgram`` -> ``cubed_program_t`` (register
  allocation of the two-address VM, constant pool, CAST insertion for the
  program's value type) + a ``cubed_task_t`` row per output chunk (the leaf
  and output views of that chunk, in a canonical dim order shared by all
  tasks: unit dims dropped, reduced dims ordered for kernel A or B, adjacent
  dims coalesced when every view allows it).
* ``CopyLaunch``: rechunk / merge_chunks / index / pure copies as a table of
  (source chunk x target chunk) boxes.
* ``GemmLaunch``: matmul / tensordot chunk products.

The task key resolution follows apply_blockwise (primitive/blockwise.py:61-84):
``block_function(('out',) + out_key)`` gives each argument's chunk key(s).
A leaf reads either one chunk (a strided sub-box), a run of unit-extent
chunks (partials being merged: one stride = the slot stride), or -- for any
other multi-chunk read -- a per-task gather into a contiguous scratch buffer.
"""

from __future__ import annotations

import ctypes
import dataclasses
import itertools
import math
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as nat
from . import ir
from .storage import (
    DeviceArray,
    HostArray,
    VirtualEmptyArray,
    VirtualFullArray,
    VirtualInMemoryArray,
    VirtualOffsetsArray,
    c_strides,
)
from .utils import block_id_to_offset, flatten_keys, offset_to_block_id


class LoweringError(RuntimeError):
    pass


LEAF_ARRAY, LEAF_PHILOX, LEAF_OFFSET, LEAF_IOTA = 0, 1, 2, 3
V_F32, V_F64, V_I64 = 0, 1, 2


# ------------------------------------------------------------------ views


@dataclass
class ArrView:
    """A strided view: base byte address + per-dim (extent, stride) in
    elements of ``dtype`` (array-dim order)."""
    base: int
    extent: List[int]
    stride: List[int]
    dtype: np.dtype


def chunk_view(arr: DeviceArray, coords, field=None) -> ArrView:
    ext = list(arr.chunk_extent(coords))
    return ArrView(arr.chunk_addr(coords, field), ext, list(c_strides(ext)),
                   arr.field_dtype(field))


def merged_view(arr: DeviceArray, keys, field=None) -> Optional[ArrView]:
    """One view over a set of chunk keys, or None if irregular.  Regular =
    along each dim either one chunk, or a contiguous run of chunks that all
    have extent 1 there (reduction partials): that dim's stride is the slot
    stride, since every chunk occupies one fixed-size slot."""
    coords = [k[1:] for k in keys]
    nd = arr.ndim
    if nd == 0:
        return chunk_view(arr, coords[0], field)
    per_dim = [sorted({c[d] for c in coords}) for d in range(nd)]
    if math.prod(len(p) for p in per_dim) != len(set(map(tuple, coords))):
        return None
    if arr.world != 1:
        return None
    first = tuple(p[0] for p in per_dim)
    base_ext = arr.chunk_extent(first)
    ext, stride = [], []
    inner = c_strides(base_ext)
    slot_elems = arr.slot_stride_elems(field)
    for d in range(nd):
        p = per_dim[d]
        if len(p) == 1:
            ext.append(base_ext[d])
            stride.append(inner[d])
            continue
        if p != list(range(p[0], p[-1] + 1)):
            return None
        if any(arr.chunk_extent(tuple(p2 if dd == d else first[dd] for dd in range(nd)))[d] != 1
               for p2 in p):
            return None
        slot_step = math.prod(arr.numblocks[d + 1:])
        ext.append(len(p))
        stride.append(slot_step * slot_elems)
    return ArrView(arr.chunk_addr(first, field), ext, stride, arr.field_dtype(field))


def region_pieces(arr, region) -> List[Tuple[Tuple[int, ...], List[Tuple[int, int, int]], List[int]]]:
    """Split a region (per dim: slice with step, int, or list) of ``arr``
    into per-chunk pieces: (chunk coords, per-dim (in-chunk start, count,
    step), per-region-dim output offsets).  Int dims produce no region dim."""
    per_dim = []
    for d, s in enumerate(region):
        n = arr.shape[d]
        pieces = []  # (chunk, local_start, count, step, out_offset)
        if isinstance(s, slice):
            start, stop, step = s.start or 0, s.stop if s.stop is not None else n, s.step or 1
            i, out = start, 0
            while i < stop:
                c = arr.chunk_of(d, i)
                cst = arr.chunk_start(tuple(c if dd == d else 0 for dd in range(arr.ndim)))[d]
                cend = cst + arr.chunk_extent(tuple(c if dd == d else 0 for dd in range(arr.ndim)))[d]
                last = min(stop, cend)
                cnt = (last - i + step - 1) // step
                pieces.append((c, i - cst, cnt, step, out))
                out += cnt
                i += cnt * step
            per_dim.append((pieces, True))
        elif isinstance(s, list):
            for j, v in enumerate(s):
                c = arr.chunk_of(d, v)
                cst = arr.chunk_start(tuple(c if dd == d else 0 for dd in range(arr.ndim)))[d]
                pieces.append((c, v - cst, 1, 1, j))
            per_dim.append((pieces, True))
        else:
            v = int(s)
            c = arr.chunk_of(d, v)
            cst = arr.chunk_start(tuple(c if dd == d else 0 for dd in range(arr.ndim)))[d]
            per_dim.append(([(c, v - cst, 1, 1, 0)], False))
    out = []
    for combo in itertools.product(*[p for p, _ in per_dim]):
        coords = tuple(c for c, *_ in combo)
        local = [(ls, cnt, st) for _, ls, cnt, st, _ in combo]
        offs = [o for (_, _, _, _, o), (_, keep) in zip(combo, per_dim) if keep]
        out.append((coords, local, offs))
    return out


def region_chunk_keys(arr: DeviceArray, region):
    """Chunk keys of a region made of whole chunks (unit-step slices aligned
    to chunk boundaries), else None."""
    ranges = []
    for d, s in enumerate(region):
        if not isinstance(s, slice) or (s.step or 1) != 1:
            return None
        start, stop = s.start or 0, s.stop if s.stop is not None else arr.shape[d]
        st = arr._starts[d]
        if start not in st or stop not in st:
            return None
        ranges.append(range(st.index(start), st.index(stop)))
    return [(arr.name,) + c for c in itertools.product(*ranges)]


def region_view(arr: DeviceArray, region, field=None) -> Optional[ArrView]:
    """View of a region that lies inside one chunk (None otherwise)."""
    pieces = region_pieces(arr, region)
    if len(pieces) != 1:
        return None
    coords, local, _ = pieces[0]
    ext = arr.chunk_extent(coords)
    inner = c_strides(ext)
    off = sum(ls * inner[d] for d, (ls, _, _) in enumerate(local))
    isz = arr.field_dtype(field).itemsize
    # int-indexed dims keep extent 1 (the leaf maps them to no space dim)
    return ArrView(arr.chunk_addr(coords, field) + off * isz,
                   [cnt for (_, cnt, _) in local],
                   [inner[d] * st for d, (_, _, st) in enumerate(local)],
                   arr.field_dtype(field))


# ------------------------------------------------------------------ box copies


@dataclass
class Box:
    src: int
    dst: int
    extent: List[int]
    sstride: List[int]
    dstride: List[int]


def boxes_for_region(src: DeviceArray, region, dst_base: int, dst_strides: Sequence[int],
                     field=None) -> List[Box]:
    """Boxes copying ``src[region]`` into a destination view whose dims are
    the region's non-int dims."""
    isz = src.field_dtype(field).itemsize
    out = []
    for coords, local, offs in region_pieces(src, region):
        ext = src.chunk_extent(coords)
        inner = c_strides(ext)
        base = src.chunk_addr(coords, field) + sum(ls * inner[d] for d, (ls, _, _) in enumerate(local)) * isz
        keep = [d for d, s in enumerate(region) if not _is_int_sel(s)]
        extent = [local[d][1] for d in keep]
        sstr = [inner[d] * local[d][2] for d in keep]
        dbase = dst_base + sum(o * s for o, s in zip(offs, dst_strides)) * isz
        out.append(Box(base, dbase, extent, sstr, list(dst_strides)))
    return out


def _is_int_sel(s):
    return not isinstance(s, (slice, list))


def canonical_boxes(boxes: List[Box]):
    """Drop unit dims, coalesce dims contiguous on both sides; returns
    (ndim, boxes) with every box padded to the same ndim."""
    canon = []
    for b in boxes:
        dims = [(e, s, d) for e, s, d in zip(b.extent, b.sstride, b.dstride) if e != 1]
        if not dims:
            dims = [(1, 1, 1)]
        merged = [list(dims[0])]
        for e, s, d in dims[1:]:
            pe, ps, pd = merged[-1]
            if ps == s * e and pd == d * e:
                merged[-1] = [pe * e, s, d]
            else:
                merged.append([e, s, d])
        canon.append((b, merged))
    nd = max(len(m) for _, m in canon)
    if nd > nat.MAX_DIMS:
        raise LoweringError(f"box with {nd} dims after coalescing")
    out = []
    for b, m in canon:
        m = [[1, 0, 0]] * (nd - len(m)) + m
        out.append(Box(b.src, b.dst, [x[0] for x in m], [x[1] for x in m], [x[2] for x in m]))
    return nd, out


COPY_FLAT = True  # tests set False to run packed pieces on the per-row kernel


class CopyLaunch:
    """One cubed_copy_boxes launch."""

    def __init__(self, boxes: List[Box], itemsize: int, device):
        import torch

        self.nboxes = len(boxes)
        if not boxes:
            return
        nd, boxes = canonical_boxes(boxes)
        self.boxes = boxes
        self.ndim = nd
        self.itemsize = itemsize
        inner_contig = all(b.sstride[-1] == 1 and b.dstride[-1] == 1 for b in boxes)
        if inner_contig:
            self.path = nat.COPY_ROWS
            lane = 16
            for b in boxes:
                vals = [b.extent[-1] * itemsize, b.src, b.dst]
                vals += [s * itemsize for s in b.sstride[:-1]] + [s * itemsize for s in b.dstride[:-1]]
                while lane > 1 and any(v % lane for v in vals):
                    lane //= 2
            self.lane = lane
            self.work = max(math.prod(b.extent[:-1]) for b in boxes)
            self.row_bytes = max(b.extent[-1] for b in boxes) * itemsize
            words = max(b.extent[0] * b.extent[1] * itemsize // lane for b in boxes) if nd == 2 else 0
            if COPY_FLAT and nd == 2 and 0 < words < 2 ** 31 and \
                    all(b.dstride[0] == b.extent[1] for b in boxes):
                # packed destinations (rechunk pieces): walk each box as one
                # run of destination words
                self.path = nat.COPY_FLAT
                self.work = words
                # source-address order: the pieces of one source row band
                # sit next to each other, so the workgroups copying the two
                # sides of a piece boundary share an XCD (cubed_copy_boxes
                # rounds workgroups per box to a multiple of 8)
                boxes = sorted(boxes, key=lambda b: b.src)
                self.boxes = boxes
        elif nd == 2 and all(b.sstride[1] == 1 and b.dstride[0] == 1 for b in boxes):
            self.path = nat.COPY_TILE
            self.lane = 0
            self.work = max(((b.extent[0] + 63) // 64) * ((b.extent[1] + 63) // 64) for b in boxes)
            self.row_bytes = 0
        else:
            self.path = nat.COPY_ELEMS
            self.lane = 0
            self.work = max(math.prod(b.extent) for b in boxes)
            self.row_bytes = 0
        rows = np.zeros(len(boxes), dtype=nat.BOX_DTYPE)
        for i, b in enumerate(boxes):
            rows[i]["src_base"] = b.src
            rows[i]["dst_base"] = b.dst
            ext = [1] * nat.MAX_DIMS
            ss = [0] * nat.MAX_DIMS
            ds = [0] * nat.MAX_DIMS
            ext[:nd] = b.extent
            ss[:nd] = b.sstride
            ds[:nd] = b.dstride
            rows[i]["extent"] = ext
            rows[i]["src_stride"] = ss
            rows[i]["dst_stride"] = ds
        self.table = torch.from_numpy(rows.view(np.uint8).copy()).to(device)

    def run(self, stream):
        if self.nboxes == 0:
            return
        L = nat.lib()
        nat.check(L.cubed_copy_boxes(self.table.data_ptr(), self.nboxes, self.ndim, self.itemsize,
                                     self.path, self.lane, self.work, self.row_bytes, stream),
                  "cubed_copy_boxes")


# ------------------------------------------------------------------ programs


class Codegen:
    """IR expressions -> two-address VM code for cubed_program_t."""

    def __init__(self, vtype: int, leaf_regs: Dict[int, int], nregs: int = nat.NREGS):
        self.vtype = vtype
        self.leaf_regs = leaf_regs       # id(leaf expr) -> register
        self.reserved = set(leaf_regs.values())
        self.free = [r for r in range(nregs) if r not in self.reserved]
        self.code: List[Tuple] = []
        self.consts: List[Tuple[str, Any]] = []
        self.cache: Dict[Any, int] = {}
        self.uses: Dict[Any, int] = {}
        self._skeys: Dict[int, Any] = {}
        self._keep: List[Any] = []

    # -- helpers --------------------------------------------------------------
    def skey(self, e):
        """Structural key (common-subexpression identity) of an expression."""
        k = self._skeys.get(id(e))
        if k is not None:
            return k
        if isinstance(e, ir.Const):
            k = ("const", repr(e.value), str(e.dtype))
        elif isinstance(e, (ir.Arg, ir.Region, ir.Philox, ir.BlockOffset, ir.Iota)):
            k = ("leaf",) + _leaf_key(e)
        elif isinstance(e, ir.Field):
            k = ("field", e.name)
        else:
            k = (type(e).__name__, getattr(e, "op", None), str(e.dtype)) + \
                tuple(self.skey(c) for c in e.children())
        self._skeys[id(e)] = k
        self._keep.append(e)
        return k

    def count_uses(self, exprs):
        seen = set()

        def walk(e):
            k = self.skey(e)
            self.uses[k] = self.uses.get(k, 0) + 1
            if k in seen:
                return
            seen.add(k)
            for c in e.children():
                walk(c)

        for e in exprs:
            walk(e)

    def alloc(self) -> int:
        if not self.free:
            raise LoweringError("fused expression needs more than 6 VM registers")
        return self.free.pop(0)

    def release(self, r):
        if r not in self.reserved and r not in self.free and r not in self.cache.values():
            self.free.append(r)
            self.free.sort()

    def const_index(self, value, dtype) -> int:
        dtype = np.dtype(dtype)
        if self.vtype == V_I64:
            item = ("i", int(np.array(value).astype(np.int64)))
        else:
            v = float(np.array(value).astype(np.float64))
            if self.vtype == V_F32 or dtype == np.float32:
                v = float(np.float32(v)) if ir.is_float(dtype) and dtype.itemsize <= 4 else v
            item = ("f", v)
        for i, c in enumerate(self.consts):
            if c == item and not (isinstance(c[1], float) and math.isnan(c[1])):
                return i
        if len(self.consts) >= nat.MAX_CONSTS:
            raise LoweringError("too many constants in one fused program")
        self.consts.append(item)
        return len(self.consts) - 1

    def natural(self, dtype) -> bool:
        """True if a value of ``dtype`` needs no re-rounding in V."""
        dtype = np.dtype(dtype)
        if dtype.kind == "b":
            return True
        if self.vtype == V_F64:
            return dtype in (np.dtype(np.float64), np.dtype(np.int64), np.dtype(np.uint64))
        if self.vtype == V_F32:
            return dtype == np.dtype(np.float32)
        return dtype in (np.dtype(np.int64), np.dtype(np.uint64))

    # -- expression codegen --------------------------------------------------
    def _last_use(self, key) -> bool:
        """Count one use of ``key``; True if it was the last one."""
        if not hasattr(self, "remaining"):
            self.remaining = dict(self.uses)
        n = self.remaining.get(key, 0) - 1
        self.remaining[key] = n
        return n == 0 and key in self.uses

    def gen(self, e) -> Tuple[int, bool]:
        """Return (register, owned) holding the value of ``e``.  A leaf or
        common subexpression at its last use is handed over as owned, so
        the consumer computes in place instead of copying it to a fresh
        register (complex products read 4 leaves and keep 2 parts live)."""
        pinned = getattr(self, "pinned", ())
        if id(e) in self.leaf_regs:
            r = self.leaf_regs[id(e)]
            if self._last_use(self.skey(e)) and r in self.reserved and r not in pinned and \
                    sum(1 for v in self.leaf_regs.values() if v == r) == 1:
                self.reserved.discard(r)  # leaves reload every element: free to overwrite
                return r, True
            return r, False
        key = self.skey(e)
        if key in self.cache:
            r = self.cache[key]
            if self._last_use(key) and r not in pinned:
                del self.cache[key]
                return r, True
            return r, False
        if isinstance(e, ir.Const):
            r = self.alloc()
            self.code.append((ir_op("CONST"), r, 0, 0, 0, self.const_index(e.value, e.dtype)))
            return self._finish(e, r)
        if isinstance(e, (ir.Arg, ir.Region, ir.Philox, ir.BlockOffset, ir.Iota, ir.Field)):
            raise LoweringError(f"leaf {e} has no register")
        if isinstance(e, ir.Cast):
            r = self.owned(*self.gen(e.x))
            self.code.append((ir_op("CAST"), r, 0, 0, ir.dtype_code(e.dtype), ir.dtype_code(e.x.dtype)))
            return self._finish(e, r, rounded=True)
        if isinstance(e, ir.Unary):
            r = self.owned(*self.gen(e.x))
            self.code.append((ir.UNARY_OPS[e.op], r, 0, 0, 0, 0))
            return self._finish(e, r)
        if isinstance(e, ir.Binary):
            ra, oa = self.gen(e.a)
            ra = self.owned(ra, oa)
            rb, ob = self.gen(e.b)
            self.code.append((ir.BINARY_OPS[e.op], ra, rb, 0, 0, 0))
            if ob:
                self.release(rb)
            return self._finish(e, ra)
        if isinstance(e, ir.Where):
            ra = self.owned(*self.gen(e.a))
            rb, ob = self.gen(e.b)
            self.pin(rb)  # read by the WHERE below: c's code must not reuse it
            rc, oc = self.gen(e.c)
            self.unpin(rb)
            self.code.append((ir_op("WHERE"), ra, rb, rc, 0, 0))
            if ob:
                self.release(rb)
            if oc:
                self.release(rc)
            return self._finish(e, ra)
        raise LoweringError(f"cannot generate code for {type(e).__name__}")

    def pin(self, r):
        """Keep register r's value intact: no later last-use handover of it
        (operands awaiting their instruction, program outputs)."""
        if not hasattr(self, "pinned"):
            self.pinned = {}
        self.pinned[r] = self.pinned.get(r, 0) + 1

    def unpin(self, r):
        self.pinned[r] -= 1
        if not self.pinned[r]:
            del self.pinned[r]

    def owned(self, r, owned) -> int:
        if owned:
            return r
        t = self.alloc()
        self.code.append((ir_op("MOV"), t, r, 0, 0, 0))
        return t

    def _finish(self, e, r, rounded=False):
        if not rounded and not self.natural(e.dtype):
            self.code.append((ir_op("CAST"), r, 0, 0, ir.dtype_code(e.dtype), ir.dtype_code(e.dtype)))
        k = self.skey(e)
        if self.uses.get(k, 0) > 1:
            self._last_use(k)  # the computing visit is one of the uses
            self.cache[k] = r
            return r, False
        return r, True


_OPCODES = {"NOP": 0, "CONST": 1, "MOV": 2, "CAST": 3, "WHERE": 4}


def ir_op(name):
    return _OPCODES[name]


def choose_vtype(exprs, leaves) -> int:
    """Register value type: I64 for all-integer programs, F32 when every
    computed node is f32-or-narrower (f64 leaves only feed casts to f32), else
    F64 (f32 nodes are then re-rounded by CAST, exact for + - * / sqrt)."""
    nodes = []
    seen = set()
    parents: Dict[int, List[Any]] = {}

    def walk(e, parent=None):
        if parent is not None:
            parents.setdefault(id(e), []).append(parent)
        if id(e) in seen:
            return
        seen.add(id(e))
        nodes.append(e)
        for c in e.children():
            walk(c, e)

    for e in exprs:
        walk(e)
    dts = [np.dtype(n.dtype) for n in nodes if not isinstance(n, ir.Field)]
    if all(d.kind in "biu" for d in dts):
        return V_I64
    small = {np.dtype(np.float32), np.dtype(np.float16), ir.bfloat16, np.dtype(np.bool_), np.dtype(np.int8),
             np.dtype(np.uint8), np.dtype(np.int16), np.dtype(np.uint16)}
    ok = True
    for n in nodes:
        d = np.dtype(n.dtype)
        if isinstance(n, (ir.Arg, ir.Region, ir.Philox)):
            if d not in small and not all(isinstance(p, ir.Cast) and np.dtype(p.dtype) in small
                                          for p in parents.get(id(n), [None])):
                ok = False
        elif isinstance(n, (ir.BlockOffset, ir.Iota)):
            ok = False
        elif isinstance(n, ir.Const):
            continue
        elif d not in small:
            ok = False
    return V_F32 if ok else V_F64


def collect_leaves(exprs) -> List[Any]:
    out, seen = [], set()
    for e in exprs:
        for leaf in ir.leaves(e):
            if isinstance(leaf, (ir.Const, ir.Field)):
                continue
            k = _leaf_key(leaf)
            if k not in seen:
                seen.add(k)
                out.append(leaf)
    return out


def _leaf_key(leaf):
    if isinstance(leaf, ir.ReshapeArg):
        return ("reshape", leaf.index, leaf.field, leaf.axes)
    if isinstance(leaf, ir.Concat):
        return ("concat", leaf.field, leaf.axes, id(leaf.region), leaf.block_arg)
    if isinstance(leaf, ir.Arg):
        return ("arg", leaf.index, leaf.field, leaf.axes)
    if isinstance(leaf, ir.Region):
        return ("region", leaf.array_name, leaf.field, leaf.axes, id(leaf.region), leaf.block_arg)
    if isinstance(leaf, ir.Philox):
        return ("philox", leaf.root_seed, leaf.block_arg, leaf.axes)
    if isinstance(leaf, ir.BlockOffset):
        return ("offset", leaf.block_arg)
    if isinstance(leaf, ir.Iota):
        return ("iota", leaf.dim, leaf.arg, leaf.axes)
    return ("other", id(leaf))


def dedupe_leaves(exprs):
    """Rewrite expressions so equal leaves are one object (one register)."""
    canon: Dict[Any, Any] = {}

    def fn(leaf):
        if isinstance(leaf, (ir.Const, ir.Field)):
            return None
        k = _leaf_key(leaf)
        if k in canon:
            return canon[k]
        canon[k] = leaf
        return leaf

    memo: Dict[int, Any] = {}
    return [ir.transform(e, fn, memo) for e in exprs]


def program_exprs(p: ir.ExprProgram):
    outs = [e for _, e in p.output_items()]
    fields = [f.expr for f in p.reduce.fields] if p.reduce else []
    return outs, fields


def program_fits(p: ir.ExprProgram) -> bool:
    """Whether an expression program fits the VM (leaves, one random stream,
    registers, instruction counts) -- checked before any constant folding,
    so it is conservative.  Used by the executor's producer fusion to only
    build fused programs it can lower."""
    try:
        outs, fields = program_exprs(p)
        exprs = dedupe_leaves(outs + fields)
        pre = exprs[:len(outs)] if p.reduce is None else exprs[len(outs):]
        leaves = collect_leaves(pre)
        if len(leaves) > nat.MAX_LEAVES or sum(isinstance(l, ir.Philox) for l in leaves) > 1:
            return False
        by_key = {_leaf_key(l): i for i, l in enumerate(leaves)}
        leaf_regs = {}
        for e in pre:
            for lf in ir.leaves(e):
                if not isinstance(lf, (ir.Const, ir.Field)):
                    leaf_regs[id(lf)] = by_key[_leaf_key(lf)]
        cg = Codegen(choose_vtype(pre, leaves), leaf_regs)
        cg.count_uses(pre)
        for e in pre:
            cg.pin(cg.gen(e)[0])  # as the lowering does: outputs stay live
        if len(cg.code) > nat.MAX_INSNS or len(cg.consts) > nat.MAX_CONSTS:
            return False
        if p.reduce is not None and not all(isinstance(e, ir.Field) for e in exprs[:len(outs)]):
            ecg = Codegen(V_F64, {}, nregs=nat.NREGS)
            nf = len(p.reduce.fields)
            ecg.reserved = set(range(nf))
            ecg.free = [r for r in range(nat.NREGS) if r not in ecg.reserved]
            fidx = {f.name: i for i, f in enumerate(p.reduce.fields)}
            for e in exprs[:len(outs)]:
                for lf in ir.leaves(e):
                    if isinstance(lf, ir.Field):
                        ecg.leaf_regs[id(lf)] = fidx[lf.name]
            ecg.count_uses(exprs[:len(outs)])
            for e in exprs[:len(outs)]:
                ecg.pin(ecg.gen(e)[0])
            if len(ecg.code) > nat.MAX_EPI:
                return False
        return True
    except (LoweringError, KeyError):
        return False


def is_pure_copy(p: ir.ExprProgram, out_dtype) -> bool:
    """A program that only moves one leaf's values (merge/index/squeeze)."""
    if p.reduce is not None or p.structured:
        return False
    e = p.outputs
    return isinstance(e, (ir.Arg, ir.Region)) and np.dtype(e.dtype) == np.dtype(out_dtype)


# ------------------------------------------------------------------ fused launch


class FusedLaunch:
    """One cubed_fused_chunks launch (+ optional scratch gathers)."""

    def __init__(self, prog_struct, table, ntasks, max_kept, max_red, ws_bytes, gathers, device):
        import torch

        self.prog = prog_struct
        raw = np.frombuffer(ctypes.string_at(ctypes.addressof(prog_struct), ctypes.sizeof(prog_struct)),
                            dtype=np.uint8)
        self.d_prog = torch.from_numpy(raw.copy()).to(device)  # read by the kernels
        self.handle = nat.compile_program(prog_struct) if nat.jit_enabled() else None
        self.table = table
        self.ntasks = ntasks
        self.max_kept = max_kept
        self.max_red = max_red
        self.gathers = gathers
        # zeroed once: the streaming kernels' split-arrival counters live at its
        # end and are reset to zero by the kernels themselves
        self.ws = torch.zeros(max(ws_bytes, 16), dtype=torch.uint8, device=device) if ws_bytes else None
        self.ws_bytes = ws_bytes

    def reprogram(self):
        """Re-upload and re-compile ``prog`` after the host changed it once
        the launch's consumer was known (mode bits and consts set by
        dist.DistPiecesLaunch for owner-major partials)."""
        import torch

        raw = np.frombuffer(ctypes.string_at(ctypes.addressof(self.prog), ctypes.sizeof(self.prog)),
                            dtype=np.uint8)
        self.d_prog = torch.from_numpy(raw.copy()).to(self.d_prog.device)
        self.handle = nat.compile_program(self.prog) if nat.jit_enabled() else None

    groups = None

    fold = None

    def set_groups(self, group_start, fold=None):
        """Rows are pieces; group_start (ngroups + 1) delimits the pieces of
        each output box (partials mode: run() adds the grouped finish).
        ``fold = (epilogue program, one task row per group)``: a lifted full
        reduction -- rows and kept elements fold to one value per group
        (cubed_fold_groups), then the epilogue runs per group."""
        import torch

        self.ngroups = len(group_start) - 1
        self.groups = torch.from_numpy(np.ascontiguousarray(group_start)).to(self.d_prog.device)
        if fold is not None:
            prog_fin, table = fold
            raw = np.frombuffer(ctypes.string_at(ctypes.addressof(prog_fin), ctypes.sizeof(prog_fin)),
                                dtype=np.uint8)
            rows_per_group = int(np.max(np.diff(group_start))) if self.ngroups else 1
            self.fold_split = int(nat.lib().cubed_fold_groups_splits(self.ngroups, rows_per_group,
                                                                     self.max_kept))
            split_ws = None
            if self.fold_split > 1:
                # split accumulators + one arrival counter per group, zeroed
                # once (the kernel leaves the counters at zero)
                split_ws = torch.zeros(8 * self.prog.nfields * self.ngroups * self.fold_split
                                       + 4 * self.ngroups, dtype=torch.uint8, device=self.d_prog.device)
            self.fold = (prog_fin, torch.from_numpy(raw.copy()).to(self.d_prog.device), table,
                         torch.empty(max(8 * self.prog.nfields * self.ngroups, 16), dtype=torch.uint8,
                                     device=self.d_prog.device), split_ws)

    def run(self, stream):
        self._run(stream)
        if self.fold is not None:
            prog_fin, d_fin, table, gsoa, split_ws = self.fold
            L = nat.lib()
            # the fold and the epilogue in one launch (the group's last
            # workgroup finishes it); specialised from the program's JIT
            # module when there is one
            if self.handle is not None and self.prog.mode & MODE_PARTIALS:
                nat.check(L.cubed_fold_groups_compiled(
                    self.handle, self.prog, self.table.data_ptr(), self.ntasks, self.max_kept,
                    self.ws.data_ptr(), self.groups.data_ptr(), self.ngroups, gsoa.data_ptr(), self.fold_split,
                    split_ws.data_ptr() if split_ws is not None else None, table.data_ptr(), stream),
                    "cubed_fold_groups_compiled")
                return
            nat.check(L.cubed_fold_groups(self.prog, self.d_prog.data_ptr(), self.table.data_ptr(),
                                          self.ntasks, self.max_kept, self.ws.data_ptr(),
                                          self.groups.data_ptr(), self.ngroups, gsoa.data_ptr(),
                                          self.fold_split,
                                          split_ws.data_ptr() if split_ws is not None else None,
                                          prog_fin, d_fin.data_ptr(), table.data_ptr(), stream),
                      "cubed_fold_groups")
        elif self.groups is not None:
            nat.check(nat.lib().cubed_fused_finish_groups(
                self.prog, self.d_prog.data_ptr(), self.table.data_ptr(), self.ntasks, self.max_kept,
                self.ws.data_ptr(), self.groups.data_ptr(), self.ngroups, stream),
                "cubed_fused_finish_groups")

    def _run(self, stream):
        for g in self.gathers:
            g.run(stream)
        L = nat.lib()
        if self.handle is not None:
            nat.check(L.cubed_fused_chunks_compiled(
                self.handle, self.prog, self.d_prog.data_ptr(), self.table.data_ptr(), self.ntasks,
                self.max_kept, self.max_red, self.ws.data_ptr() if self.ws is not None else None,
                self.ws_bytes, stream), "cubed_fused_chunks_compiled")
            return
        nat.check(L.cubed_fused_chunks(self.prog, self.d_prog.data_ptr(), self.table.data_ptr(),
                                       self.ntasks, self.max_kept,
                                       self.max_red, self.ws.data_ptr() if self.ws is not None else None,
                                       self.ws_bytes, stream), "cubed_fused_chunks")


class GemmLaunch:
    """Chained chunk GEMMs of one matmul / tensordot (``cubed_gemm_chain``):
    one task per output chunk, each summing its segment products in one K
    loop (a per-chunk product is a chain of one segment).  The hand-written
    kernels of csrc/gemm_chain.hip run every dtype (MFMA for bf16 / f32)."""

    GRID = True  # probes set False to time the per-chunk tiling
    # input dtypes whose UNPACKED kernels take the grid tiling (when the packed
    # path below is not taken): f32 measured 133.6 TF
    # grid vs 129-130 per chunk.  bf16 stays per chunk: on config 5 the
    # one-wave full-line kernel runs 1251-1256 TF per chunk vs 1076-1080 grid
    # (its grid form keeps per-lane chunk selects live through the K loop;
    # profiles/r05_gemm_bf16_ab.log, ping-pong grid 1048-1050)
    GRID_INPUTS = {ir.dtype_code(np.float32)}  # (tools/gemm_ab.sh widens it for A/B runs)
    # bf16 / f32 chunk grids of one product take the packed-operand kernels
    # (cubed_gemm_chain_packed): both operands rewritten once into the GEMM's
    # LDS image, then whole-matrix tiles -- config 5 bf16 GEMM 1316 TF vs 1214
    # for the per-chunk w4l kernel (+ 2.6 ms of packing,
    # profiles/r05_gemm_bf16_w4p.log); f32 143.3 TF incl. packing vs 132.5 for
    # the grid kernel (profiles/r05_gemm_f32_w4p.log)
    PACKED = True  # probes set False to time the unpacked kernels
    PACKED_INPUTS = {ir.dtype_code(ir.bfloat16), ir.dtype_code(np.float32)}

    def __init__(self, tasks, segs, in_code, out_code, device, zero_ptr, path=None, grid=None, scratch=None):
        import torch

        self.n = len(tasks)
        self.in_code, self.out_code = in_code, out_code
        self.tasks = np.ascontiguousarray(tasks)
        self.segs = np.ascontiguousarray(segs) if len(segs) else np.zeros(1, dtype=nat.SEG_DTYPE)
        self.zero = zero_ptr
        self.path = nat.GEMM_AUTO if path is None else path
        # (ti, tj): the tasks are the C-order chunk grid of one output; the
        # f32 MFMA kernel then tiles the whole matrix (cubed_gemm_chain_grid)
        self.grid = None
        if grid is not None and self.GRID and in_code in self.GRID_INPUTS and self.path == nat.GEMM_AUTO and \
                grid[0] * grid[1] == self.n and \
                nat.lib().cubed_gemm_grid_check(self.tasks.ctypes.data, grid[0], grid[1], self.segs.ctypes.data,
                                                len(self.segs), in_code, out_code) == 0:
            self.grid = tuple(grid)
        # packed: (workspace pointer, bytes) from scratch(nbytes), which returns
        # None when the workspace does not fit beside the plan's arrays
        self.packed = None
        if grid is not None and self.GRID and self.PACKED and scratch is not None and in_code in self.PACKED_INPUTS and \
                self.path == nat.GEMM_AUTO and grid[0] * grid[1] == self.n:
            nbytes = nat.lib().cubed_gemm_pack_bytes(self.tasks.ctypes.data, grid[0], grid[1], self.segs.ctypes.data,
                                                     len(self.segs), in_code, out_code)
            ws = scratch(nbytes) if nbytes > 0 else None
            if ws is not None:
                self.packed = (ws, nbytes)
                self.grid = tuple(grid)
        self.flops = 2.0 * float(sum(int(t["m"]) * int(t["n"]) * int(t["ktot"]) for t in self.tasks))
        if not self.n:
            return
        self.d_tasks = torch.from_numpy(self.tasks.view(np.uint8).copy()).to(device)
        self.d_segs = torch.from_numpy(self.segs.view(np.uint8).copy()).to(device)

    def kernel_path(self) -> int:
        """CUBED_GEMM_MFMA or CUBED_GEMM_ANY (host-side decision)."""
        if self.path != nat.GEMM_AUTO:
            return self.path
        return nat.lib().cubed_gemm_chain_path(self.tasks.ctypes.data, self.n, self.segs.ctypes.data,
                                               self.in_code, self.out_code)

    def run(self, stream):
        if not self.n:
            return
        L = nat.lib()
        if self.packed is not None:
            nat.check(L.cubed_gemm_chain_packed(self.tasks.ctypes.data, self.d_tasks.data_ptr(), self.grid[0],
                                                self.grid[1], self.segs.ctypes.data, self.d_segs.data_ptr(),
                                                len(self.segs), self.in_code, self.out_code, self.packed[0],
                                                self.packed[1], stream), "cubed_gemm_chain_packed")
            return
        if self.grid is not None:
            nat.check(L.cubed_gemm_chain_grid(self.tasks.ctypes.data, self.d_tasks.data_ptr(), self.grid[0],
                                              self.grid[1], self.segs.ctypes.data, self.d_segs.data_ptr(),
                                              len(self.segs), self.in_code, self.out_code, self.zero, stream),
                      "cubed_gemm_chain_grid")
            return
        nat.check(L.cubed_gemm_chain(self.tasks.ctypes.data, self.d_tasks.data_ptr(), self.n,
                                     self.segs.ctypes.data, self.d_segs.data_ptr(), len(self.segs),
                                     self.in_code, self.out_code, self.zero, self.path, stream),
                  "cubed_gemm_chain")


class Lowerer:
    """Lowers pipelines for one executor context (device, scratch buffers,
    uploaded small arrays)."""

    def __init__(self, ctx):
        self.ctx = ctx

    # -- argument resolution ---------------------------------------------------
    def resolve_target(self, name, reads_map):
        proxy = reads_map.get(name)
        if proxy is None:
            raise LoweringError(f"array {name} is not an input of this pipeline")
        return self.ctx.device_source(proxy.array)

    def lower_expr_pipeline(self, program: ir.ExprProgram, spec, target: DeviceArray, task_keys,
                            rows_fn=None, sample_key=None, partials=False, lift=True,
                            merge_kept_groups=False, host_count=False):
        """Build the FusedLaunch (or CopyLaunch) for a blockwise pipeline.
        ``rows_fn(leaves, kinds) -> (rows, reduced dims)`` overrides the
        per-task views (reduction-chain fusion, cubed_amd/chains.py)."""
        outs, field_exprs = program_exprs(program)
        exprs = dedupe_leaves(outs + field_exprs)
        outs2, fields2 = exprs[:len(outs)], exprs[len(outs):]
        out_items = [(n, e) for (n, _), e in zip(program.output_items(), outs2)]
        rfields = []
        if program.reduce is not None:
            rfields = [ir.ReduceField(f.name, f.rop, e, f.dtype) for f, e in zip(program.reduce.fields, fields2)]

        # pure copies go through the box-copy kernel
        if rows_fn is None and program.reduce is None and not program.structured and \
                is_pure_copy(program, target.dtype):
            try:
                return self.lower_copy_program(program, spec, target, task_keys)
            except _NotACopy:
                pass  # a constant source: the fused path materialises it

        pre_exprs = [e for _, e in out_items] if program.reduce is None else [f.expr for f in rfields]
        leaves = collect_leaves(pre_exprs)
        if len(leaves) > nat.MAX_LEAVES:
            raise LoweringError(f"fused program reads {len(leaves)} inputs (max {nat.MAX_LEAVES})")

        # constant-fold leaves that resolve to constants (virtual full / scalars)
        sample_args = spec.block_function(("out",) + tuple(task_keys[0] if sample_key is None else sample_key))
        const_leaves = {}
        for leaf in leaves:
            c = self.constant_value(leaf, sample_args, spec.reads_map)
            if c is not None:
                const_leaves[_leaf_key(leaf)] = c
        if const_leaves:
            def fold(leaf):
                k = _leaf_key(leaf) if not isinstance(leaf, (ir.Const, ir.Field)) else None
                if k in const_leaves:
                    return ir.Const(const_leaves[k], leaf.dtype)
                return None
            memo = {}
            pre_exprs = [ir.transform(e, fold, memo) for e in pre_exprs]
            if program.reduce is None:
                out_items = [(n, e) for (n, _), e in zip(out_items, pre_exprs)]
            else:
                rfields = [ir.ReduceField(f.name, f.rop, e, f.dtype) for f, e in zip(rfields, pre_exprs)]
            leaves = collect_leaves(pre_exprs)

        if sum(isinstance(l, ir.Philox) for l in leaves) > 1:
            # cubed_task_t carries one Philox key per task
            raise LoweringError("fused program draws from more than one random stream")
        vtype = choose_vtype(pre_exprs, leaves)
        leaf_regs = {}
        by_key = {_leaf_key(l): i for i, l in enumerate(leaves)}

        def index_leaves(e):
            for lf in ir.leaves(e):
                if not isinstance(lf, (ir.Const, ir.Field)):
                    leaf_regs[id(lf)] = by_key[_leaf_key(lf)]

        for e in pre_exprs:
            index_leaves(e)
        cg = Codegen(vtype, leaf_regs)
        cg.count_uses(pre_exprs)

        P = nat.Program()
        P.vtype = vtype
        P.nleaves = len(leaves)
        structured_out = program.structured
        out_fields = [n for n, _ in out_items]
        if program.reduce is None:
            srcs = []
            for _, e in out_items:
                r, _ = cg.gen(e)
                cg.pin(r)
                srcs.append(r)
            P.nfields = 0
            P.nepi = -1
            out_regs = srcs
        else:
            P.nfields = len(rfields)
            if P.nfields > nat.MAX_FIELDS:
                raise LoweringError("too many reduced fields")
            for i, f in enumerate(rfields):
                r, _ = cg.gen(f.expr)
                cg.pin(r)
                P.field_src[i] = r
                P.field_rop[i] = ir.ROPS[f.rop]
                P.field_acc[i] = 1 if ir.acc_is_int(f.rop, f.dtype) else 0
            # epilogue over fields (double registers 0..nf-1)
            fidx = {f.name: i for i, f in enumerate(rfields)}
            direct = all(isinstance(e, ir.Field) for _, e in out_items)
            if direct:
                P.nepi = -1
                out_regs = [fidx[e.name] for _, e in out_items]
            else:
                ecg = Codegen(V_F64, {}, nregs=nat.NREGS)
                ecg.reserved = set(range(len(rfields)))
                ecg.free = [r for r in range(nat.NREGS) if r not in ecg.reserved]
                ecg.consts = cg.consts  # shared pool
                ecg.count_uses([e for _, e in out_items])
                field_regs = {}

                def bind_fields(e):
                    for lf in ir.leaves(e):
                        if isinstance(lf, ir.Field):
                            field_regs[id(lf)] = fidx[lf.name]

                for _, e in out_items:
                    bind_fields(e)
                ecg.leaf_regs = field_regs
                out_regs = []
                for _, e in out_items:
                    r, _ = ecg.gen(e)
                    ecg.pin(r)
                    out_regs.append(r)
                if len(ecg.code) > nat.MAX_EPI:
                    raise LoweringError("epilogue too long")
                P.nepi = len(ecg.code)
                for i, ins in enumerate(ecg.code):
                    _set_insn(P.epi[i], ins)
                cg.consts = ecg.consts
        if len(cg.code) > nat.MAX_INSNS:
            raise LoweringError("fused program too long")
        P.ninsns = len(cg.code)
        for i, ins in enumerate(cg.code):
            _set_insn(P.insns[i], ins)
        for i, (kind, v) in enumerate(cg.consts):
            if kind == "i":
                P.consts[i].i = v
            else:
                P.consts[i].f = v

        # outputs
        fields_of_target = target.fields
        if len(out_items) > nat.MAX_OUTS:
            raise LoweringError(f"fused program writes {len(out_items)} outputs (max {nat.MAX_OUTS})")
        P.nouts = len(out_items)
        for o, (name, _) in enumerate(out_items):
            fname = name if structured_out else None
            if fname is not None and fname not in fields_of_target:
                raise LoweringError(f"output field {fname} missing in target")
            P.out_dtype[o] = ir.dtype_code(target.field_dtype(fname))
            P.out_src[o] = out_regs[o]

        for i, leaf in enumerate(leaves):
            P.leaf_kind[i] = self.leaf_kind(leaf)
            P.leaf_dtype[i] = ir.dtype_code(leaf.dtype) if P.leaf_kind[i] == LEAF_ARRAY else 0

        # ---- per-task views
        kinds = [self.leaf_kind(l) for l in leaves]
        gathers = []
        group_start = None
        merge_ok = MERGE_ROWS and not partials and all(k == LEAF_ARRAY for k in kinds)
        if rows_fn is not None:
            res = rows_fn(leaves, kinds)
            rows, red_axes = res[0], res[1]
            n = len(rows[0].extent)
            if len(res) > 2:
                # rows of several groups (chain_piece_rows): partials + grouped finish
                group_keys = res[2]
                gathers += res[3]
                if merge_ok:
                    rows, group_keys = _merge_group_rows(rows, group_keys, red_axes, leaves)
                starts = [i for i in range(len(group_keys)) if i == 0 or group_keys[i] != group_keys[i - 1]]
                group_start = np.array(starts + [len(group_keys)], dtype=np.int64)
                partials = partials or len(starts) < len(group_keys)
        else:
            red_axes = set(program.reduce.axes) if program.reduce is not None else set()
            n = program.ndim
            rows, group_keys = [], []
            for key in task_keys:
                r, gk = self.task_pieces(program, spec, target, key, leaves, out_items,
                                         structured_out, gathers)
                rows += r
                group_keys += gk
            if merge_ok and program.reduce is not None and len(set(group_keys)) < len(group_keys):
                rows, group_keys = _merge_group_rows(rows, group_keys, red_axes, leaves)
            if program.reduce is not None and len(set(group_keys)) < len(group_keys):
                # pieces reduce into shared outputs: partials + grouped finish
                partials = True
                starts = [i for i in range(len(group_keys))
                          if i == 0 or group_keys[i] != group_keys[i - 1]]
                group_start = np.array(starts + [len(group_keys)], dtype=np.int64)
        # full reductions with long inner rows run "lifted": the inner dims
        # are walked as kept dims (every lane streams), then folded per task
        lifted = set()
        if lift and LIFT_ENABLED and program.reduce is not None and n >= 2 and set(range(n)) <= set(red_axes):
            lifted = _lift_dims(rows, n)
        if lifted:
            partials = True
            # the main kernel writes no output (the fold + epilogue do), so
            # output strides must not stop the inner dims from coalescing
            rows = [dataclasses.replace(r, ostrides=[[0] * len(st) for st in r.ostrides]) for r in rows]
            if group_start is None:
                group_start = np.arange(len(rows) + 1, dtype=np.int64)
        layout = canonicalize(rows, n, set(red_axes) - lifted, leaves, kinds,
                              check_outputs=not lifted)
        P.ndim = layout.ndim
        P.nred = layout.nred
        P.mode = layout.mode
        stream = _stream_ok(layout, leaves, kinds, P.vtype, check_outputs=not lifted)
        if stream and merge_ok and MERGE_KEPT and not partials and not lifted and \
                (group_start is None or len(group_start) == len(rows) + 1):
            out_isz = [target.field_dtype(n if structured_out else None).itemsize for n, _ in out_items]
            merged = _merge_kept_runs(layout, [np.dtype(l.dtype).itemsize for l in leaves], out_isz)
            if merged is not None:
                layout = merged
                rows = layout.rows
                if group_start is not None:
                    group_start = np.arange(len(rows) + 1, dtype=np.int64)
        group_layout = None
        if stream and merge_kept_groups and merge_kept_groups() and MERGE_KEPT and partials and not lifted \
                and group_start is None:
            # one row per output group (DistPiecesLaunch): consecutive groups
            # whose rows continue each other along the packed kept dim stream
            # as one wide task.  The main kernel writes only SoA partials, so
            # outputs do not constrain the merge; kept only when the merged
            # SoA [task][kept] is byte-identical to the per-group SoA
            # [group][kept] (every task and every group the same extent).
            merged = _merge_kept_runs(layout, [np.dtype(l.dtype).itemsize for l in leaves], [])
            if merged is not None and \
                    all(r.extent[-1] == merged.max_kept for r in merged.rows) and \
                    all(_apply_groups(r, layout.groups)[0][-1] == layout.max_kept for r in layout.rows) and \
                    len(merged.rows) * merged.max_kept == len(layout.rows) * layout.max_kept:
                group_layout = layout
                layout = merged
                rows = layout.rows
        if stream:
            P.mode |= MODE_STREAM | _stream_groups_mode(P, len(rows), layout.max_kept)
            if STREAM_EVEN and P.nfields > 0 and len({_red_extent(r, layout) for r in rows}) == 1:
                # every task the same reduced extent: a split launch may cut
                # the (task, column block, row) units into equal runs per
                # workgroup (stream_body's balanced split)
                P.mode |= MODE_STREAM_EVEN
        if partials:
            if P.nfields == 0:
                raise LoweringError("partials mode needs a reduction")
            P.mode |= MODE_PARTIALS
            if group_layout is not None or (host_count() if callable(host_count) else host_count):
                # per-group SoA straight from the kernel (DistPiecesLaunch), or
                # a chain whose global count the host knows (PartialsLaunch):
                # its plain COUNT fields hold the global counts, filled by the
                # host once, never reduced across the ranks
                P.mode |= MODE_HOST_COUNT
        table = layout.table(self.ctx.device)
        ws = nat.lib().cubed_fused_workspace_bytes(P, len(rows), layout.max_kept, layout.max_red)
        launch = FusedLaunch(P, table, len(rows), layout.max_kept, layout.max_red, ws,
                             gathers, self.ctx.device)
        launch.layout = layout
        launch.group_layout = group_layout
        if lifted:
            # the epilogue program: same instructions, every dim reduced (one output per task)
            fin = nat.Program()
            ctypes.memmove(ctypes.addressof(fin), ctypes.addressof(P), ctypes.sizeof(P))
            fin.nred = fin.ndim
            fin.mode = 0
            gt = dataclasses.replace(layout, rows=[layout.rows[i] for i in group_start[:-1]])
            launch.set_groups(group_start, fold=(fin, gt.table(self.ctx.device)))
        elif group_start is not None:
            launch.set_groups(group_start)
        return launch

    def leaf_kind(self, leaf) -> int:
        if isinstance(leaf, ir.Philox):
            return LEAF_PHILOX
        if isinstance(leaf, ir.BlockOffset):
            return LEAF_OFFSET
        if isinstance(leaf, ir.Iota):
            return LEAF_IOTA
        return LEAF_ARRAY

    def constant_value(self, leaf, args, reads_map):
        """Value of a leaf that reads a constant (virtual full array, 1-element
        in-memory array), else None."""
        if isinstance(leaf, ir.Arg):
            spec = args[leaf.index]
            if not isinstance(spec, tuple):
                return None
            arr = reads_map[spec[0]].array
        elif isinstance(leaf, ir.Region):
            arr = leaf.target
        else:
            return None
        if isinstance(arr, VirtualFullArray):
            v = arr.fill_value
            if np.dtype(arr.dtype).kind == "c" and leaf.field in ("real", "imag"):
                return getattr(complex(v), leaf.field)
            return v
        if isinstance(arr, VirtualInMemoryArray) and arr.array.size == 1:
            v = arr.array.reshape(-1)[0]
            if np.dtype(arr.dtype).kind == "c" and leaf.field in ("real", "imag"):
                return getattr(v, leaf.field).item()
            if leaf.field is not None:
                v = v[leaf.field]
            return v.item()
        return None

    # -- one task's views (program space order) --------------------------------
    def task_layout(self, program, spec, target, key, leaves, out_items, structured_out, gathers,
                    straddles=None):
        """One task's TaskRow.  With ``straddles`` (a list), Region leaves
        whose region spans several source chunks are not gathered: they get
        a placeholder view (the region's own C strides, base 0) and are
        recorded as (leaf index, array, region, field) for task_pieces."""
        n = program.ndim
        key = tuple(key)
        args = spec.block_function(("out",) + key)
        args = [list(a) if not isinstance(a, (tuple, list, str)) else a for a in args]
        extent = [None] * n
        leaf_views = []
        for i, leaf in enumerate(leaves):
            if straddles is not None and isinstance(leaf, ir.Region):
                sv = self.straddle_view(leaf, args)
                if sv is not None:
                    straddles.append((i,) + sv[1:])
                    leaf_views.append((LEAF_ARRAY, sv[0]))
                    continue
            leaf_views.append(self.leaf_view(leaf, args, spec, gathers, key))
        # output views
        out_views = []
        out_ext = target.chunk_extent(key) if target.ndim else ()
        for name, _ in out_items:
            fname = name if structured_out else None
            out_views.append(chunk_view(target, key, fname) if target.ndim else
                             ArrView(target.chunk_addr((), fname), [], [], target.field_dtype(fname)))
        for j, s in enumerate(program.out_axes):
            if s is not None:
                extent[s] = out_ext[j]
        # leaf extents fill / check the space
        for leaf, (kind, v) in zip(leaves, leaf_views):
            axes = getattr(leaf, "axes", None)
            if axes is None or v is None:
                continue
            for d, s in enumerate(axes):
                e = v.extent[d]
                if s is None:
                    if e != 1:
                        raise LoweringError(f"leaf dim {d} of extent {e} has no space dim")
                    continue
                if extent[s] is None or extent[s] == 1:
                    extent[s] = e if extent[s] is None or e != 1 else extent[s]
                elif e != 1 and e != extent[s]:
                    raise LoweringError(f"extent mismatch on space dim {s}: {e} vs {extent[s]}")
        extent = [1 if e is None else e for e in extent]
        # strides per space dim
        lstrides, bases = [], []
        for leaf, (kind, v) in zip(leaves, leaf_views):
            st = [0] * n
            axes = getattr(leaf, "axes", ())
            if v is not None:
                for d, s in enumerate(axes):
                    if s is not None and v.extent[d] != 1:
                        st[s] = v.stride[d]
                    elif s is not None and v.extent[d] == 1 and extent[s] != 1:
                        st[s] = 0
                bases.append(v.base)
            else:
                bases.append(0)
            lstrides.append(st)
        ostrides = []
        for (name, _), v in zip(out_items, out_views):
            st = [0] * n
            for j, s in enumerate(program.out_axes):
                if s is not None and j < len(v.stride):
                    st[s] = v.stride[j] if extent[s] != 1 else 0
            ostrides.append(st)
        obases = [v.base for v in out_views]
        key_lo = key_hi = 0
        block_offset = 0
        for leaf, (kind, v) in zip(leaves, leaf_views):
            if kind == LEAF_PHILOX:
                key_lo, key_hi = v.key
            if kind in (LEAF_PHILOX, LEAF_OFFSET):
                block_offset = v.block_offset
        return TaskRow(extent, bases, lstrides, obases, ostrides, key_lo, key_hi, block_offset)

    def straddle_view(self, leaf, args):
        """(placeholder view, array, region, field) for a Region leaf whose
        unit-step slice region spans several chunks, else None."""
        if isinstance(leaf, ir.Concat):
            return None
        block_id = tuple(args[leaf.block_arg][1:])
        region = leaf.region(block_id)
        if any(isinstance(r, list) or (isinstance(r, slice) and (r.step or 1) != 1) for r in region):
            return None
        arr = self.ctx.device_source(leaf.target)
        if not isinstance(arr, DeviceArray):
            return None
        if region_view(arr, region, leaf.field) is not None:
            return None
        keys = region_chunk_keys(arr, region)
        if keys is not None and merged_view(arr, keys, leaf.field) is not None:
            return None
        ext = []
        for d, r in enumerate(region):
            if isinstance(r, slice):
                start, stop = r.start or 0, r.stop if r.stop is not None else arr.shape[d]
                ext.append(max(0, stop - start))
            else:
                ext.append(1)
        v = ArrView(0, ext, list(c_strides(ext)), arr.field_dtype(leaf.field))
        return v, arr, region, leaf.field

    def task_pieces(self, program, spec, target, key, leaves, out_items, structured_out, gathers,
                    reads_out=None):
        """The task as one or more TaskRows: when Region leaves straddle
        source chunks (``a[1:]`` of index, core/ops.py:374-486, whose output
        chunks overlap two input chunks), the task's space is cut at the
        chunk boundaries into pieces that each read single chunks in place --
        instead of gathering the region into scratch (a full extra write +
        read).  Returns (rows, group keys): pieces of one task with equal
        kept-dim intervals form one group, whose partials (if the program
        reduces across a cut) are combined before the epilogue.

        ``reads_out`` (a list) receives, per returned row, the
        (array, chunk coords, field) of every Region chunk the row reads
        (the multi-GPU executor runs each piece where that chunk lives)."""
        straddles = [] if not any(isinstance(l, ir.Philox) for l in leaves) else None
        row = self.task_layout(program, spec, target, key, leaves, out_items, structured_out,
                               gathers, straddles=straddles)
        if not straddles:
            if reads_out is not None:
                reads_out.append([r[:3] for r in self._region_chunks(leaves, spec, key)])
            return [row], [(tuple(key), ())]
        n = program.ndim
        red = set(program.reduce.axes) if program.reduce is not None else set()
        cuts = [{0, row.extent[d]} for d in range(n)]
        piece_lists = []
        for l, arr, region, field in straddles:
            axes = leaves[l].axes
            plist = []
            for coords, local, offs in region_pieces(arr, region):
                off_d, k = [], 0
                for d, r in enumerate(region):
                    if isinstance(r, slice):
                        off_d.append(offs[k])
                        k += 1
                    else:
                        off_d.append(0)
                iv = {}
                for d, sd in enumerate(axes):
                    if sd is not None and isinstance(region[d], slice):
                        lo, cnt = off_d[d], local[d][1]
                        iv[sd] = (lo, lo + cnt, d)
                        cuts[sd].update((lo, lo + cnt))
                plist.append((coords, local, iv))
            piece_lists.append(plist)
        bounds = [sorted(c) for c in cuts]
        intervals = [list(zip(b[:-1], b[1:])) for b in bounds]
        rows, groups, reads = [], [], []
        kept = [d for d in range(n) if d not in red]
        straddled = {l for l, *_ in straddles}
        fixed = [r for r in self._region_chunks(leaves, spec, key) if r[3] not in straddled]
        for box in itertools.product(*intervals):
            row_reads = [r[:3] for r in fixed]
            lo = [b[0] for b in box]
            ext = [b[1] - b[0] for b in box]
            bases = list(row.bases)
            lstr = [list(st) for st in row.lstrides]
            for l in range(len(leaves)):
                if isinstance(leaves[l], (ir.Arg, ir.Region)) or isinstance(leaves[l], ir.Iota):
                    isz = np.dtype(leaves[l].dtype).itemsize if not isinstance(leaves[l], ir.Iota) else 1
                    bases[l] = row.bases[l] + sum(lo[d] * row.lstrides[l][d] for d in range(n)) * isz
            for (l, arr, region, field), plist in zip(straddles, piece_lists):
                hit = None
                for coords, local, iv in plist:
                    if all(iv[sd][0] <= lo[sd] and lo[sd] + ext[sd] <= iv[sd][1] for sd in iv):
                        hit = (coords, local, iv)
                        break
                if hit is None:
                    raise LoweringError("region piece not found for a task sub-box")
                coords, local, iv = hit
                row_reads.append((arr, tuple(coords), field))
                inner = c_strides(arr.chunk_extent(coords))
                isz = arr.field_dtype(field).itemsize
                axes = leaves[l].axes
                off = 0
                st = [0] * n
                for d, r in enumerate(region):
                    ls, _, step = local[d]
                    sd = axes[d]
                    pos = ls
                    if sd is not None and sd in iv:
                        pos += (lo[sd] - iv[sd][0]) * step
                        st[sd] = inner[d] * step if ext[sd] != 1 else 0
                    off += pos * inner[d]
                bases[l] = arr.chunk_addr(coords, field) + off * isz
                lstr[l] = st
            obases = [row.obases[o] + sum(lo[d] * row.ostrides[o][d] for d in range(n)) *
                      np.dtype(_out_dtype(target, out_items[o][0], structured_out)).itemsize
                      for o in range(len(row.obases))]
            rows.append(TaskRow(ext, bases, lstr, obases, [list(x) for x in row.ostrides],
                                row.key_lo, row.key_hi, row.block_offset))
            groups.append((tuple(key), tuple(lo[d] for d in kept)))
            reads.append(row_reads)
        # pieces of one group contiguous, in order along the cut reduced dims
        order = sorted(range(len(rows)), key=lambda i: (groups[i][1], i))
        if reads_out is not None:
            reads_out += [reads[i] for i in order]
        return [rows[i] for i in order], [groups[i] for i in order]

    def _region_chunks(self, leaves, spec, key):
        """(array, coords, field, leaf index) of every chunk the task's
        Region leaves read."""
        args = spec.block_function(("out",) + tuple(key))
        args = [list(a) if not isinstance(a, (tuple, list, str)) else a for a in args]
        out = []
        for l, leaf in enumerate(leaves):
            if isinstance(leaf, ir.Concat):
                for ai, region, _ in leaf.region(tuple(args[leaf.block_arg][1:])):
                    arr = self.ctx.device_source(leaf.sources[ai])
                    if isinstance(arr, DeviceArray):
                        for coords, _, _ in region_pieces(arr, region):
                            out.append((arr, tuple(coords), leaf.field, l))
            elif isinstance(leaf, ir.Region):
                arr = self.ctx.device_source(leaf.target)
                if not isinstance(arr, DeviceArray):
                    continue
                region = leaf.region(tuple(args[leaf.block_arg][1:]))
                for coords, _, _ in region_pieces(arr, region):
                    out.append((arr, tuple(coords), leaf.field, l))
        return out

    def leaf_view(self, leaf, args, spec, gathers, out_key):
        """(kind, view) for one leaf of one task."""
        if isinstance(leaf, ir.ReshapeArg):
            a = args[leaf.index]
            arr = self.resolve_target(a[0], spec.reads_map)
            v = chunk_view(arr, a[1:], leaf.field)
            return LEAF_ARRAY, _reshaped_view(leaf, a[1:], v)
        if isinstance(leaf, ir.Concat):
            block_id = tuple(args[leaf.block_arg][1:])
            srcs = [self.ctx.device_source(t) for t in leaf.sources]
            return LEAF_ARRAY, self.ctx.gather_concat(srcs, leaf.region(block_id), leaf.axis,
                                                      leaf.field, gathers)
        if isinstance(leaf, ir.Arg):
            a = args[leaf.index]
            if isinstance(a, tuple):
                arr = self.resolve_target(a[0], spec.reads_map)
                if isinstance(arr, _OffsetsSource):
                    return LEAF_OFFSET, _Scalar(block_id_to_offset(a[1:], arr.shape))
                return LEAF_ARRAY, (chunk_view(arr, a[1:], leaf.field) if arr.ndim else
                                    ArrView(arr.chunk_addr((), leaf.field), [], [], arr.field_dtype(leaf.field)))
            keys = flatten_keys(a)
            arr = self.resolve_target(keys[0][0], spec.reads_map)
            v = merged_view(arr, keys, leaf.field)
            if v is None:
                v = self.ctx.gather_keys(arr, keys, leaf.field, gathers)
            return LEAF_ARRAY, v
        if isinstance(leaf, ir.Region):
            block_id = tuple(args[leaf.block_arg][1:])
            region = leaf.region(block_id)
            arr = self.ctx.device_source(leaf.target)
            v = region_view(arr, region, leaf.field)
            if v is None:
                keys = region_chunk_keys(arr, region)
                if keys is not None:
                    v = merged_view(arr, keys, leaf.field)
            if v is None:
                v = self.ctx.gather_region(arr, region, leaf.field, gathers)
            return LEAF_ARRAY, v
        if isinstance(leaf, ir.Philox):
            block_id = tuple(args[leaf.block_arg][1:])
            off = block_id_to_offset(block_id, leaf.numblocks)
            from .random import philox_key

            ext = [leaf.chunks[d][b] for d, b in enumerate(block_id)]
            v = ArrView(0, ext, list(c_strides(ext)), np.dtype(np.float64))
            v.key = philox_key(leaf.root_seed, off)
            v.block_offset = off
            return LEAF_PHILOX, v
        if isinstance(leaf, ir.BlockOffset):
            block_id = tuple(args[leaf.block_arg][1:])
            return LEAF_OFFSET, _Scalar(block_id_to_offset(block_id, leaf.numblocks))
        if isinstance(leaf, ir.Iota):
            block_id = tuple(args[leaf.arg][1:])
            nd = len(leaf.chunks)
            ext = [leaf.chunks[d][b] for d, b in enumerate(block_id)]
            start = sum(leaf.chunks[leaf.dim][:block_id[leaf.dim]])
            st = [1 if d == leaf.dim else 0 for d in range(nd)]
            return LEAF_IOTA, ArrView(start, ext, st, np.dtype(np.int64))
        raise LoweringError(f"unsupported leaf {type(leaf).__name__}")

    # -- copies ---------------------------------------------------------------
    def lower_copy_program(self, program, spec, target, task_keys):
        """merge_chunks / index / identity maps as box copies."""
        leaf = program.outputs
        boxes = []
        for key in task_keys:
            key = tuple(key)
            args = spec.block_function(("out",) + key)
            dst = chunk_view(target, key) if target.ndim else ArrView(target.chunk_addr(()), [], [], target.dtype)
            if isinstance(leaf, ir.Concat):
                block_id = tuple(args[leaf.block_arg][1:])
                dstr = _dst_strides_for(leaf.axes, program.out_axes, dst)
                isz = target.dtype.itemsize
                for ai, region, off in leaf.region(block_id):
                    src = self.ctx.device_source(leaf.sources[ai])
                    if not isinstance(src, DeviceArray):
                        raise _NotACopy()
                    boxes += boxes_for_region(src, region, dst.base + off * dstr[leaf.axis] * isz,
                                              dstr, leaf.field)
            elif isinstance(leaf, ir.ReshapeArg):
                a = args[leaf.index]
                src = self.resolve_target(a[0], spec.reads_map)
                if not isinstance(src, DeviceArray):
                    raise _NotACopy()
                sv = _reshaped_view(leaf, a[1:], chunk_view(src, a[1:], leaf.field))
                n = math.prod(sv.extent)
                if n:
                    boxes.append(Box(sv.base, dst.base, [n], [1], [1]))
            elif isinstance(leaf, ir.Region):
                block_id = tuple(args[leaf.block_arg][1:])
                region = leaf.region(block_id)
                src = self.ctx.device_source(leaf.target)
                if isinstance(src, _ConstSource):
                    raise LoweringError("copy from a constant")
                # destination strides for the region's kept (non-int) dims
                dstr = _dst_strides_for(leaf.axes, program.out_axes, dst)
                dstr = [st for st, r in zip(dstr, region) if not _is_int_sel(r)]
                boxes += boxes_for_region(src, region, dst.base, dstr, leaf.field)
            else:
                a = args[leaf.index]
                keys = [a] if isinstance(a, tuple) else flatten_keys(a)
                src = self.resolve_target(keys[0][0], spec.reads_map)
                dstr = _dst_strides_for(leaf.axes, program.out_axes, dst)
                n_src = sum(math.prod(src.chunk_extent(k[1:])) if src.ndim else 1 for k in keys)
                if n_src != (math.prod(dst.extent) if target.ndim else 1):
                    raise _NotACopy()  # a broadcast (broadcast_to, meshgrid): the fused path
                for k in keys:
                    sv = chunk_view(src, k[1:], leaf.field) if src.ndim else \
                        ArrView(src.chunk_addr((), leaf.field), [], [], src.dtype)
                    # position of this chunk inside the merged destination
                    boxes.append(Box(sv.base, dst.base + _merged_offset(src, keys, k, dstr) * target.dtype.itemsize,
                                     sv.extent, sv.stride, dstr[:len(sv.extent)]))
        return CopyLaunch(boxes, target.dtype.itemsize, self.ctx.device)


class _NotACopy(Exception):
    """A copy program whose source is not an HBM array (constant, offsets)."""


def _reshaped_view(leaf, in_coords, v: ArrView) -> ArrView:
    """The input chunk (compact C order in its slot) seen with the extents
    of the reshaped output chunk of the same linear block offset
    (reshape_chunks' block_function, manipulation_functions.py:258-265)."""
    off = block_id_to_offset(tuple(in_coords), leaf.in_numblocks)
    oc = offset_to_block_id(off, tuple(len(c) for c in leaf.out_chunks))
    ext = [leaf.out_chunks[d][b] for d, b in enumerate(oc)]
    if math.prod(ext) != math.prod(v.extent):
        raise LoweringError(f"reshape of a {v.extent} chunk into {ext}")
    return ArrView(v.base, ext, list(c_strides(ext)), v.dtype)


def _out_dtype(target, name, structured):
    return target.field_dtype(name if structured else None)


def _merged_offset(src, keys, k, dstr):
    if len(keys) == 1:
        return 0
    first = [min(kk[d + 1] for kk in keys) for d in range(src.ndim)]
    off = 0
    for d in range(src.ndim):
        pos = sum(src._norm_chunks[d][first[d]:k[d + 1]])
        off += pos * dstr[d]
    return off


def _dst_strides_for(leaf_axes, out_axes, dst: ArrView):
    """Destination element strides for each leaf dim (0 for unit dims)."""
    space_to_out = {s: j for j, s in enumerate(out_axes) if s is not None}
    out = []
    for s in leaf_axes:
        if s is None or s not in space_to_out:
            out.append(0)
        else:
            out.append(dst.stride[space_to_out[s]] if dst.stride else 0)
    return out


class _Scalar:
    def __init__(self, offset):
        self.block_offset = offset
        self.base = 0
        self.extent = []
        self.stride = []


class _ConstSource:
    def __init__(self, value, arr):
        self.value = value
        self.array = arr


class _OffsetsSource:
    def __init__(self, arr):
        self.shape = arr.shape
        self.ndim = arr.ndim


def _set_insn(slot, ins):
    op, a, b, c, t, imm = ins
    slot.op, slot.a, slot.b, slot.c, slot.t, slot.imm = op, a, b, c, t, imm


# ------------------------------------------------------------------ canonical layout


@dataclass
class TaskRow:
    extent: List[int]
    bases: List[int]
    lstrides: List[List[int]]
    obases: List[int]
    ostrides: List[List[int]]
    key_lo: int
    key_hi: int
    block_offset: int


@dataclass
class Layout:
    order: List[int]          # groups of program dims (after coalescing) in kernel order
    groups: List[List[int]]
    ndim: int
    nred: int
    mode: int
    rows: List[TaskRow]
    max_kept: int
    max_red: int

    def table(self, device):
        import torch

        arr = np.zeros(len(self.rows), dtype=nat.TASK_DTYPE)
        for i, r in enumerate(self.rows):
            ext, ls, os_ = _apply_groups(r, self.groups)
            e = [1] * nat.MAX_DIMS
            e[:len(ext)] = ext
            arr[i]["extent"] = e
            for l in range(len(r.bases)):
                arr[i]["leaf_base"][l] = r.bases[l]
                s = [0] * nat.MAX_DIMS
                s[:len(ext)] = ls[l]
                arr[i]["leaf_stride"][l] = s
            for o in range(len(r.obases)):
                arr[i]["out_base"][o] = r.obases[o]
                s = [0] * nat.MAX_DIMS
                s[:len(ext)] = os_[o]
                arr[i]["out_stride"][o] = s
            arr[i]["key_lo"] = np.uint64(r.key_lo)
            arr[i]["key_hi"] = np.uint64(r.key_hi)
            arr[i]["block_offset"] = r.block_offset
        return torch.from_numpy(arr.view(np.uint8).copy()).to(device)


def _apply_groups(r: TaskRow, groups):
    """Coalesce program dims into kernel dims (each group = contiguous run,
    outermost first; the group's stride is its innermost dim's)."""
    ext = [math.prod(r.extent[d] for d in g) for g in groups]
    ls = [[st[g[-1]] for g in groups] for st in r.lstrides]
    os_ = [[st[g[-1]] for g in groups] for st in r.ostrides]
    return ext, ls, os_


def canonicalize(rows: List[TaskRow], n: int, red_axes, leaves, kinds, check_outputs=True) -> Layout:
    if n == 0:
        groups = []
    else:
        groups = None
    # 1. dims of extent 1 in every task are dropped
    live = [d for d in range(n) if any(r.extent[d] != 1 for r in rows)]
    if not live:
        live = [n - 1] if n else []
    kept = [d for d in live if d not in red_axes]
    red = [d for d in live if d in red_axes]
    innermost = live[-1] if live else None
    use_b = False
    if red and innermost is not None and innermost in red_axes:
        inner_ext = max(r.extent[innermost] for r in rows)
        contig = all(st[innermost] in (0, 1) for r in rows for st in r.lstrides)
        use_b = inner_ext >= 64 and contig
    order = (kept + red) if use_b else (red + kept)

    def can_merge(a, b):
        # a then b adjacent in `order`, same reduced status
        if (a in red_axes) != (b in red_axes):
            return False
        for r in rows:
            for st in r.lstrides + r.ostrides:
                if st[a] != st[b] * r.extent[b]:
                    return False
        return True

    groups = []
    for d in order:
        if groups and can_merge(groups[-1][-1], d) and _groups_contiguous(groups[-1], d, order):
            groups[-1].append(d)
        else:
            groups.append([d])
    if not groups:
        groups = [[0]] if n else []
    nred = sum(1 for g in groups if g[0] in red_axes)
    ndim = len(groups)
    if ndim > nat.MAX_DIMS:
        raise LoweringError(f"task needs {ndim} iteration dims after coalescing (max {nat.MAX_DIMS})")
    if ndim == 0:
        # 0-d program: one element per task
        groups = [[]]
        ndim = 1

    def gext(r, g):
        return math.prod(r.extent[d] for d in g) if g else 1

    kept_groups = [g for g in groups if not (g and g[0] in red_axes)]
    red_groups = [g for g in groups if g and g[0] in red_axes]
    max_kept = max(math.prod(gext(r, g) for g in kept_groups) for r in rows) if rows else 1
    max_red = max(math.prod(gext(r, g) for g in red_groups) for r in rows) if rows else 1
    # vectorisation (VEC=4) along the innermost kernel dim
    inner = groups[-1]
    mode = 1 if use_b else 0
    if inner and _vec_ok(rows, inner, kinds, leaves, use_b or not check_outputs):
        mode |= 4
    rows2 = []
    for r in rows:
        if not groups[0]:
            rows2.append(TaskRow([1], r.bases, [[0] for _ in r.lstrides], r.obases,
                                 [[0] for _ in r.ostrides], r.key_lo, r.key_hi, r.block_offset))
        else:
            rows2.append(r)
    lay = Layout(order, groups if groups[0] else [[0]], ndim, nred, mode, rows2,
                 max(1, max_kept), max(1, max_red))
    if not groups[0]:
        lay.groups = [[0]]
        for r in rows2:
            r.extent = [1]
    return lay


LIFT_MIN_ELEMS = 4096  # inner elements per task for a lifted full reduction
LIFT_MIN_ROWS = 32     # outer (reduced) rows per kept element: partials stay small


def _lift_dims(rows, n):
    """Innermost dims a full reduction walks as kept dims: the shortest
    innermost run with >= LIFT_MIN_ELEMS elements in the largest task, if the
    remaining outer dims still give >= LIFT_MIN_ROWS rows on average (so the
    per-element partials cost little next to the rows they summarise)."""
    big = max(rows, key=lambda r: math.prod(r.extent))
    inner, prod = [], 1
    for d in range(n - 1, 0, -1):
        inner.append(d)
        prod *= big.extent[d]
        if prod >= LIFT_MIN_ELEMS:
            break
    if prod < LIFT_MIN_ELEMS:
        return set()
    vol = sum(math.prod(r.extent) for r in rows)
    kept = sum(math.prod(r.extent[d] for d in inner) for r in rows)
    if not kept or vol / kept < LIFT_MIN_ROWS:
        return set()
    return set(inner)
LIFT_ENABLED = True
MODE_STREAM = 8  # include/cubed_amd.h CUBED_MODE_STREAM
MODE_PARTIALS = 16  # include/cubed_amd.h CUBED_MODE_PARTIALS
_VTYPE_DTYPE = {V_F32: np.dtype(np.float32), V_F64: np.dtype(np.float64), V_I64: np.dtype(np.int64)}


MODE_STREAM_W2 = 32  # include/cubed_amd.h CUBED_MODE_STREAM_W2
MODE_STREAM_W4 = 64  # include/cubed_amd.h CUBED_MODE_STREAM_W4
MODE_HOST_COUNT = 128  # include/cubed_amd.h CUBED_MODE_HOST_COUNT
MODE_STREAM_EVEN = 256  # include/cubed_amd.h CUBED_MODE_STREAM_EVEN
MODE_OWNER_MAJOR = 512  # include/cubed_amd.h CUBED_MODE_OWNER_MAJOR
# The balanced split keeps all 256 CUs streaming where the uniform split of
# 49 column blocks x 5 leaves 11 idle, but measured 4-8 % SLOWER on every
# split workload (per-rank share 0.221 vs 0.203 ms, config 1 0.464 vs 0.456,
# elided rechunk + mean 1.459 vs 1.404; profiles/r04_even_ab.log): 245 CUs
# already saturate HBM, and 256 runs at 256 different row offsets read HBM
# less sequentially than 49 column blocks x 5 row bands.  Off by default;
# probes and tests set it.
STREAM_EVEN = False


def _red_extent(row, layout) -> int:
    """Reduced extent of one streaming task (stream_body's nrd)."""
    ext = _apply_groups(row, layout.groups)[0]
    return int(np.prod(ext[:layout.nred], dtype=np.int64))


def _stream_unroll(itemsize: int, nleaves: int) -> int:
    """Rows in flight per lane of the streaming kernel (fused_common.h
    stream_unroll)."""
    if itemsize == 4:
        return 8 if nleaves <= 1 else 4 if nleaves == 2 else 2
    return 4 if nleaves <= 1 else 2


FORCE_STREAM_W = None  # tests set 1 / 2 / 4 to run one program at every W


def _stream_groups_mode(P, ntasks: int, max_kept: int) -> int:
    """Mode bits for the kept groups per thread (W) of a streaming JIT kernel.

    W gives each lane about 256 B of loads in flight (U rows x leaves x W
    groups x 4 elements), e.g. W = 2 for quad-means' two f32 leaves -- but
    only when the W-wide grid still fills the CUs without a time split
    (>= 96 KiB of loads in flight per CU; config 1's split grid ran 2.7x
    slower with W = 2)
    and a task's kept extent fills at least 8 workgroups of 1024 W elements
    (the elided rechunk+mean's 1000-wide pieces left half of every
    workgroup idle with W = 2: 2.7x slower; profiles/r02_stream_ab.log)."""
    isz = 4 if P.vtype == V_F32 else 8
    nl = max(1, P.nleaves)
    if FORCE_STREAM_W is not None:  # tests: every W on one program
        w = FORCE_STREAM_W
    else:
        w0 = 256 // (_stream_unroll(isz, nl) * nl * 4 * isz)
        # f32 two-leaf programs (quad-means, var / std of a product): W = 4
        # with ONE row per lane in flight (jit.hip) -- quad-means 1.149-1.153
        # ms against 1.173-1.179 for W = 2 with 2 rows and 1.164-1.169 with 1
        # (profiles/r06_stream_unroll.log); W = 2 where W = 4 does not fit
        cands = [4, 2] if isz == 4 and nl == 2 else [4 if w0 >= 4 else 2 if w0 >= 2 else 1]
        w = 1
        for c in cands:
            slots = -(-max_kept // (256 * c)) * 64
            # the W-wide grid must hold >= 96 KiB of loads in flight per CU
            # unsplit (fused.hip plan_launch splits below that)
            inflight = 256 * _stream_unroll(isz, nl) * nl * c * 4 * isz
            if c == 1 or (ntasks * -(-slots // 256) * inflight >= 256 * 96 * 1024 and max_kept >= 8 * 1024 * c):
                w = c
                break
    return MODE_STREAM_W4 if w == 4 else MODE_STREAM_W2 if w == 2 else 0


def _stream_ok(layout: Layout, leaves, kinds, vtype, check_outputs=True) -> bool:
    """Geometry of the streaming fast path (stream_impl.h): kernel A with VEC=4,
    one kept kernel dim (packed in every leaf and output) after at most two
    reduced dims (chunk index x rows), every leaf an array chunk in the VM's
    own dtype."""
    if layout.mode != 4 or layout.nred > 2 or layout.ndim != layout.nred + 1 or not leaves:
        return False
    want = _VTYPE_DTYPE.get(vtype)
    for l, kind in enumerate(kinds):
        if kind != LEAF_ARRAY or np.dtype(leaves[l].dtype) != want:
            return False
    for r in layout.rows:
        ext, ls, os_ = _apply_groups(r, layout.groups)
        for l, st in enumerate(ls):
            if st[-1] != 1 or r.bases[l] % 16:
                return False
            for d in range(layout.nred):
                if ext[d] != 1 and st[d] % 4:
                    return False
        for st in os_:
            if check_outputs and st[-1] != 1:
                return False
    return True


MERGE_ROWS = True  # tests set False to run the unmerged task / piece rows
MERGE_KEPT = True  # probes set False to keep one task per output chunk


def _merge_group_rows(rows, group_keys, red_axes, leaves):
    """Rows of one output group (pieces of a task cut at source-chunk
    boundaries, chain_piece_rows' per-chunk rows) that continue each other
    along a reduced dim IN MEMORY -- the stacked row bands of one HBM array
    are one run of addresses -- merged into one row per run: config 3's
    read-through column block walks its 50000 rows as one row instead of 50
    pieces combined by a grouped finish.  Only the association of the
    (associative) field reductions changes.  Returns (rows, group keys)."""
    from .chains import _try_merge

    isz = [np.dtype(l.dtype).itemsize for l in leaves]
    red = sorted(red_axes)
    out_rows, out_keys = [], []
    i = 0
    while i < len(rows):
        j = i
        while j < len(rows) and group_keys[j] == group_keys[i]:
            j += 1
        acc = []
        for r in rows[i:j]:
            for a, q in enumerate(acc):
                if q.obases != r.obases or q.ostrides != r.ostrides or \
                        (q.key_lo, q.key_hi, q.block_offset) != (r.key_lo, r.key_hi, r.block_offset):
                    continue
                m = _try_merge(q, r, red, isz)
                if m is None:
                    m = _try_merge(r, q, red, isz)
                if m is not None:
                    acc[a] = m
                    break
            else:
                acc.append(r)
        out_rows += acc
        out_keys += [group_keys[i]] * len(acc)
        i = j
    return out_rows, out_keys


def _merge_kept_runs(layout: Layout, leaf_isz, out_isz):
    """A streaming layout whose consecutive tasks continue each other along
    the packed kept dim -- same reduced extents and strides, every leaf and
    output base exactly one kept extent further on -- as fewer, wider tasks
    (None when nothing merges).  The column blocks of one row-major array
    read through an elided rechunk are such tasks: 50 tasks of 4000-B piece
    rows that start mid-line become one task of whole 200000-B rows, so
    workgroup boundaries fall on 128-B lines and no boundary line is fetched
    twice.  Rows come back in kernel dims (identity groups); each output
    element still sums the same rows of the same leaves."""
    krows = []
    for r in layout.rows:
        ext, ls, os_ = _apply_groups(r, layout.groups)
        krows.append(TaskRow(list(ext), list(r.bases), [list(s) for s in ls], list(r.obases),
                             [list(s) for s in os_], r.key_lo, r.key_hi, r.block_offset))
    out = [krows[0]]
    for b in krows[1:]:
        a = out[-1]
        n = a.extent[-1]
        if a.extent[:-1] == b.extent[:-1] and a.lstrides == b.lstrides and a.ostrides == b.ostrides and \
                all(bb == ab + n * s for ab, bb, s in zip(a.bases, b.bases, leaf_isz)) and \
                all(bb == ab + n * s for ab, bb, s in zip(a.obases, b.obases, out_isz)):
            a.extent[-1] += b.extent[-1]
        else:
            out.append(b)
    if len(out) == len(krows):
        return None
    nd = layout.ndim
    return Layout(list(range(nd)), [[d] for d in range(nd)], nd, layout.nred, layout.mode, out,
                  max(1, max(r.extent[-1] for r in out)), layout.max_red)


def _groups_contiguous(group, d, order):
    return order.index(d) == order.index(group[-1]) + 1


def _vec_ok(rows, inner, kinds, leaves, use_b) -> bool:
    for r in rows:
        e = math.prod(r.extent[d] for d in inner)
        if e % 4:
            return False
        d_in = inner[-1]
        for l, (st, kind) in enumerate(zip(r.lstrides, kinds)):
            s_in = st[d_in]
            if kind == LEAF_ARRAY:
                if s_in not in (0, 1):
                    return False
                if s_in == 1:
                    isz = np.dtype(leaves[l].dtype).itemsize
                    if r.bases[l] % (4 * isz):
                        return False
                    if any(st[d] % 4 for d in range(len(st)) if d not in inner and r.extent[d] != 1):
                        return False
            elif kind == LEAF_PHILOX:
                if s_in != 1:
                    return False
        if not use_b:
            for o, st in enumerate(r.ostrides):
                if st[d_in] != 1:
                    return False
                if r.obases[o] % 32:
                    return False
                if any(st[d] % 4 for d in range(len(st)) if d not in inner and r.extent[d] != 1):
                    return False
    return True
