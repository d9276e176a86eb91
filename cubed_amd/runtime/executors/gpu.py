"""The MI355X DAG executor.

Replaces the reference's task loop (``PythonDagExecutor``,
runtime/executors/python.py:14-32, and the thread-pool
``AsyncPythonDagExecutor``, python_async.py:121-142) behind the same plug-in
interface ``execute_dag(dag, callbacks, array_names, resume, spec)``:

* each op node of the finalized DAG (one fused pipeline) is lowered once to
  one or two kernel launches over ALL its tasks (cubed_amd/lowering.py) and
  cached on the executor, so re-executing a plan replays the launches;
* launches are stream-ordered on one HIP stream (torch's current stream by
  default); nothing synchronises inside ``execute_dag`` -- reading a result
  back (``compute()``) or the caller's ``torch.cuda.synchronize()`` does;
* intermediates stay resident in HBM (``DeviceArray`` slabs allocated by the
  create-arrays node); ``resume=True`` skips ops whose targets were already
  written by an earlier compute (the reference's resume, runtime/pipeline.py
  :8-35);
* one ``TaskEndEvent(array_name, num_tasks)`` per pipeline, so the
  reference's callbacks (task counters, history, progress) keep working.

There is no CPU path: a pipeline whose chunk function cannot be lowered
raises ``LoweringError`` instead of running host code.
"""

from __future__ import annotations

import itertools
import math
import time
import weakref
from typing import Dict, List, Optional

import networkx as nx
import numpy as np

from ... import _native as nat
from ... import ir
from ...core.ops import UploadSpec, upload_stage
from ...core.plan import create_arrays_stage
from ...lowering import (
    ArrView,
    Box,
    CopyLaunch,
    FusedLaunch,
    GemmLaunch,
    LoweringError,
    Lowerer,
    _OffsetsSource,
    boxes_for_region,
    chunk_view,
)
from ...primitive.blockwise import apply_blockwise
from ...primitive.rechunk import copy_read_to_write
from ...storage import (
    DeviceArray,
    HostArray,
    VirtualEmptyArray,
    VirtualFullArray,
    VirtualInMemoryArray,
    VirtualOffsetsArray,
    c_strides,
)
from ..pipeline import visit_nodes
from ..types import DagExecutor, TaskEndEvent

HBM_BYTES_PER_GPU = 288 * 10**9
# multi-GPU matmuls whose A k chunks / C columns each live on one rank run as
# dist.DistGemmLaunch (packed A image exchanged in place); tests flip it to
# compare with the whole-chunk fetch path
DIST_GEMM = True


def gather_to_host(arr: DeviceArray) -> np.ndarray:
    import torch

    if arr.world > 1:
        from .dist import gather_distributed

        return gather_distributed(arr)
    torch.cuda.synchronize(arr.device)
    return arr.to_numpy()


class LaunchTimer:
    """Per-launch HIP events recorded on the executor's stream (torch's
    current stream), for bench.py's live roofline figure."""

    def __init__(self):
        self.records = []

    def events(self):
        import torch

        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def add(self, key, ev0, ev1):
        self.records.append((key, ev0, ev1))

    def summary(self):
        """{launch key: (count, mean ms)} after a device synchronize."""
        out = {}
        for key, a, b in self.records:
            c, s = out.get(key, (0, 0.0))
            out[key] = (c + 1, s + a.elapsed_time(b))
        return {k: (c, s / c) for k, (c, s) in out.items()}


class _Alloc:
    def __init__(self, ctx, targets):
        self.ctx = ctx
        self.targets = list(targets)

    def run(self, stream):
        for t in self.targets:
            if id(t) not in self.ctx.elided:
                self.ctx.allocate(t)


class _Upload:
    def __init__(self, ctx, cfg: UploadSpec):
        self.ctx = ctx
        self.cfg = cfg

    def run(self, stream):
        from ...zarr_io import ZarrV2Array, upload_zarr

        self.ctx.allocate(self.cfg.target)
        if isinstance(self.cfg.source, ZarrV2Array):
            upload_zarr(self.cfg.source, self.cfg.target)
        else:
            self.cfg.target.from_numpy(np.asarray(self.cfg.source.array))


class GpuDagExecutor(DagExecutor):
    """Runs Cubed plans on one MI355X (one process per GPU)."""

    def __init__(self, device=None, stream=None, check_memory: bool = True, comm="auto"):
        """``comm``: a ``cubed_amd.runtime.comm.Comm`` for multi-GPU execution
        (one process per GPU; every rank runs the same plan), ``None`` for a
        single GPU, or "auto" = the torch.distributed world group when it has
        more than one rank."""
        import torch

        if not torch.cuda.is_available():
            raise nat.NativeError("GpuDagExecutor needs a visible GPU (cubed_amd has no CPU path)")
        nat.lib()
        self._init_state(torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}"),
                         stream, check_memory)
        if comm == "auto":
            from ..comm import default_comm

            comm = default_comm()
        self.set_comm(comm)

    def set_comm(self, comm):
        self.comm = comm
        self.rank, self.world = (comm.rank, comm.world) if comm is not None else (0, 1)

    def _init_state(self, device, stream, check_memory):
        self.device = device
        self._stream = stream
        self.check_memory = check_memory
        self._cache: Dict[int, tuple] = {}
        self._uploads: Dict[int, DeviceArray] = {}
        # device buffers made while lowering (scratch gathers, split
        # temporaries) go to the cache entry being built, so they live as
        # long as the launches that use them; outside a compile they belong
        # to the executor
        self._scratch: List = []
        self._sink: List = self._scratch
        self._schedules: Dict = {}
        self.last_schedule = None  # the schedule the last non-replayed execute_dag recorded
        self.replays = 0  # execute_dag calls served from a recorded schedule
        self.lowerer = Lowerer(self)
        self.comm = None
        self.rank, self.world = 0, 1
        self.timing: Optional[LaunchTimer] = None
        self.fuse_reductions = True
        self.fuse_gemm_sums = True
        self._chains: Dict = {}
        self._exec_dags: Dict = {}
        self.fuse_producers = True
        self.elide_rechunks = True
        self._agreed = set()
        self.elided = set()
        self._resident_bytes = 0

    # -- plumbing used by the lowerer ------------------------------------------
    @property
    def stream(self) -> int:
        import torch

        if self._stream is not None:
            return self._stream.cuda_stream if hasattr(self._stream, "cuda_stream") else int(self._stream)
        return torch.cuda.current_stream(self.device).cuda_stream

    def allocate(self, t: DeviceArray):
        if not t.allocated:
            t.allocate(self.device, self.rank, self.world)
            t.comm = self.comm

    def device_source(self, arr):
        """A readable device-side representation of an input array."""
        if isinstance(arr, DeviceArray):
            if not arr.allocated:
                self.allocate(arr)
            return arr
        if isinstance(arr, VirtualOffsetsArray):
            return _OffsetsSource(arr)
        if isinstance(arr, (VirtualInMemoryArray, VirtualFullArray, HostArray)):
            key = id(arr)
            d = self._uploads.get(key)
            if d is None:
                d = DeviceArray(arr.shape, arr.dtype, arr.chunks if arr.ndim else (),
                                name=f"virtual-{key}")
                d.allocate(self.device, 0, 1)  # small constants: replicated on every rank
                if isinstance(arr, VirtualFullArray):
                    self._fill(d, arr.fill_value)
                else:
                    d.from_numpy(np.asarray(arr.array))
                d.written = True
                self._uploads[key] = d
                # the cache entry (and its HBM) lives as long as the source
                # array: id() may be reused once the array is collected
                weakref.finalize(arr, _drop_upload, weakref.ref(self), key)
            return d
        if isinstance(arr, VirtualEmptyArray):
            raise LoweringError("a chunk function reads an empty (template) array")
        raise LoweringError(f"unsupported source array {type(arr).__name__}")

    def _fill(self, d: DeviceArray, value):
        import torch

        tdt = {np.dtype(np.float64): torch.float64, np.dtype(np.float32): torch.float32,
               np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32,
               np.dtype(np.int16): torch.int16, np.dtype(np.int8): torch.int8,
               np.dtype(np.uint8): torch.uint8, np.dtype(np.bool_): torch.bool}
        for f in d.fields:
            dt = d.field_dtype(f)
            if d.dtype.kind == "c":
                v = complex(value)
                value_f = v.real if f == "real" else v.imag
            else:
                value_f = value if f is None else value[f]
            if dt in tdt:
                d.slabs[f].view(tdt[dt]).fill_(value_f)
            else:
                raw = np.full(d.slabs[f].numel() // dt.itemsize, value_f, dtype=dt)
                d.slabs[f].copy_(torch.from_numpy(raw.view(np.uint8)))

    def scratch(self, nbytes: int) -> int:
        import torch

        from ...storage import _GEOMETRY_ONLY

        if _GEOMETRY_ONLY[0]:
            return 0

        buf = torch.empty(max(nbytes, 16) + 256, dtype=torch.uint8, device=self.device)
        self._sink.append(buf)
        p = buf.data_ptr()
        return (p + 255) // 256 * 256

    def own(self, arr: DeviceArray):
        """Tie an HBM temporary made while lowering (cubed_amd/split.py) to
        the cache entry being built, after checking it fits next to the
        plan's resident arrays."""
        need = sum(arr.slot_bytes(f) for f in arr.fields) * arr.nchunks
        if self.check_memory and self._resident_bytes + self.owned_bytes() + need > HBM_BYTES_PER_GPU:
            raise MemoryError(f"a {need}-byte split temporary does not fit next to the plan's "
                              f"{self._resident_bytes} bytes of HBM-resident arrays")
        self._sink.append(arr)

    def owned_bytes(self) -> int:
        """HBM held by buffers of cached launches and of the executor."""
        total = sum(_nbytes(b) for b in self._scratch)
        for entry in self._cache.values():
            total += sum(_nbytes(b) for b in entry[2])
        return total

    def _cache_put(self, key, obj, launches, owned):
        """Cache ``launches`` (and the buffers they own) for ``obj``; the
        entry goes when ``obj`` is collected (its id may then be reused).
        The launches hold device addresses: an entry recorded before an
        array was released or moved (storage.alloc_epoch) is not reused."""
        from ...storage import alloc_epoch

        self._cache[key] = (weakref.ref(obj), launches, owned, alloc_epoch())
        weakref.finalize(obj, _drop_entry, weakref.ref(self), "_cache", key)

    def _cache_hit(self, key, obj):
        from ...storage import alloc_epoch

        entry = self._cache.get(key)
        if entry is not None and entry[0]() is obj and entry[3] == alloc_epoch():
            return entry
        return None

    class _Collect:
        def __init__(self, ex):
            self.ex, self.owned = ex, []

        def __enter__(self):
            self.prev, self.ex._sink = self.ex._sink, self.owned
            return self.owned

        def __exit__(self, *exc):
            self.ex._sink = self.prev
            return False

    def gather_region(self, arr: DeviceArray, region, field, gathers) -> ArrView:
        """Copy a multi-chunk region into contiguous scratch; return its view
        in array-dim order (int-indexed dims as extent 1)."""
        ext_all, keep_ext = [], []
        for d, s in enumerate(region):
            if isinstance(s, slice):
                start, stop, step = s.start or 0, s.stop, s.step or 1
                e = max(0, (stop - start + step - 1) // step)
                ext_all.append(e)
                keep_ext.append(e)
            elif isinstance(s, list):
                ext_all.append(len(s))
                keep_ext.append(len(s))
            else:
                ext_all.append(1)
        dt = arr.field_dtype(field)
        base = self.scratch(math.prod(keep_ext) * dt.itemsize)
        dstr = list(c_strides(keep_ext))
        gathers.append((boxes_for_region(arr, region, base, dstr, field), dt.itemsize))
        strides_all, k = [], 0
        for d, s in enumerate(region):
            if isinstance(s, (slice, list)):
                strides_all.append(dstr[k])
                k += 1
            else:
                strides_all.append(0)
        return ArrView(base, ext_all, strides_all, dt)

    def gather_concat(self, srcs, parts, axis, field, gathers) -> ArrView:
        """Assemble a concat output block (parts = (source index, region,
        offset along ``axis``)) into contiguous scratch."""
        dt = srcs[parts[0][0]].field_dtype(field)
        ext = None
        for ai, region, off in parts:
            e = [max(0, (s.stop - (s.start or 0))) for s in region]
            if ext is None:
                ext = list(e)
                ext[axis] = 0
            ext[axis] = max(ext[axis], off + e[axis])
        base = self.scratch(max(1, math.prod(ext)) * dt.itemsize)
        dstr = list(c_strides(ext))
        boxes = []
        for ai, region, off in parts:
            boxes += boxes_for_region(srcs[ai], region, base + off * dstr[axis] * dt.itemsize, dstr, field)
        gathers.append((boxes, dt.itemsize))
        return ArrView(base, ext, dstr, dt)

    def gather_keys(self, arr: DeviceArray, keys, field, gathers) -> ArrView:
        coords = [k[1:] for k in keys]
        region = []
        for d in range(arr.ndim):
            lo = min(c[d] for c in coords)
            hi = max(c[d] for c in coords)
            start = arr.chunk_start(tuple(lo if dd == d else 0 for dd in range(arr.ndim)))[d]
            stop_c = tuple(hi if dd == d else 0 for dd in range(arr.ndim))
            stop = arr.chunk_start(stop_c)[d] + arr.chunk_extent(stop_c)[d]
            region.append(slice(start, stop, 1))
        return self.gather_region(arr, tuple(region), field, gathers)

    # -- lowering --------------------------------------------------------------
    def _task_keys(self, target: DeviceArray):
        if target.ndim == 0:
            return [()]
        return list(itertools.product(*[range(n) for n in target.numblocks]))

    def lower_node(self, name, node) -> list:
        pipeline = node["pipeline"]
        fn = pipeline.function
        cfg = pipeline.config
        if fn is create_arrays_stage:
            return [_Alloc(self, pipeline.mappable)]
        if fn is upload_stage:
            return [_Upload(self, cfg)]
        if fn is copy_read_to_write:
            return [self._lower_rechunk(cfg)]
        if fn is apply_blockwise:
            target = cfg.write.array
            self.allocate(target)
            program = cfg.function
            keys = self._task_keys(target)
            if isinstance(program, ir.OpaqueProgram):
                raise LoweringError(
                    f"op {name}: {program.func!r} cannot run on the MI355X executor "
                    "(not expressible as a fused chunk program)")
            if isinstance(program, (ir.ExprProgram, ir.MatmulProgram, ir.TensordotProgram,
                                    ir.PerBlockProgram)):
                return self._lower_part(program, cfg, target, keys)
            if isinstance(program, ir.GemmThenProgram):
                from types import SimpleNamespace

                from ...primitive.types import CubedArrayProxy

                gt = program.gemm_target
                self.allocate(gt)
                gcfg = SimpleNamespace(block_function=program.gemm_block_function,
                                       reads_map=program.gemm_reads)
                launches = self._lower_part(program.gemm, gcfg, gt, self._task_keys(gt))
                if not isinstance(program.then, ir.ExprProgram):
                    raise LoweringError(f"op {name}: GEMM consumer {program.then!r} is not lowerable")
                tcfg = SimpleNamespace(block_function=program.then_block_function,
                                       reads_map={gt.name: CubedArrayProxy(gt, gt.chunks)},
                                       write=cfg.write)
                return launches + self._lower_part(program.then, tcfg, target, keys)
            raise LoweringError(f"op {name}: unsupported program {type(program).__name__}")
        raise LoweringError(f"op {name}: unknown stage function {getattr(fn, '__name__', fn)}")

    # -- one blockwise part: (fetch of remote inputs) + its launch --------------
    def _lower_part(self, program, cfg, target, keys):
        """Launches of one blockwise program over the tasks this rank owns.
        With several GPUs, chunks the owned tasks read from other ranks are
        fetched first (FetchLaunch) and the task views point at the copies."""
        if isinstance(program, ir.PerBlockProgram):
            # traced per output block; blocks with equal programs share a launch
            groups = {}
            for key in keys:
                try:
                    p = program.trace(key)
                except ir.FusionError as e:
                    raise LoweringError(str(e)) from None
                groups.setdefault(repr(p.outputs), (p, []))[1].append(key)
            out = []
            for p, ks in groups.values():
                out += self._lower_part(p, cfg, target, ks)
            return out
        if self.world == 1:
            return self._lower_local(program, cfg, target, keys)
        if isinstance(program, ir.ExprProgram) and program.reduce is not None and \
                any(isinstance(l, ir.Region) for l in ir.leaves_of_program(program)) and \
                not any(isinstance(l, ir.Concat) for l in ir.leaves_of_program(program)):
            launches = self._lower_pieces_dist(program, cfg, target, keys)
            # every rank must take the same path (their collectives pair up)
            if self.comm.all_ok(launches is not None):
                return launches
        owned = [k for k in keys if target.owner(k) == self.rank]
        fetch, arrays = self._plan_fetch(
            {k: target.owner(k) for k in keys},
            lambda k: self._task_reads(program, cfg, k))
        out = [fetch] if fetch is not None else []
        if not owned:
            return out
        with _remote_chunks(fetch, arrays):
            out += self._lower_local(program, cfg, target, owned)
        return out

    def _lower_pieces_dist(self, program, cfg, target, keys):
        """A reduction over Region leaves (index / merge regions, a rechunk
        read through) on several GPUs: every task is cut into pieces at the
        source chunk boundaries and each piece runs on the rank that holds its
        chunk (dist.DistPiecesLaunch), so the source never crosses xGMI --
        only per-group partials do.  None when the program does not fit this
        shape (the caller then fetches whole chunks instead)."""
        import dataclasses

        from ...lowering import MODE_HOST_COUNT
        from ...storage import geometry_only
        from .dist import DistPiecesLaunch

        rank = self.rank
        low = self.lowerer
        red = set(program.reduce.axes)
        meta = {"discard": self.scratch(max(target.slot_bytes(f) for f in target.fields))}

        def home_of(reads, key):
            for arr, coords, _ in reads:
                if arr.world > 1:
                    return arr.owner(coords)
            return target.owner(key)

        def rows_fn(leaves, kinds):
            out_items = list(program.output_items())
            # pass 1: geometry of every piece of every task -> homes, fetch needs
            per_task = {}
            with geometry_only():
                for key in keys:
                    reads, gathers = [], []
                    r, g = low.task_pieces(program, cfg, target, key, leaves, out_items,
                                           program.structured, gathers, reads_out=reads)
                    if gathers:
                        raise LoweringError("pieces need a scratch gather")
                    per_task[key] = reads
            arg_reads = {key: self._task_reads(program, cfg, key, regions=False) for key in keys}
            home = {(key, i): home_of(rd, key) for key, reads in per_task.items()
                    for i, rd in enumerate(reads)}
            fetch, arrays = self._plan_fetch(
                home, lambda item: list(per_task[item[0]][item[1]]) + arg_reads[item[0]])
            meta["fetch"] = fetch
            # pass 2: this rank's pieces with real addresses (fetched chunks
            # resolved); other ranks' pieces only give their group's shape
            rows, gkeys = [], []
            mko = 1
            counts = {}
            with _remote_chunks(fetch, arrays), geometry_only():
                for key in keys:
                    r, g = low.task_pieces(program, cfg, target, key, leaves, out_items,
                                           program.structured, [])
                    owned_out = target.owner(key) == rank
                    by_group = {}
                    for i, (row, gk) in enumerate(zip(r, g)):
                        by_group.setdefault(gk, []).append((i, row))
                    for gk, items in by_group.items():
                        # the group's global element count along the reduced
                        # dims: its pieces on every rank together
                        counts[(key, gk)] = sum(math.prod(row.extent[d] for d in red) for _, row in items)
                        first = items[0][1]
                        mko = max(mko, math.prod(first.extent[d] for d in range(len(first.extent))
                                                 if d not in red))
                        mine = [row for i, row in items if home[(key, i)] == rank]
                        if not mine:  # no piece here: an empty row yields the identity
                            e = list(first.extent)
                            for d in red:
                                e[d] = 0
                            mine = [dataclasses.replace(first, extent=e, bases=[0] * len(first.bases))]
                        for row in mine:
                            if not owned_out:
                                row = dataclasses.replace(row, obases=[meta["discard"]] * len(row.obases))
                            rows.append(row)
                            gkeys.append((key, gk))
            from ... import lowering as L

            if L.MERGE_ROWS and all(k == L.LEAF_ARRAY for k in kinds):
                # this rank's row bands of one group continue each other in its
                # slab (its chunks' slots are consecutive): one row per run
                rows, gkeys = L._merge_group_rows(rows, gkeys, red, leaves)
            meta["starts"] = [i for i in range(len(gkeys)) if i == 0 or gkeys[i] != gkeys[i - 1]]
            meta["nrows"] = len(rows)
            meta["kept_ok"] = all(math.prod(r.extent[d] for d in range(len(r.extent)) if d not in red) == mko
                                  for r in rows)
            meta["mko"] = mko
            meta["counts"] = [counts[gkeys[i]] for i in meta["starts"]]
            # the output block of every group (several groups per key when the
            # pieces cut a kept dim): the combine's owner of each group
            meta["group_keys"] = [gkeys[i][0] for i in meta["starts"]]
            return rows, red

        def one_row_per_group():
            return meta["nrows"] == len(meta["starts"]) and meta["kept_ok"]

        try:
            launch = low.lower_expr_pipeline(program, cfg, target, keys, rows_fn=rows_fn,
                                             sample_key=keys[0], partials=True, lift=False,
                                             merge_kept_groups=one_row_per_group)
        except LoweringError:
            return None
        starts = meta["starts"]
        lay = launch.group_layout or launch.layout
        table = dataclasses.replace(lay, rows=[lay.rows[i] for i in starts]).table(self.device)
        rops = [f.rop for f in program.reduce.fields]
        acc_int = [bool(launch.prog.field_acc[i]) for i in range(len(rops))]
        # one row per group streamed as wide merged tasks: the kernel's SoA
        # partials already are the per-group partials (no combine_groups)
        soa_direct = launch.group_layout is not None and len(starts) == len(lay.rows) and \
            lay.max_kept == meta["mko"]
        assert launch.group_layout is None or soa_direct, "merged kept runs need one row per group"
        out = [meta["fetch"]] if meta.get("fetch") is not None else []
        glay = dataclasses.replace(lay, rows=[lay.rows[i] for i in starts])
        out.append(DistPiecesLaunch(self, launch, np.array(starts + [len(lay.rows)], dtype=np.int64),
                                    table, meta["mko"], rops, acc_int,
                                    [target.owner(k) for k in meta["group_keys"]],
                                    soa_direct=soa_direct,
                                    host_counts=meta["counts"] if launch.prog.mode & MODE_HOST_COUNT else None,
                                    group_layout=glay, discard=meta["discard"], group_counts=meta["counts"]))
        return out

    def _lower_local(self, program, cfg, target, keys):
        if isinstance(program, ir.ExprProgram):
            try:
                return _with_gathers(self.lowerer.lower_expr_pipeline(program, cfg, target, keys), self.device)
            except LoweringError:
                from ...lowering import program_fits

                if program_fits(program):
                    raise
                # more inputs / instructions than one fused program holds:
                # factor parts out into HBM temporaries (cubed_amd/split.py)
                from ...split import split_launches

                return split_launches(self, program, cfg, target, keys)
        return [self._lower_gemm(program, cfg, target, keys)]

    def _task_reads(self, program, cfg, key, regions=True):
        """(array, chunk coords, field) of every distributed chunk one task
        reads (the apply_blockwise key resolution, primitive/blockwise.py
        :70-76, plus map_direct regions)."""
        from ...lowering import collect_leaves, program_exprs, region_pieces
        from ...utils import flatten_keys

        args = cfg.block_function(("out",) + tuple(key))
        args = [list(a) if not isinstance(a, (tuple, list, str)) else a for a in args]
        out = []

        def add_key(k, field):
            src = self.device_source(cfg.reads_map[k[0]].array)
            if isinstance(src, DeviceArray) and src.world > 1:
                out.append((src, tuple(k[1:]), field))

        if isinstance(program, (ir.MatmulProgram, ir.TensordotProgram)):
            for a in args[:2]:
                for k in ([a] if isinstance(a, tuple) else flatten_keys(a)):
                    add_key(k, None)
            return out
        outs, fields = program_exprs(program)
        for leaf in collect_leaves(outs + fields):
            if isinstance(leaf, ir.Arg):
                a = args[leaf.index]
                if isinstance(a, str):
                    continue
                for k in ([a] if isinstance(a, tuple) else flatten_keys(a)):
                    add_key(k, leaf.field)
            elif isinstance(leaf, ir.Concat):
                block_id = tuple(args[leaf.block_arg][1:])
                for ai, region, _ in leaf.region(block_id):
                    src = self.device_source(leaf.sources[ai])
                    if isinstance(src, DeviceArray) and src.world > 1:
                        for coords, _, _ in region_pieces(src, region):
                            out.append((src, tuple(coords), leaf.field))
            elif isinstance(leaf, ir.Region) and regions:
                src = self.device_source(leaf.target)
                if isinstance(src, DeviceArray) and src.world > 1:
                    block_id = tuple(args[leaf.block_arg][1:])
                    for coords, _, _ in region_pieces(src, leaf.region(block_id)):
                        out.append((src, tuple(coords), leaf.field))
        return out

    def _plan_fetch(self, task_owner, reads_of):
        """FetchLaunch for the remote chunks of a set of tasks ({key: owner
        rank}), or None when no rank reads a chunk it does not own."""
        from ..exchange import plan_fetch
        from .dist import FetchLaunch, chunk_nbytes

        needs: Dict[int, set] = {}
        arrays: Dict[str, DeviceArray] = {}
        remote = False
        for key, r in task_owner.items():
            for arr, coords, field in reads_of(key):
                if arr.name is None:
                    raise LoweringError("distributed arrays need names")
                prev = arrays.setdefault(arr.name, arr)
                if prev is not arr:
                    raise LoweringError(f"two arrays named {arr.name}")
                needs.setdefault(r, set()).add((arr.name, coords, field))
                remote = remote or arr.owner(coords) != r
        if not remote:
            return None, arrays
        plan = plan_fetch(needs, lambda ref: arrays[ref[0]].owner(ref[1]),
                          lambda ref: chunk_nbytes(arrays[ref[0]], ref[1], ref[2]),
                          self.rank, self.world)
        return FetchLaunch(self, plan, arrays), arrays

    def _lower_rechunk(self, cfg):
        src = self.device_source(cfg.read.array)
        dst = cfg.write.array
        self.allocate(dst)
        if self.world > 1:
            from ..exchange import plan_rechunk
            from .dist import RechunkLaunch

            replicated = src.world == 1
            plan = plan_rechunk(src, dst, self.rank, self.world, dst.dtype.itemsize,
                                src_world=1 if replicated else self.world)
            return RechunkLaunch(self, plan, src, dst, replicated)
        boxes: List[Box] = []
        for f in dst.fields:  # complex / structured arrays: every slab
            for key in self._task_keys(dst):
                region = tuple(slice(s, s + e) for s, e in zip(dst.chunk_start(key), dst.chunk_extent(key)))
                dv = chunk_view(dst, key, f)
                boxes += boxes_for_region(src, region, dv.base, dv.stride, f)
        if len({dst.field_dtype(f).itemsize for f in dst.fields}) != 1:
            raise LoweringError("rechunk of fields of different widths is not lowered")
        # source order: workgroups in flight together read neighbouring source
        # rows (measured 3.6 vs 4.05 ms on the 50000^2 rows -> columns case)
        boxes.sort(key=lambda b: b.src)
        return CopyLaunch(boxes, dst.field_dtype(dst.fields[0]).itemsize, self.device)

    def _lower_gemm(self, program, cfg, target, keys):
        """Per-chunk products (each task a chain of one segment): the matmul
        blockwise op when its k-sum is not fused (gemm_chains.py)."""
        tasks = np.zeros(len(keys), dtype=nat.CHAIN_DTYPE)
        segs = np.zeros(len(keys), dtype=nat.SEG_DTYPE)
        in_dt = None
        for i, key in enumerate(keys):
            args = cfg.block_function(("out",) + tuple(key))
            a_key, b_key = args[0], args[1]
            A = self.device_source(cfg.reads_map[a_key[0]].array)
            B = self.device_source(cfg.reads_map[b_key[0]].array)
            if A.ndim != 2 or B.ndim != 2:
                raise LoweringError("batched matmul chunks are not lowered yet")
            if A.dtype != B.dtype or (in_dt is not None and A.dtype != in_dt):
                raise LoweringError(f"matmul of {A.dtype} x {B.dtype} -> {target.dtype} is not lowered "
                                    "(operands of one dtype only)")
            in_dt = A.dtype
            if A.dtype not in (np.float32, np.float64, np.int64, ir.bfloat16):
                raise LoweringError(f"matmul of {A.dtype} is not lowered (f32, bf16, f64, int64)")
            am, ak = A.chunk_extent(a_key[1:])
            bk, bn = B.chunk_extent(b_key[1:])
            if ak != bk:
                raise LoweringError("contracted chunk extents differ")
            segs[i] = (A.chunk_addr(a_key[1:]), B.chunk_addr(b_key[1:]), ak, ak, bn, 0)
            tasks[i] = (target.chunk_addr(key), am, bn, bn, i, 1, ak, 0)
        return GemmLaunch(tasks, segs, ir.dtype_code(in_dt or target.dtype), ir.dtype_code(target.dtype),
                          self.device, self.zero_page())

    def zero_page(self) -> int:
        """Device address of 4 KiB of zeros (k past a GEMM chain's end)."""
        import torch

        from ...storage import _GEOMETRY_ONLY

        if _GEOMETRY_ONLY[0]:
            return 0
        z = getattr(self, "_zero", None)
        if z is None:
            z = self._zero = torch.zeros(4096, dtype=torch.uint8, device=self.device)
        return (z.data_ptr() + 255) // 256 * 256

    # -- execution -------------------------------------------------------------
    def compiled(self, name, node):
        pipeline = node["pipeline"]
        entry = self._cache_hit(id(pipeline), pipeline)
        if entry is not None:
            return entry[1]
        err = None
        with self._Collect(self) as owned:
            try:
                launches = self.lower_node(name, node)
            except LoweringError as e:
                err = e
        if self.world > 1 and not self.comm.all_ok(err is None):
            # a pipeline that cannot be lowered on one rank fails on all of them
            # (instead of leaving the others waiting in a collective)
            raise err or LoweringError(f"op {name} could not be lowered on another rank")
        if err is not None:
            raise err
        self._cache_put(id(pipeline), pipeline, launches, owned)
        return launches

    def chains_of(self, dag, array_names):
        """Reduction chains of this DAG (cubed_amd/chains.py), cached."""
        key = (id(dag), tuple(array_names or ()))
        entry = self._chains.get(key)
        if entry is not None and entry[0]() is dag:
            return entry[1]
        from ...chains import find_chains
        from ...gemm_chains import find_gemm_chains

        chains = find_gemm_chains(dag, array_names) if self.fuse_gemm_sums else {}
        taken = {m for ch in chains.values() for m in ch.nodes}
        if self.fuse_reductions:
            chains.update(find_chains(dag, array_names, exclude=taken))
        members = {}
        nodes = dict(dag.nodes(data=True))
        for first, ch in chains.items():
            for m in ch.nodes[1:]:
                members[m] = first
            # partials of all but the last level are never materialised
            for m in ch.nodes[:-1]:
                for out in dag.successors(m):
                    t = nodes[out].get("target")
                    if isinstance(t, DeviceArray):
                        self.elided.add(id(t))
            for t in getattr(ch, "extra_targets", ()):
                if t is not ch.final_target:
                    self.elided.add(id(t))
        self._chains[key] = (weakref.ref(dag), (chains, members))
        weakref.finalize(dag, _drop_entry, weakref.ref(self), "_chains", key)
        return chains, members

    def compiled_chain(self, chain):
        from ...gemm_chains import GemmChain

        key = ("gemm" if isinstance(chain, GemmChain) else "chain", id(chain.first_spec))
        entry = self._cache_hit(key, chain.first_spec)
        if entry is not None:
            return entry[1]
        with self._Collect(self) as owned:
            if isinstance(chain, GemmChain):
                launches = self._lower_gemm_chain(chain)
            else:
                launches = self._lower_chain(chain)
        self._cache_put(key, chain.first_spec, launches, owned)
        return launches

    def _lower_chain(self, chain):
        from ...chains import chain_rows, contributing_keys

        target = chain.final_target
        self.allocate(target)
        keys = self._task_keys(target)
        if chain.regions:
            if self.world > 1:
                # the distributed pieces path (DistPiecesLaunch) runs these per op
                raise LoweringError("region chains run op by op on several GPUs")
            from ...chains import chain_piece_rows

            launch = self.lowerer.lower_expr_pipeline(
                chain.program, chain.first_spec, target, keys,
                rows_fn=lambda leaves, kinds: chain_piece_rows(self.lowerer, chain, leaves, kinds, keys),
                sample_key=contributing_keys(chain, keys[0])[0])
            return _with_gathers(launch, self.device)
        if self.world > 1:
            return self._compiled_chain_dist(chain, target, keys)
        launch = self.lowerer.lower_expr_pipeline(
            chain.program, chain.first_spec, target, keys,
            rows_fn=lambda leaves, kinds: chain_rows(self.lowerer, chain, leaves, kinds, keys),
            sample_key=contributing_keys(chain, keys[0])[0])
        return _with_gathers(launch, self.device)

    def _lower_gemm_chain(self, chain):
        """matmul's chunk products + k-sum as ONE cubed_gemm_chain launch
        (gemm_chains.py); with several GPUs each rank computes the output
        chunks it owns, after fetching the A row / B column chunks it lacks."""
        from ...gemm_chains import K_AXIS, chain_tables

        F = chain.final_target
        self.allocate(F)
        keys = self._task_keys(F)
        out = []
        if F.dtype.kind == "c":
            from ...gemm_chains import complex_chain_tables

            if self.world > 1:
                raise LoweringError("complex matmul runs on one GPU")
            pre, tasks, segs, in_dt, out_dt = complex_chain_tables(self, chain, keys)
            return pre + [GemmLaunch(tasks, segs, ir.dtype_code(in_dt), ir.dtype_code(out_dt), self.device,
                                     self.zero_page())]
        if self.world > 1 and DIST_GEMM:
            from .dist import DistGemmLaunch, dist_gemm_plan

            plan = dist_gemm_plan(self, chain, F)
            ok = plan is not None
            if ok:
                A = plan[0]
                need = nat.lib().cubed_gemm_dist_image_bytes(A.shape[0], A.shape[1],
                                                             ir.dtype_code(A.dtype))
                ok = not (self.check_memory and
                          self._resident_bytes + self.owned_bytes() + need > HBM_BYTES_PER_GPU)
            # every rank takes the same path (their transfers pair up)
            if self.comm.all_ok(ok):
                A, B, ti, nk, nj = plan
                code = ir.dtype_code(A.dtype)
                return [DistGemmLaunch(self, A, B, F, ti, nk, nj, code, ir.dtype_code(F.dtype),
                                       A.dtype.itemsize)]
        if self.world > 1:
            def reads(k):
                G = chain.gemm_target
                res = []
                for kk in range(G.numblocks[K_AXIS]):
                    args = chain.gemm_spec.block_function(("out", k[0], kk, k[-1]))
                    for a in args[:2]:
                        src = self.device_source(chain.gemm_spec.reads_map[a[0]].array)
                        if isinstance(src, DeviceArray) and src.world > 1:
                            res.append((src, tuple(a[1:]), None))
                return res

            fetch, arrays = self._plan_fetch({k: F.owner(k) for k in keys}, reads)
            owned = [k for k in keys if F.owner(k) == self.rank]
            if fetch is not None:
                out.append(fetch)
            with _remote_chunks(fetch, arrays):
                tasks, segs, in_dt, out_dt = chain_tables(self, chain, owned)
        else:
            tasks, segs, in_dt, out_dt = chain_tables(self, chain, keys)
        in_dt = in_dt if in_dt is not None else out_dt
        if in_dt not in (np.float32, np.float64, np.int64, ir.bfloat16):
            raise LoweringError(f"matmul of {in_dt} is not lowered (f32, bf16, f64, int64)")
        # one GPU, every output chunk in C order: tiles may cover the whole
        # matrix (cubed_gemm_chain_grid checks the grid and the dtype)
        grid = (F.numblocks[0], F.numblocks[-1]) if self.world == 1 and len(tasks) > 1 else None
        out.append(GemmLaunch(tasks, segs, ir.dtype_code(in_dt), ir.dtype_code(out_dt), self.device,
                              self.zero_page(), grid=grid, scratch=self._gemm_workspace))
        return out

    def _gemm_workspace(self, nbytes):
        """HBM workspace of the packed GEMMs (both operands rewritten once),
        or None when it would not fit beside the plan's arrays -- the chain
        set then runs on the per-chunk kernel, which needs none -- or when
        lowering only for geometry (no address exists).  Each packed launch
        owns its workspace for the life of its cached plan: a repeated step
        allocates nothing, and launches that run concurrently
        (compute_arrays_in_parallel) never share one."""
        if self.check_memory and self._resident_bytes + self.owned_bytes() + nbytes > HBM_BYTES_PER_GPU:
            return None
        return self.scratch(nbytes) or None

    def _compiled_chain_dist(self, chain, target, keys):
        """A reduction chain over chunks spread across the ranks: each rank
        reduces the first-level tasks it owns (the chunks of the chain's
        input it holds) for EVERY output block into SoA partials; RCCL then
        combines the partials and the owners run the epilogue
        (dist.PartialsLaunch).  Same fields and composition as the 1-GPU
        chain, with the sum over ranks as the outermost association."""
        from ...chains import chain_rows, contributing_keys
        from .dist import PartialsLaunch

        first = chain.first_target
        world, rank = self.world, self.rank

        def first_owner(t):
            return first.chunk_offset(t) % world

        contrib = {K: contributing_keys(chain, K) for K in keys}
        p1 = chain.first_spec.function
        task_owner = {t: first_owner(t) for K in keys for t in contrib[K]}
        fetch, arrays = self._plan_fetch(task_owner,
                                         lambda t: self._task_reads(p1, chain.first_spec, t))
        discard = self.scratch(max(target.slot_bytes(f) for f in target.fields))
        select = {K: [t for t in contrib[K] if first_owner(t) == rank] for K in keys}
        rops = [f.rop for f in chain.program.reduce.fields]
        meta = {}

        def rows_fn(leaves, kinds):
            rows = chain_rows(self.lowerer, chain, leaves, kinds, keys, select=select,
                              out_owned=lambda K: target.owner(K) == rank, discard=discard)
            # from geometry every rank derives alike (same decision everywhere)
            meta["count"] = _chain_global_count(self.lowerer, chain, rops, keys, contrib, leaves)
            return rows

        with _remote_chunks(fetch, arrays):
            launch = self.lowerer.lower_expr_pipeline(
                chain.program, chain.first_spec, target, keys, rows_fn=rows_fn,
                sample_key=contrib[keys[0]][0], partials=True, lift=False,
                host_count=lambda: meta.get("count") is not None)
        launches = [fetch] if fetch is not None else []
        launches += _with_gathers(launch, self.device)
        acc_int = [bool(launch.prog.field_acc[i]) for i in range(len(rops))]
        launches.append(PartialsLaunch(self, launch, rops, acc_int, [target.owner(K) for K in keys],
                                       host_count=meta.get("count"), discard=discard))
        return launches

    def exec_dag(self, dag, array_names):
        """The DAG this executor runs: the plan's finalized DAG with
        single-consumer rechunks read through by their consumer
        (rewrites.elide_rechunks) and single-consumer elementwise maps fused
        into their consumers (chains.fuse_elementwise_producers), cached per
        plan DAG."""
        key = (id(dag), tuple(array_names or ()))
        entry = self._exec_dags.get(key)
        if entry is not None and entry[0]() is dag:
            return entry[1]
        from ...chains import fuse_elementwise_producers
        from ...rewrites import compose_rechunks, elide_rechunks, split_complex

        new, absorbed = compose_rechunks(split_complex(dag), array_names)
        if self.elide_rechunks:
            new, more = elide_rechunks(new, array_names)
            absorbed += more
        if self.fuse_producers:
            new, more = fuse_elementwise_producers(new, array_names)
            absorbed += more
        for t in absorbed:
            if isinstance(t, DeviceArray):
                self.elided.add(id(t))
        self._exec_dags[key] = (weakref.ref(dag), new)
        weakref.finalize(dag, _drop_entry, weakref.ref(self), "_exec_dags", key)
        return new

    def execute_dag(self, dag, callbacks=None, array_names=None, resume=None, spec=None,
                    compute_arrays_in_parallel=None, **kwargs):
        """``compute_arrays_in_parallel`` (the async executors' flag,
        ``runtime/executors/python_async.py:86-114``): the pipelines of one
        topological generation are independent, so each runs on its own HIP
        stream (up to ``PARALLEL_STREAMS``), joined back into the executor's
        stream before the next generation.  With several ranks only ops made
        of local kernel launches (copy / fused / GEMM) fork; every op that
        holds a collective (partials, pieces, exchanges, fetches) stays on
        the executor's stream, so each rank issues its collectives in one
        order on one stream, as RCCL requires."""
        from ..reference_dag import execute_reference_dag, is_reference_dag

        if is_reference_dag(dag):
            # a plan built by the reference cubed: converted (targets to HBM,
            # chunk functions traced), run, outputs written to their Zarr stores
            execute_reference_dag(self, dag, callbacks=callbacks, array_names=array_names, resume=resume,
                                  spec=spec, compute_arrays_in_parallel=compute_arrays_in_parallel, **kwargs)
            return
        parallel = bool(compute_arrays_in_parallel)
        if self.world > 1 and self._stream is not None and self.device.type == "cuda":
            # collectives are issued on torch's current stream: make it the
            # executor's, so the pack / exchange / unpack sequence of a
            # RechunkLaunch or FetchLaunch stays stream-ordered
            import torch

            st = self._stream if isinstance(self._stream, torch.cuda.Stream) else \
                torch.cuda.ExternalStream(int(self._stream), device=self.device)
            with torch.cuda.stream(st):
                return self._execute_dag(dag, callbacks, array_names, resume, parallel)
        return self._execute_dag(dag, callbacks, array_names, resume, parallel)

    def _execute_dag(self, dag, callbacks, array_names, resume, parallel=False):
        stream = self.stream
        key = (id(dag), tuple(array_names or ()), bool(resume), self.elide_rechunks, self.fuse_producers,
               self.fuse_reductions, self.fuse_gemm_sums, parallel)
        book = self._schedules.get(key)
        if book is not None and book.dag_ref() is dag:
            sched = book.lookup()
            if sched is not None:
                self.replays += 1
                return self._run_schedule(sched, stream, callbacks)
        plan_dag = dag
        dag = self.exec_dag(dag, array_names)
        nodes = dict(dag.nodes(data=True))
        chains, members = self.chains_of(dag, array_names)
        if self.check_memory:
            self._check_hbm(dag)
        targets = [d["target"] for _, d in dag.nodes(data=True) if isinstance(d.get("target"), DeviceArray)]
        state = target_state(targets)
        gen_of = {}
        if parallel:
            for g, names in enumerate(nx.topological_generations(dag)):
                for n in names:
                    gen_of[n] = g
        steps = []
        try:
            self._lower_steps(dag, nodes, chains, members, gen_of, resume, steps)
        except LoweringError:
            # the ops before the one that cannot be lowered run (and are marked
            # written), as the reference's executor runs op by op: a resume
            # then picks up after them
            if steps:
                self._run_schedule(_Schedule(steps, parallel), stream, callbacks)
            raise
        sched = _Schedule(steps, parallel)
        self.last_schedule = sched
        self._run_schedule(sched, stream, callbacks)
        # later calls with the same plan, names, resume flag and written
        # state replay the launch list without re-walking the DAG
        if book is None or book.dag_ref() is not plan_dag:
            book = self._schedules[key] = _Schedules(plan_dag, targets)
            weakref.finalize(plan_dag, _drop_entry, weakref.ref(self), "_schedules", key)
        book.add(state, sched)

    def _lower_steps(self, dag, nodes, chains, members, gen_of, resume, steps):
        """The recorded steps of one execute_dag, appended to ``steps`` op by
        op (so a LoweringError leaves the lowered prefix in ``steps``)."""
        for name, node in visit_nodes(dag, resume=resume):
            gen = gen_of.get(name, 0)
            if name in members:
                launches = []  # ran as part of its chain's fused launch
            elif name in chains:
                ch = chains[name]
                if resume and ch.final_target.written:
                    launches = []
                else:
                    try:
                        launches = self.compiled_chain(ch)
                        ok = True
                    except LoweringError:
                        ok = False
                    if self.world > 1 and (name, id(ch)) not in self._agreed:
                        # every rank must take the same path (their collectives pair up)
                        ok = self.comm.all_ok(ok)
                        self._agreed.add((name, id(ch)))
                        if not ok:
                            self._cache.pop(("chain", id(ch.first_spec)), None)
                            self._cache.pop(("gemm", id(ch.first_spec)), None)
                    if not ok:
                        # not fusable after all: run the chain's pipelines one by one
                        chains.pop(name)
                        for m in ch.nodes[1:]:
                            members.pop(m, None)
                        for m in ch.nodes[:-1]:
                            for out in dag.successors(m):
                                t = nodes[out].get("target")
                                if isinstance(t, DeviceArray):
                                    self.elided.discard(id(t))
                                    self.allocate(t)
                        for t in getattr(ch, "extra_targets", ()):
                            self.elided.discard(id(t))
                        launches = self.compiled(name, node)
                    else:
                        # the fused launch reads every member's inputs: in a
                        # generation walk it runs with the chain's last member
                        gen = max(gen_of.get(m, 0) for m in ch.nodes)
            else:
                launches = self.compiled(name, node)
            marks = []
            if name not in chains:  # a chain head's partials are never materialised
                marks = [nodes[out].get("target") for out in dag.successors(name)
                         if isinstance(nodes[out].get("target"), DeviceArray)]
            op = node.get("primitive_op")
            events = list(node.get("fused_from", ())) + [(name, op.num_tasks if op is not None else 1)]
            steps.append((name, tuple(launches), tuple(marks), tuple(events), gen))

    PARALLEL_STREAMS = 4  # GPU_MAX_HW_QUEUES on the box: one hardware queue each

    def _side_streams(self):
        import torch

        if getattr(self, "_sides", None) is None:
            self._sides = [torch.cuda.Stream(device=self.device) for _ in range(self.PARALLEL_STREAMS - 1)]
        return [s.cuda_stream for s in self._sides]

    def _run_schedule(self, sched, stream, callbacks):
        """Run a recorded schedule.  Sequential: every launch on ``stream``.
        Parallel: per generation, the ops whose launches are all native
        kernel launches fork onto the side streams (each waits for the
        generation's start on ``stream``), everything else runs on
        ``stream`` first, and ``stream`` waits for every side stream before
        the next generation -- the only dependencies a generation has are on
        earlier generations."""
        timing = self.timing
        gpu_events = callbacks is not None and self.device.type == "cuda"
        fork_ok = sched.parallel and self.device.type == "cuda"
        use_events = gpu_events or fork_ok
        if use_events:
            import torch

            ext_cache = {}

            def ext(h):
                e = ext_cache.get(h)
                if e is None:
                    e = ext_cache[h] = torch.cuda.ExternalStream(h, device=self.device)
                return e

            def record(h):
                ev = torch.cuda.Event(enable_timing=gpu_events)
                ev.record(ext(h))
                return ev
        nsteps = len(sched.steps)
        start_ev = [None] * nsteps
        end_ev = [None] * nsteps
        host = [time.time()]
        t0_ev = record(stream) if gpu_events else None

        def run_step(i, h):
            name, launches, marks, _, _ = sched.steps[i]
            if timing is None:
                for launch in launches:
                    launch.run(h)
            else:
                for j, launch in enumerate(launches):
                    ev0, ev1 = timing.events()
                    if use_events:
                        ev0.record(ext(h))
                    else:
                        ev0.record()
                    launch.run(h)
                    if use_events:
                        ev1.record(ext(h))
                    else:
                        ev1.record()
                    timing.add((name, j, type(launch).__name__), ev0, ev1)
            for t in marks:
                t.written = True

        for group in sched.groups:
            if len(group) == 1 or not fork_ok:
                for i in group:
                    start_ev[i] = end_ev[i - 1] if i > 0 else t0_ev
                    run_step(i, stream)
                    if gpu_events:
                        end_ev[i] = record(stream)
                    elif callbacks is not None:
                        host.append(time.time())
                continue
            # host-side steps (allocations, uploads) and single-launch
            # generations stay on the executor's stream
            forked = [i for i in group if sched.forkable[i]]
            for i in group:
                if i not in forked:
                    start_ev[i] = t0_ev if gpu_events else None
                    run_step(i, stream)
                    if gpu_events:
                        end_ev[i] = record(stream)
            fork = record(stream)
            sides = self._side_streams()
            used = set()
            for k, i in enumerate(forked):
                h = stream if k == 0 else sides[(k - 1) % len(sides)]
                if h != stream and h not in used:
                    ext(h).wait_event(fork)
                    used.add(h)
                start_ev[i] = fork if gpu_events else None
                run_step(i, h)
                if gpu_events:
                    end_ev[i] = record(h)
            for h in used:
                ext(stream).wait_event(record(h))
            self.parallel_forks = getattr(self, "parallel_forks", 0) + 1
        if callbacks is None:
            return
        if gpu_events:
            # TaskEndEvents carry completion times: each op's end is its
            # stream event, placed on the host clock from one final event
            last = record(stream)
            last.synchronize()
            t_end = time.time()

            def at(ev):
                return t_end - ev.elapsed_time(last) * 1e-3

            starts = [at(e if e is not None else t0_ev) for e in start_ev]
            ends = [at(e if e is not None else last) for e in end_ev]
        else:
            starts, ends = host[:-1], host[1:]
        for i, (_, _, _, events, _) in enumerate(sched.steps):
            for aname, ntasks in events:
                ev = TaskEndEvent(array_name=aname, num_tasks=ntasks, function_start_tstamp=starts[i],
                                  function_end_tstamp=ends[i])
                ev.task_result_tstamp = ends[i]
                for cb in callbacks:
                    cb.on_task_end(ev)

    def _check_hbm(self, dag):
        total = 0
        for _, d in dag.nodes(data=True):
            t = d.get("target")
            if isinstance(t, DeviceArray) and id(t) not in self.elided:
                if t.allocated:
                    total += t.device_bytes()
                else:  # this rank's block-cyclic share, at most
                    total += -(-t.nchunks // self.world) * sum(t.slot_bytes(f) for f in t.fields)
        # uploaded host / in-memory sources are replicated on every rank
        total += sum(d.device_bytes() for d in self._uploads.values() if d.allocated)
        self._resident_bytes = total
        # scratch gathers and split temporaries of cached launches
        total += self.owned_bytes()
        if total > HBM_BYTES_PER_GPU:
            raise MemoryError(f"plan needs {total} bytes of HBM-resident arrays, more than one "
                              f"MI355X holds ({HBM_BYTES_PER_GPU})")


def _chain_global_count(lowerer, chain, rops, keys, contrib, leaves):
    """The global COUNT of a chain run over several ranks, when the host
    knows it: a plain ``count`` field of a sum-only chain (mean's ``n``)
    counts the elements of the reduced dims of every first-level task that
    contributes to an output block -- on every rank together.  Taken from the
    lowering geometry of ALL contributing tasks (``geometry_only``: the same
    extents on every rank, whoever owns the chunks), in the program's own
    iteration space, so permuted or reshaped leaves, broadcast inputs and
    chains ending before the last round count what the kernel counts.  None
    when blocks differ (the counts are then reduced over RCCL)."""
    from ...storage import geometry_only
    from .dist import SUM_ROPS

    if "count" not in rops or not all(r in SUM_ROPS for r in rops) or chain.regions:
        return None
    p1 = chain.first_spec.function
    axes = tuple(chain.program.reduce.axes)
    counts = set()
    with geometry_only():
        for K in keys:
            c = 0
            for t in contrib[K]:
                lay = lowerer.task_layout(p1, chain.first_spec, chain.first_target, t, leaves,
                                          [], p1.structured, [])
                c += math.prod(int(lay.extent[a]) for a in axes)
            counts.add(c)
    return counts.pop() if len(counts) == 1 else None


class _Schedule:
    """One recorded execute_dag: per op, its launches, the targets it marks
    written, the TaskEndEvents it emits and its topological generation
    (``groups``: consecutive runs of steps, one per generation when the
    schedule runs generations in parallel)."""

    def __init__(self, steps, parallel=False):
        from ...storage import alloc_epoch

        self.parallel = parallel
        if parallel:
            # a stable sort by generation: a chain's fused launch moved to
            # its last member's generation keeps its place among that
            # generation's ops
            steps = sorted(steps, key=lambda st: st[4])
            groups = {}
            for i, st in enumerate(steps):
                groups.setdefault(st[4], []).append(i)
            self.groups = list(groups.values())
        else:
            self.groups = [[i] for i in range(len(steps))]
        self.steps = steps
        self.forkable = [bool(st[1]) and all(isinstance(l, (CopyLaunch, FusedLaunch, GemmLaunch)) for l in st[1])
                         for st in steps]
        self.epoch = alloc_epoch()


def target_state(targets):
    """What a recorded schedule depends on: which targets are written (in
    HBM) or complete in their Zarr store (resume)."""
    return tuple((t.written, bool(getattr(t, "zarr_complete", False))) for t in targets)


class _Schedules:
    """The recorded schedules of one (plan DAG, array names, resume) by the
    written state of the plan's targets they start from.  A schedule is
    replayed while the DAG is alive and no array was released or moved
    since it was recorded (storage.alloc_epoch)."""

    def __init__(self, dag, targets):
        self.dag_ref = weakref.ref(dag)
        self.targets = targets
        self.by_state = {}

    def lookup(self):
        from ...storage import alloc_epoch

        sched = self.by_state.get(target_state(self.targets))
        if sched is not None and sched.epoch == alloc_epoch():
            return sched
        return None

    def add(self, state, sched):
        if len(self.by_state) > 16:
            self.by_state.clear()
        self.by_state[state] = sched


def _nbytes(b) -> int:
    if isinstance(b, DeviceArray):
        return b.device_bytes() if b.allocated else 0
    return b.numel() * b.element_size()


def _drop_entry(ex_ref, attr, key):
    """Finalizer: drop a cache entry whose key object was collected (unless
    the slot was already reused by a live object)."""
    ex = ex_ref()
    if ex is None:
        return
    cache = getattr(ex, attr)
    entry = cache.get(key)
    if entry is None:
        return
    ref = entry.dag_ref if isinstance(entry, _Schedules) else entry[0]
    if ref() is None:
        cache.pop(key, None)


def _drop_upload(ex_ref, key):
    ex = ex_ref()
    if ex is not None:
        ex._uploads.pop(key, None)


class _remote_chunks:
    """Installs a FetchLaunch's chunk copies on the arrays while one pipeline
    is lowered (DeviceArray.chunk_addr resolves non-owned chunks to them)."""

    def __init__(self, fetch, arrays):
        self.fetch, self.arrays = fetch, arrays

    def __enter__(self):
        if self.fetch is not None:
            for name, m in self.fetch.remote.items():
                self.arrays[name].remote = m
        return self

    def __exit__(self, *exc):
        for arr in self.arrays.values():
            arr.remote = None
        return False


def _with_gathers(launch, device):
    """Turn collected scratch gathers into CopyLaunches run before ``launch``."""
    gathers = getattr(launch, "gathers", None)
    if not gathers:
        return [launch]
    by_size: Dict[int, List[Box]] = {}
    for boxes, isz in gathers:
        by_size.setdefault(isz, []).extend(boxes)
    launch.gathers = [CopyLaunch(b, isz, device) for isz, b in by_size.items()]
    return [launch]
