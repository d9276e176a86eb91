"""Multi-GPU pieces of the MI355X executor (one process per GPU, RCCL).

The reference scales by mapping independent tasks onto workers that share
Zarr storage (runtime/executors/python_async.py:121-142, lithops.py); here
each GPU owns a block-cyclic share of every array's chunks
(cubed_amd/storage.py) and runs the tasks whose output chunk it owns.  Data
crosses GPUs only where a task reads a chunk it does not own:

* ``FetchLaunch``   -- whole chunks read by local tasks but owned elsewhere
  (pack -> RCCL all-to-all -> the task views point into the receive buffer);
* ``RechunkLaunch`` -- rechunk: local pieces copied in place, the rest moved
  by grouped point-to-point transfers in 1-4 slices (the pack of slice k+1
  and the local copies overlap the transfers of slice k); pieces contiguous
  in their target chunk are received straight into its slot, pieces
  contiguous in their source chunk are sent from it;
* ``PartialsLaunch``-- a fused reduction chain whose inputs are spread over
  the ranks: every rank reduces its own chunks to per-field partials
  (CUBED_MODE_PARTIALS), RCCL reduces them (SUM fields) or all-gathers them
  (max/min/prod/any/all, folded in rank order by cubed_combine_partials), and
  the owner(s) of the output run the epilogue (cubed_fused_finish).

Every rank walks the same DAG in the same order and derives the same plans
from chunk geometry alone, so the collectives always match.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np

from ... import _native as nat
from ...lowering import Box, CopyLaunch
from ...storage import DeviceArray, c_strides
from ..exchange import FetchExchange, RechunkExchange, box_offset

FETCH_ROW = 4096  # bytes per row of a whole-chunk pack copy (one wave moves 4 KiB)
SCATTER = True  # multi-owner sum reductions combine by reduce-scatter (ScatterCombine); tests flip it
OWNER_MAJOR = True  # ... with the stream kernel writing the owner-major order itself; tests flip it
ROP_COUNT = 3  # ir.ROPS["count"], include/cubed_amd.h CUBED_R_COUNT
OP_CONST = 1  # include/cubed_amd.h CUBED_OP_CONST (r[a] = consts[imm])


def consts_used(P):
    """Const slots a fused program reads (CONST instructions of its prologue
    and epilogue)."""
    ins = list(P.insns[:P.ninsns]) + list(P.epi[:max(P.nepi, 0)])
    return max([i.imm + 1 for i in ins if i.op == OP_CONST], default=0)


def _round(n, a):
    return (n + a - 1) // a * a


def chunk_nbytes(arr: DeviceArray, coords, field) -> int:
    return math.prod(arr.chunk_extent(coords)) * arr.field_dtype(field).itemsize


def _flat_boxes(pairs):
    """Contiguous byte copies (src, dst, nbytes: a multiple of 256 that never
    runs past the source slot) as 4 KiB-row boxes plus a tail row."""
    boxes = []
    for src, dst, nb in pairs:
        rows, tail = divmod(nb, FETCH_ROW)
        if rows:
            boxes.append(Box(src, dst, [rows, FETCH_ROW], [FETCH_ROW, 1], [FETCH_ROW, 1]))
        if tail:
            o = rows * FETCH_ROW
            boxes.append(Box(src + o, dst + o, [1, tail], [tail, 1], [tail, 1]))
    return boxes


class FetchLaunch:
    """Brings the remote chunks one pipeline reads into a local buffer."""

    def __init__(self, ctx, plan: FetchExchange, arrays: Dict[str, DeviceArray]):
        import torch

        self.ctx = ctx
        self.plan = plan
        self.send = torch.empty(max(sum(plan.send_splits), 16), dtype=torch.uint8, device=ctx.device)
        self.recv = torch.empty(max(sum(plan.recv_splits), 16), dtype=torch.uint8, device=ctx.device)
        sbase, rbase = self.send.data_ptr(), self.recv.data_ptr()
        pairs = []
        for lst in plan.send:
            for (name, coords, field), off, nb in lst:
                arr = arrays[name]
                pairs.append((arr.chunk_addr(coords, field), sbase + off, nb))
        self.pack = CopyLaunch(_flat_boxes(pairs), 1, ctx.device)
        # remote chunk maps, installed on the arrays while the pipeline lowers
        self.remote: Dict[str, Dict] = {}
        for lst in plan.recv:
            for (name, coords, field), off, nb in lst:
                self.remote.setdefault(name, {})[(tuple(coords), field)] = rbase + off

    def run(self, stream):
        self.pack.run(stream)
        self.ctx.comm.all_to_all(self.recv, self.send, self.plan.recv_splits, self.plan.send_splits)


SLICE_BYTES = 256 << 20  # exchanges moving more than this per rank run in slices
MAX_SLICES = 4


class RechunkLaunch:
    """copy_read_to_write over all target chunks owned here."""

    def __init__(self, ctx, plan: RechunkExchange, src: DeviceArray, dst: DeviceArray,
                 src_replicated: bool):
        import torch

        self.ctx = ctx
        self.plan = plan
        isz = plan.itemsize
        self.pack_buf = torch.empty(max(plan.pack_bytes, 16), dtype=torch.uint8, device=ctx.device)
        self.stage_buf = torch.empty(max(plan.stage_bytes, 16), dtype=torch.uint8, device=ctx.device)
        pbase, sbase = self.pack_buf.data_ptr(), self.stage_buf.data_ptr()

        def src_at(p):
            ext = src.chunk_extent(p.src)
            return src.chunk_addr(p.src) + box_offset(ext, p.src_start) * isz, list(c_strides(ext))

        def dst_at(p):
            ext = dst.chunk_extent(p.dst)
            return dst.chunk_addr(p.dst) + box_offset(ext, p.dst_start) * isz, list(c_strides(ext))

        def slab_view(arr, addr, nbytes):
            slab = arr.slabs[None]
            o = addr - slab.data_ptr()
            return slab[o:o + nbytes]

        local = []
        for p in plan.local:
            s_, ss = src_at(p)
            d_, ds = dst_at(p)
            local.append(Box(s_, d_, list(p.extent), ss, ds))
        local.sort(key=lambda b: b.src)
        self.local = CopyLaunch(local, isz, ctx.device)
        moved = plan.send_bytes + plan.recv_bytes
        nslices = 1 if moved <= SLICE_BYTES else min(MAX_SLICES, -(-moved // SLICE_BYTES))
        self.slices = []
        unpack = []
        for lo, hi in plan.slice_bounds(nslices):
            pack, sends, recvs = [], [], []
            for peer, lst in enumerate(plan.send):
                for x in lst:
                    if not lo <= x.index < hi:
                        continue
                    a, ss = src_at(x.piece)
                    if x.direct:
                        sends.append((slab_view(src, a, x.nbytes), peer))
                    else:
                        pack.append(Box(a, pbase + x.offset, list(x.piece.extent), ss,
                                        list(c_strides(x.piece.extent))))
                        sends.append((self.pack_buf[x.offset:x.offset + x.nbytes], peer))
            for peer, lst in enumerate(plan.recv):
                for x in lst:
                    if not lo <= x.index < hi:
                        continue
                    a, ds = dst_at(x.piece)
                    if x.direct:
                        recvs.append((slab_view(dst, a, x.nbytes), peer))
                    else:
                        recvs.append((self.stage_buf[x.offset:x.offset + x.nbytes], peer))
                        unpack.append(Box(sbase + x.offset, a, list(x.piece.extent),
                                          list(c_strides(x.piece.extent)), ds))
            pack.sort(key=lambda b: b.src)
            self.slices.append((CopyLaunch(pack, isz, ctx.device), sends, recvs))
        self.unpack = CopyLaunch(unpack, isz, ctx.device)
        self.exchange = plan.exchanges
        self.collective = True  # every rank takes part, even with nothing to move

    def run(self, stream):
        timing = getattr(self.ctx, "timing", None)
        if timing is not None and getattr(self.ctx.comm, "backend", None) == "loopback":
            return self._run_phases(stream, timing)
        pending = []
        for pack, sends, recvs in self.slices:
            pack.run(stream)
            pending.append(self.ctx.comm.exchange(sends, recvs))
        self.local.run(stream)  # overlaps the transfers
        for p in pending:
            p.wait()
        self.unpack.run(stream)

    def _run_phases(self, stream, timing):
        """A rehearsed rank (LoopbackComm) under bench timing: the same
        launches, with HIP events around each phase (pack, the slot writes
        of the arriving bytes, local copies, unpack) -- on one stream, so the
        phases run back to back instead of overlapping the transfers."""
        import torch

        cur = torch.cuda.current_stream()

        def timed(name, fn):
            e0, e1 = timing.events()
            e0.record(cur)
            fn()
            e1.record(cur)
            timing.add(("rechunk", 0, name), e0, e1)

        pending = []
        for pack, sends, recvs in self.slices:
            timed("pack", lambda: pack.run(stream))
            timed("slot_writes", lambda: pending.append(self.ctx.comm.exchange(sends, recvs)))
        timed("local_copies", lambda: self.local.run(stream))
        for p in pending:
            p.wait()
        timed("unpack", lambda: self.unpack.run(stream))


SUM_ROPS = {"sum", "nansum", "count", "count_nonnan"}


class ScatterCombine:
    """The cross-rank combine of a sum-only reduction whose output blocks
    have SEVERAL owners, as one RCCL reduce-scatter instead of an all-reduce
    of every block's partials (each rank finishes only its own blocks, so it
    needs only their sums).

    The SoA partials ([field][group][kept], group = output block) are
    scattered by one box copy (cubed_copy_boxes) into owner-major order, [rank][field]
    [slot][kept] with ``L`` slots per rank (the most blocks any rank owns;
    unused slots stay zero), and ``reduce_scatter`` leaves each rank the
    summed [field][slot][kept] of its own blocks -- straight in the finish's
    SoA buffer, whose host-count fields (mean's n) are filled once here.
    The finish runs over this rank's blocks only (padding slots write to a
    discard buffer).  Payload per rank: (W-1)/W of W*L*kept*8 B per field
    on a ring, against 2(W-1)/W of the whole G*kept*8 for the all-reduce.

    Used when every field sums (SUM_ROPS), the plain COUNT fields' global
    values are known on the host (geometry: the same on every rank) and the
    summed fields are one contiguous run of one accumulator dtype.  When the
    partials come from a streaming program with ONE summed field and the
    owners are block-cyclic, the stream kernel writes the owner-major order
    itself (``use_direct``, CUBED_MODE_OWNER_MAJOR) and the permute goes."""

    def __init__(self, ctx, fused, rows, group_owner, nf, mko, f0, f1, acc_int, host_counts, discard, src):
        import dataclasses

        import torch

        W, rank = ctx.world, ctx.rank
        G = len(group_owner)
        per = [[g for g in range(G) if group_owner[g] == q] for q in range(W)]
        L = max(1, max(len(p) for p in per))
        pos = {g: i for q in range(W) for i, g in enumerate(per[q])}
        nfr = f1 - f0
        self.ctx, self.fused = ctx, fused
        self.G, self.L, self.mko, self.nf, self.f0, self.f1 = G, L, mko, nf, f0, f1
        self.mine = per[rank]
        dt = torch.int64 if acc_int else torch.float64
        dst = [(group_owner[g] * nfr + fr) * L + pos[g] for fr in range(nfr) for g in range(G)]
        self.dst = torch.tensor(dst, dtype=torch.int64, device=ctx.device)  # (unpermute: tests)
        self.perm = torch.zeros(W * nfr * L * mko, dtype=dt, device=ctx.device)
        # the owner-major scatter: one row of mko 8-B words per (field, group),
        # one cubed_copy_boxes launch (src: the [field][group][kept] partials)
        pb, rb = self.perm.data_ptr(), mko * 8
        self.permute = CopyLaunch([Box(src + ((f0 + fr) * G + g) * rb, pb + dst[fr * G + g] * rb, [mko], [1], [1])
                                   for fr in range(nfr) for g in range(G)], 8, ctx.device)
        self.fin = torch.zeros(max(nf * L * mko, 2), dtype=torch.int64, device=ctx.device).view(torch.uint8)
        self.fin_red = self.fin[f0 * L * mko * 8:f1 * L * mko * 8].view(dt)
        for f, counts in (host_counts or {}).items():
            v = self.fin[f * L * mko * 8:(f + 1) * L * mko * 8].view(torch.int64).view(L, mko)
            vals = [int(counts[g]) for g in self.mine] + [1] * (L - len(self.mine))
            v.copy_(torch.tensor(vals, dtype=torch.int64, device=ctx.device)[:, None].expand(L, mko))
        self.finish_here = bool(self.mine)
        if self.finish_here:
            tmpl = rows.rows[self.mine[0]]
            pad = dataclasses.replace(tmpl, obases=[discard] * len(tmpl.obases))
            fin_rows = [rows.rows[g] for g in self.mine] + [pad] * (L - len(self.mine))
            self.table = dataclasses.replace(rows, rows=fin_rows).table(ctx.device)

    @staticmethod
    def plan(rops, counts_known, acc_int):
        """(f0, f1) of the summed fields when the reduce-scatter form applies
        (``counts_known``: the host knows every plain COUNT field's value)."""
        if not all(r in SUM_ROPS for r in rops) or ("count" in rops and not counts_known):
            return None
        red = [f for f, r in enumerate(rops) if r != "count"]
        if not red:
            return None
        if red != list(range(red[0], red[-1] + 1)) or len({bool(acc_int[f]) for f in red}) != 1:
            return None
        return red[0], red[-1] + 1

    def direct_ok(self, fused, owners, n):
        """True when the partials kernel can write the owner-major order
        itself (CUBED_MODE_OWNER_MAJOR): a streaming partials program with ONE
        summed field (every COUNT host-filled), block-cyclic group owners (g
        mod W, so a group's slot is g // W), three free const slots and the
        W x L x mko slots inside the SoA block (nf x n words)."""
        from ...lowering import MODE_HOST_COUNT, MODE_PARTIALS, MODE_STREAM

        P, W = fused.prog, self.ctx.world
        need = MODE_STREAM | MODE_PARTIALS | MODE_HOST_COUNT
        return (P.mode & need) == need and self.f1 - self.f0 == 1 and \
            sum(P.field_rop[f] != ROP_COUNT for f in range(P.nfields)) == 1 and \
            all(o == g % W for g, o in enumerate(owners)) and \
            consts_used(P) <= nat.MAX_CONSTS - 3 and W * self.L * self.mko <= self.nf * n

    def use_direct(self, fused, gsoa):
        """The stream kernel writes field f0's partials owner-major into the
        start of its SoA block (``gsoa``): that block is the reduce-scatter's
        input and the box-copy permute goes."""
        from ...lowering import MODE_OWNER_MAJOR

        P, W = fused.prog, self.ctx.world
        P.mode |= MODE_OWNER_MAJOR
        P.consts[nat.MAX_CONSTS - 3].i = self.mko
        P.consts[nat.MAX_CONSTS - 2].i = W
        P.consts[nat.MAX_CONSTS - 1].i = self.L
        fused.reprogram()
        self.perm = gsoa[: W * self.L * self.mko * 8].view(self.perm.dtype)
        self.perm.zero_()  # padding slots (groups >= G) are never written
        self.permute = None

    def run(self, stream):
        """The partials at ``src`` ([field][group][kept], 8-B words) to every
        rank's owned blocks, then the finish."""
        if self.permute is not None:
            self.permute.run(stream)
        self.ctx.comm.reduce_scatter_sum(self.fin_red, self.perm)
        if self.finish_here:
            fused_finish(self.fused, self.table, self.L, self.mko, self.fin, stream)

    def unpermute(self, perm_sum):
        """[field][group][kept] from an owner-major buffer (tests: the sum of
        every rank's recorded reduce-scatter input)."""
        return perm_sum.view(-1, self.mko)[self.dst].view(self.f1 - self.f0, self.G, self.mko)



class BlockCount:
    """A plain COUNT field (mean's n) holds one value per output block --
    every kept element of a block counts the same rows -- so only that value
    crosses the ranks (8 B per block instead of 8 B per element).  Two
    cubed_copy_boxes launches: the first word of every block into a compact
    vector before the collective, and that vector back over the block's
    words after it."""

    def __init__(self, view, mk, device):
        import torch

        self.nblk = view.numel() // mk
        self.view = view
        self.compact = torch.empty(self.nblk, dtype=view.dtype, device=device)
        src, dst = view.data_ptr(), self.compact.data_ptr()
        self.gather = CopyLaunch([Box(src, dst, [self.nblk], [mk], [1])], 8, device)
        self.spread = CopyLaunch([Box(dst, src, [self.nblk, mk], [1, 0], [mk, 1])], 8, device)


def _sum_fields(ctx, fields, root, stream):
    """The SUM combine of a sum-only reduction's partial fields: (view,
    BlockCount or None) per field, reduced to ``root`` (or all-reduced)."""
    comm = ctx.comm
    for v, bc in fields:
        if bc is not None:
            bc.gather.run(stream)
            v = bc.compact
        if root is not None:
            comm.reduce_sum(v, root)
        else:
            comm.all_reduce_sum(v)
        if bc is not None and (root is None or ctx.rank == root):
            bc.spread.run(stream)


class PartialsLaunch:
    """Cross-rank combine + epilogue of a reduction chain run in partials
    mode (the FusedLaunch before it leaves SoA partials in its workspace)."""

    def __init__(self, ctx, fused, rops: List[str], acc_int: List[bool], owners: List[int], host_count=None,
                 discard=0):
        import torch

        self.ctx = ctx
        self.fused = fused
        self.nf = len(rops)
        self.n = fused.ntasks * fused.max_kept
        self.sum_only = all(r in SUM_ROPS for r in rops)
        self.acc_int = acc_int
        # host_count (CUBED_MODE_HOST_COUNT, sum-only chains): the kernel
        # leaves the COUNT fields alone; they hold the global count (the whole
        # reduced extent), filled here once -- one collective fewer per step
        self.host_count = [r == "count" and host_count is not None for r in rops]
        if host_count is not None:
            assert self.sum_only and fused.prog.mode & 128
            for f in range(self.nf):
                if self.host_count[f]:
                    self.field_view(f).fill_(int(host_count))
        # a plain COUNT field (mean's n) holds one value per output block --
        # every kept element of a task counts the same rows -- so only that
        # value crosses the ranks (8 B per block instead of 8 B per element:
        # quad-means' RCCL payload halves, 16.6 -> 8.3 MB per rank)
        self.uniform = [r == "count" for r in rops]
        group_owner = list(owners)
        owners = sorted(set(owners))
        # one owner for every output block (e.g. a full reduction): RCCL reduce
        # to it; otherwise reduce-scatter in owner-major order (ScatterCombine)
        # or, where that does not apply, all-reduce; every rank finishes its
        # own blocks
        self.root = owners[0] if len(owners) == 1 else None
        self.finish_here = ctx.rank in owners
        self.scatter = None
        fr = ScatterCombine.plan(rops, host_count is not None, acc_int) if self.root is None and SCATTER else None
        if fr is not None and fused.ntasks == len(group_owner):
            self.scatter = ScatterCombine(
                ctx, fused, fused.layout, group_owner, self.nf, fused.max_kept, fr[0], fr[1], acc_int[fr[0]],
                {f: [int(host_count)] * len(group_owner) for f, r in enumerate(rops) if r == "count"},
                discard, fused.ws.data_ptr())
            self.finish_here = self.scatter.finish_here
            if OWNER_MAJOR and self.scatter.direct_ok(fused, group_owner, fused.ntasks * fused.max_kept):
                self.scatter.use_direct(fused, fused.ws)
        if self.sum_only and self.scatter is None:
            mk = fused.max_kept
            self.sum_views = [(self.field_view(f), BlockCount(self.field_view(f), mk, ctx.device)
                               if self.uniform[f] and mk > 1 else None)
                              for f in range(self.nf) if not self.host_count[f]]
        if not self.sum_only:
            self.gathered = torch.empty(ctx.world * self.nf * self.n * 8, dtype=torch.uint8,
                                        device=ctx.device)

    def soa(self):
        return self.fused.ws[: self.nf * self.n * 8]

    def field_view(self, f):
        import torch

        raw = self.fused.ws[f * self.n * 8:(f + 1) * self.n * 8]
        return raw.view(torch.int64 if self.acc_int[f] else torch.float64)

    def run(self, stream):
        comm = self.ctx.comm
        L = nat.lib()
        if self.scatter is not None:
            self.scatter.run(stream)
            return
        if self.sum_only:
            _sum_fields(self.ctx, self.sum_views, self.root, stream)
        else:
            comm.all_gather(self.gathered, self.soa())
            if self.finish_here:
                nat.check(L.cubed_combine_partials(self.fused.prog, self.fused.d_prog.data_ptr(),
                                                   self.gathered.data_ptr(), comm.world, self.n,
                                                   self.fused.ws.data_ptr(), stream),
                          "cubed_combine_partials")
        if self.finish_here:
            fused_finish(self.fused, self.fused.table, self.fused.ntasks, self.fused.max_kept,
                         self.fused.ws, stream)


def fused_finish(F, table, ntasks, max_kept, partials, stream):
    """The epilogue over combined SoA partials of ``F``'s program: the JIT
    module's specialised finish when the program was compiled, else the
    interpreted kernel (CUBED_AMD_JIT=0)."""
    L = nat.lib()
    if F.handle is not None:
        nat.check(L.cubed_fused_finish_compiled(F.handle, F.prog, table.data_ptr(), ntasks, max_kept,
                                                partials.data_ptr(), stream), "cubed_fused_finish_compiled")
    else:
        nat.check(L.cubed_fused_finish(F.prog, F.d_prog.data_ptr(), table.data_ptr(), ntasks, max_kept,
                                       partials.data_ptr(), stream), "cubed_fused_finish")


def gather_distributed(arr: DeviceArray) -> np.ndarray:
    """Assemble a block-cyclically stored array on every rank: each rank
    broadcasts its slab (all its chunks), then chunks are decoded on the
    host.  Used to return compute() results, not on the hot path."""
    import itertools

    import torch

    comm = arr.comm
    out = np.empty(arr.shape, dtype=arr.dtype)
    if arr.size == 0:
        return out
    torch.cuda.synchronize(arr.device)
    for r in range(arr.world):
        nslots = (arr.nchunks - r + arr.world - 1) // arr.world if arr.nchunks > r else 0
        if nslots == 0:
            continue
        for f in arr.fields:
            nb = nslots * arr.slot_bytes(f)
            if r == arr.rank:
                buf = arr.slabs[f][:nb].clone()
            else:
                buf = torch.empty(nb, dtype=torch.uint8, device=arr.device)
            comm.broadcast(buf, r)
            host = buf.cpu().numpy()
            dt = arr.field_dtype(f)
            for coords in itertools.product(*[range(n) for n in arr.numblocks]):
                if arr.chunk_offset(coords) % arr.world != r:
                    continue
                slot = arr.chunk_offset(coords) // arr.world
                ext = arr.chunk_extent(coords)
                start = slot * arr.slot_bytes(f)
                vals = host[start:start + math.prod(ext) * dt.itemsize].view(dt).reshape(ext)
                sl = tuple(slice(s, s + e) for s, e in zip(arr.chunk_start(coords), ext))
                if f is None:
                    out[sl] = vals
                else:
                    out[f][sl] = vals
    return out


class DistPiecesLaunch:
    """A reduction whose tasks are cut into pieces at source-chunk boundaries
    (index regions, rechunk read-through) run where the pieces' chunks live:
    each rank reduces its pieces of EVERY output group in partials mode,
    folds them per group (cubed_combine_groups), the per-group partials are
    combined over RCCL, and the owners of the outputs run the epilogue
    (cubed_fused_finish over one row per group)."""

    def __init__(self, ctx, fused, group_start, group_table, max_kept_out, rops, acc_int, owners,
                 soa_direct=False, host_counts=None, group_layout=None, discard=0, group_counts=None):
        import torch

        self.ctx = ctx
        self.fused = fused
        self.ngroups = len(group_start) - 1
        self.gs = torch.from_numpy(np.ascontiguousarray(group_start, dtype=np.int64)).to(ctx.device)
        self.group_table = group_table
        self.mko = max_kept_out
        self.nf = len(rops)
        self.n = self.ngroups * max_kept_out
        # soa_direct: the fused launch streamed this rank's one row per group as
        # merged kept runs; its SoA partials [f][task][kept] are byte for byte
        # the per-group partials [f][group][kept], so no combine_groups pass
        self.soa_direct = soa_direct
        if soa_direct:
            assert fused.ntasks * fused.max_kept == self.n
            self.gsoa = fused.ws
        else:
            self.gsoa = torch.empty(max(self.nf * self.n * 8, 16), dtype=torch.uint8, device=ctx.device)
        # a plain COUNT field (mean's n) is uniform over the kept elements of a
        # group: one int64 per group crosses the ranks (as in PartialsLaunch)
        self.uniform = [r == "count" for r in rops]
        self.sum_only = all(r in SUM_ROPS for r in rops)
        self.acc_int = acc_int
        # host_counts (CUBED_MODE_HOST_COUNT, soa_direct only): the kernel leaves
        # the COUNT fields alone; they hold each group's global count, filled
        # here once, and never cross the ranks
        self.host_count = [r == "count" and host_counts is not None for r in rops]
        if host_counts is not None:
            assert soa_direct and len(host_counts) == self.ngroups
            hc = torch.as_tensor(np.asarray(host_counts, dtype=np.int64), device=ctx.device)
            for f in range(self.nf):
                if self.host_count[f]:
                    self.field_view(f).view(self.ngroups, self.mko).copy_(hc[:, None].expand(self.ngroups, self.mko))
        # owners: the rank finishing each GROUP (one entry per group; a key
        # cut along a kept dim has several groups, all owned by its owner)
        if len(owners) != self.ngroups:
            raise ValueError(f"{len(owners)} owners for {self.ngroups} groups")
        uniq = sorted(set(owners))
        self.root = uniq[0] if len(uniq) == 1 else None
        self.finish_here = ctx.rank in uniq
        self.scatter = None
        # group_counts: every group's global element count (geometry, all ranks)
        fr = ScatterCombine.plan(rops, group_counts is not None, acc_int) \
            if self.root is None and group_layout is not None and SCATTER else None
        if fr is not None:
            self.scatter = ScatterCombine(
                ctx, fused, group_layout, list(owners), self.nf, max_kept_out, fr[0], fr[1], acc_int[fr[0]],
                {f: list(group_counts) for f, r in enumerate(rops) if r == "count"}, discard,
                self.gsoa.data_ptr())
            self.finish_here = self.scatter.finish_here
            if OWNER_MAJOR and soa_direct and self.scatter.direct_ok(fused, owners, self.n):
                self.scatter.use_direct(fused, self.gsoa)
        if self.sum_only and self.scatter is None:
            mk = self.mko
            self.sum_views = [(self.field_view(f), BlockCount(self.field_view(f), mk, ctx.device)
                               if self.uniform[f] and mk > 1 else None)
                              for f in range(self.nf) if not self.host_count[f]]
        if not self.sum_only:
            self.gathered = torch.empty(ctx.world * self.nf * self.n * 8, dtype=torch.uint8, device=ctx.device)

    def field_view(self, f):
        import torch

        raw = self.gsoa[f * self.n * 8:(f + 1) * self.n * 8]
        return raw.view(torch.int64 if self.acc_int[f] else torch.float64)

    def run(self, stream):
        F = self.fused
        L = nat.lib()
        F.run(stream)
        if not self.soa_direct:
            nat.check(L.cubed_combine_groups(F.prog, F.d_prog.data_ptr(), F.table.data_ptr(), F.ntasks,
                                             F.max_kept, F.ws.data_ptr(), self.gs.data_ptr(), self.ngroups,
                                             self.mko, self.gsoa.data_ptr(), stream), "cubed_combine_groups")
        comm = self.ctx.comm
        if self.scatter is not None:
            self.scatter.run(stream)
            return
        if self.sum_only:
            _sum_fields(self.ctx, self.sum_views, self.root, stream)
        else:
            comm.all_gather(self.gathered, self.gsoa[: self.nf * self.n * 8])
            if self.finish_here:
                nat.check(L.cubed_combine_partials(F.prog, F.d_prog.data_ptr(), self.gathered.data_ptr(),
                                                   comm.world, self.n, self.gsoa.data_ptr(), stream),
                          "cubed_combine_partials")
        if self.finish_here:
            fused_finish(F, self.group_table, self.ngroups, self.mko, self.gsoa, stream)


# k block of the packed GEMM images (bf16: 64-deep tiles of 32 KiB per
# 256-row panel; f32: 16-deep steps of 16 KiB), csrc/gemm_bf16_w4p.h / _f32_
KBLOCK = {2: (64, 32768), 4: (16, 16384)}
LINK_GBPS = 153.0  # ASSUMED xGMI rate per link and direction (MI355X_MICROARCH.md); rehearsal predictions only


class DistGemmLaunch:
    """A matmul's chunk products + k-sum (linear_algebra_functions.py:35-78)
    on W ranks, when the block-cyclic ownership gives every k chunk q of A
    ONE rank (q mod W: A's chunk columns nk % W == 0) and every chunk column j
    of C and of B one rank (j mod W: nj % W == 0) -- config 5's 8 x 8 grid at
    W = 1, 2, 4, 8.  Rank r computes its C columns from ALL of A and its own
    B columns, so A is the only operand that moves:

    1. halo: the owner of chunk q+1 sends the first h_q columns of its A
       chunks (the part of the k block straddling the q / q+1 edge) to the
       owner of q (h_q < one k block; one small box copy + p2p);
    2. pack A: each rank packs the k blocks starting in its own chunks into
       ONE k-major image of the whole packed A (cubed_gemm_dist_pack_a);
    3. exchange: each rank sends its blocks (one contiguous run per owned k
       chunk) to every peer, received in place into the same image (grouped
       point-to-point: every peer pair on its own xGMI link, no pack and no
       unpack); B's pack (its own chunks, cubed_gemm_dist_pack_b) runs
       meanwhile;
    4. GEMM: the single-GPU packed kernel over the rank's C columns
       (cubed_gemm_dist_gemm).

    The image holds exactly the single-GPU packed A (same blocks, same
    order of k), so every element is the same f32 chain over K: the result
    is bit-identical to one GPU's."""

    def __init__(self, ctx, A, B, F, ti, nk, nj, in_code, out_code, isz):
        import torch

        from ... import ir

        W, r = ctx.world, ctx.rank
        self.ctx = ctx
        self.in_code, self.out_code = in_code, out_code
        T, blk = KBLOCK[isz]
        kw = [A.chunk_extent((0, q))[1] for q in range(nk)]
        ks = [sum(kw[:q]) for q in range(nk + 1)]
        K = ks[-1]
        M = A.shape[0]
        rows = [A.chunk_extent((i, 0))[0] for i in range(ti)]
        TM = -(-M // 256)
        KTL = -(-K // T)
        self.K, self.M, self.TM, self.KTL, self.blk = K, M, TM, KTL, blk
        L = nat.lib()
        self.image_bytes = int(L.cubed_gemm_dist_image_bytes(M, K, in_code))
        assert self.image_bytes == KTL * TM * blk
        dev = ctx.device
        self.image = torch.empty(self.image_bytes, dtype=torch.uint8, device=dev)
        ib = self.image.data_ptr()
        # k blocks packed by the owner of chunk q: those starting inside it
        self.ranges = [(-(-ks[q] // T), min(KTL, -(-ks[q + 1] // T))) for q in range(nk)]
        self.halo_w = [min(K, self.ranges[q][1] * T) - ks[q + 1] for q in range(nk)]
        self.owned = [q for q in range(nk) if q % W == r]
        # -- halo buffers: [M][h_q] per owned q whose last block reaches into q+1
        self.halo = {}
        sends, recvs, hboxes = [], [], []
        off = 0
        need = {q: M * self.halo_w[q] * isz for q in self.owned if self.halo_w[q] > 0}
        self.halo_buf = torch.empty(max(sum(need.values()), 16), dtype=torch.uint8, device=dev)
        for q in self.owned:
            if self.halo_w[q] > 0:
                self.halo[q] = (self.halo_buf.data_ptr() + off, off)
                off += need[q]
        out_halo = [q for q in range(nk - 1) if (q + 1) % W == r and self.halo_w[q] > 0]
        send_bytes = sum(M * self.halo_w[q] * isz for q in out_halo)
        self.halo_send = torch.empty(max(send_bytes, 16), dtype=torch.uint8, device=dev)
        so = 0
        for q in out_halo:
            h = self.halo_w[q]
            base = self.halo_send.data_ptr() + so
            row0 = 0
            for i in range(ti):
                src = A.chunk_addr((i, q + 1))
                hboxes.append(Box(src, base + row0 * h * isz, [rows[i], h], [kw[q + 1], 1], [h, 1]))
                row0 += rows[i]
            sends.append((self.halo_send[so:so + M * h * isz], q % W))
            so += M * h * isz
        for q in self.owned:
            if q in self.halo:
                o = self.halo[q][1]
                recvs.append((self.halo_buf[o:o + need[q]], (q + 1) % W))
        self.halo_pack = CopyLaunch(hboxes, isz, dev)
        self.halo_sends, self.halo_recvs = sends, recvs
        # -- A pack tables: task I = chunk row I, segment q = A(I, q) here, the
        # halo of q+1 where q is ours, else absent (0)
        nat_tasks = np.zeros(ti, dtype=nat.CHAIN_DTYPE)
        nat_segs = np.zeros(ti * nk, dtype=nat.SEG_DTYPE)
        for i in range(ti):
            row0 = sum(rows[:i])
            for q in range(nk):
                a, lda = 0, kw[q]
                if q % W == r:
                    a = A.chunk_addr((i, q))
                elif q >= 1 and (q - 1) in self.halo:
                    h = self.halo_w[q - 1]
                    a, lda = self.halo[q - 1][0] + row0 * h * isz, h
                nat_segs[i * nk + q] = (a, 0, kw[q], lda, 1, 0)
            nat_tasks[i] = (0, rows[i], 1, 1, i * nk, nk, K, 0)
        self.a_tasks, self.a_segs = nat_tasks, nat_segs
        self.d_a_tasks = torch.from_numpy(nat_tasks.view(np.uint8).copy()).to(dev)
        self.d_a_segs = torch.from_numpy(nat_segs.view(np.uint8).copy()).to(dev)
        # -- the image's exchange: every owned range to every peer, in place
        rs, rr = [], []
        self.bytes_out = 0
        for q in range(nk):
            lo, hi = self.ranges[q]
            view = self.image[lo * TM * blk:hi * TM * blk]
            if q % W == r:
                for p in range(W):
                    if p != r:
                        rs.append((view, p))
                self.bytes_out += (W - 1) * view.numel()
            else:
                rr.append((view, q % W))
        self.region_sends, self.region_recvs = rs, rr
        self.bytes_in = sum(v.numel() for v, _ in rr)
        self.own_bytes = {p: sum((self.ranges[q][1] - self.ranges[q][0]) * TM * blk
                                 for q in range(nk) if q % W == p) for p in range(W)}
        # -- the rank's C grid: rows I, its chunk columns j = r, r + W, ...
        cols = [j for j in range(nj) if j % W == r]
        self.ti, self.tj = ti, len(cols)
        tasks = np.zeros(ti * len(cols), dtype=nat.CHAIN_DTYPE)
        segs = np.zeros(ti * len(cols) * nk, dtype=nat.SEG_DTYPE)
        self.flops = 0.0
        for i in range(ti):
            for jl, j in enumerate(cols):
                t = i * len(cols) + jl
                key = (i, j) if F.ndim == 2 else (i, 0, j)
                m, n = F.chunk_extent(key)[0], F.chunk_extent(key)[-1]
                for q in range(nk):
                    a = A.chunk_addr((i, q)) if q % W == r else 0
                    segs[t * nk + q] = (a, B.chunk_addr((q, j)), kw[q], kw[q], n, 0)
                tasks[t] = (F.chunk_addr(key), m, n, n, t * nk, nk, K, 0)
                self.flops += 2.0 * m * n * K
        self.tasks, self.segs = tasks, segs
        self.b_bytes = int(L.cubed_gemm_dist_b_bytes(tasks.ctypes.data, ti, len(cols), segs.ctypes.data,
                                                     len(segs), in_code, out_code))
        if self.b_bytes < 0:
            nat.check(int(self.b_bytes), "cubed_gemm_dist_b_bytes")
        self.bws = torch.empty(max(self.b_bytes, 256), dtype=torch.uint8, device=dev)
        self.d_tasks = torch.from_numpy(tasks.view(np.uint8).copy()).to(dev)
        self.d_segs = torch.from_numpy(segs.view(np.uint8).copy()).to(dev)
        self.collective = True
        self.phase_ms = {}

    def _pack_a(self, stream):
        L = nat.lib()
        for q in self.owned:
            lo, hi = self.ranges[q]
            nat.check(L.cubed_gemm_dist_pack_a(self.a_tasks.ctypes.data, self.d_a_tasks.data_ptr(), self.ti,
                                               self.a_segs.ctypes.data, self.d_a_segs.data_ptr(),
                                               len(self.a_segs), self.in_code, lo, hi, self.image.data_ptr(),
                                               self.image_bytes, stream), "cubed_gemm_dist_pack_a")

    def _pack_b(self, stream):
        nat.check(nat.lib().cubed_gemm_dist_pack_b(self.tasks.ctypes.data, self.d_tasks.data_ptr(), self.ti,
                                                   self.tj, self.segs.ctypes.data, self.d_segs.data_ptr(),
                                                   len(self.segs), self.in_code, self.out_code,
                                                   self.bws.data_ptr(), self.b_bytes, stream),
                  "cubed_gemm_dist_pack_b")

    def _gemm(self, stream):
        nat.check(nat.lib().cubed_gemm_dist_gemm(self.tasks.ctypes.data, self.d_tasks.data_ptr(), self.ti, self.tj,
                                                 self.segs.ctypes.data, len(self.segs), self.in_code,
                                                 self.out_code, self.image.data_ptr(), self.image_bytes,
                                                 self.bws.data_ptr(), self.b_bytes, stream),
                  "cubed_gemm_dist_gemm")

    def run(self, stream):
        timing = getattr(self.ctx, "timing", None)
        if timing is not None and getattr(self.ctx.comm, "backend", None) == "loopback":
            return self._run_phases(stream, timing)
        comm = self.ctx.comm
        self.halo_pack.run(stream)
        comm.exchange(self.halo_sends, self.halo_recvs).wait()
        self._pack_a(stream)
        pending = comm.exchange(self.region_sends, self.region_recvs)
        self._pack_b(stream)  # overlaps the transfers
        pending.wait()
        self._gemm(stream)

    def _run_phases(self, stream, timing):
        """A rehearsed rank under bench timing: the same launches with HIP
        events around each phase, back to back on one stream."""
        import torch

        cur = torch.cuda.current_stream()
        comm = self.ctx.comm

        def timed(name, fn):
            e0, e1 = timing.events()
            e0.record(cur)
            fn()
            e1.record(cur)
            timing.add(("matmul", 0, name), e0, e1)

        timed("halo", lambda: (self.halo_pack.run(stream), comm.exchange(self.halo_sends, self.halo_recvs).wait()))
        timed("pack_a", lambda: self._pack_a(stream))
        timed("slot_writes", lambda: comm.exchange(self.region_sends, self.region_recvs).wait())
        timed("pack_b", lambda: self._pack_b(stream))
        timed("gemm", lambda: self._gemm(stream))

    def predicted_xfer_ms(self, gbps=LINK_GBPS):
        """The exchange at ``gbps`` per link and direction, every peer pair
        on its own link: the busiest link carries one rank's whole blocks."""
        return max(self.own_bytes.values()) / (gbps * 1e9) * 1e3


def dist_gemm_plan(ex, chain, F):
    """(A, B, ti, nk, nj) when the chain runs as a DistGemmLaunch on ex's
    ranks, else None (the fetch path runs it)."""
    from ... import ir
    from ...gemm_chains import K_AXIS
    from ...storage import DeviceArray

    W = ex.world
    G = chain.gemm_target
    nk = G.numblocks[K_AXIS]
    ti, nj = F.numblocks[0], F.numblocks[-1]
    args = chain.gemm_spec.block_function(("out", 0, 0, 0))
    A = ex.device_source(chain.gemm_spec.reads_map[args[0][0]].array)
    B = ex.device_source(chain.gemm_spec.reads_map[args[1][0]].array)
    if not all(isinstance(x, DeviceArray) and x.world == W and x.ndim == 2 for x in (A, B)) or F.world != W:
        return None
    if A.dtype != B.dtype or A.dtype not in (np.dtype(np.float32), ir.bfloat16):
        return None
    if A.numblocks != (ti, nk) or B.numblocks != (nk, nj) or nk % W or nj % W:
        return None
    for i in (0, ti - 1):
        for k in (0, nk - 1):
            for j in (0, nj - 1):
                a, b = chain.gemm_spec.block_function(("out", i, k, j))[:2]
                if tuple(a[1:]) != (i, k) or tuple(b[1:]) != (k, j):
                    return None
    T, _ = KBLOCK[A.dtype.itemsize]
    kw = [A.chunk_extent((0, q))[1] for q in range(nk)]
    if min(kw) < T or any(w % (16 // A.dtype.itemsize) for w in kw):
        return None
    # the packed kernels' own geometry rules (tile vs chunk widths, row
    # alignment), asked of the native check on the rank's C grid with zero
    # addresses: the same answer on every rank
    cols = [j for j in range(nj) if j % W == ex.rank]
    K = sum(kw)
    tasks = np.zeros(ti * len(cols), dtype=nat.CHAIN_DTYPE)
    segs = np.zeros(ti * len(cols) * nk, dtype=nat.SEG_DTYPE)
    for i in range(ti):
        for jl, j in enumerate(cols):
            t = i * len(cols) + jl
            key = (i, j) if F.ndim == 2 else (i, 0, j)
            m, n = F.chunk_extent(key)[0], F.chunk_extent(key)[-1]
            for q in range(nk):
                segs[t * nk + q] = (0, 0, kw[q], kw[q], n, 0)
            tasks[t] = (0, m, n, n, t * nk, nk, K, 0)
    code = ir.dtype_code(A.dtype)
    if nat.lib().cubed_gemm_dist_b_bytes(tasks.ctypes.data, ti, len(cols), segs.ctypes.data, len(segs), code,
                                         ir.dtype_code(F.dtype)) < 0:
        return None
    return A, B, ti, nk, nj
