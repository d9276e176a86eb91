"""Inter-GPU communication for the multi-GPU executor.

The reference has no collective layer: every byte between tasks moves
through shared Zarr storage (cubed/core/plan.py:44-48).  On one
MI355X node the executor runs one process per GPU and moves chunks over
xGMI with RCCL (torch.distributed's "nccl" backend is RCCL on ROCm):

* ``exchange`` -- the piece transfers of a rechunk: grouped point-to-point
  sends / receives (``batch_isend_irecv``, one RCCL group), so pieces land
  straight in their target chunk slots; started on torch's current stream
  and waited for by it (``Pending.wait``), so kernels queued in between
  (the next slice's pack, the local pieces) overlap the transfers;
* ``all_to_all`` -- whole-chunk fetches of pipelines whose tasks read chunks
  owned by another rank (one ``all_to_all_single`` of a packed byte buffer,
  issued on torch's current stream, so it is ordered with the pack kernel
  before it);
* ``reduce`` / ``all_reduce`` / ``reduce_scatter`` -- the final combine
  round of a reduction (SUM of f64 totals / i64 counts): to the one owner of
  the output, or, with several owners, a reduce-scatter of the partials in
  owner-major order (dist.ScatterCombine);
* ``all_gather`` -- partials whose combine RCCL cannot express with numpy's
  semantics (max/min with NaN, prod, any/all), folded afterwards by
  ``cubed_combine_partials`` in rank order;
* ``broadcast`` -- assembling a computed result on every rank.

With the ``gloo`` backend (CPU tests, or several ranks sharing one GPU in a
test) device tensors are staged through host memory; the data path is
otherwise identical.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence


class Comm:
    """A process group plus the backend-specific tensor plumbing."""

    def __init__(self, group=None):
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("Comm needs an initialised torch.distributed process group")
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = str(dist.get_backend(group)).lower()
        self.staged = self.backend == "gloo"
        # control-plane agreements (all_ok) go over a host-side gloo group:
        # a device all-reduce + .item() would wait for every kernel queued on
        # the stream, serialising the first step of each new plan across the
        # ranks.  One per process and world group (control_group).
        self.ctrl = control_group(dist) if not self.staged and group is None else None

    # -- helpers --------------------------------------------------------------
    def _stage(self, t):
        if self.staged and t.device.type != "cpu":
            return t.cpu(), True
        return t, False

    def _unstage(self, host, dev, staged):
        if staged:
            dev.copy_(host)

    def barrier(self):
        self.dist.barrier(group=self.group)

    # -- collectives ------------------------------------------------------------
    def all_to_all(self, recv, send, recv_splits: Sequence[int], send_splits: Sequence[int]):
        """Byte exchange: rank r's ``send[sum(send_splits[:j]) : +send_splits[j]]``
        lands in rank j's ``recv`` at ``sum(recv_splits[:r])``."""
        rs, ss = list(map(int, recv_splits)), list(map(int, send_splits))
        send, recv = send[:sum(ss)], recv[:sum(rs)]  # buffers may carry padding
        s, _ = self._stage(send)
        r, staged = self._stage(recv)
        self.dist.all_to_all_single(r, s, rs, ss, group=self.group)
        self._unstage(r, recv, staged)

    def exchange(self, sends, recvs) -> "Pending":
        """Start grouped point-to-point transfers: ``sends`` / ``recvs`` are
        (byte tensor, peer rank) lists; per peer, both ends list their
        transfers in the same order.  Returns a handle whose ``wait()``
        orders the current stream (RCCL) or the host (gloo) after them."""
        dist = self.dist
        ops, fixups = [], []
        for t, peer in sends:
            h, _ = self._stage(t)
            ops.append(dist.P2POp(dist.isend, h, self._global(peer), group=self.group))
        for t, peer in recvs:
            if self.staged and t.device.type != "cpu":
                h = t.new_empty(t.shape, device="cpu")
                fixups.append((h, t))
            else:
                h = t
            ops.append(dist.P2POp(dist.irecv, h, self._global(peer), group=self.group))
        works = dist.batch_isend_irecv(ops) if ops else []
        return Pending(works, fixups)

    def all_reduce_sum(self, t):
        h, staged = self._stage(t)
        self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM, group=self.group)
        self._unstage(h, t, staged)

    def reduce_scatter_sum(self, out, t):
        """SUM of every rank's ``t`` (world equal parts), rank r keeping part
        r in ``out``.  gloo has no reduce-scatter: all-reduce, keep a part."""
        if self.staged:
            h = t.cpu() if t.device.type != "cpu" else t.clone()
            self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM, group=self.group)
            out.copy_(h.view(self.world, -1)[self.rank])
            return
        self.dist.reduce_scatter_tensor(out, t, op=self.dist.ReduceOp.SUM, group=self.group)

    def reduce_sum(self, t, dst: int):
        h, staged = self._stage(t)
        self.dist.reduce(h, dst=self._global(dst), op=self.dist.ReduceOp.SUM, group=self.group)
        if self.rank == dst:
            self._unstage(h, t, staged)

    def all_gather(self, out, t):
        """``out`` (world * t.numel() elements) receives every rank's ``t`` in
        rank order."""
        h, _ = self._stage(t)
        o, staged = self._stage(out)
        self.dist.all_gather_into_tensor(o, h, group=self.group)
        self._unstage(o, out, staged)

    def broadcast(self, t, src: int):
        h, staged = self._stage(t)
        self.dist.broadcast(h, src=self._global(src), group=self.group)
        if self.rank != src:
            self._unstage(h, t, staged)

    def all_ok(self, ok: bool) -> bool:
        """True iff every rank passes True (plan-time agreement, e.g. whether
        a reduction chain could be fused on all ranks)."""
        import torch

        if self.ctrl is not None:
            t = torch.tensor([1 if ok else 0], dtype=torch.int32)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.ctrl)
            return bool(t.item())
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=collective_device(self.dist, self.group))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
        return bool(t.item())

    def _global(self, r: int) -> int:
        if self.group is None:
            return r
        return self.dist.get_global_rank(self.group, r)


_CTRL: dict = {}


def collective_device(dist, group=None):
    """The device a device-group collective of this process runs on: CPU
    for gloo, else the GPU the process group was bound to at init
    (``init_process_group(device_id=...)``), else the current device -- never
    a bare "cuda" that would put every rank of a launcher that skipped
    ``torch.cuda.set_device`` on GPU 0."""
    import torch

    if str(dist.get_backend(group)).lower() == "gloo":
        return torch.device("cpu")
    pg = group if group is not None else dist.group.WORLD
    bound = getattr(pg, "bound_device_id", None)
    if bound is not None:
        return bound
    return torch.device("cuda", torch.cuda.current_device())


def control_group(dist):
    """The host-side gloo group beside the world group, created ONCE per
    process and world group (``dist.new_group`` is collective and opens its
    own connections, so building one per executor would leak them).  Every
    rank agrees on the result over the world group before using it: if the
    gloo group could not be made on some rank, all ranks fall back to the
    device group (None)."""
    import torch

    world = dist.group.WORLD
    key = id(world)
    if key in _CTRL and _CTRL[key][0] is world:
        return _CTRL[key][1]
    try:
        ctrl = dist.new_group(backend="gloo")
    except Exception:  # noqa: BLE001 -- agreed below
        ctrl = None
    t = torch.tensor([0 if ctrl is None else 1], dtype=torch.int32, device=collective_device(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    if not int(t.item()):
        ctrl = None
    _CTRL.clear()  # a re-initialised world drops the previous one's group
    _CTRL[key] = (world, ctrl)
    return ctrl


class Pending:
    """Transfers started by ``Comm.exchange``."""

    def __init__(self, works, fixups):
        self.works, self.fixups = works, fixups

    def wait(self):
        for w in self.works:
            w.wait()
        for host, dev in self.fixups:
            dev.copy_(host)
        self.works, self.fixups = [], []


class LoopbackMesh:
    """The point-to-point transfers of several ``LoopbackComm`` ranks
    rehearsed in one process, matched by (sender, receiver) pair and issue
    order -- the pairing RCCL's grouped send / receive gives
    (``batch_isend_irecv``: per peer, both ends list their transfers in the
    same order).  Two phases, set by the caller:

    * ``"record"``: every rank's sends are copied into its mailboxes
      ``box[(src, dst)]`` (run every rank once); receives are left as they
      are (their senders may not have run yet);
    * ``"replay"``: a receive from ``src`` takes the next recorded send of
      that pair (a per-pair cursor that wraps, so every step of a rank
      consumes the pair's sequence once) -- the bytes land exactly where the
      peer's RCCL send would put them, so the assembled target of all ranks
      can be checked bit for bit.  A replayed send overwrites its recorded
      bytes (a send cursor per pair), so sends that depend on earlier
      receives (a halo received, then packed into what is sent on) are
      right after one more replay pass.

    Collectives (all-reduce, reduce, reduce-scatter, all-gather, all-to-all,
    broadcast) are matched by their per-rank issue index the same way: the
    record pass keeps every rank's inputs, a replay pass overwrites the
    rank's own input and computes its output from ALL ranks' inputs of that
    index, summed in rank order (RCCL's association on a ring is not
    specified; rank order is the reference association the tests use)."""

    def __init__(self, world: int):
        self.world = world
        self.phase = "record"
        self.box: Dict = {}
        self.cursor: Dict = {}
        self.scursor: Dict = {}
        self.coll: Dict = {}  # rank -> [(kind, {name: tensor or splits})] in issue order
        self.ccursor: Dict = {}
        self.log: List = []  # (src, dst, nbytes) of every recorded send, in issue order

    def bytes_between(self, src: int, dst: int) -> int:
        return sum(t.numel() * t.element_size() for t in self.box.get((src, dst), ()))

    def collective(self, rank: int, kind: str, parts: Dict):
        """Record (record phase) or refresh (replay) rank ``rank``'s inputs of
        its next collective; in replay returns every rank's inputs of that
        index, in rank order (None while recording)."""
        lst = self.coll.setdefault(rank, [])
        if self.phase == "record":
            lst.append((kind, {k: v.detach().clone() if hasattr(v, "detach") else v for k, v in parts.items()}))
            return None
        if not lst:
            raise RuntimeError(f"rank {rank}: no collective recorded")
        i = self.ccursor.get(rank, 0)
        self.ccursor[rank] = (i + 1) % len(lst)
        rk, rec = lst[i]
        if rk != kind:
            raise RuntimeError(f"rank {rank}: collective {i} is {kind}, recorded {rk}")
        for k, v in parts.items():
            if hasattr(v, "detach"):
                if rec[k].shape != v.shape:
                    raise RuntimeError(f"rank {rank}: collective {i} ({kind}) changed shape")
                rec[k].copy_(v)
            else:
                rec[k] = v
        out = []
        for q in range(self.world):
            ql = self.coll.get(q)
            if not ql or len(ql) <= i or ql[i][0] != kind:
                raise RuntimeError(f"rank {q} has no {kind} at index {i} (rank {rank} has)")
            out.append(ql[i][1])
        return out


class LoopbackComm:
    """Rank ``rank`` of a ``world``-rank job, rehearsed in ONE process on one
    GPU: the executor plans, allocates and launches exactly what that rank
    runs (its block-cyclic share of every array, its pieces, its partials),
    and every collective becomes a local device copy of the same bytes on the
    current stream -- the HBM traffic the rank's own side of the collective
    causes, without the xGMI transfer.  Values are NOT combined across ranks
    (there are no other ranks): a rehearsal times the per-rank launch list; a
    test folds the recorded partials of all ``world`` rehearsed ranks itself
    (``record=True`` keeps a copy of every reduce / all-reduce input, in
    issue order, in ``self.records``).

    Point-to-point exchanges (``exchange``) are matched by peer and order:
    with a shared ``LoopbackMesh`` the receives get the bytes the peer rank
    sent (see there); alone, every receive is written from a scratch buffer
    of its size (the write traffic of the arriving bytes, values
    meaningless)."""

    backend = "loopback"
    staged = False

    def __init__(self, rank: int, world: int, record: bool = False, mesh: Optional[LoopbackMesh] = None):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside a world of {world}")
        if mesh is not None and mesh.world != world:
            raise ValueError(f"a mesh of {mesh.world} ranks for a world of {world}")
        self.rank, self.world = rank, world
        self.record = record
        self.records: List = []
        self._scratch = None
        self.mesh = mesh
        self.sent_bytes = 0  # bytes this rank's exchanges sent / received (per call, cumulative)
        self.recv_bytes = 0

    def _copy(self, t):
        """Read + write ``t``'s bytes once (into a scratch buffer)."""
        import torch

        flat = t.reshape(-1)
        if self._scratch is None or self._scratch.numel() < flat.numel() * flat.element_size() \
                or self._scratch.device != flat.device:
            self._scratch = torch.empty(max(flat.numel() * flat.element_size(), 16), dtype=torch.uint8,
                                        device=flat.device)
        self._scratch[:flat.numel() * flat.element_size()].view(flat.dtype).copy_(flat)

    def barrier(self):
        pass

    def all_to_all(self, recv, send, recv_splits, send_splits):
        rs, ss = list(map(int, recv_splits)), list(map(int, send_splits))
        got = self._meshed("all_to_all", send=send[:sum(ss)], splits=ss)
        if got is not None:
            # the segment from rank q is q's send segment addressed to this rank
            o = 0
            for q in range(self.world):
                qs = got[q]["splits"]
                if qs[self.rank] != rs[q]:
                    raise RuntimeError(f"rank {self.rank}: rank {q} sends {qs[self.rank]} B, "
                                       f"{rs[q]} B expected")
                s0 = sum(qs[:self.rank])
                recv[o:o + rs[q]].copy_(got[q]["send"][s0:s0 + rs[q]])
                o += rs[q]
            return
        n = min(sum(rs), sum(ss))
        if n:
            recv[:n].copy_(send[:n])

    def _scratch_of(self, nbytes, device):
        import torch

        if self._scratch is None or self._scratch.numel() < nbytes or self._scratch.device != device:
            self._scratch = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=device)
        return self._scratch

    def exchange(self, sends, recvs) -> "Pending":
        mesh = self.mesh
        for t, peer in sends:
            if not 0 <= peer < self.world or peer == self.rank:
                raise ValueError(f"rank {self.rank} sends to {peer}")
            nb = t.numel() * t.element_size()
            self.sent_bytes += nb
            if mesh is not None and mesh.phase == "record":
                mesh.box.setdefault((self.rank, peer), []).append(t.detach().reshape(-1).clone())
                mesh.log.append((self.rank, peer, nb))
            elif mesh is not None:
                key = (self.rank, peer)
                box = mesh.box.get(key)
                if not box:
                    raise RuntimeError(f"rank {self.rank}: no send to rank {peer} recorded")
                i = mesh.scursor.get(key, 0)
                mesh.scursor[key] = (i + 1) % len(box)
                if box[i].numel() * box[i].element_size() != nb:
                    raise RuntimeError(f"rank {self.rank}: send {i} to rank {peer} changed size")
                box[i].copy_(t.detach().reshape(-1))
        for t, peer in recvs:
            if not 0 <= peer < self.world or peer == self.rank:
                raise ValueError(f"rank {self.rank} receives from {peer}")
            import torch

            flat = t.reshape(-1).view(torch.uint8)
            nb = flat.numel()
            self.recv_bytes += nb
            if mesh is None:
                flat.copy_(self._scratch_of(nb, flat.device)[:nb])
                continue
            if mesh.phase != "replay":
                continue
            key = (peer, self.rank)
            box = mesh.box.get(key)
            if not box:
                raise RuntimeError(f"rank {self.rank}: nothing recorded from rank {peer}")
            i = mesh.cursor.get(key, 0)
            mesh.cursor[key] = (i + 1) % len(box)
            src = box[i].view(torch.uint8)
            if src.numel() != nb:
                raise RuntimeError(f"rank {self.rank}: transfer {i} from rank {peer} is "
                                   f"{src.numel()} B, the receive {nb} B")
            flat.copy_(src)
        return Pending([], [])

    # timing only: reduce / all-reduce / reduce-scatter / all-gather /
    # broadcast become no-ops (values meaningless), so a rehearsal can time
    # the step without the local copies that stand in for RCCL's collective
    skip_collectives = False

    def _reduce(self, kind, t):
        if self.record:
            self.records.append((kind, t.detach().clone()))
        if not self.skip_collectives and self.mesh is None:
            self._copy(t)

    def _meshed(self, kind, **parts):
        """Every rank's inputs of this collective (replay), else None."""
        if self.mesh is None:
            return None
        return self.mesh.collective(self.rank, kind, parts)

    @staticmethod
    def _sum(ts):
        acc = ts[0].clone()
        for t in ts[1:]:
            acc += t
        return acc

    def all_reduce_sum(self, t):
        self._reduce("all_reduce_sum", t)
        got = self._meshed("all_reduce_sum", t=t)
        if got is not None:
            t.copy_(self._sum([g["t"] for g in got]))

    def reduce_sum(self, t, dst: int):
        self._reduce("reduce_sum", t)
        got = self._meshed("reduce_sum", t=t)
        if got is not None and self.rank == dst:
            t.copy_(self._sum([g["t"] for g in got]))

    def reduce_scatter_sum(self, out, t):
        self._reduce("reduce_scatter_sum", t)
        got = self._meshed("reduce_scatter_sum", t=t)
        if got is not None:
            out.copy_(self._sum([g["t"] for g in got]).view(self.world, -1)[self.rank])
        elif not self.skip_collectives:
            out.copy_(t.view(self.world, -1)[self.rank])

    def all_gather(self, out, t):
        got = self._meshed("all_gather", t=t)
        flat = t.reshape(-1)
        o = out.reshape(-1)
        if got is not None:
            for r in range(self.world):
                o[r * flat.numel():(r + 1) * flat.numel()].copy_(got[r]["t"].reshape(-1))
            return
        if self.skip_collectives:
            return
        for r in range(self.world):
            o[r * flat.numel():(r + 1) * flat.numel()].copy_(flat)

    def broadcast(self, t, src: int):
        got = self._meshed("broadcast", t=t)
        if got is not None:
            if self.rank != src:
                t.copy_(got[src]["t"])
            return
        if not self.skip_collectives:
            self._copy(t)

    def all_ok(self, ok: bool) -> bool:
        return bool(ok)


def default_comm() -> Optional[Comm]:
    """The world process group when torch.distributed runs with > 1 rank."""
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return Comm()
    return None


def splits_to_offsets(splits: List[int]) -> List[int]:
    out, o = [], 0
    for s in splits:
        out.append(o)
        o += s
    return out
