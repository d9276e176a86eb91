"""Host-side planning of the multi-GPU chunk exchanges.

Ownership is block-cyclic: chunk ``c`` of an array lives on rank
``block_id_to_offset(c) % world`` (the C-order offset of
cubed/utils.py:38-40), so every rank can compute, without communicating,
which bytes every other rank sends and receives.  Two plans:

* ``RechunkExchange`` -- ``copy_read_to_write`` (cubed/primitive/rechunk.py
  :187-192) over a whole target array: each target chunk is assembled from
  pieces of source chunks; pieces whose source and target chunks share an
  owner are copied locally, the rest move as point-to-point transfers (one
  send / receive pair per piece, grouped).  A piece whose box is contiguous
  in its TARGET chunk (e.g. a row band of a column chunk: config 3's
  (1000 rows x 1000 cols) pieces of a (50000, 1000) target) is received
  straight into the chunk's slot -- no unpack pass; one contiguous in its
  SOURCE chunk is sent from the slot -- no pack pass.  Pieces are
  enumerated in (target chunk, source chunk) C order on every rank, so both
  ends of every peer pair post their transfers in the same order.
* ``FetchExchange`` -- whole chunks a pipeline's tasks read but do not own
  (inputs on a different chunk grid, merge regions spanning ranks, matmul
  operand panels).  Each needed (array, chunk, field) is fetched once per
  rank into a receive buffer the task views then point into.

Pure Python over chunk geometry (no device, no torch): the executor turns
the pieces into box-copy tables, and the CPU tests drive the same plans with
numpy copies over a gloo process group.
"""

from __future__ import annotations

import itertools
import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

ALIGN = 256  # bytes; every packed piece starts 256-B aligned (16-B lanes)


def round_up(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


def owner_of(grid, coords, world: int) -> int:
    return grid.chunk_offset(coords) % world


@dataclass(frozen=True)
class Piece:
    """A box of ``extent`` elements moved from source chunk ``src`` (starting
    at in-chunk position ``src_start``) to target chunk ``dst`` (at
    ``dst_start``)."""
    src: Tuple[int, ...]
    src_start: Tuple[int, ...]
    dst: Tuple[int, ...]
    dst_start: Tuple[int, ...]
    extent: Tuple[int, ...]

    @property
    def size(self) -> int:
        return math.prod(self.extent)


def rechunk_pieces(src_grid, dst_grid) -> List[Piece]:
    """All pieces of a rechunk, in (target chunk, source chunk) C order."""
    out = []
    nd = src_grid.ndim
    for dkey in itertools.product(*[range(n) for n in dst_grid.numblocks]):
        dstart = dst_grid.chunk_start(dkey)
        dext = dst_grid.chunk_extent(dkey)
        ranges = []
        for d in range(nd):
            lo, hi = dstart[d], dstart[d] + dext[d]
            if hi <= lo:
                ranges.append(range(0))
                continue
            ranges.append(range(src_grid.chunk_of(d, lo), src_grid.chunk_of(d, hi - 1) + 1))
        for skey in itertools.product(*ranges):
            sstart = src_grid.chunk_start(skey)
            sext = src_grid.chunk_extent(skey)
            a = [max(dstart[d], sstart[d]) for d in range(nd)]
            b = [min(dstart[d] + dext[d], sstart[d] + sext[d]) for d in range(nd)]
            if any(x >= y for x, y in zip(a, b)):
                continue
            out.append(Piece(skey, tuple(a[d] - sstart[d] for d in range(nd)), dkey,
                             tuple(a[d] - dstart[d] for d in range(nd)),
                             tuple(b[d] - a[d] for d in range(nd))))
    return out


def box_contiguous(chunk_extent, start, extent) -> bool:
    """Whether a box of a C-order chunk is one contiguous byte run: every dim
    after the first one the box spans (> 1) is taken whole."""
    nd = len(extent)
    k = next((d for d in range(nd) if extent[d] > 1), nd - 1)
    return all(start[d] == 0 and extent[d] == chunk_extent[d] for d in range(k + 1, nd))


def box_offset(chunk_extent, start) -> int:
    """Element offset of a box's first element inside its C-order chunk."""
    st, o = 1, 0
    for d in range(len(chunk_extent) - 1, -1, -1):
        o += start[d] * st
        st *= chunk_extent[d]
    return o


@dataclass(frozen=True)
class Xfer:
    """One point-to-point transfer of a rechunk piece.  ``direct``: the
    bytes go straight from the source slot (send) or into the target slot
    (receive); otherwise through the pack (send) or staging (receive)
    buffer at byte ``offset``.  ``index``: the piece's position in the
    global piece order (slices of the exchange are index ranges)."""
    piece: Piece
    index: int
    direct: bool
    offset: int
    nbytes: int


@dataclass
class RechunkExchange:
    """What one rank does in a distributed rechunk."""
    rank: int
    world: int
    itemsize: int
    npieces: int
    local: List[Piece]          # src and dst chunk both owned here
    send: List[List[Xfer]]      # per dst rank, in piece order
    recv: List[List[Xfer]]      # per src rank, in piece order
    pack_bytes: int             # pack buffer (sends whose source box is strided)
    stage_bytes: int            # staging buffer (receives whose target box is strided)

    @property
    def exchanges(self) -> bool:
        return any(self.send) or any(self.recv)

    @property
    def send_bytes(self) -> int:
        return sum(x.nbytes for lst in self.send for x in lst)

    @property
    def recv_bytes(self) -> int:
        return sum(x.nbytes for lst in self.recv for x in lst)

    def slice_bounds(self, nslices: int) -> List[Tuple[int, int]]:
        """``nslices`` ranges of piece indices (the same on every rank)."""
        n = max(1, self.npieces)
        return [(n * k // nslices, n * (k + 1) // nslices) for k in range(nslices)]


def plan_rechunk(src_grid, dst_grid, rank: int, world: int, itemsize: int,
                 pieces: Optional[List[Piece]] = None, src_world: Optional[int] = None) -> RechunkExchange:
    """``src_world=1``: the source is replicated on every rank (a small
    uploaded constant), so every piece is local to its target's owner."""
    pieces = rechunk_pieces(src_grid, dst_grid) if pieces is None else pieces
    replicated = src_world == 1
    local = []
    send: List[List[Xfer]] = [[] for _ in range(world)]
    recv: List[List[Xfer]] = [[] for _ in range(world)]
    packed = staged = 0
    for i, p in enumerate(pieces):
        d = owner_of(dst_grid, p.dst, world)
        s = d if replicated else owner_of(src_grid, p.src, world)
        if s == d:
            if s == rank:
                local.append(p)
            continue
        nbytes = p.size * itemsize
        if s == rank:
            direct = box_contiguous(src_grid.chunk_extent(p.src), p.src_start, p.extent)
            send[d].append(Xfer(p, i, direct, 0 if direct else packed, nbytes))
            if not direct:
                packed += round_up(nbytes)
        if d == rank:
            direct = box_contiguous(dst_grid.chunk_extent(p.dst), p.dst_start, p.extent)
            recv[s].append(Xfer(p, i, direct, 0 if direct else staged, nbytes))
            if not direct:
                staged += round_up(nbytes)
    return RechunkExchange(rank, world, itemsize, len(pieces), local, send, recv, packed, staged)


def prefix(xs: Sequence[int]) -> List[int]:
    out, o = [], 0
    for x in xs:
        out.append(o)
        o += x
    return out


# ------------------------------------------------------------------ fetches

ChunkRef = Tuple[str, Tuple[int, ...], Optional[str]]  # (array name, chunk coords, field)


@dataclass
class FetchExchange:
    """Whole-chunk fetches of one pipeline, for one rank."""
    rank: int
    world: int
    send: List[List[Tuple[ChunkRef, int, int]]]   # per dst: (chunk, byte offset, nbytes)
    recv: List[List[Tuple[ChunkRef, int, int]]]   # per src: (chunk, byte offset, nbytes)
    send_splits: List[int]
    recv_splits: List[int]

    @property
    def exchanges(self) -> bool:
        return any(self.send_splits) or any(self.recv_splits)

    def recv_offsets(self) -> Dict[ChunkRef, int]:
        return {ref: off for lst in self.recv for ref, off, _ in lst}


def plan_fetch(needs: Dict[int, set], owner, nbytes, rank: int, world: int) -> FetchExchange:
    """``needs[r]`` = chunk refs rank r's tasks read; ``owner(ref)`` its owner
    rank; ``nbytes(ref)`` its compact size.  Refs a rank owns are not
    fetched."""
    send: List[List] = [[] for _ in range(world)]
    recv: List[List] = [[] for _ in range(world)]
    sent = [0] * world
    got = [0] * world
    for r in range(world):
        for ref in sorted(needs.get(r, ()), key=_ref_key):
            o = owner(ref)
            if o == r:
                continue
            nb = round_up(nbytes(ref))
            if o == rank:
                send[r].append((ref, sent[r], nb))
                sent[r] += nb
            if r == rank:
                recv[o].append((ref, got[o], nb))
                got[o] += nb
    soff = prefix(sent)
    roff = prefix(got)
    send = [[(ref, off + soff[j], nb) for ref, off, nb in lst] for j, lst in enumerate(send)]
    recv = [[(ref, off + roff[j], nb) for ref, off, nb in lst] for j, lst in enumerate(recv)]
    return FetchExchange(rank, world, send, recv, sent, got)


def _ref_key(ref):
    name, coords, field = ref
    return (name, tuple(coords), field or "")
