"""Array targets: where a Cubed array's chunks live.

The reference stores every array as a Zarr array -- ``LazyZarrArray`` for
intermediates (cubed/storage/zarr.py:8-103), created by the ``create-arrays``
op before the first task -- plus never-materialised virtual arrays for
constants, templates and block ids (cubed/storage/virtual.py:14-182).

Here intermediates are HBM-resident ``DeviceArray``s instead: chunk-major
"slabs" with one fixed-size slot per chunk (edge chunks stored compact at the
start of their slot), one slab per structured field (SoA), chunks owned
block-cyclically by rank (chunk offset mod world size).  Because every slot
has the same size, the chunks along any axis sit at a constant stride, so a
run of chunks (a merge_chunks region, a partial_reduce group) is one strided
view -- the kernels read merged chunks in place instead of copying them.
Zarr is only a source/sink format (``cubed_amd.zarr_io``).
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .utils import (
    chunk_starts,
    memory_repr,
    normalize_chunks,
    normalize_shape,
    to_chunksize,
)

# bytes between chunk slots: four 8-byte elements, the alignment the
# vectorised kernels need of every chunk base (lowering._vec_ok).  Slots are
# otherwise packed end to end, so the stacked row bands of an array are one
# run of addresses and consecutive output chunks continue each other -- the
# executor walks such runs as single task rows (lowering._merge_group_rows /
# _merge_kept_runs)
SLOT_ALIGN = 32

_GEOMETRY_ONLY = [False]


class geometry_only:
    """Context in which chunks owned by other ranks have address 0 instead of
    raising: the multi-GPU executor uses it to derive the shape of a task it
    does not run (its extents and strides), never to read through it."""

    def __enter__(self):
        self._prev = _GEOMETRY_ONLY[0]
        _GEOMETRY_ONLY[0] = True
        return self

    def __exit__(self, *exc):
        _GEOMETRY_ONLY[0] = self._prev
        return False


class ChunkGrid:
    """Geometry shared by all chunked targets."""

    def __init__(self, shape, dtype, chunks):
        self.shape = normalize_shape(shape)
        self.dtype = np.dtype(dtype)
        if isinstance(chunks, tuple) and chunks and isinstance(chunks[0], tuple):
            norm = chunks
        else:
            norm = normalize_chunks(chunks, self.shape, dtype=self.dtype)
        self._norm_chunks = norm
        self.chunks = to_chunksize(norm) if self.shape else ()
        self.ndim = len(self.shape)
        self.numblocks = tuple(len(c) for c in norm)
        self._starts = [chunk_starts(c) for c in norm]

    @property
    def size(self) -> int:
        return math.prod(self.shape)

    @property
    def nbytes(self) -> int:
        return self.size * self.dtype.itemsize

    @property
    def nchunks(self) -> int:
        return math.prod(self.numblocks)

    def chunk_extent(self, coords: Sequence[int]) -> Tuple[int, ...]:
        return tuple(self._norm_chunks[d][c] for d, c in enumerate(coords))

    def chunk_start(self, coords: Sequence[int]) -> Tuple[int, ...]:
        return tuple(self._starts[d][c] for d, c in enumerate(coords))

    def chunk_offset(self, coords: Sequence[int]) -> int:
        o = 0
        for c, n in zip(coords, self.numblocks):
            o = o * n + c
        return o

    def chunk_of(self, d: int, pos: int) -> int:
        """Index of the chunk holding global position ``pos`` along dim d."""
        st = self._starts[d]
        # regular chunks: direct division, clamped for the edge chunk
        c = pos // self.chunks[d] if self.chunks[d] else 0
        return min(c, len(st) - 2)


def c_strides(extent: Sequence[int]) -> Tuple[int, ...]:
    s, out = 1, []
    for e in reversed(extent):
        out.append(s)
        s *= e
    return tuple(reversed(out))


_ALLOC_EPOCH = [0]


def alloc_epoch() -> int:
    """Bumped whenever an allocated array's slabs are freed or replaced."""
    return _ALLOC_EPOCH[0]


class DeviceArray(ChunkGrid):
    """HBM-resident chunked array (replaces LazyZarrArray for intermediates).

    Allocation is lazy (``allocate``); a structured dtype gets one slab per
    field.  ``rank``/``world`` select the block-cyclic subset of chunks this
    process owns."""

    def __init__(self, shape, dtype, chunks, name: Optional[str] = None):
        super().__init__(shape, dtype, chunks)
        self.name = name
        # structured dtypes: one slab per field; complex: a real and an
        # imaginary slab (cubed_amd/complex.py)
        self.fields: Tuple[Optional[str], ...] = (
            tuple(self.dtype.names) if self.dtype.names else
            ("real", "imag") if self.dtype.kind == "c" else (None,))
        self.slabs: Dict[Optional[str], object] = {}
        self.rank, self.world = 0, 1
        self.written = False
        self.device = None
        self.alias: Optional["DeviceArray"] = None  # same values, other chunking
        # multi-GPU: fetched copies of chunks owned by other ranks, visible
        # while the executor lowers one pipeline ((coords, field) -> address)
        self.remote: Optional[Dict] = None
        self.comm = None

    # -- layout ---------------------------------------------------------------
    def field_dtype(self, field: Optional[str]) -> np.dtype:
        if field is None:
            return self.dtype
        if self.dtype.kind == "c":
            return np.dtype(f"f{self.dtype.itemsize // 2}")
        return self.dtype.fields[field][0]

    @property
    def slot_elems(self) -> int:
        return max(1, math.prod(self.chunks)) if self.ndim else 1

    def slot_bytes(self, field=None) -> int:
        b = self.slot_elems * self.field_dtype(field).itemsize
        return (b + SLOT_ALIGN - 1) // SLOT_ALIGN * SLOT_ALIGN

    def slot_stride_elems(self, field=None) -> int:
        """Distance between consecutive slots in elements of the field."""
        isz = self.field_dtype(field).itemsize
        sb = self.slot_bytes(field)
        assert sb % isz == 0
        return sb // isz

    def owner(self, coords) -> int:
        return self.chunk_offset(coords) % self.world

    def local_slot(self, coords) -> int:
        return self.chunk_offset(coords) // self.world

    def local_nslots(self) -> int:
        n = self.nchunks
        return (n - self.rank + self.world - 1) // self.world if n > self.rank else 0

    def device_bytes(self) -> int:
        return sum(self.local_nslots() * self.slot_bytes(f) for f in self.fields)

    # -- allocation -----------------------------------------------------------
    def allocate(self, device, rank: int = 0, world: int = 1):
        import torch

        if self.slabs and self.device == device and (self.rank, self.world) == (rank, world):
            return
        if self.slabs:  # addresses change: recorded launch lists are stale
            _ALLOC_EPOCH[0] += 1
        self.rank, self.world, self.device = rank, world, device
        self.slabs = {}
        for f in self.fields:
            nbytes = max(self.local_nslots() * self.slot_bytes(f), SLOT_ALIGN)
            self.slabs[f] = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.written = False

    def release(self):
        """Free the slabs.  Launch lists the executor recorded against them
        are invalidated (alloc_epoch)."""
        if self.slabs:
            _ALLOC_EPOCH[0] += 1
        self.slabs = {}
        self.written = False

    @property
    def allocated(self) -> bool:
        return bool(self.slabs)

    def base_addr(self, field=None) -> int:
        return self.slabs[field].data_ptr()

    def chunk_addr(self, coords, field=None) -> int:
        if self.owner(coords) != self.rank:
            if self.remote is not None:
                a = self.remote.get((tuple(coords), field))
                if a is not None:
                    return a
            if _GEOMETRY_ONLY[0]:
                return 0
            raise KeyError(f"chunk {coords} of {self.name} is owned by rank {self.owner(coords)}")
        return self.base_addr(field) + self.local_slot(coords) * self.slot_bytes(field)

    # -- host transfer --------------------------------------------------------
    def _slab_view(self, field, slot, extent):
        import torch

        dt = self.field_dtype(field)
        nb = math.prod(extent) * dt.itemsize
        start = slot * self.slot_bytes(field)
        raw = self.slabs[field][start:start + nb]
        return raw, dt

    def read_chunk(self, coords, field=None) -> np.ndarray:
        if field is None and self.dtype.kind == "c":
            out = np.empty(self.chunk_extent(coords), dtype=self.dtype)
            out.real = self.read_chunk(coords, "real")
            out.imag = self.read_chunk(coords, "imag")
            return out
        ext = self.chunk_extent(coords)
        raw, dt = self._slab_view(field, self.local_slot(coords), ext)
        host = raw.cpu().numpy()
        return host.view(dt).reshape(ext)

    def write_chunk(self, coords, value: np.ndarray, field=None):
        import torch

        if field is None and self.dtype.kind == "c":
            v = np.asarray(value, dtype=self.dtype)
            self.write_chunk(coords, v.real, "real")
            self.write_chunk(coords, v.imag, "imag")
            return

        ext = self.chunk_extent(coords)
        dt = self.field_dtype(field)
        arr = np.array(np.broadcast_to(np.asarray(value, dtype=dt), ext), order="C", copy=True)
        raw, _ = self._slab_view(field, self.local_slot(coords), ext)
        raw.copy_(torch.from_numpy(arr.reshape(-1).view(np.uint8)))

    def to_numpy(self) -> np.ndarray:
        """Assemble the whole array on the host (owned chunks only when
        world > 1; callers gather first)."""
        import itertools

        out = np.empty(self.shape, dtype=self.dtype)
        if self.size == 0:
            return out
        for coords in itertools.product(*[range(n) for n in self.numblocks]):
            if self.owner(coords) != self.rank:
                continue
            st = self.chunk_start(coords)
            ext = self.chunk_extent(coords)
            sl = tuple(slice(s, s + e) for s, e in zip(st, ext))
            if self.dtype.names:
                for f in self.fields:
                    out[f][sl] = self.read_chunk(coords, f)
            else:
                out[sl] = self.read_chunk(coords)
        return out

    def from_numpy(self, arr: np.ndarray):
        import itertools

        arr = np.asarray(arr)
        for coords in itertools.product(*[range(n) for n in self.numblocks]):
            if self.owner(coords) != self.rank:
                continue
            st = self.chunk_start(coords)
            ext = self.chunk_extent(coords)
            sl = tuple(slice(s, s + e) for s, e in zip(st, ext))
            if self.dtype.names:
                for f in self.fields:
                    self.write_chunk(coords, arr[f][sl], f)
            else:
                self.write_chunk(coords, arr[sl])
        self.written = True

    def __repr__(self):
        return (f"DeviceArray<{self.name}, shape={self.shape}, dtype={self.dtype}, "
                f"chunks={self.chunks}, {memory_repr(self.nbytes)}>")


def device_empty(shape, *, dtype, chunks, name=None) -> DeviceArray:
    return DeviceArray(shape, dtype, chunks, name=name)


# ------------------------------------------------------------------ virtual


class VirtualEmptyArray(ChunkGrid):
    """Never materialised; reading it is an error (cubed/storage/virtual.py:14)."""


class VirtualFullArray(ChunkGrid):
    """A single fill value (cubed/storage/virtual.py:44); lowered to a constant."""

    def __init__(self, shape, dtype, chunks, fill_value=None):
        super().__init__(shape, dtype, chunks)
        self.fill_value = fill_value


class VirtualOffsetsArray(ChunkGrid):
    """Block offsets: element i is the C-order offset of block i
    (cubed/storage/virtual.py:82); lowered to the task's block id."""

    def __init__(self, shape):
        shape = normalize_shape(shape)
        super().__init__(shape, np.int32, (1,) * len(shape))


class VirtualInMemoryArray(ChunkGrid):
    """A small host array (<= 1 MB, cubed/storage/virtual.py:105-150).  0-d
    and single-element arrays lower to constants; larger ones are uploaded to
    HBM once per executor."""

    def __init__(self, array: np.ndarray, chunks, max_nbytes: int = 10**6):
        if array.nbytes > max_nbytes:
            raise ValueError(
                f"Size of in memory array is {memory_repr(array.nbytes)} which exceeds maximum "
                f"of {memory_repr(max_nbytes)}. Consider loading the array from storage using `from_array`."
            )
        super().__init__(array.shape, array.dtype, chunks)
        self.array = array
        self.device_copy: Optional[DeviceArray] = None


class HostArray(ChunkGrid):
    """An in-memory numpy (or array-like) source of ``from_array``, uploaded
    chunk by chunk by the executor."""

    def __init__(self, array, chunks):
        super().__init__(array.shape, array.dtype, chunks)
        self.array = array


def virtual_empty(shape, *, dtype, chunks):
    return VirtualEmptyArray(shape, dtype, chunks)


def virtual_full(shape, fill_value, *, dtype, chunks):
    return VirtualFullArray(shape, dtype, chunks, fill_value)


def virtual_offsets(shape):
    return VirtualOffsetsArray(shape)


def virtual_in_memory(array, chunks):
    return VirtualInMemoryArray(array, chunks)
