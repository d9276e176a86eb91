"""Primitive operation metadata (mirrors cubed/primitive/types.py:11-75)."""

from dataclasses import dataclass
from typing import Any, Optional, Tuple

from ..runtime.types import CubedPipeline


@dataclass(frozen=True)
class PrimitiveOperation:
    """Metadata about a ``blockwise`` or ``rechunk`` primitive operation."""

    pipeline: CubedPipeline
    target_array: Any
    projected_mem: int
    allowed_mem: int
    reserved_mem: int
    num_tasks: int
    fusable: bool = True
    write_chunks: Optional[Tuple[int, ...]] = None


class CubedArrayProxy:
    """An array (target or source) plus the chunking tasks use on it."""

    def __init__(self, array, chunks):
        self.array = array
        self.chunks = chunks

    def open(self):
        return self.array


@dataclass(frozen=True)
class CubedCopySpec:
    read: CubedArrayProxy
    write: CubedArrayProxy


class MemoryModeller:
    """Models peak memory usage for a series of operations."""

    def __init__(self):
        self.current_mem = 0
        self.peak_mem = 0

    def allocate(self, num_bytes):
        self.current_mem += num_bytes
        self.peak_mem = max(self.peak_mem, self.current_mem)

    def free(self, num_bytes):
        self.current_mem -= num_bytes
        self.peak_mem = max(self.peak_mem, self.current_mem)
