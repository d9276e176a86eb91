"""Seeded random arrays (cubed/random.py:13-36).

``random(size, chunks, spec)`` draws ``root_seed = random.getrandbits(128)``
from Python's global ``random`` state at graph-build time, exactly like the
reference, and block b is ``Generator(Philox(key=root_seed + offset(b)))
.random(shape)``.  On the MI355X the chunk is produced by the Philox leaf of a
fused program (csrc/common.h philox4x64_10), bit-identical to numpy, so a
``random(...)`` followed by elementwise ops and a reduction runs as one kernel
without materialising the random array."""

import random as pyrandom

import numpy as np

from . import ir
from .core.ops import _BlockIdProgram, map_blocks
from .utils import normalize_chunks, normalize_shape


def random(size, *, chunks=None, spec=None):
    """Return random floats in the half-open interval [0.0, 1.0)."""
    shape = normalize_shape(size)
    dtype = np.dtype(np.float64)
    chunks = normalize_chunks(chunks, shape=shape, dtype=dtype)
    numblocks = tuple(map(len, chunks))
    root_seed = pyrandom.getrandbits(128)
    ndim = len(shape)

    def build(block_arg):
        leaf = ir.Philox(root_seed=root_seed, numblocks=numblocks, block_arg=block_arg,
                         axes=tuple(range(ndim)), chunks=chunks)
        return ir.ExprProgram(ndim=ndim, nargs=block_arg + 1, outputs=leaf,
                              out_axes=tuple(range(ndim)), name="random")

    return map_blocks(_BlockIdProgram(build, 0), dtype=dtype, chunks=chunks, spec=spec)


def philox_key(root_seed: int, stream_id: int):
    """(key_lo, key_hi) numpy derives from ``Philox(key=root_seed + stream_id)``."""
    k = root_seed + stream_id
    if k >= 2**128:
        raise ValueError("Philox key must fit in 128 bits")
    return k & (2**64 - 1), k >> 64
