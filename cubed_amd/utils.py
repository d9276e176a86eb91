"""Chunk geometry and size helpers.

Restates the helpers the reference keeps in ``cubed/utils.py`` (chunk_memory
:28-30, offset/block-id conversion :33-40, get_item :43-48, to_chunksize
:109-125, convert_to_bytes :201-258, memory_repr :65-88, split_into, map_nested
:270-293) and the chunk normalisation it vendors from dask
(``cubed/vendor/dask/array/core.py:103-407`` normalize_chunks / auto_chunks /
blockdims_from_blockshape, ``common_blockdim``).  Pure host code used at plan
time only.
"""

from __future__ import annotations

import itertools
import math
from collections import Counter
from numbers import Integral, Number
from typing import Dict, Iterable, Sequence, Tuple, Union

import numpy as np

DEFAULT_CHUNK_BYTES = 128 * 2**20  # dask's "array.chunk-size" default (128 MiB)


# ---------------------------------------------------------------- sizes


def chunk_memory(dtype, chunksize) -> int:
    """Bytes used by one chunk of ``chunksize`` elements of ``dtype``."""
    return np.dtype(dtype).itemsize * math.prod(chunksize)


_SI = {"kB": 1, "MB": 2, "GB": 3, "TB": 4, "PB": 5}


def _is_number(s: str) -> bool:
    try:
        float(s)
    except ValueError:
        return False
    return True


def convert_to_bytes(size: Union[int, float, str]) -> int:
    """Parse ``500kB`` / ``2GB`` / ``123`` into a byte count (SI, powers of 1000)."""
    if isinstance(size, str):
        s = size.replace(" ", "")
        if _is_number(s):
            value, factor = s, 1
        elif s.endswith("B") and _is_number(s[:-1]):
            value, factor = s[:-1], 1
        elif s[-2:] in _SI and _is_number(s[:-2]):
            value, factor = s[:-2], 1000 ** _SI[s[-2:]]
        else:
            raise ValueError(
                f"Invalid value: {size}. Expected the string to be a numeric value ending with an SI prefix."
            )
        size = float(value) * factor
    if isinstance(size, float):
        if not size.is_integer():
            raise ValueError(
                f"Invalid value: {size}. Can't have a non-integer number of bytes"
            )
        size = int(size)
    if size < 0:
        raise ValueError(f"Invalid value: {size}. Must be a positive value")
    return size


def memory_repr(num: int) -> str:
    """Human readable decimal byte count (1 KB = 1000 bytes)."""
    if num < 0:
        raise ValueError(f"Invalid value: {num}. Expected a positive integer.")
    if num < 1000.0:
        return f"{num} bytes"
    val = num / 1000.0
    for unit in ["KB", "MB", "GB", "TB", "PB"]:
        if val < 1000.0:
            return f"{val:3.1f} {unit}"
        val /= 1000.0
    return f"{num:.1e} bytes"


_BYTE_SUFFIX = {
    "b": 1, "kb": 10**3, "mb": 10**6, "gb": 10**9, "tb": 10**12, "pb": 10**15,
    "kib": 2**10, "mib": 2**20, "gib": 2**30, "tib": 2**40, "pib": 2**50,
    "k": 10**3, "m": 10**6, "g": 10**9, "t": 10**12, "p": 10**15,
    "ki": 2**10, "mi": 2**20, "gi": 2**30, "ti": 2**40,
}


def parse_bytes(s) -> int:
    """dask-style byte parser used for chunk specs like ``"1kiB"``."""
    if isinstance(s, (int, float)):
        return int(s)
    t = s.replace(" ", "").lower()
    i = 0
    while i < len(t) and (t[i].isdigit() or t[i] in ".e"):
        i += 1
    num = float(t[:i]) if i else 1.0
    suffix = t[i:] or "b"
    if suffix not in _BYTE_SUFFIX:
        raise ValueError(f"Could not interpret '{suffix}' as a byte unit")
    return int(num * _BYTE_SUFFIX[suffix])


# ---------------------------------------------------------------- block ids


def offset_to_block_id(offset: int, numblocks: Tuple[int, ...]) -> Tuple[int, ...]:
    """C-order block offset -> block coordinates."""
    return tuple(int(i) for i in np.unravel_index(offset, numblocks))


def block_id_to_offset(block_id: Tuple[int, ...], numblocks: Tuple[int, ...]) -> int:
    """Block coordinates -> C-order block offset (cubed/utils.py:38-40)."""
    return int(np.ravel_multi_index(block_id, numblocks))


def chunk_starts(chunks_1d: Sequence[int]) -> Tuple[int, ...]:
    out = [0]
    for c in chunks_1d:
        out.append(out[-1] + c)
    return tuple(out)


def get_item(chunks, idx: Tuple[int, ...]) -> Tuple[slice, ...]:
    """Slices selecting block ``idx`` of an array with normalized ``chunks``."""
    out = []
    for c, i in zip(chunks, idx):
        st = chunk_starts(c)
        out.append(slice(st[i], st[i + 1], None))
    return tuple(out)


def _check_regular_chunks(chunkset) -> bool:
    for chunks in chunkset:
        if len(chunks) == 1:
            continue
        if len(set(chunks[:-1])) > 1:
            return False
        if chunks[-1] > chunks[0]:
            return False
    return True


def to_chunksize(chunkset) -> Tuple[int, ...]:
    """Regular chunk set -> chunk size tuple (first chunk of each dim)."""
    if not _check_regular_chunks(chunkset):
        raise ValueError(f"Array must have regular chunks, but found chunks={chunkset}")
    return tuple(c[0] for c in chunkset)


def numblocks_of(chunks) -> Tuple[int, ...]:
    return tuple(len(c) for c in chunks)


# ---------------------------------------------------------------- normalize


def blockdims_from_blockshape(shape, blockshape):
    """(10,), (4,) -> ((4, 4, 2),)"""
    out = []
    for d, bd in zip(shape, blockshape):
        if d == 0:
            out.append((0,))
        elif bd == 0:
            out.append((0,))
        else:
            full, rem = divmod(int(d), int(bd))
            out.append((int(bd),) * full + ((rem,) if rem else ()))
    return tuple(out)


def _round_to(c, s):
    """Chunk length near ``c`` aligned with ``s`` (as dask's round_to)."""
    if c <= s:
        return max(1, int(c))
    return math.floor(c / s) * s


def _auto_chunks(chunks, shape, limit, dtype, previous_chunks=None):
    chunks = list(chunks)
    autos = {i for i, c in enumerate(chunks) if c == "auto"}
    if not autos:
        return tuple(chunks)
    if limit is None:
        limit = DEFAULT_CHUNK_BYTES
    if isinstance(limit, str):
        limit = parse_bytes(limit)
    if dtype is None:
        raise TypeError("dtype must be known for auto-chunking")
    limit = max(1, limit)
    largest = math.prod(
        c if isinstance(c, Number) else max(c) for c in chunks if c != "auto"
    )
    if previous_chunks:
        prev = tuple(c if isinstance(c, tuple) else (c,) for c in previous_chunks)
        result = {a: float(np.median(prev[a])) for a in autos}
        ideal = []
        for i, s in enumerate(shape):
            mode, count = max(Counter(prev[i]).items(), key=lambda kv: kv[1])
            ideal.append(mode if (mode > 1 and count >= len(prev[i]) / 2) else s)

        def multiplier():
            return limit / dtype.itemsize / largest / math.prod(r for r in result.values() if r)

        m = multiplier()
        last_m, last_autos = 0, set()
        while m != last_m or autos != last_autos:
            last_m, last_autos = m, set(autos)
            for a in sorted(autos):
                if ideal[a] == 0:
                    result[a] = 0
                    continue
                proposed = result[a] * m ** (1 / len(autos))
                if proposed > shape[a]:
                    autos.remove(a)
                    largest *= shape[a]
                    chunks[a] = shape[a]
                    del result[a]
                else:
                    result[a] = _round_to(proposed, ideal[a])
            m = multiplier()
        for k, v in result.items():
            chunks[k] = v
        return tuple(chunks)
    size = (limit / dtype.itemsize / largest) ** (1 / len(autos))
    small = [i for i in autos if shape[i] < size]
    if small:
        for i in small:
            chunks[i] = (shape[i],)
        return _auto_chunks(chunks, shape, limit, dtype)
    for i in autos:
        chunks[i] = _round_to(size, shape[i])
    return tuple(chunks)


def normalize_chunks(chunks, shape=None, limit=None, dtype=None, previous_chunks=None):
    """Normalize a chunk spec to a tuple of tuples (dask semantics).

    Accepts ints, tuples, tuples-of-tuples, dicts, -1/None (full extent),
    "auto" and byte strings.
    """
    if dtype is not None and not isinstance(dtype, np.dtype):
        dtype = np.dtype(dtype)
    if chunks is None:
        raise ValueError("chunks cannot be None")
    if isinstance(chunks, list):
        chunks = tuple(chunks)
    if isinstance(chunks, (Number, str)):
        chunks = (chunks,) * len(shape)
    if isinstance(chunks, dict):
        chunks = tuple(chunks.get(i, None) for i in range(len(shape)))
    if isinstance(chunks, np.ndarray):
        chunks = tuple(chunks.tolist())
    if not chunks and shape and all(s == 0 for s in shape):
        chunks = ((0,),) * len(shape)
    if (
        shape
        and len(shape) == 1
        and len(chunks) > 1
        and all(isinstance(c, (Number, str)) for c in chunks)
    ):
        chunks = (chunks,)
    if shape and len(chunks) != len(shape):
        raise ValueError(
            "Chunks and shape must be of the same length/dimension. "
            f"Got chunks={chunks}, shape={shape}"
        )
    if shape is not None:
        chunks = tuple(s if (c is None or (isinstance(c, Number) and c == -1)) else c
                       for c, s in zip(chunks, shape))
    for c in chunks:
        if isinstance(c, str) and c != "auto":
            parsed = parse_bytes(c)
            if limit is None:
                limit = parsed
            elif parsed != limit:
                raise ValueError("Only one consistent value of limit or chunk is allowed.")
    chunks = tuple("auto" if isinstance(c, str) else c for c in chunks)
    if any(c == "auto" for c in chunks):
        chunks = _auto_chunks(chunks, shape, limit, dtype, previous_chunks)
    if chunks and shape is not None:
        out = []
        for s, c in zip(shape, chunks):
            if isinstance(c, (tuple, list)):
                out.append(tuple(int(x) for x in c))
            else:
                out.extend(blockdims_from_blockshape((s,), (c,)))
        chunks = tuple(out)
    else:
        chunks = tuple(tuple(c) if isinstance(c, (tuple, list)) else (c,) for c in chunks)
    for c in chunks:
        if not c:
            raise ValueError(
                "Empty tuples are not allowed in chunks. Express "
                "zero length dimensions with 0(s) in chunks"
            )
    if shape is not None:
        if len(chunks) != len(shape):
            raise ValueError(
                f"Input array has {len(shape)} dimensions but the supplied "
                f"chunks has only {len(chunks)} dimensions"
            )
        if not all(sum(c) == s for c, s in zip(chunks, shape)):
            raise ValueError(f"Chunks do not add up to shape. Got chunks={chunks}, shape={shape}")
    return tuple(tuple(int(x) for x in c) for c in chunks)


def normalize_shape(shape) -> Tuple[int, ...]:
    if isinstance(shape, Integral):
        return (int(shape),)
    return tuple(int(s) for s in shape)


def common_blockdim(blockdims):
    """Common refinement of several 1-d chunkings of the same extent
    (dask's common_blockdim, used by unify_chunks)."""
    if not any(blockdims):
        return ()
    non_trivial = {b for b in blockdims if len(b) > 1 or (len(b) == 1 and b[0] != 1)}
    if len(non_trivial) == 1:
        return next(iter(non_trivial))
    if len(non_trivial) == 0:
        return next(iter(blockdims))
    if len({sum(b) for b in non_trivial}) > 1:
        raise ValueError("Chunks do not add up to same value", blockdims)
    bounds = sorted({x for b in non_trivial for x in chunk_starts(b)})
    return tuple(b - a for a, b in zip(bounds[:-1], bounds[1:]))


# ---------------------------------------------------------------- misc


def split_into(iterable, sizes):
    it = iter(iterable)
    for size in sizes:
        if size is None:
            yield list(it)
            return
        yield list(itertools.islice(it, size))


def map_nested(func, seq):
    """Apply ``func`` to leaves of nested lists/iterators, keeping structure."""
    if isinstance(seq, list):
        return [map_nested(func, item) for item in seq]
    if isinstance(seq, Iterable) and not isinstance(seq, (tuple, str, bytes)):
        return map(lambda s: map_nested(func, s), seq)
    return func(seq)


def flatten_keys(seq):
    """Flatten nested lists / iterators of chunk keys into a list of keys."""
    if isinstance(seq, tuple):
        return [seq]
    out = []
    for s in seq:
        out.extend(flatten_keys(s))
    return out


def gensym_factory(prefix: str):
    counter = itertools.count(1)

    def gensym(name: str = prefix) -> str:
        return f"{name}-{next(counter):03}"

    return gensym
