from .array import CoreArray, compute, gensym, measure_reserved_mem, visualize
from .ops import (
    blockwise,
    elemwise,
    from_array,
    from_zarr,
    map_blocks,
    map_direct,
    merge_chunks,
    partial_reduce,
    rechunk,
    reduction,
    squeeze,
    store,
    to_zarr,
    tree_reduce,
    unify_chunks,
)
from .plan import Plan

__all__ = [
    "CoreArray", "Plan", "blockwise", "compute", "elemwise", "from_array", "from_zarr",
    "gensym", "map_blocks", "map_direct", "measure_reserved_mem", "merge_chunks",
    "partial_reduce", "rechunk", "reduction", "squeeze", "store", "to_zarr", "tree_reduce",
    "unify_chunks", "visualize",
]
