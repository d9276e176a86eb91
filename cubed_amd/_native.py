"""ctypes binding of libcubed_amd.so (the C ABI in include/cubed_amd.h).

The library is built in-tree (``make`` / ``__graft_entry__.build()``) and is
the only compute path: if it is missing, or no GPU is visible, every call
raises -- there is no host fallback.  torch is imported first so the HIP
runtime torch ships (soname libamdhip64.so.7) is the one the library binds
to; streams and device pointers therefore come straight from torch.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import (
    POINTER,
    Structure,
    Union,
    c_char_p,
    c_double,
    c_int,
    c_int32,
    c_int64,
    c_uint8,
    c_uint16,
    c_uint64,
    c_void_p,
)

import numpy as np

MAX_DIMS = 6
MAX_LEAVES = 4
MAX_FIELDS = 3
MAX_OUTS = 3
MAX_INSNS = 48
MAX_EPI = 16
MAX_CONSTS = 16
NREGS = 6

ABI_VERSION = 16  # include/cubed_amd.h CUBED_ABI_VERSION
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcubed_amd.so")


class Insn(Structure):
    _fields_ = [("op", c_uint8), ("a", c_uint8), ("b", c_uint8), ("c", c_uint8),
                ("t", c_uint8), ("pad", c_uint8), ("imm", c_uint16)]


class ConstVal(Union):
    _fields_ = [("f", c_double), ("i", c_int64)]


class Program(Structure):
    _fields_ = [
        ("vtype", c_int32), ("ndim", c_int32), ("nred", c_int32), ("mode", c_int32),
        ("nleaves", c_int32),
        ("leaf_kind", c_uint8 * MAX_LEAVES), ("leaf_dtype", c_uint8 * MAX_LEAVES),
        ("nfields", c_int32),
        ("field_rop", c_uint8 * MAX_FIELDS), ("field_acc", c_uint8 * MAX_FIELDS),
        ("field_src", c_uint8 * MAX_FIELDS), ("pad0", c_uint8 * 3),
        ("nouts", c_int32),
        ("out_dtype", c_uint8 * MAX_OUTS), ("out_src", c_uint8 * MAX_OUTS), ("pad1", c_uint8 * 2),
        ("ninsns", c_int32), ("nepi", c_int32),
        ("insns", Insn * MAX_INSNS), ("epi", Insn * MAX_EPI),
        ("consts", ConstVal * MAX_CONSTS),
    ]


# numpy mirror of cubed_task_t (one row per task, uploaded as bytes)
TASK_DTYPE = np.dtype([
    ("extent", np.int64, (MAX_DIMS,)),
    ("leaf_base", np.int64, (MAX_LEAVES,)),
    ("leaf_stride", np.int64, (MAX_LEAVES, MAX_DIMS)),
    ("out_base", np.int64, (MAX_OUTS,)),
    ("out_stride", np.int64, (MAX_OUTS, MAX_DIMS)),
    ("key_lo", np.uint64), ("key_hi", np.uint64),
    ("block_offset", np.int64), ("pad", np.int64),
])

BOX_DTYPE = np.dtype([
    ("src_base", np.int64), ("dst_base", np.int64),
    ("extent", np.int64, (MAX_DIMS,)),
    ("src_stride", np.int64, (MAX_DIMS,)),
    ("dst_stride", np.int64, (MAX_DIMS,)),
])

# cubed_gemm_chain_t / cubed_gemm_seg_t (chained chunk GEMMs)
CHAIN_DTYPE = np.dtype([
    ("c", np.int64), ("m", np.int64), ("n", np.int64), ("ldc", np.int64),
    ("seg0", np.int64), ("nseg", np.int64), ("ktot", np.int64), ("accumulate", np.int64),
])
SEG_DTYPE = np.dtype([
    ("a", np.int64), ("b", np.int64), ("k", np.int64), ("lda", np.int64), ("ldb", np.int64),
    ("pad", np.int64),
])
GEMM_AUTO, GEMM_ANY, GEMM_MFMA = -1, 0, 1

COPY_ROWS, COPY_ELEMS, COPY_TILE, COPY_FLAT = 0, 1, 2, 3


class NativeError(RuntimeError):
    pass


_lib = None


def lib():
    """Load (once) and return the native library; raise if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- bind to torch's HIP runtime first

    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()); "
            "cubed_amd has no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    L.cubed_fused_chunks.argtypes = [POINTER(Program), c_void_p, c_void_p, c_int64, c_int64, c_int64,
                                     c_void_p, c_int64, c_void_p]
    L.cubed_fused_chunks.restype = c_int
    L.cubed_fused_workspace_bytes.argtypes = [POINTER(Program), c_int64, c_int64, c_int64]
    L.cubed_fused_workspace_bytes.restype = c_int64
    L.cubed_stream_split_target.argtypes = [c_int64]
    L.cubed_stream_split_target.restype = c_int64
    L.cubed_random_chunks.argtypes = [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p]
    L.cubed_random_chunks.restype = c_int
    L.cubed_copy_boxes.argtypes = [c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32,
                                   c_int64, c_int64, c_void_p]
    L.cubed_copy_boxes.restype = c_int
    L.cubed_gemm_chain_path.argtypes = [c_void_p, c_int64, c_void_p, c_int32, c_int32]
    L.cubed_gemm_chain_path.restype = c_int
    L.cubed_gemm_grid_check.argtypes = [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_int32]
    L.cubed_gemm_grid_check.restype = c_int
    L.cubed_gemm_chain_grid.argtypes = [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_int64,
                                        c_int32, c_int32, c_void_p, c_void_p]
    L.cubed_gemm_chain_grid.restype = c_int
    L.cubed_gemm_pack_bytes.argtypes = [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_int32]
    L.cubed_gemm_pack_bytes.restype = c_int64
    L.cubed_gemm_chain_packed.argtypes = [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_int64,
                                          c_int32, c_int32, c_void_p, c_int64, c_void_p]
    L.cubed_gemm_chain_packed.restype = c_int
    L.cubed_gemm_dist_image_bytes.argtypes = [c_int64, c_int64, c_int32]
    L.cubed_gemm_dist_image_bytes.restype = c_int64
    L.cubed_gemm_dist_pack_a.argtypes = [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int32,
                                         c_int64, c_int64, c_void_p, c_int64, c_void_p]
    L.cubed_gemm_dist_pack_a.restype = c_int
    L.cubed_gemm_dist_b_bytes.argtypes = [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_int32]
    L.cubed_gemm_dist_b_bytes.restype = c_int64
    L.cubed_gemm_dist_pack_b.argtypes = [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_int64,
                                         c_int32, c_int32, c_void_p, c_int64, c_void_p]
    L.cubed_gemm_dist_pack_b.restype = c_int
    L.cubed_gemm_dist_gemm.argtypes = [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_int32,
                                       c_void_p, c_int64, c_void_p, c_int64, c_void_p]
    L.cubed_gemm_dist_gemm.restype = c_int
    L.cubed_gemm_chain.argtypes = [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                   c_void_p, c_int32, c_void_p]
    L.cubed_gemm_chain.restype = c_int
    L.cubed_fused_compile.argtypes = [POINTER(Program), c_char_p, POINTER(c_void_p)]
    L.cubed_fused_compile.restype = c_int
    L.cubed_fused_chunks_compiled.argtypes = [c_void_p, POINTER(Program), c_void_p, c_void_p, c_int64,
                                              c_int64, c_int64, c_void_p, c_int64, c_void_p]
    L.cubed_fused_chunks_compiled.restype = c_int
    L.cubed_fused_source.argtypes = [c_void_p]
    L.cubed_fused_source.restype = c_char_p
    L.cubed_fused_code_bytes.argtypes = [c_void_p]
    L.cubed_fused_code_bytes.restype = c_int64
    L.cubed_fused_finish.argtypes = [POINTER(Program), c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                     c_void_p]
    L.cubed_fused_finish.restype = c_int
    L.cubed_stream_force_split.argtypes = [c_int64]
    L.cubed_stream_force_split.restype = c_int64
    L.cubed_fused_finish_compiled.argtypes = [c_void_p, POINTER(Program), c_void_p, c_int64, c_int64,
                                              c_void_p, c_void_p]
    L.cubed_fused_finish_compiled.restype = c_int
    L.cubed_fused_finish_groups.argtypes = [POINTER(Program), c_void_p, c_void_p, c_int64, c_int64,
                                            c_void_p, c_void_p, c_int64, c_void_p]
    L.cubed_fused_finish_groups.restype = c_int
    L.cubed_combine_groups.argtypes = [POINTER(Program), c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                       c_void_p, c_int64, c_int64, c_void_p, c_void_p]
    L.cubed_combine_groups.restype = c_int
    L.cubed_fold_groups.argtypes = [POINTER(Program), c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                    c_void_p, c_int64, c_void_p, c_int64, c_void_p, POINTER(Program),
                                    c_void_p, c_void_p, c_void_p]
    L.cubed_fold_groups.restype = c_int
    L.cubed_fold_groups_compiled.argtypes = [c_void_p, POINTER(Program), c_void_p, c_int64, c_int64, c_void_p,
                                             c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]
    L.cubed_fold_groups_compiled.restype = c_int
    L.cubed_fold_groups_splits.argtypes = [c_int64, c_int64, c_int64]
    L.cubed_fold_groups_splits.restype = c_int64
    L.cubed_combine_partials.argtypes = [POINTER(Program), c_void_p, c_void_p, c_int32, c_int64, c_void_p,
                                         c_void_p]
    L.cubed_combine_partials.restype = c_int
    L.cubed_blosc_header.argtypes = [c_void_p, c_int64, POINTER(c_int64), POINTER(c_int64),
                                     POINTER(c_int), POINTER(c_int)]
    L.cubed_blosc_header.restype = c_int
    L.cubed_blosc_decompress.argtypes = [c_void_p, c_int64, c_void_p, c_int64]
    L.cubed_blosc_decompress.restype = c_int
    L.cubed_blosc_max_compressed.argtypes = [c_int64]
    L.cubed_blosc_max_compressed.restype = c_int64
    L.cubed_blosc_compress.argtypes = [c_void_p, c_int64, c_int, c_int, c_void_p, c_int64]
    L.cubed_blosc_compress.restype = c_int64
    for fn in (L.cubed_zstd_decompress, L.cubed_lz4_chunk_decompress):
        fn.argtypes = [c_void_p, c_int64, c_void_p, c_int64]
        fn.restype = c_int
    L.cubed_abi_version.restype = c_int
    L.cubed_last_error.restype = c_char_p
    L.cubed_device_count.restype = c_int
    if L.cubed_abi_version() != ABI_VERSION:
        raise NativeError("libcubed_amd.so ABI version mismatch; rebuild it")
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().cubed_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed with code {rc}: {msg}")


EXPORTED_SYMBOLS = (
    "cubed_fused_chunks", "cubed_fused_workspace_bytes", "cubed_stream_split_target", "cubed_stream_force_split", "cubed_random_chunks",
    "cubed_copy_boxes", "cubed_abi_version", "cubed_last_error",
    "cubed_device_count", "cubed_fused_compile", "cubed_fused_chunks_compiled", "cubed_fused_source",
    "cubed_fused_code_bytes", "cubed_fused_finish", "cubed_fused_finish_compiled", "cubed_combine_partials",
    "cubed_fused_finish_groups", "cubed_combine_groups", "cubed_fold_groups", "cubed_fold_groups_splits", "cubed_fold_groups_compiled",
    "cubed_blosc_header", "cubed_blosc_decompress", "cubed_blosc_max_compressed",
    "cubed_blosc_compress", "cubed_zstd_decompress", "cubed_lz4_chunk_decompress", "cubed_gemm_chain", "cubed_gemm_chain_path",
    "cubed_gemm_grid_check", "cubed_gemm_chain_grid", "cubed_gemm_pack_bytes", "cubed_gemm_chain_packed",
    "cubed_gemm_dist_image_bytes", "cubed_gemm_dist_pack_a", "cubed_gemm_dist_b_bytes", "cubed_gemm_dist_pack_b",
    "cubed_gemm_dist_gemm",
)


INCLUDE_DIRS = ";".join([os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc"),
                         os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")])


def jit_enabled() -> bool:
    """Runtime-specialised fused kernels (default).  CUBED_AMD_JIT=0 selects
    the ahead-of-time interpreter kernels instead (for comparison/debug)."""
    return os.environ.get("CUBED_AMD_JIT", "1") != "0"


def compile_program(prog: "Program"):
    """Compile (or fetch from the process cache) the specialised kernels of
    one fused program; returns the opaque handle."""
    h = c_void_p()
    check(lib().cubed_fused_compile(ctypes.byref(prog), INCLUDE_DIRS.encode(), ctypes.byref(h)),
          "cubed_fused_compile")
    return h


def program_source(handle) -> str:
    return lib().cubed_fused_source(handle).decode()
