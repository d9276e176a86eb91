"""The C-ABI library (include/cubed_amd.h) loads and matches its header (CPU).

No compute entry point is called here (there is no GPU in the build
container); the struct layouts the host writes into the task tables are
checked against the C compiler's view of the header, and every function the
header declares must be exported by libcubed_amd.so.
"""

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cubed_amd.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b(cubed_\w+)\s*\(", src)))


def test_header_declares_entry_points():
    fns = header_functions()
    for f in ("cubed_fused_chunks", "cubed_copy_boxes", "cubed_random_chunks", "cubed_gemm_chain"):
        assert f in fns


def test_library_exports_every_header_symbol(built):
    from cubed_amd import _native as nat

    lib = ctypes.CDLL(nat.LIB_PATH)
    for f in header_functions():
        assert hasattr(lib, f), f"{f} declared in include/cubed_amd.h but not exported"
    assert set(nat.EXPORTED_SYMBOLS) <= set(header_functions())


def test_library_loads_through_binding(built):
    from cubed_amd import _native as nat

    L = nat.lib()
    assert L.cubed_abi_version() == nat.ABI_VERSION


def test_workspace_query_is_host_only(built):
    """cubed_fused_workspace_bytes is pure host logic: callable without a GPU."""
    from cubed_amd import _native as nat

    P = nat.Program()
    P.ndim, P.nred, P.mode, P.nleaves, P.nfields, P.nouts = 2, 1, 0, 1, 1, 1
    n = nat.lib().cubed_fused_workspace_bytes(ctypes.byref(P), 1, 1 << 20, 1 << 12)
    assert n >= 0


def test_fold_split_counts_are_host_only(built):
    """cubed_fold_groups_splits (ABI 13): few groups of many elements are cut
    into runs of >= 512 SoA entries, toward 1024 workgroups; many groups or
    small ones are not split."""
    from cubed_amd import _native as nat

    f = nat.lib().cubed_fold_groups_splits
    assert f(1, 10, 72000) == 1024         # 720000 entries: 1024 runs
    assert f(1, 720, 136) == 191           # the vorticity fold: 97920 entries, runs of >= 512
    assert f(1, 8, 136) == 2
    assert f(100, 1000, 1000) == 11        # ~1024 workgroups over 100 groups
    assert f(600, 1000, 1000) == 1         # >= 512 groups: one workgroup each
    assert f(1, 1, 1000) == 1              # one short row


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "cubed_amd.h"
#define P(T, F) printf(#T "." #F " %zu\n", offsetof(T, F))
#define S(T) printf(#T " %zu\n", sizeof(T))
int main(void) {
  S(cubed_insn_t); S(cubed_program_t); S(cubed_task_t); S(cubed_box_t);
  P(cubed_program_t, insns); P(cubed_program_t, epi); P(cubed_program_t, consts);
  P(cubed_program_t, leaf_kind); P(cubed_program_t, out_dtype); P(cubed_program_t, ninsns);
  P(cubed_task_t, leaf_base); P(cubed_task_t, leaf_stride); P(cubed_task_t, out_base);
  P(cubed_task_t, out_stride); P(cubed_task_t, key_lo); P(cubed_task_t, block_offset);
  P(cubed_box_t, src_stride); P(cubed_box_t, dst_stride);
  S(cubed_gemm_chain_t); S(cubed_gemm_seg_t);
  P(cubed_gemm_chain_t, seg0); P(cubed_gemm_chain_t, ktot); P(cubed_gemm_chain_t, accumulate);
  P(cubed_gemm_seg_t, k); P(cubed_gemm_seg_t, ldb);
  return 0;
}
"""


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("abi")
    src = d / "layout.c"
    src.write_text(LAYOUT_C)
    exe = d / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return {k: int(v) for k, v in (line.split() for line in out.splitlines())}


def test_header_is_plain_c(c_layout):
    assert c_layout["cubed_task_t"] > 0


def test_struct_layouts_match_binding(c_layout):
    from cubed_amd import _native as nat

    assert ctypes.sizeof(nat.Insn) == c_layout["cubed_insn_t"]
    assert ctypes.sizeof(nat.Program) == c_layout["cubed_program_t"]
    for f in ("insns", "epi", "consts", "leaf_kind", "out_dtype", "ninsns"):
        assert getattr(nat.Program, f).offset == c_layout[f"cubed_program_t.{f}"], f
    assert nat.TASK_DTYPE.itemsize == c_layout["cubed_task_t"]
    for f in ("leaf_base", "leaf_stride", "out_base", "out_stride", "key_lo", "block_offset"):
        assert nat.TASK_DTYPE.fields[f][1] == c_layout[f"cubed_task_t.{f}"], f
    assert nat.BOX_DTYPE.itemsize == c_layout["cubed_box_t"]
    for f in ("src_stride", "dst_stride"):
        assert nat.BOX_DTYPE.fields[f][1] == c_layout[f"cubed_box_t.{f}"], f
    assert nat.CHAIN_DTYPE.itemsize == c_layout["cubed_gemm_chain_t"]
    for f in ("seg0", "ktot", "accumulate"):
        assert nat.CHAIN_DTYPE.fields[f][1] == c_layout[f"cubed_gemm_chain_t.{f}"], f
    assert nat.SEG_DTYPE.itemsize == c_layout["cubed_gemm_seg_t"]
    for f in ("k", "ldb"):
        assert nat.SEG_DTYPE.fields[f][1] == c_layout[f"cubed_gemm_seg_t.{f}"], f


def _chain(m, n, ks, lda=None, ldb=None, align=0):
    from cubed_amd import _native as nat

    segs = np.zeros(len(ks), dtype=nat.SEG_DTYPE)
    for i, k in enumerate(ks):
        segs[i] = (4096 * (i + 1) + align, 1 << 20, k, lda or k, ldb or n, 0)
    tasks = np.zeros(1, dtype=nat.CHAIN_DTYPE)
    tasks[0] = (1 << 24, m, n, n, 0, len(ks), sum(ks), 0)
    return tasks, segs


@pytest.mark.parametrize("case,in_dt,out_dt,expect", [
    (dict(m=5000, n=5000, ks=[5000] * 8), "bf16", "bf16", 1),    # config 5, bf16
    (dict(m=5000, n=5000, ks=[5000] * 8), "bf16", "f32", 1),
    (dict(m=5000, n=5000, ks=[5000] * 8), "f32", "f32", 1),      # config 5, f32
    (dict(m=100, n=100, ks=[100, 60]), "bf16", "bf16", 0),       # a segment shorter than BK=64
    (dict(m=100, n=100, ks=[100, 100]), "f32", "f32", 1),         # f32: BK = 32
    (dict(m=100, n=101, ks=[104]), "bf16", "bf16", 0),           # ragged n: no 16-B rows
    (dict(m=100, n=96, ks=[100]), "bf16", "bf16", 0),            # k % 8 != 0
    (dict(m=100, n=96, ks=[104], align=8), "bf16", "bf16", 0),   # operand not 16-B aligned
    (dict(m=64, n=64, ks=[64]), "f64", "f64", 0),                # f64 / int64: element kernel
])
def test_gemm_chain_path_selection(built, case, in_dt, out_dt, expect):
    """cubed_gemm_chain_path is pure host logic: which kernel a chain set
    would take (the MFMA tiles' alignment / segment-length preconditions)."""
    from cubed_amd import _native as nat

    codes = {"bf16": 12, "f32": 9, "f64": 10}
    tasks, segs = _chain(case["m"], case["n"], case["ks"], align=case.get("align", 0))
    got = nat.lib().cubed_gemm_chain_path(tasks.ctypes.data, len(tasks), segs.ctypes.data,
                                          codes[in_dt], codes[out_dt])
    assert got == expect


def _product_grid(ti, tj, cm, cn, ks, last_m=None, last_n=None):
    """Tables of ONE chunked product: task (I, J), segment s = A(I, s) @ B(s, J)."""
    from cubed_amd import _native as nat

    ns = len(ks)
    tasks = np.zeros(ti * tj, dtype=nat.CHAIN_DTYPE)
    segs = np.zeros(ti * tj * ns, dtype=nat.SEG_DTYPE)
    for I in range(ti):
        for J in range(tj):
            t = I * tj + J
            m = last_m if (I == ti - 1 and last_m) else cm
            n = last_n if (J == tj - 1 and last_n) else cn
            tasks[t] = ((1 << 30) + t * (1 << 24), m, n, n, t * ns, ns, sum(ks), 0)
            for s, k in enumerate(ks):
                segs[t * ns + s] = ((1 << 32) + (I * ns + s) * (1 << 24), (1 << 36) + (s * tj + J) * (1 << 24),
                                    k, k, n, 0)
    return tasks, segs


CTR = 8 * 128  # the bf16 GEMM's per-XCD round counters after the two images


def test_gemm_pack_bytes(built):
    """cubed_gemm_pack_bytes (host logic): the packed path's workspace is
    (256-row panels over M + 256-column panels over N) x k blocks -- bf16
    64-k tiles of 32 KiB, f32 16-k steps of 16 KiB; sets that are not one
    chunked product of a regular grid, or not bf16 / f32, are refused with a
    negative code."""
    from cubed_amd import _native as nat
    from cubed_amd import ir

    L_ = nat.lib()
    bf, f32 = ir.dtype_code(ir.bfloat16), ir.dtype_code(np.float32)
    tasks, segs = _product_grid(8, 8, 5000, 5000, [5000] * 8)  # config 5
    args = (tasks.ctypes.data, 8, 8, segs.ctypes.data, len(segs))
    assert L_.cubed_gemm_pack_bytes(*args, bf, bf) == (157 + 157) * 625 * 32768 + CTR  # + round counters
    assert L_.cubed_gemm_pack_bytes(*args, bf, f32) == (157 + 157) * 625 * 32768 + CTR
    assert L_.cubed_gemm_pack_bytes(*args, f32, f32) == (157 + 157) * 2500 * 16384 + CTR  # f32: 16-k steps of 16 KiB
    assert L_.cubed_gemm_pack_bytes(*args, ir.dtype_code(np.float64), ir.dtype_code(np.float64)) < 0
    tasks, segs = _product_grid(3, 2, 300, 256, [520, 520, 104], last_m=100, last_n=136)
    args = (tasks.ctypes.data, 3, 2, segs.ctypes.data, len(segs))
    assert L_.cubed_gemm_pack_bytes(*args, bf, bf) == (3 + 2) * 18 * 32768 + CTR  # M 700, N 392, K 1144
    segs["a"][len(segs) - 1] += 4096  # task (2, 1) reads another A chunk than (2, 0)
    assert L_.cubed_gemm_pack_bytes(*args, bf, bf) < 0
    assert b"not one chunked product" in L_.cubed_last_error()


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No CPU fallback: a missing extension is an error, not a silent path."""
    from cubed_amd import _native as nat

    monkeypatch.setattr(nat, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(nat, "_lib", None)
    with pytest.raises(nat.NativeError):
        nat.lib()


def test_product_library_has_no_vendor_blas(built):
    """One GEMM path: the product library links no rocBLAS / hipBLASLt and
    exports no library-comparator entry points."""
    from cubed_amd import _native as nat

    out = subprocess.run(["ldd", nat.LIB_PATH], capture_output=True, text=True).stdout
    assert "rocblas" not in out and "hipblas" not in out
    lib = ctypes.CDLL(nat.LIB_PATH)
    for f in ("cubed_gemm_batched", "cubed_gemm_chunks"):
        assert not hasattr(lib, f)


def test_no_environment_switches_in_kernels():
    """The C library's launch paths read no environment variables (no A/B
    switch can silently change the kernel that runs)."""
    csrc = os.path.join(ROOT, "cubed_amd", "csrc")
    for name in os.listdir(csrc):
        if name.endswith((".hip", ".h", ".cpp")):
            assert "getenv" not in open(os.path.join(csrc, name)).read(), name
