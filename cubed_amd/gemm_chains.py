"""Matmul k-sum fusion (an executor-side optimization of the plan).

The reference's ``matmul`` (cubed/array_api/linear_algebra_functions.py
:13-59) is two stages: a blockwise op over (i, k, j) whose every task is one
chunk product ``A_ik @ B_kj`` written as a (m, 1, n) partial (``_matmul``
:62-64), then ``_sum_wo_cat`` (:67-78), a sum reduction over the k axis that
reads those partials back (merge_chunks rounds + ``_chunk_sum``).  At BASELINE
config 5 (40000^2 in 5000^2 chunks) the partial-product array alone is
51.2 GB of f32, written once and read once more per reduction round.

On the MI355X the whole thing is one launch of chained chunk GEMMs
(``cubed_gemm_chain``): for every OUTPUT chunk (i, j) one task walks
k = 0, 1, ... in a single continuous K loop over the segment pairs
(A_ik, B_kj), so the partial products never exist.  This pass recognises the
pattern in the finalized DAG -- the GEMM node (a plain MatmulProgram, or the
optimizer's GemmThenProgram whose ``then`` is the per-chunk ``_chunk_sum``
over the unit k dim) followed by reduction nodes that only sum over the k
axis -- and hands the executor a ``GemmChain`` in place of those nodes.

Legality: the reference sums f32 chunk products in f32 (each product rounded
to f32, then ``np.sum(..., dtype=f32)`` over k); here the sum is one f32
accumulation chain through the MFMA accumulators -- a different association
of the same f32 sum, within the error bound the tests state
(tests/test_gpu_matmul.py).  Task bookkeeping (a TaskEndEvent per original
pipeline) is unchanged.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from types import SimpleNamespace
from typing import Dict, List, Optional

import numpy as np

from . import ir
from .primitive.blockwise import apply_blockwise
from .storage import DeviceArray

K_AXIS = 1  # matmul of 2-d operands: blockwise output (i, k, j)


@dataclass
class GemmChain:
    nodes: List[str]              # the GEMM node, then the k-sum reduction nodes
    gemm: ir.MatmulProgram
    gemm_spec: object             # block_function / reads_map of the (i, k, j) tasks
    gemm_target: DeviceArray      # the (M, nk, N) partial-product geometry
    final_target: DeviceArray     # (M, N) or (M, 1, N): sum over k
    first_spec: object = None     # the GEMM node's BlockwiseSpec (cache key)
    extra_targets: List[DeviceArray] = field(default_factory=list)  # never materialised


def _is_ksum(p, src_leaf_ok) -> Optional[ir.ReduceField]:
    """The program if it is ``sum over the k axis`` of one input (the
    ``_chunk_sum`` of linear_algebra_functions.py:77-78, with or without a
    merge region and a squeeze), else None.  A complex k-sum split into its
    parts (rewrites.split_complex: fields ``v#re`` / ``v#im`` over the
    input's real / imag slabs, output {real, imag}) counts too."""
    if isinstance(p, ir.ExprProgram) and p.reduce is not None and p.structured:
        return _is_split_complex_ksum(p, src_leaf_ok)
    if not isinstance(p, ir.ExprProgram) or p.reduce is None or p.structured:
        return None
    if tuple(p.reduce.axes) != (K_AXIS,) or p.ndim != 3 or len(p.reduce.fields) != 1:
        return None
    f = p.reduce.fields[0]
    if f.rop != "sum" or not src_leaf_ok(f.expr):
        return None
    if not (isinstance(p.outputs, ir.Field) and p.outputs.name == f.name):
        return None
    if np.dtype(p.outputs.dtype) != np.dtype(f.dtype) or np.dtype(f.expr.dtype) != np.dtype(f.dtype):
        return None
    return f


def _is_split_complex_ksum(p, src_leaf_ok):
    if tuple(p.reduce.axes) != (K_AXIS,) or p.ndim != 3 or len(p.reduce.fields) != 2:
        return None
    re, im = p.reduce.fields
    if not (re.name.endswith("#re") and im.name == re.name[:-3] + "#im"):
        return None
    for f, part in ((re, "real"), (im, "imag")):
        if f.rop != "sum" or not src_leaf_ok(f.expr) or getattr(f.expr, "field", None) != part:
            return None
        if np.dtype(f.expr.dtype) != np.dtype(f.dtype):
            return None
    outs = dict(p.outputs)
    if set(outs) != {"real", "imag"}:
        return None
    if not all(isinstance(outs[k], ir.Field) and outs[k].name == f.name
               for k, f in (("real", re), ("imag", im))):
        return None
    return re


def find_gemm_chains(dag, array_names) -> Dict[str, GemmChain]:
    nodes = dict(dag.nodes(data=True))
    requested = set(array_names or ())
    out = {}
    for n in dag.nodes():
        d = nodes[n]
        if "pipeline" not in d or d["pipeline"].function is not apply_blockwise:
            continue
        cfg = d["pipeline"].config
        prog = cfg.function
        extra = []
        if isinstance(prog, ir.MatmulProgram):
            gemm, gspec, gtarget = prog, cfg, cfg.write.array
        elif isinstance(prog, ir.GemmThenProgram) and isinstance(prog.gemm, ir.MatmulProgram):
            if _is_ksum(prog.then, lambda e: isinstance(e, ir.Arg) and e.index == 0) is None:
                continue
            gtarget = prog.gemm_target
            if gtarget.ndim != 3 or gtarget.chunks[K_AXIS] != 1:
                continue
            gemm = prog.gemm
            gspec = SimpleNamespace(block_function=prog.gemm_block_function, reads_map=prog.gemm_reads)
            extra.append(gtarget)
        else:
            continue
        if not isinstance(gtarget, DeviceArray) or gtarget.ndim != 3:
            continue
        members = [n]
        cur = n
        final = None
        while True:
            outs = list(dag.successors(cur))
            if len(outs) != 1:
                break
            arr = outs[0]
            t = nodes[arr].get("target")
            if not isinstance(t, DeviceArray) or t.ndim not in (2, 3):
                break
            if t.ndim == 2 or t.numblocks[K_AXIS] == 1:
                final = t  # summed over k: the chain's output
                break
            # still split along k: it must feed exactly one k-sum round
            if arr in requested or dag.out_degree(arr) != 1:
                break
            nxt = next(iter(dag.successors(arr)))
            nd = nodes[nxt]
            if "pipeline" not in nd or nd["pipeline"].function is not apply_blockwise:
                break
            if _is_ksum(nd["pipeline"].config.function,
                        lambda e, src=t: isinstance(e, ir.Region) and e.target is src) is None:
                break
            members.append(nxt)
            extra.append(t)
            cur = nxt
        if final is None or (len(members) < 2 and not extra):
            continue
        out[n] = GemmChain(members, gemm, gspec, gtarget, final, cfg, extra)
    return out


def chain_tables(ex, chain: GemmChain, keys):
    """(tasks, segs, in dtype, out dtype) of the cubed_gemm_chain launch for
    the final-output blocks ``keys`` (2-d (i, j) or 3-d (i, 0, j))."""
    from . import _native as nat
    from .lowering import LoweringError

    F = chain.final_target
    G = chain.gemm_target
    nk = G.numblocks[K_AXIS]
    tasks = np.zeros(len(keys), dtype=nat.CHAIN_DTYPE)
    segs = np.zeros(len(keys) * nk, dtype=nat.SEG_DTYPE)
    in_dt = None
    si = 0
    for t, key in enumerate(keys):
        i, j = key[0], key[-1]
        m, n = F.chunk_extent(key)[0], F.chunk_extent(key)[-1]
        ktot = 0
        for k in range(nk):
            args = chain.gemm_spec.block_function(("out", i, k, j))
            a_key, b_key = args[0], args[1]
            A = ex.device_source(chain.gemm_spec.reads_map[a_key[0]].array)
            B = ex.device_source(chain.gemm_spec.reads_map[b_key[0]].array)
            if A.ndim != 2 or B.ndim != 2:
                raise LoweringError("chained GEMM needs 2-d operands")
            if A.dtype != B.dtype:
                raise LoweringError(f"matmul of {A.dtype} x {B.dtype} is not lowered")
            if in_dt is None:
                in_dt = A.dtype
            elif A.dtype != in_dt:
                raise LoweringError("operand dtypes differ between chunks")
            am, ak = A.chunk_extent(a_key[1:])
            bk, bn = B.chunk_extent(b_key[1:])
            if ak != bk or am != m or bn != n:
                raise LoweringError("operand chunks do not match the output chunk")
            segs[si] = (A.chunk_addr(a_key[1:]), B.chunk_addr(b_key[1:]), ak, ak, bn, 0)
            si += 1
            ktot += ak
        tasks[t] = (F.chunk_addr(key), m, n, n, t * nk, nk, ktot, 0)
    return tasks, segs[:si], in_dt, F.dtype


def complex_chain_tables(ex, chain: GemmChain, keys):
    """Complex matmul as real chained GEMMs over the part slabs
    (cubed_amd/complex.py's SoA layout): for every output chunk two tasks,

        C.real = sum_k Ar_k Br_k + sum_k Ai_k (-Bi_k)
        C.imag = sum_k Ar_k Bi_k + sum_k Ai_k Br_k

    each one K loop over 2 nk segments, so the four real products of
    numpy's complex dot (linear_algebra_functions.py:62-64 on complex
    chunks) run on the f32 MFMA kernel (complex64) or the f64 element kernel
    (complex128).  -Bi is one negated copy of B's imaginary slab per chunk
    (a map launch, returned in ``pre``).  Returns (pre launches, tasks,
    segs, part dtype, part dtype)."""
    from types import SimpleNamespace

    from . import _native as nat
    from .complex import is_complex, part_dtype
    from .lowering import LoweringError
    from .primitive.types import CubedArrayProxy

    F = chain.final_target
    G = chain.gemm_target
    nk = G.numblocks[K_AXIS]
    pdt = part_dtype(F.dtype)
    negs = {}
    pre = []

    def neg_imag(B):
        """Device array holding -B.imag (same chunk grid), made once."""
        if id(B) in negs:
            return negs[id(B)]
        T = DeviceArray(B.shape, part_dtype(B.dtype), B.chunks, name=f"{B.name}-negimag")
        ex.own(T)
        ex.allocate(T)
        axes = tuple(range(B.ndim))
        prog = ir.ExprProgram(ndim=B.ndim, nargs=1,
                              outputs=ir.Unary("negative", ir.Arg(0, np.dtype(T.dtype), axes, "imag"),
                                               np.dtype(T.dtype)),
                              out_axes=axes, name="neg_imag")
        cfg = SimpleNamespace(block_function=lambda out_key, _n=B.name: [(_n,) + tuple(out_key[1:])],
                              reads_map={B.name: CubedArrayProxy(B, B.chunks)})
        import itertools

        tkeys = list(itertools.product(*[range(n) for n in B.numblocks]))
        from .runtime.executors.gpu import _with_gathers

        pre.extend(_with_gathers(ex.lowerer.lower_expr_pipeline(prog, cfg, T, tkeys), ex.device))
        negs[id(B)] = T
        return T

    tasks = np.zeros(2 * len(keys), dtype=nat.CHAIN_DTYPE)
    segs = np.zeros(2 * len(keys) * 2 * nk, dtype=nat.SEG_DTYPE)
    si = 0
    for t, key in enumerate(keys):
        i, j = key[0], key[-1]
        m, n = F.chunk_extent(key)[0], F.chunk_extent(key)[-1]
        pairs = []
        for k in range(nk):
            args = chain.gemm_spec.block_function(("out", i, k, j))
            a_key, b_key = args[0], args[1]
            A = ex.device_source(chain.gemm_spec.reads_map[a_key[0]].array)
            B = ex.device_source(chain.gemm_spec.reads_map[b_key[0]].array)
            if A.ndim != 2 or B.ndim != 2:
                raise LoweringError("chained GEMM needs 2-d operands")
            if not (is_complex(A.dtype) and is_complex(B.dtype) and A.dtype == B.dtype == F.dtype):
                raise LoweringError(f"matmul of {A.dtype} x {B.dtype} -> {F.dtype} is not lowered "
                                    "(complex operands of the output's dtype)")
            am, ak = A.chunk_extent(a_key[1:])
            bk, bn = B.chunk_extent(b_key[1:])
            if ak != bk or am != m or bn != n:
                raise LoweringError("operand chunks do not match the output chunk")
            pairs.append((A, a_key[1:], B, b_key[1:], ak))
        for part in ("real", "imag"):
            seg0, ktot = si, 0
            for A, ac, B, bc, kk in pairs:  # Ar x (Br | Bi)
                b = B.chunk_addr(bc, "real" if part == "real" else "imag")
                segs[si] = (A.chunk_addr(ac, "real"), b, kk, kk, B.chunk_extent(bc)[1], 0)
                si += 1
                ktot += kk
            for A, ac, B, bc, kk in pairs:  # Ai x (-Bi | Br)
                b = neg_imag(B).chunk_addr(bc) if part == "real" else B.chunk_addr(bc, "real")
                segs[si] = (A.chunk_addr(ac, "imag"), b, kk, kk, B.chunk_extent(bc)[1], 0)
                si += 1
                ktot += kk
            tasks[2 * t + (part == "imag")] = (F.chunk_addr(key, part), m, n, n, seg0, 2 * nk, ktot, 0)
    return pre, tasks, segs[:si], pdt, pdt
