"""The fused-program code generator (lowering.Codegen) against a direct
numpy evaluation: random expression DAGs over 3 leaves (shared
subexpressions, WHERE, one or two outputs) are compiled to two-address VM
code, the code is interpreted on the host with numpy ops in place of the
kernels' register ops, and every output register must hold the expression's
value.  Guards the register handover (a leaf or common subexpression at its
last use is computed in place) against clobbering an operand that is still
pending or an output already produced.  CPU only; no kernel runs."""
import random

import numpy as np

from cubed_amd import ir
from cubed_amd.lowering import _OPCODES, V_F64, Codegen, LoweringError

UNARY_BY_CODE = {v: k for k, v in ir.UNARY_OPS.items() if v is not None}
BINARY_BY_CODE = {v: k for k, v in ir.BINARY_OPS.items()}
NP_UNARY = {"negative": np.negative, "abs": np.abs, "exp": np.exp}
NP_BINARY = {"add": np.add, "subtract": np.subtract, "multiply": np.multiply,
             "maximum": np.maximum, "less": np.less}
F8 = np.dtype("f8")


def rand_expr(leaves, depth, rng):
    """A random expression DAG (leaves are shared objects: CSE and reuse)."""
    if depth == 0 or rng.random() < 0.25:
        return rng.choice(leaves)
    k = rng.random()
    if k < 0.25:
        return ir.Unary(rng.choice(list(NP_UNARY)), rand_expr(leaves, depth - 1, rng), F8)
    if k < 0.8:
        op = rng.choice(["add", "subtract", "multiply", "maximum"])
        return ir.Binary(op, rand_expr(leaves, depth - 1, rng), rand_expr(leaves, depth - 1, rng), F8)
    c = ir.Binary("less", rand_expr(leaves, depth - 1, rng), rand_expr(leaves, depth - 1, rng),
                  np.dtype("bool"))
    return ir.Where(c, rand_expr(leaves, depth - 1, rng), rand_expr(leaves, depth - 1, rng), F8)


def evaluate(e, vals):
    if isinstance(e, ir.Arg):
        return vals[e.index]
    if isinstance(e, ir.Unary):
        return NP_UNARY[e.op](evaluate(e.x, vals))
    if isinstance(e, ir.Binary):
        return NP_BINARY[e.op](evaluate(e.a, vals), evaluate(e.b, vals)).astype(float)
    return np.where(evaluate(e.c, vals) != 0, evaluate(e.a, vals), evaluate(e.b, vals))


def run(code, regs):
    """Interpret two-address VM code (vm.h run_vm) with numpy ops."""
    for op, a, b, c, _t, _imm in code:
        if op == _OPCODES["MOV"]:
            regs[a] = regs[b].copy()
        elif op == _OPCODES["WHERE"]:
            regs[a] = np.where(regs[c] != 0, regs[a], regs[b])
        elif op == _OPCODES["CAST"]:
            pass  # f64 values in f64 registers
        elif op in BINARY_BY_CODE:
            regs[a] = NP_BINARY[BINARY_BY_CODE[op]](regs[a], regs[b]).astype(float)
        else:
            regs[a] = NP_UNARY[UNARY_BY_CODE[op]](regs[a])


def test_codegen_matches_numpy_on_random_programs():
    rng = random.Random(5)
    tried = 0
    with np.errstate(all="ignore"):
        for trial in range(1500):
            leaves = [ir.Arg(i, np.dtype("f8"), (0,)) for i in range(3)]
            outs = [rand_expr(leaves, 4, rng) for _ in range(rng.choice([1, 2]))]
            lr = {}
            for e in outs:
                for lf in ir.leaves(e):
                    lr[id(lf)] = lf.index
            cg = Codegen(V_F64, lr)
            cg.count_uses(outs)
            try:
                regs_out = []
                for e in outs:
                    r, _ = cg.gen(e)
                    cg.pin(r)
                    regs_out.append(r)
            except LoweringError:
                continue  # needs more than the VM's registers: split.py's case
            tried += 1
            vals = [np.random.default_rng(trial).standard_normal(8) for _ in range(3)]
            regs = {i: vals[i].copy() for i in range(3)}
            for i in range(3, 6):
                regs[i] = np.full(8, np.nan)
            run(cg.code, regs)
            for e, r in zip(outs, regs_out):
                assert np.array_equal(regs[r], evaluate(e, vals), equal_nan=True), (trial, e)
    assert tried > 500


def test_common_subexpression_handed_over_at_last_use():
    """t = exp(x0) is used twice: first as the left operand of t * x1 (it
    stays cached, so that use copies it), last as the left operand of
    t - x2: handed over in place, no second MOV."""
    x = [ir.Arg(i, F8, (0,)) for i in range(3)]
    t = ir.Unary("exp", x[0], F8)
    out = ir.Binary("add", ir.Binary("multiply", t, x[1], F8), ir.Binary("subtract", t, x[2], F8), F8)
    cg = Codegen(V_F64, {id(a): a.index for a in x})
    cg.count_uses([out])
    r, _ = cg.gen(out)
    movs = [c for c in cg.code if c[0] == _OPCODES["MOV"]]
    assert len(movs) == 1, cg.code
    vals = [np.linspace(-1, 1, 8) * (i + 1) for i in range(3)]
    regs = {i: vals[i].copy() for i in range(3)}
    for i in range(3, 6):
        regs[i] = np.full(8, np.nan)
    run(cg.code, regs)
    assert np.array_equal(regs[r], np.exp(vals[0]) * vals[1] + (np.exp(vals[0]) - vals[2]))
