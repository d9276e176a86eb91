"""Split a chunk program that exceeds the fused VM into several launches.

A fused program reads at most CUBED_MAX_LEAVES (4) inputs and runs at most
48 instructions over 6 registers (include/cubed_amd.h).  The reference has
no such limit: its chunk function is a numpy closure over any number of
chunks (primitive/blockwise.py:61-84).  Rather than refusing a pipeline such
as ``a * b + c * d + e`` (five inputs), the executor factors out
subexpressions that do fit, computes each into an HBM-resident temporary with
the task space's geometry (one extra fused launch over the same tasks), and
runs the remainder -- which now reads the temporary as one leaf -- as the
op's launch.  Values are unchanged: a subexpression is stored at its own
node dtype, which is exactly the rounding the fused evaluation applies to it
(every node is rounded to its dtype).

Supported: maps whose output space is the task space (out_axes identity) and
reductions whose inputs are single chunks at the task's own block (the
per-chunk stage of ``reduction``, core/ops.py:838-847).  A program drawing
from more than one random stream (the VM carries one Philox key per task)
materialises all but one stream the same way: ``mean(u * v)`` of two
unmaterialised ``random`` arrays (the reference's own quad_means test).  On
several GPUs the temporaries are block-cyclic like every array: the task
space's block grid is the temporary's, so each rank computes and reads only
the chunks of the tasks it owns (inputs it lacks are fetched first, as for
any pipeline), and the reduction rounds after a split per-chunk stage combine
across ranks as usual.  Anything else keeps raising LoweringError (there is
no host path).
"""

from __future__ import annotations

import itertools
from types import SimpleNamespace
from typing import Dict, List, Optional

from . import ir
from .lowering import LoweringError, collect_leaves, program_fits
from .primitive.types import CubedArrayProxy
from .storage import DeviceArray

_temp_ids = itertools.count()


def _nodes(e: ir.Expr, out: List[ir.Expr], seen: set):
    if id(e) in seen:
        return
    seen.add(id(e))
    for c in e.children():
        _nodes(c, out, seen)
    out.append(e)


def _pre_exprs(p: ir.ExprProgram) -> List[ir.Expr]:
    if p.reduce is None:
        return [e for _, e in p.output_items()]
    return [f.expr for f in p.reduce.fields]


def _with_pre(p: ir.ExprProgram, new: List[ir.Expr], nargs: int) -> ir.ExprProgram:
    import dataclasses

    if p.reduce is None:
        if p.structured:
            outs = tuple((n, e) for (n, _), e in zip(p.output_items(), new))
        else:
            outs = new[0]
        return dataclasses.replace(p, outputs=outs, nargs=nargs)
    fields = tuple(dataclasses.replace(f, expr=e) for f, e in zip(p.reduce.fields, new))
    return dataclasses.replace(p, reduce=dataclasses.replace(p.reduce, fields=fields), nargs=nargs)


def pick_subexpr(p: ir.ExprProgram) -> Optional[ir.Expr]:
    """The non-leaf subexpression with the most distinct leaves (>= 2) that
    fits the VM as a map program of its own."""
    pre = _pre_exprs(p)
    nodes, seen = [], set()
    for e in pre:
        _nodes(e, nodes, seen)
    best, best_key = None, None
    for e in nodes:
        if isinstance(e, ir.LEAF_TYPES):
            continue
        lv = collect_leaves([e])
        if len(lv) < 2 or any(not type(l) is ir.Arg for l in lv):
            continue
        sub = ir.ExprProgram(ndim=p.ndim, nargs=p.nargs, outputs=e, out_axes=tuple(range(p.ndim)),
                             name=f"{p.name}/part")
        if not program_fits(sub):
            continue
        k = (len(lv), len(collect_leaves_nodes(e)))
        if best_key is None or k > best_key:
            best, best_key = e, k
    if best is None:
        # one random stream per fused program (cubed_task_t carries one
        # Philox key): u * v of two unmaterialised random arrays
        # (test_core.py:540-570 quad_means) materialises all but one stream
        rnd = [l for l in collect_leaves(pre) if isinstance(l, ir.Philox)]
        if len(rnd) > 1:
            for e in nodes:
                if isinstance(e, ir.Philox) and _full_space(e, p.ndim):
                    return e
    return best


def _full_space(leaf, ndim: int) -> bool:
    return tuple(leaf.axes) == tuple(range(ndim))


def collect_leaves_nodes(e):
    out, seen = [], set()
    _nodes(e, out, seen)
    return out


def split_program(p: ir.ExprProgram, max_parts: int = 32):
    """[(subexpression program, its dtype)], remainder program: the parts
    are computed first, in order; part i is read by the remainder (and by
    later parts) as Arg(p.nargs + i) with identity axes."""
    parts = []
    cur = p
    nargs = p.nargs
    while not program_fits(cur):
        if len(parts) >= max_parts:
            raise LoweringError(f"{p.name}: chunk program too large to split into fused launches")
        e = pick_subexpr(cur)
        if e is None:
            raise LoweringError(f"{p.name}: chunk program exceeds the fused VM and has no part that fits")
        sub = ir.ExprProgram(ndim=cur.ndim, nargs=nargs, outputs=e, out_axes=tuple(range(cur.ndim)),
                             name=f"{p.name}/part{len(parts)}")
        parts.append((sub, e.dtype))
        new_leaf = ir.Arg(nargs, e.dtype, tuple(range(cur.ndim)))
        memo: Dict[int, ir.Expr] = {}
        pre = [_replace_node(x, id(e), new_leaf, memo) for x in _pre_exprs(cur)]
        nargs += 1
        cur = _with_pre(cur, pre, nargs)
    return parts, cur


def _replace_node(e: ir.Expr, target_id: int, new: ir.Expr, memo: Dict[int, ir.Expr]) -> ir.Expr:
    if id(e) == target_id:
        return new
    if id(e) in memo:
        return memo[id(e)]
    if isinstance(e, ir.LEAF_TYPES):
        out = e
    else:
        ch = tuple(_replace_node(c, target_id, new, memo) for c in e.children())
        out = e.with_children(ch) if any(a is not b for a, b in zip(ch, e.children())) else e
    memo[id(e)] = out
    return out


def _space_geometry(ex, program: ir.ExprProgram, cfg, target: DeviceArray, keys):
    """(shape, chunks, key -> temp block coords) of the task space."""
    if program.reduce is None:
        if tuple(program.out_axes) != tuple(range(program.ndim)) or target.ndim != program.ndim:
            raise LoweringError("split: map output is not the task space")
        return target.shape, target.chunks, {tuple(k): tuple(k) for k in keys}
    # a reduction over single chunks: the space is an input array's geometry
    ident = tuple(range(program.ndim))
    ref = None
    for leaf in collect_leaves(_pre_exprs(program)):
        if type(leaf) is ir.Arg and tuple(leaf.axes) == ident:  # any field: same geometry
            ref = leaf
            break
    if ref is None:
        # only random inputs: the random array's own blocks are the space
        for leaf in collect_leaves(_pre_exprs(program)):
            if isinstance(leaf, ir.Philox) and tuple(leaf.axes) == ident:
                coords = {}
                for k in keys:
                    a = cfg.block_function(("out",) + tuple(k))[leaf.block_arg]
                    coords[tuple(k)] = tuple(a[1:])
                shape = tuple(int(sum(c)) for c in leaf.chunks)
                return shape, tuple(tuple(c) for c in leaf.chunks), coords
        raise LoweringError("split: no full-space input defines the reduction's space")
    coords = {}
    arr = None
    for k in keys:
        a = cfg.block_function(("out",) + tuple(k))[ref.index]
        if not (isinstance(a, tuple) and a and isinstance(a[0], str)):
            raise LoweringError("split: a reduction input is not a single chunk per task")
        arr = ex.device_source(cfg.reads_map[a[0]].array)
        coords[tuple(k)] = tuple(a[1:])
    return arr.shape, arr.chunks, coords


def split_launches(ex, program: ir.ExprProgram, cfg, target: DeviceArray, keys):
    """Launches computing ``program`` over ``keys`` as several fused
    programs through HBM temporaries (see the module docstring)."""
    parts, rest = split_program(program)
    shape, chunks, coords = _space_geometry(ex, program, cfg, target, keys)
    launches = []
    temps = []
    orig_bf = cfg.block_function
    reads = dict(cfg.reads_map)
    for sub, dt in parts:
        name = f"split-{next(_temp_ids)}"
        T = DeviceArray(shape, dt, chunks, name=name)
        ex.own(T)  # fits next to the plan? then it lives as long as the cached launches
        ex.allocate(T)
        # several GPUs: the temporary is block-cyclic like every array; the
        # chunk a task writes must be one this rank holds (it is when the
        # space's block grid is the task grid: the same C-order offsets)
        for k in keys:
            if T.owner(coords[tuple(k)]) != ex.rank:
                raise LoweringError(f"{program.name}: split temporary chunk {coords[tuple(k)]} of task {k} "
                                    f"lives on rank {T.owner(coords[tuple(k)])}")
        prev = list(temps)

        def bf_sub(out_key, _prev=prev, _inv={v: k for k, v in coords.items()}):
            k = _inv[tuple(out_key[1:])]
            return list(orig_bf(("out",) + k)) + [(t.name,) + coords[k] for t in _prev]

        sub_cfg = SimpleNamespace(block_function=bf_sub, reads_map=dict(reads))
        tkeys = sorted(set(coords.values()))
        launches += _lower(ex, sub, sub_cfg, T, tkeys)
        reads[name] = CubedArrayProxy(T, T.chunks)
        temps.append(T)

    def bf_rest(out_key, _temps=tuple(temps)):
        k = tuple(out_key[1:])
        return list(orig_bf(out_key)) + [(t.name,) + coords[k] for t in _temps]

    rest_cfg = SimpleNamespace(block_function=bf_rest, reads_map=reads)
    launches += _lower(ex, rest, rest_cfg, target, keys)
    return launches


def _lower(ex, program, cfg, target, keys):
    from .runtime.executors.gpu import _with_gathers

    return _with_gathers(ex.lowerer.lower_expr_pipeline(program, cfg, target, list(keys)), ex.device)
