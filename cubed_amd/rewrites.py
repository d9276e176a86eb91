"""Executor-side rewrites of a finalized DAG that remove whole passes over
HBM without changing any value.

``elide_rechunks``: a rechunk (cubed/core/ops.py:702-758 ->
primitive/rechunk.py:23-98, one copy op or two through an intermediate)
whose result feeds exactly ONE blockwise op and is not requested is not
materialised.  The consumer reads the rechunk's SOURCE instead: each of its
tasks reads the box its input chunk covers, as a ``Region`` of the source
(the same leaf kind as ``index``/``merge_chunks``' map_direct regions,
core/ops.py:374-517, 646-699).  The lowering cuts such tasks at the source
chunk boundaries into pieces that read in place (lowering.task_pieces); a
reduction combines its pieces' partials before the epilogue.  Rechunk is a
pure layout change (values bit-identical), so the consumer computes the same
elementwise values; reductions regroup their per-field sums at the source's
chunk boundaries (within the DESIGN.md tolerances).

The copy (2 x the array in HBM traffic) and the consumer's re-read of the
copy disappear: ``rechunk + mean`` reads the source once.
"""

from __future__ import annotations

import dataclasses
from typing import List

from . import ir
from .primitive.blockwise import apply_blockwise
from .primitive.rechunk import copy_read_to_write
from .primitive.types import CubedArrayProxy
from .storage import DeviceArray


def _box_of(grid):
    def region(block_id):
        return tuple(slice(s, s + e) for s, e in zip(grid.chunk_start(block_id), grid.chunk_extent(block_id)))
    return region


def elide_rechunks(dag, array_names):
    """Returns (rewritten DAG copy, elided targets)."""
    import networkx as nx

    from .chains import _arg_arrays
    from .core.optimization import predecessors

    requested = set(array_names or ())
    dag = dag.copy()
    elided: List = []
    for name in list(nx.topological_sort(dag)):
        if name not in dag:
            continue
        nd = dag.nodes[name]
        if "pipeline" not in nd or nd["pipeline"].function is not apply_blockwise:
            continue
        spec = nd["pipeline"].config
        program = spec.function
        if not isinstance(program, ir.ExprProgram):
            continue
        target = nd["primitive_op"].target_array
        args_names = _arg_arrays(spec, target)
        if args_names is None:
            continue
        sample = spec.block_function(("out",) + (0,) * len(getattr(target, "numblocks", ())))
        for i, yname in enumerate(args_names):
            if yname not in dag or yname in requested or dag.out_degree(yname) != 1:
                continue
            if not isinstance(sample[i], tuple):
                continue  # the consumer reads several chunks per task: keep the rechunk
            if any(isinstance(l, ir.ReshapeArg) and l.index == i for l in ir.leaves_of_program(program)):
                continue  # a chunk reshape needs the rechunked chunk's bytes in C order
            # walk back through the rechunk's copy op(s): y <- R [<- int <- R1] <- x
            removed, cur, x_name, x_target = [], yname, None, None
            while True:
                pres = list(predecessors(dag, cur))
                if len(pres) != 1:
                    break
                op = pres[0]
                od = dag.nodes[op]
                if "pipeline" not in od or od["pipeline"].function is not copy_read_to_write:
                    break
                srcs = [p for p in predecessors(dag, op) if p != "arrays"]
                if len(srcs) != 1:
                    break
                removed += [op, cur]
                cur = srcs[0]
                x_name, x_target = cur, od["pipeline"].config.read.array
                cd = dag.nodes[cur]
                is_int = any("pipeline" in dag.nodes[p] and
                             dag.nodes[p]["pipeline"].function is copy_read_to_write
                             for p in predecessors(dag, cur))
                if not (is_int and dag.out_degree(cur) == 1 and cur not in requested):
                    break
            if x_name is None or not isinstance(x_target, DeviceArray):
                continue
            y_target = dag.nodes[yname].get("target")
            if y_target is None or tuple(y_target.shape) != tuple(x_target.shape):
                continue
            region_fn = _box_of(y_target)

            def swap(leaf, i=i, region_fn=region_fn, x_name=x_name, x_target=x_target):
                if isinstance(leaf, ir.Arg) and leaf.index == i:
                    return ir.Region(x_name, leaf.dtype, leaf.axes, region_fn, i, leaf.field, x_target)
                return None

            memo = {}
            if program.structured:
                outputs = tuple((n, ir.transform(e, swap, memo)) for n, e in program.outputs)
            else:
                outputs = ir.transform(program.outputs, swap, memo)
            reduce = program.reduce
            if reduce is not None:
                reduce = dataclasses.replace(reduce, fields=tuple(
                    dataclasses.replace(f, expr=ir.transform(f.expr, swap, memo)) for f in reduce.fields))
            program = dataclasses.replace(program, outputs=outputs, reduce=reduce)
            reads = dict(spec.reads_map)
            reads[x_name] = CubedArrayProxy(x_target, x_target.chunks)
            spec = dataclasses.replace(spec, function=program, reads_map=reads)
            pipeline = dataclasses.replace(nd["pipeline"], config=spec)
            nd["pipeline"] = pipeline
            nd["primitive_op"] = dataclasses.replace(nd["primitive_op"], pipeline=pipeline)
            fused_from = list(nd.get("fused_from", ()))
            for n2 in removed:
                d2 = dag.nodes[n2]
                if "primitive_op" in d2:
                    fused_from.append((n2, d2["primitive_op"].num_tasks))
                elif isinstance(d2.get("target"), DeviceArray):
                    elided.append(d2["target"])
            nd["fused_from"] = fused_from
            for n2 in removed:
                dag.remove_node(n2)
            dag.add_edge(x_name, name)
    return dag, elided


def compose_rechunks(dag, array_names):
    """A two-op rechunk (source -> ``{name}-int`` -> target, primitive/
    rechunk.py:144-155, planned when the source and target chunks do not fit
    ``max_mem`` together) whose intermediate is read only by the second copy
    and is not requested becomes ONE copy from the source straight into the
    target chunks: every target chunk is assembled from the source chunk
    pieces it covers (the intermediate's chunk grid only bounded the
    reference's per-task memory, which HBM-resident boxes do not need).
    Values are bit-identical; the first op keeps its TaskEndEvent and task
    count (``fused_from``).  Returns (DAG copy, elided targets)."""
    import networkx as nx

    from .core.optimization import predecessors

    requested = set(array_names or ())
    todo = []
    for name, nd in dag.nodes(data=True):
        if "pipeline" not in nd or nd["pipeline"].function is not copy_read_to_write:
            continue
        srcs = [p for p in predecessors(dag, name) if p != "arrays"]
        if len(srcs) != 1:
            continue
        mid = srcs[0]
        if mid in requested or dag.out_degree(mid) != 1:
            continue
        pres = [p for p in predecessors(dag, mid)]
        if len(pres) != 1:
            continue
        op1 = pres[0]
        od = dag.nodes[op1]
        if "pipeline" not in od or od["pipeline"].function is not copy_read_to_write:
            continue
        x = [p for p in predecessors(dag, op1) if p != "arrays"]
        if len(x) != 1:
            continue
        todo.append((op1, mid, name, x[0]))
    if not todo:
        return dag, []
    dag = nx.MultiDiGraph(dag)  # an unfrozen copy
    elided = []
    for op1, mid, op2, x in todo:
        d1, d2 = dag.nodes[op1], dag.nodes[op2]
        read = d1["pipeline"].config.read
        spec = dataclasses.replace(d2["pipeline"].config, read=read)
        pipeline = dataclasses.replace(d2["pipeline"], config=spec)
        d2["pipeline"] = pipeline
        d2["primitive_op"] = dataclasses.replace(d2["primitive_op"], pipeline=pipeline)
        d2["fused_from"] = list(d1.get("fused_from", ())) + [(op1, d1["primitive_op"].num_tasks)] + \
            list(d2.get("fused_from", ()))
        t = dag.nodes[mid].get("target")
        if isinstance(t, DeviceArray):
            elided.append(t)
        dag.remove_node(op1)
        dag.remove_node(mid)
        dag.add_edge(x, op2)
    return dag, elided


def _constant_args(spec):
    """{argument index: value} of a blockwise spec's arguments that read a
    constant array (a promoted scalar: VirtualFullArray, or a one-element
    in-memory array), resolved through the key function of block 0."""
    from .storage import VirtualFullArray, VirtualInMemoryArray

    out = {}
    try:
        nd = spec.write.array.ndim
        args = spec.block_function(("out",) + (0,) * nd)
    except Exception:  # noqa: BLE001 - no resolvable block: no constants
        return out
    for i, a in enumerate(args):
        if not isinstance(a, tuple) or not a or a[0] not in spec.reads_map:
            continue
        arr = spec.reads_map[a[0]].array
        if isinstance(arr, VirtualFullArray):
            out[i] = arr.fill_value
        elif isinstance(arr, VirtualInMemoryArray) and arr.array.size == 1:
            out[i] = arr.array.reshape(-1)[0].item()
    return out


def split_complex(dag):
    """Every blockwise program that computes complex values rewritten into
    real expressions over the values' real / imaginary slabs
    (cubed_amd/complex.py).  Returns the DAG (a copy when anything changed)."""
    from .complex import program_has_complex, split_program

    todo = [n for n, d in dag.nodes(data=True)
            if "pipeline" in d and d["pipeline"].function is apply_blockwise
            and program_has_complex(d["pipeline"].config.function)]
    if not todo:
        return dag
    dag = dag.copy()
    for name in todo:
        nd = dag.nodes[name]
        spec = nd["pipeline"].config
        spec = dataclasses.replace(spec, function=split_program(spec.function, _constant_args(spec)))
        pipeline = dataclasses.replace(nd["pipeline"], config=spec)
        nd["pipeline"] = pipeline
        nd["primitive_op"] = dataclasses.replace(nd["primitive_op"], pipeline=pipeline)
    return dag
