"""DAG optimizers: which ops become one fused pipeline (one kernel launch).

Mirrors cubed/core/optimization.py: ``simple_optimize_dag`` (the default
linear-chain map fusion, :11-68), ``multiple_inputs_optimize_dag`` with
``max_total_source_arrays`` (:97-209), ``fuse_all_optimize_dag`` (:212-216) and
``fuse_only_optimize_dag`` (:219-226).  Same decisions, so task counts match
the reference; fusion composes IR programs (primitive/blockwise.py).
"""

import networkx as nx

from ..primitive.blockwise import (
    can_fuse_multiple_primitive_ops,
    can_fuse_primitive_ops,
    fuse,
    fuse_multiple,
)


def simple_optimize_dag(dag):
    """Apply map blocks fusion (single in-degree chains)."""
    dag = dag.copy()
    nodes = {n: d for (n, d) in dag.nodes(data=True)}

    def can_fuse(n):
        op2 = n
        if "primitive_op" not in nodes[op2]:
            return False
        if dag.in_degree(op2) != 1:
            return False
        op2_input = next(dag.predecessors(op2))
        if dag.out_degree(op2_input) != 1:
            return False
        op1 = next(dag.predecessors(op2_input))
        if dag.out_degree(op1) != 1:
            return False
        if "primitive_op" not in nodes[op1]:
            return False
        return can_fuse_primitive_ops(nodes[op1]["primitive_op"], nodes[op2]["primitive_op"])

    for n in list(dag.nodes()):
        if can_fuse(n):
            op2 = n
            op2_input = next(dag.predecessors(op2))
            op1 = next(dag.predecessors(op2_input))
            op1_inputs = list(dag.predecessors(op1))
            primitive_op = fuse(nodes[op1]["primitive_op"], nodes[op2]["primitive_op"])
            nodes[op2]["primitive_op"] = primitive_op
            nodes[op2]["pipeline"] = primitive_op.pipeline
            for i in op1_inputs:
                dag.add_edge(i, op2)
            dag.remove_node(op2_input)
            dag.remove_node(op1)
    return dag


def predecessors(dag, name):
    """A node's predecessors, with repeats for multiple edges."""
    for pre, _ in dag.in_edges(name):
        yield pre


def predecessor_ops(dag, name):
    for inp in predecessors(dag, name):
        for pre in predecessors(dag, inp):
            yield pre


def is_fusable(node_dict):
    return "primitive_op" in node_dict and node_dict["primitive_op"].fusable


def can_fuse_predecessors(dag, name, *, max_total_source_arrays=4, always_fuse=None,
                          never_fuse=None):
    nodes = dict(dag.nodes(data=True))
    if not is_fusable(nodes[name]):
        return False
    if all(not is_fusable(nodes[pre]) for pre in predecessor_ops(dag, name)):
        return False
    if never_fuse is not None and name in never_fuse:
        return False
    if always_fuse is not None and name in always_fuse:
        return True
    if len(list(predecessor_ops(dag, name))) > 1:
        total = sum(len(list(predecessors(dag, pre))) if is_fusable(nodes[pre]) else 1
                    for pre in predecessor_ops(dag, name))
        if total > max_total_source_arrays:
            return False
    preds = [nodes[pre]["primitive_op"] for pre in predecessor_ops(dag, name)
             if is_fusable(nodes[pre])]
    return can_fuse_multiple_primitive_ops(nodes[name]["primitive_op"], *preds)


def fuse_predecessors(dag, name, *, max_total_source_arrays=4, always_fuse=None, never_fuse=None):
    """Fuse a node with its immediate predecessors."""
    if not can_fuse_predecessors(dag, name, max_total_source_arrays=max_total_source_arrays,
                                 always_fuse=always_fuse, never_fuse=never_fuse):
        return dag
    nodes = dict(dag.nodes(data=True))
    primitive_op = nodes[name]["primitive_op"]
    preds = [nodes[pre]["primitive_op"] if is_fusable(nodes[pre]) else None
             for pre in predecessor_ops(dag, name)]
    fused_op = fuse_multiple(primitive_op, *preds)
    fused_dag = dag.copy()
    fused_nodes = dict(fused_dag.nodes(data=True))
    fused_nodes[name]["primitive_op"] = fused_op
    fused_nodes[name]["pipeline"] = fused_op.pipeline
    for inp in predecessors(dag, name):
        pre = next(predecessors(dag, inp))
        if not is_fusable(fused_nodes[pre]):
            continue
        fused_dag.remove_edge(inp, name)
    for pre in predecessor_ops(dag, name):
        if not is_fusable(fused_nodes[pre]):
            continue
        for inp in predecessors(dag, pre):
            fused_dag.add_edge(inp, name)
    for inp in predecessors(dag, name):
        if fused_dag.out_degree(inp) == 0:
            for pre in list(predecessors(fused_dag, inp)):
                fused_dag.remove_node(pre)
            fused_dag.remove_node(inp)
    return fused_dag


def multiple_inputs_optimize_dag(dag, *, max_total_source_arrays=4, always_fuse=None,
                                 never_fuse=None):
    """Fuse multiple inputs."""
    for name in list(nx.topological_sort(dag)):
        dag = fuse_predecessors(dag, name, max_total_source_arrays=max_total_source_arrays,
                                always_fuse=always_fuse, never_fuse=never_fuse)
    return dag


def fuse_all_optimize_dag(dag):
    """Force all operations to be fused."""
    dag = dag.copy()
    always_fuse = [op for op in dag.nodes() if op.startswith("op-")]
    return multiple_inputs_optimize_dag(dag, always_fuse=always_fuse)


def fuse_only_optimize_dag(dag, *, only_fuse=None):
    """Force only the specified operations to be fused."""
    dag = dag.copy()
    always_fuse = only_fuse
    never_fuse = set(op for op in dag.nodes() if op.startswith("op-")) - set(only_fuse)
    return multiple_inputs_optimize_dag(dag, always_fuse=always_fuse, never_fuse=never_fuse)
