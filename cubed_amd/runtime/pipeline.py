"""DAG traversal (mirrors cubed/runtime/pipeline.py:8-57)."""

from typing import Any, Dict, Optional

import networkx as nx


def _target_complete(target) -> bool:
    """An HBM target written by an earlier compute (and still resident), or
    one whose Zarr store holds every chunk (``zarr_complete``, set for a
    resumed reference DAG: the reference's nchunks_initialized check,
    cubed/runtime/pipeline.py:25-33)."""
    return bool(getattr(target, "written", None)) or bool(getattr(target, "zarr_complete", False))


def already_computed(name, dag, nodes: Dict[str, Any], resume: Optional[bool] = None) -> bool:
    """True if the node has no pipeline, or (with ``resume``) every output
    target already holds its data -- for HBM targets, that they were written
    by an earlier compute and are still resident."""
    pipeline = nodes[name].get("pipeline", None)
    if pipeline is None:
        return True
    if all(nodes[o].get("target", None) is None for o in dag.successors(name)):
        return False
    if resume:
        for o in dag.successors(name):
            target = nodes[o].get("target", None)
            if target is not None and not _target_complete(target):
                return False
        return True
    return False


def visit_nodes(dag, resume=None):
    """Nodes to run, in topological order."""
    nodes = {n: d for (n, d) in dag.nodes(data=True)}
    for name in list(nx.topological_sort(dag)):
        if already_computed(name, dag, nodes, resume=resume):
            continue
        yield name, nodes[name]


def visit_node_generations(dag, resume=None):
    nodes = {n: d for (n, d) in dag.nodes(data=True)}
    for names in nx.topological_generations(dag):
        gen = [(n, nodes[n]) for n in names if not already_computed(n, dag, nodes, resume=resume)]
        if gen:
            yield gen
