"""Deferred computation plan (mirrors cubed/core/plan.py:30-247).

A networkx ``MultiDiGraph`` of op and array nodes.  ``execute`` finalizes the
DAG (optimize + a ``create-arrays`` node, lru-cached) and hands it to an
executor -- the plug-in point the MI355X executor sits behind.
"""

from __future__ import annotations

import inspect
import uuid
from datetime import datetime
from typing import Callable, Optional

import networkx as nx

from ..primitive.types import PrimitiveOperation
from ..runtime.pipeline import visit_nodes
from ..runtime.types import CubedPipeline
from ..storage import DeviceArray
from ..utils import gensym_factory

CONTEXT_ID = f"cubed-{datetime.now().strftime('%Y%m%dT%H%M%S')}-{uuid.uuid4()}"

gensym = gensym_factory("op")


class Plan:
    """Deferred computation plan for a graph of arrays."""

    def __init__(self, dag):
        self.dag = dag

    @classmethod
    def _new(cls, name, op_name, target, primitive_op=None, hidden=False, *source_arrays):
        dag = nx.MultiDiGraph() if not source_arrays else arrays_to_dag(*source_arrays)
        op_name_unique = gensym()
        attrs = dict(name=op_name_unique, op_name=op_name, type="op", hidden=hidden)
        if primitive_op is not None:
            attrs.update(primitive_op=primitive_op, pipeline=primitive_op.pipeline)
        dag.add_node(op_name_unique, **attrs)
        dag.add_node(name, name=name, type="array", target=target, hidden=hidden)
        dag.add_edge(op_name_unique, name)
        for x in source_arrays:
            if hasattr(x, "name"):
                dag.add_edge(x.name, op_name_unique)
        return Plan(dag)

    @classmethod
    def arrays_to_plan(cls, *arrays):
        return Plan(arrays_to_dag(*arrays))

    def optimize(self, optimize_function: Optional[Callable[..., nx.MultiDiGraph]] = None):
        from .optimization import simple_optimize_dag

        if optimize_function is None:
            optimize_function = simple_optimize_dag
        return Plan(optimize_function(self.dag))

    def _create_arrays_node(self, dag):
        """Add the ``create-arrays`` op (the reference creates the Zarr
        intermediates there, core/plan.py:136-176); here it marks where the
        executor allocates HBM targets."""
        pipeline_nodes, targets = [], []
        allowed_mem = reserved_mem = 0
        for n, d in dag.nodes(data=True):
            if "primitive_op" in d:
                pipeline_nodes.append(n)
                allowed_mem = max(allowed_mem, d["primitive_op"].allowed_mem)
                reserved_mem = max(reserved_mem, d["primitive_op"].reserved_mem)
            if isinstance(d.get("target"), DeviceArray):
                targets.append(d["target"])
        if targets:
            name = "create-arrays"
            op = create_arrays_op(targets, allowed_mem, reserved_mem)
            dag.add_node(name, name=name, op_name=name, type="op", primitive_op=op,
                         pipeline=op.pipeline)
            dag.add_node("arrays", name="arrays", target=None)
            dag.add_edge(name, "arrays")
            for n in pipeline_nodes:
                dag.add_edge("arrays", n)
        return dag

    def _finalize_dag(self, optimize_graph: bool = True, optimize_function=None) -> nx.MultiDiGraph:
        # cached on the plan (the reference's lru_cache, core/plan.py:178, would
        # keep up to 128 finalized DAGs -- and the HBM of the launches an
        # executor caches for them -- alive after their plans are dropped)
        cache = self.__dict__.setdefault("_finalized", {})
        key = (optimize_graph, optimize_function)
        dag = cache.get(key)
        if dag is None:
            dag = self.optimize(optimize_function).dag if optimize_graph else self.dag
            dag = dag.copy()
            dag = self._create_arrays_node(dag)
            dag = cache[key] = nx.freeze(dag)
        return dag

    def execute(self, executor=None, callbacks=None, optimize_graph=True, optimize_function=None,
                resume=None, spec=None, array_names=None, **kwargs):
        dag = self._finalize_dag(optimize_graph, optimize_function)
        if callbacks is not None:
            [cb.on_compute_start(dag, resume=resume) for cb in callbacks]
        executor.execute_dag(dag, callbacks=callbacks, array_names=array_names, resume=resume,
                             spec=spec, **kwargs)
        if callbacks is not None:
            [cb.on_compute_end(dag) for cb in callbacks]

    def num_tasks(self, optimize_graph=True, optimize_function=None, resume=None):
        dag = self._finalize_dag(optimize_graph, optimize_function)
        return sum(node["primitive_op"].num_tasks for _, node in visit_nodes(dag, resume=resume))

    def num_arrays(self, optimize_graph: bool = True, optimize_function=None) -> int:
        dag = self._finalize_dag(optimize_graph, optimize_function)
        return sum(d.get("type") == "array" for _, d in dag.nodes(data=True))

    def max_projected_mem(self, optimize_graph=True, optimize_function=None, resume=None):
        dag = self._finalize_dag(optimize_graph, optimize_function)
        vals = [node["primitive_op"].projected_mem for _, node in visit_nodes(dag, resume=resume)]
        return max(vals) if vals else 0

    def total_nbytes(self, optimize_graph: bool = True, optimize_function=None) -> int:
        dag = self._finalize_dag(optimize_graph, optimize_function)
        return sum(d["target"].nbytes for _, d in dag.nodes(data=True)
                   if d.get("type") == "array" and isinstance(d.get("target"), DeviceArray))

    def visualize(self, filename="cubed", format=None, optimize_graph=True,
                  optimize_function=None, show_hidden=False):
        """Write the plan as a Graphviz dot file (no rendering: graphviz is
        not a dependency of this build)."""
        dag = self._finalize_dag(optimize_graph, optimize_function)
        lines = ["digraph {"]
        for n, d in dag.nodes(data=True):
            if d.get("hidden") and not show_hidden:
                continue
            label = d.get("op_name", n)
            lines.append(f'  "{n}" [label="{label}"];')
        for u, v in dag.edges():
            lines.append(f'  "{u}" -> "{v}";')
        lines.append("}")
        path = str(filename)
        if not path.endswith(".dot"):
            path += ".dot"
        with open(path, "w") as f:
            f.write("\n".join(lines))
        return None


def arrays_to_dag(*arrays):
    from .array import check_array_specs

    check_array_specs(arrays)
    dags = [x.plan.dag for x in arrays if hasattr(x, "plan")]
    return nx.compose_all(dags)


def arrays_to_plan(*arrays):
    plans = [x.plan for x in arrays if hasattr(x, "plan")]
    if len(plans) == 0:
        raise ValueError(f"No plans found for arrays: {arrays}")
    return plans[0].arrays_to_plan(*arrays)


def new_temp_path(name, suffix=".zarr", spec=None):
    """Name for an intermediate target (kept for API parity; HBM targets are
    named, not stored at a path)."""
    return f"{CONTEXT_ID}/{name}{suffix}"


def create_arrays_stage(targets, *, config=None):
    raise TypeError("create-arrays runs only through the MI355X executor")


class _TargetList:
    def __init__(self, targets):
        self.targets = list(targets)

    def __iter__(self):
        return iter(self.targets)

    def __len__(self):
        return len(self.targets)


def create_arrays_op(targets, allowed_mem, reserved_mem) -> PrimitiveOperation:
    pipeline = CubedPipeline(create_arrays_stage, "create-arrays", _TargetList(targets), None)
    projected_mem = max([t.dtype.itemsize for t in targets], default=0) + reserved_mem
    return PrimitiveOperation(pipeline=pipeline, target_array=None, projected_mem=projected_mem,
                              allowed_mem=allowed_mem, reserved_mem=reserved_mem,
                              num_tasks=len(targets), fusable=False)
