"""Executor plug-in interface (mirrors cubed/runtime/types.py:9-87)."""

from dataclasses import dataclass
from typing import Any, Callable, Iterable, Optional


class DagExecutor:
    """``execute_dag(dag, callbacks=None, array_names=None, resume=None,
    spec=None, **kwargs)`` runs every op node of a finalized plan DAG."""

    def execute_dag(self, dag, **kwargs) -> None:
        raise NotImplementedError  # pragma: no cover


Executor = DagExecutor


@dataclass(frozen=True)
class CubedPipeline:
    """Stage function, name, iterable of task keys and the stage config."""

    function: Callable[..., Any]
    name: str
    mappable: Iterable
    config: Any


class Callback:
    """Object to receive callback events during array computation."""

    def on_compute_start(self, dag, resume):
        pass  # pragma: no cover

    def on_compute_end(self, dag):
        pass  # pragma: no cover

    def on_task_end(self, event):
        pass  # pragma: no cover


@dataclass
class TaskEndEvent:
    """Callback information about a completed task (or tasks)."""

    array_name: str
    num_tasks: int = 1
    task_create_tstamp: Optional[float] = None
    function_start_tstamp: Optional[float] = None
    function_end_tstamp: Optional[float] = None
    task_result_tstamp: Optional[float] = None
    peak_measured_mem_start: Optional[int] = None
    peak_measured_mem_end: Optional[int] = None
