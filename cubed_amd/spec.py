"""Resource specification (mirrors cubed/spec.py:7-102)."""

from typing import Optional, Union

from .utils import convert_to_bytes


class Spec:
    """Specification of resources available to run a computation.

    ``allowed_mem`` bounds the projected memory of one task, exactly as in the
    reference (it drives the reduction merge factor and the rechunk plan).
    On the MI355X executor a task's chunks live in HBM; the executor
    additionally checks that the resident intermediates of a plan fit the
    device (288 GB per MI355X), see DESIGN.md.
    """

    def __init__(self, work_dir: Union[str, None] = None, allowed_mem: Union[int, str, None] = None,
                 reserved_mem: Union[int, str, None] = 0, executor=None,
                 storage_options: Union[dict, None] = None):
        self._work_dir = work_dir
        self._reserved_mem = convert_to_bytes(reserved_mem or 0)
        if allowed_mem is None:
            self._allowed_mem = self.reserved_mem
        else:
            self._allowed_mem = convert_to_bytes(allowed_mem)
        self._executor = executor
        self._storage_options = storage_options

    @property
    def work_dir(self) -> Optional[str]:
        return self._work_dir

    @property
    def allowed_mem(self) -> int:
        return self._allowed_mem

    @property
    def reserved_mem(self) -> int:
        return self._reserved_mem

    @property
    def executor(self):
        return self._executor

    @property
    def storage_options(self) -> Optional[dict]:
        return self._storage_options

    def __repr__(self) -> str:
        return (f"cubed.Spec(work_dir={self._work_dir}, allowed_mem={self._allowed_mem}, "
                f"reserved_mem={self._reserved_mem}, executor={self._executor}, "
                f"storage_options={self._storage_options})")

    def __eq__(self, other):
        if isinstance(other, Spec):
            return (self.work_dir == other.work_dir and self.allowed_mem == other.allowed_mem
                    and self.reserved_mem == other.reserved_mem
                    and self.executor == other.executor
                    and self.storage_options == other.storage_options)
        return False
