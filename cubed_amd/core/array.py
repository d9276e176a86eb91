"""Chunked array metadata and ``compute`` (mirrors cubed/core/array.py)."""

from __future__ import annotations

from operator import mul
from functools import reduce
from typing import Optional, TypeVar

import numpy as np

from .. import ir
from ..runtime.types import Callback, Executor
from ..spec import Spec
from ..utils import chunk_memory, gensym_factory, normalize_chunks

gensym = gensym_factory("array")

T_ChunkedArray = TypeVar("T_ChunkedArray", bound="CoreArray")


class CoreArray:
    """Chunked array backed by an HBM target (or a virtual array)."""

    def __init__(self, name, zarray, spec, plan):
        self.name = name
        self._zarray = zarray
        self._shape = tuple(zarray.shape)
        self._dtype = np.dtype(zarray.dtype)
        self._chunks = normalize_chunks(zarray.chunks, shape=self.shape, dtype=self.dtype)
        # default spec as the reference: 200 MB allowed, 100 MB reserved
        self.spec = spec or Spec(None, allowed_mem=200_000_000, reserved_mem=100_000_000)
        self.plan = plan

    @property
    def zarray_maybe_lazy(self):
        return self._zarray

    @property
    def zarray(self):
        return self._zarray

    @property
    def chunkmem(self):
        return chunk_memory(self.dtype, self.chunksize)

    @property
    def chunksize(self):
        return tuple(max(c) for c in self.chunks)

    @property
    def chunks(self):
        return self._chunks

    @property
    def dtype(self):
        return self._dtype

    @property
    def ndim(self):
        return len(self.shape)

    @property
    def numblocks(self):
        return tuple(map(len, self.chunks))

    @property
    def npartitions(self):
        return reduce(mul, self.numblocks, 1)

    @property
    def shape(self):
        return self._shape

    @property
    def size(self):
        return reduce(mul, self.shape, 1)

    @property
    def nbytes(self) -> int:
        return self.size * self.dtype.itemsize

    @property
    def itemsize(self) -> int:
        return self.dtype.itemsize

    def _read_stored(self):
        """Copy the computed array back to a host numpy array."""
        from ..storage import DeviceArray, VirtualFullArray, VirtualInMemoryArray

        t = self._zarray
        if self.size == 0:
            return np.empty(self.shape, dtype=self.dtype)
        if isinstance(t, DeviceArray):
            if not t.written:
                raise RuntimeError(f"array {self.name} has not been computed")
            from ..runtime.executors.gpu import gather_to_host

            out = gather_to_host(t)
            if out.dtype == ir.bfloat16:  # numpy has no bfloat16: widen exactly to f32
                out = ir.bf16_to_numpy(out)
            return out
        if isinstance(t, VirtualInMemoryArray):
            return np.array(t.array)
        if isinstance(t, VirtualFullArray):
            return np.full(self.shape, t.fill_value, dtype=self.dtype)
        raise RuntimeError(f"array {self.name} has no stored values")

    def compute(self, *, executor=None, callbacks=None, optimize_graph=True,
                optimize_function=None, resume=None, **kwargs):
        result = compute(self, executor=executor, callbacks=callbacks,
                         optimize_graph=optimize_graph, optimize_function=optimize_function,
                         resume=resume, **kwargs)
        if result:
            return result[0]

    def rechunk(self: T_ChunkedArray, chunks) -> T_ChunkedArray:
        from .ops import rechunk

        return rechunk(self, chunks)

    def visualize(self, filename="cubed", format=None, optimize_graph=True,
                  optimize_function=None, show_hidden=False):
        return visualize(self, filename=filename, format=format, optimize_graph=optimize_graph,
                         optimize_function=optimize_function, show_hidden=show_hidden)

    def __getitem__(self: T_ChunkedArray, key, /) -> T_ChunkedArray:
        from .ops import index

        return index(self, key)

    def __repr__(self):
        return f"cubed.core.CoreArray<{self.name}, shape={self.shape}, dtype={self.dtype}, chunks={self.chunks}>"


def check_array_specs(arrays):
    specs = [a.spec for a in arrays if hasattr(a, "spec")]
    if not all(s == specs[0] for s in specs):
        raise ValueError(f"Arrays must have same spec in single computation. Specs: {specs}")
    return arrays[0].spec


def default_executor():
    from ..runtime.executors.gpu import GpuDagExecutor

    return GpuDagExecutor()


def compute(*arrays, executor=None, callbacks=None, optimize_graph=True, optimize_function=None,
            resume=None, **kwargs):
    """Compute multiple arrays at once.  The default executor is the MI355X
    ``GpuDagExecutor`` (the reference defaults to PythonDagExecutor,
    core/array.py:275-280)."""
    from .plan import arrays_to_plan

    spec = check_array_specs(arrays)
    plan = arrays_to_plan(*arrays)
    if executor is None:
        executor = arrays[0].spec.executor
        if executor is None:
            executor = default_executor()
    _return_in_memory_array = kwargs.pop("_return_in_memory_array", True)
    plan.execute(executor=executor, callbacks=callbacks, optimize_graph=optimize_graph,
                 optimize_function=optimize_function, resume=resume,
                 array_names=[a.name for a in arrays], spec=spec, **kwargs)
    if _return_in_memory_array:
        return tuple(a._read_stored() for a in arrays)


def visualize(*arrays, filename="cubed", format=None, optimize_graph=True,
              optimize_function=None, show_hidden=False):
    from .plan import arrays_to_plan

    plan = arrays_to_plan(*arrays)
    return plan.visualize(filename=filename, format=format, optimize_graph=optimize_graph,
                          optimize_function=optimize_function, show_hidden=show_hidden)


class PeakMeasuredMemoryCallback(Callback):
    def on_task_end(self, event):
        self.peak_measured_mem = event.peak_measured_mem_end


def measure_reserved_mem(executor: Executor, work_dir: Optional[str] = None, **kwargs) -> int:
    """Reserved (non-data) memory of a task: for the GPU executor the host
    process peak RSS while running a trivial computation."""
    from .. import array_api as xp

    a = xp.ones((1,), spec=Spec(work_dir, allowed_mem="500MB"))
    b = xp.negative(a)
    cb = PeakMeasuredMemoryCallback()
    b.compute(executor=executor, callbacks=[cb], **kwargs)
    return cb.peak_measured_mem
