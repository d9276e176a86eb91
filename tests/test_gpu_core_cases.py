"""The reference's core-API behaviour cases (cubed/tests/test_core.py:
from_array / Zarr I/O, map_blocks forms, rechunk, reductions, merge_chunks,
compute of several arrays, specs) run on the MI355X executor (``-m gpu``).
Integer and copy results are exact; the float mean uses numpy's value."""

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
from cubed_amd import zarr_io as Z
from cubed_amd.core.ops import merge_chunks, partial_reduce, tree_reduce
from cubed_amd.runtime.types import Callback

pytestmark = pytest.mark.gpu

M3 = [[1, 2, 3], [4, 5, 6], [7, 8, 9]]


@pytest.fixture(scope="module")
def ex(gpu_executor):
    return gpu_executor


@pytest.fixture
def spec(ex):
    return cubed.Spec(None, allowed_mem=100000, executor=ex)


class TaskCounter(Callback):
    def __init__(self):
        self.value = 0

    def on_task_end(self, event):
        self.value += event.num_tasks


class Wrapped:
    """An array-like that is not a numpy array (reference WrappedArray)."""

    def __init__(self, x):
        self.x, self.dtype, self.shape, self.ndim = x, x.dtype, x.shape, x.ndim

    def __array__(self, dtype=None, copy=None):
        return np.asarray(self.x, dtype=dtype)

    def __getitem__(self, i):
        return Wrapped(self.x[i])


@pytest.mark.parametrize("x, chunks, asarray", [
    (np.arange(25).reshape(5, 5), (5, 5), None),
    (np.arange(25).reshape(5, 5), (3, 2), True),
    (np.arange(25).reshape(5, 5), -1, True),
    (np.array([[1]]), 1, None),
])
def test_from_array(spec, x, chunks, asarray):
    a = cubed.from_array(Wrapped(x), chunks=chunks, asarray=asarray, spec=spec)
    assert isinstance(a, cubed.Array)
    assert np.array_equal(a.compute(), x)


def test_zarr_source_and_sinks(spec, tmp_path):
    src = Z.open_array(str(tmp_path / "source.zarr"), mode="w", shape=(3, 3), dtype=np.int64, chunks=(2, 2))
    src[...] = np.array(M3)
    assert np.array_equal(cubed.from_zarr(str(tmp_path / "source.zarr"), spec=spec).compute(), M3)
    assert np.array_equal(cubed.from_array(src, spec=spec).compute(), M3)
    a = xp.asarray(M3, chunks=(2, 2), spec=spec)
    b = xp.asarray(np.ones((3, 3), int), chunks=(2, 2), spec=spec)
    t1 = Z.open_array(str(tmp_path / "t1.zarr"), mode="w", shape=(3, 3), dtype=np.int64, chunks=(2, 2))
    t2 = Z.open_array(str(tmp_path / "t2.zarr"), mode="w", shape=(3, 3), dtype=np.int64, chunks=(2, 2))
    cubed.store([a, b], [t1, t2])
    assert np.array_equal(t1[...], M3) and np.array_equal(t2[...], np.ones((3, 3)))
    with pytest.raises(ValueError, match=r"Different number of sources \(2\) and targets \(1\)"):
        cubed.store([a, b], [t1])
    with pytest.raises(ValueError, match="All sources must be cubed array objects"):
        cubed.store([1], [t1])
    cubed.to_zarr(a, str(tmp_path / "output.zarr"))
    assert np.array_equal(Z.open_array(str(tmp_path / "output.zarr"))[:], M3)


def test_map_blocks_with_kwargs(spec):
    a = xp.asarray(np.arange(10), chunks=5, spec=spec)
    b = cubed.map_blocks(np.max, a, axis=0, keepdims=True, dtype=a.dtype, chunks=(1,))
    assert np.array_equal(b.compute(), [4, 9])


def test_map_blocks_with_block_id(spec):
    def func(block, block_id=None, c=0):
        return np.ones_like(block) * int(sum(block_id)) + c

    a = xp.arange(10, dtype="int64", chunks=(2,), spec=spec)
    assert np.array_equal(cubed.map_blocks(func, a, dtype="int64").compute(), [0, 0, 1, 1, 2, 2, 3, 3, 4, 4])
    m = xp.asarray(M3, chunks=(2, 2), spec=spec)
    exp = np.array([[0, 0, 1], [0, 0, 1], [1, 1, 2]])
    assert np.array_equal(cubed.map_blocks(func, m, dtype="int64").compute(), exp)
    assert np.array_equal(cubed.map_blocks(func, m, dtype="int64", c=1).compute(), exp + 1)


def test_map_blocks_no_array_args(spec):
    def func(block, block_id=None):
        return np.ones_like(block) * int(sum(block_id))

    a = cubed.map_blocks(func, dtype="int64", chunks=((5, 3),), spec=spec)
    assert a.chunks == ((5, 3),)
    assert np.array_equal(a.compute(), [0, 0, 0, 0, 0, 1, 1, 1])


def test_map_blocks_with_different_block_shapes(spec):
    a = xp.asarray([[[12, 13]]], spec=spec)
    b = xp.asarray([14, 15], spec=spec)
    c = cubed.map_blocks(lambda x, y: x, a, b, dtype="int64", chunks=(1, 1, 2), drop_axis=2, new_axis=2)
    assert np.array_equal(c.compute(), [[[12, 13]]])


def test_multiple_ops_and_idempotent_compute(spec):
    a = xp.asarray(M3, chunks=(2, 2), spec=spec)
    d = xp.negative(xp.add(a, xp.asarray(np.ones((3, 3), int), chunks=(2, 2), spec=spec)))
    assert np.array_equal(d.compute(), -(np.array(M3) + 1))
    assert np.array_equal(d.compute(), -(np.array(M3) + 1))


@pytest.mark.parametrize("new_chunks", [(1, 2), {0: 1, 1: 2}])
def test_rechunk(spec, new_chunks):
    a = xp.asarray(M3, chunks=(2, 1), spec=spec)
    assert np.array_equal(a.rechunk(new_chunks).compute(), M3)


def test_rechunk_same_chunks_runs_no_task(spec):
    b = xp.asarray(M3, chunks=(2, 1), spec=spec).rechunk((2, 1))
    tc = TaskCounter()
    assert np.array_equal(b.compute(callbacks=[tc]), M3)
    assert tc.value == 0


def test_rechunk_intermediate(ex):
    s = cubed.Spec(None, allowed_mem=4 * 8 * 4, executor=ex)
    b = xp.ones((4, 4), chunks=(1, 4), spec=s).rechunk((4, 1))
    assert np.array_equal(b.compute(), np.ones((4, 4)))
    assert len([n for n, d in b.plan.dag.nodes(data=True) if "-int" in d["name"]]) == 1


def test_reduction_multiple_rounds(ex):
    s = cubed.Spec(None, allowed_mem=1000, executor=ex)
    b = xp.sum(xp.ones((100, 10), dtype=np.uint8, chunks=(1, 10), spec=s), axis=0, dtype=np.uint8)
    assert len([n for n, d in b.plan.dag.nodes(data=True) if d.get("op_name") == "blockwise"]) > 1
    assert b.plan.max_projected_mem() <= 1000
    assert np.array_equal(b.compute(), np.ones((100, 10)).sum(axis=0))
    s50 = cubed.Spec(None, allowed_mem=50, executor=ex)
    with pytest.raises(ValueError, match="Not enough memory for reduction"):
        xp.sum(xp.ones((100, 10), dtype=np.uint8, chunks=(1, 10), spec=s50), axis=0, dtype=np.uint8)


def test_partial_and_tree_reduce(spec):
    x = np.arange(242).reshape(11, 22)
    a = xp.asarray(x, chunks=(3, 4), spec=spec)
    c = partial_reduce(partial_reduce(a, np.sum, split_every={0: 2}), np.sum, split_every={0: 2})
    assert np.array_equal(c.compute(), x.sum(axis=0, keepdims=True))
    t = tree_reduce(a, np.sum, axis=0, dtype=np.int64, split_every={0: 2})
    assert np.array_equal(t.compute(), x.sum(axis=0, keepdims=True))


@pytest.mark.parametrize("target, expected", [((2, 3), None), ((4, 3), None), ((2, 6), None), ((4, 6), None),
                                              ((12, 12), (10, 10))])
def test_merge_chunks(spec, target, expected):
    b = merge_chunks(xp.ones((10, 10), dtype=np.uint8, chunks=(2, 3), spec=spec), target)
    assert b.chunksize == (expected or target)
    assert np.array_equal(b.compute(), np.ones((10, 10)))


@pytest.mark.parametrize("target", [(2,), (2, 3, 1), (3, 2), (1, 3), (5, 5), (10, 10)])
def test_merge_chunks_fails(spec, target):
    with pytest.raises(ValueError):
        merge_chunks(xp.ones((10, 10), dtype=np.uint8, chunks=(2, 3), spec=spec), target)


def test_compute_multiple(spec):
    a = xp.asarray(M3, chunks=(2, 2), spec=spec)
    c = xp.add(a, xp.asarray(np.ones((3, 3), int), chunks=(2, 2), spec=spec))
    g = xp.asarray(M3, chunks=(2, 2), spec=spec) * 4
    dc, ec, gc = cubed.compute(c * 2, c * 3, g)
    cn = np.array(M3) + 1
    assert np.array_equal(dc, cn * 2) and np.array_equal(ec, cn * 3) and np.array_equal(gc, np.array(M3) * 4)


def test_different_specs_fail(ex):
    s1 = cubed.Spec(None, allowed_mem=100000, executor=ex)
    s2 = cubed.Spec(None, allowed_mem=200000, executor=ex)
    with pytest.raises(ValueError):
        xp.add(xp.ones((3, 3), chunks=(2, 2), spec=s1), xp.ones((3, 3), chunks=(2, 2), spec=s2))
    c1 = xp.add(xp.ones((3, 3), chunks=(2, 2), spec=s1), xp.ones((3, 3), chunks=(2, 2), spec=s1))
    c2 = xp.add(xp.ones((3, 3), chunks=(2, 2), spec=s2), xp.ones((3, 3), chunks=(2, 2), spec=s2))
    with pytest.raises(ValueError):
        cubed.compute(c1, c2)


def test_default_spec_limits(ex):
    # the default spec's executor is the MI355X one: needs the GPU (ex skips without it)
    a = xp.ones((3, 3), chunks=(2, 2))
    assert np.array_equal(xp.negative(a).compute(), -np.ones((3, 3)))
    with pytest.raises(ValueError):
        xp.negative(xp.ones((100000, 100000), chunks=(10000, 10000)))
