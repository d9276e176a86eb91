"""The reference's array-API behaviour cases (cubed/tests/test_array_api.py:
object, creation, data-type, elementwise, indexing, linear-algebra,
manipulation, searching, statistical and utility sections) run end to end on
the MI355X executor (``-m gpu``), under the reference's own
``Spec(allowed_mem=100000)`` so plan-time memory checks apply as there.

Cases are a table: (id, function building the cubed_amd result from the
spec, function computing numpy's expected value).  Integer / boolean /
copy results must match exactly; float results of a few elementwise ops on
small integers are exact too, so every case uses ``array_equal`` except
linspace (numpy's own rounding, allclose as in the reference)."""

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
from cubed_amd.array_api.manipulation_functions import reshape_chunks

pytestmark = pytest.mark.gpu

M3 = [[1, 2, 3], [4, 5, 6], [7, 8, 9]]
M4 = [[1, 2, 3, 4], [5, 6, 7, 8], [9, 10, 11, 12], [13, 14, 15, 16]]
ARGM = [[11, 12, 13], [11, 11, 14], [10, 13, 11]]


@pytest.fixture(scope="module")
def spec(gpu_executor):
    return cubed.Spec(None, allowed_mem=100000, executor=gpu_executor)


def a3(s, dtype=None):
    return xp.asarray(np.array(M3, dtype=dtype) if dtype else M3, chunks=(2, 2), spec=s)


def a4(s):
    return xp.asarray(M4, chunks=(2, 2), spec=s)


CASES = [
    # array object
    ("bool_all_false", lambda s: xp.all(xp.asarray(np.zeros((3, 3), bool), chunks=(2, 2), spec=s)),
     lambda: np.False_),
    ("bool_all_true", lambda s: xp.all(xp.asarray(np.ones((3, 3), bool), chunks=(2, 2), spec=s)),
     lambda: np.True_),
    ("mT", lambda s: a3(s).mT, lambda: np.array(M3).T),
    ("T", lambda s: a3(s).T, lambda: np.array(M3).T),
    ("reflected_sub", lambda s: 1 - a3(s), lambda: 1 - np.array(M3)),
    # creation
    ("arange", lambda s: xp.arange(12, chunks=(5,), spec=s), lambda: np.arange(12)),
    ("arange_step", lambda s: xp.arange(20, step=3, chunks=(5,), spec=s), lambda: np.arange(20, step=3)),
    ("asarray", lambda s: a3(s), lambda: np.array(M3)),
    ("eye_m1", lambda s: xp.eye(5, k=-1, chunks=(2, 2), spec=s), lambda: np.eye(5, k=-1)),
    ("eye_0", lambda s: xp.eye(5, k=0, chunks=(2, 2), spec=s), lambda: np.eye(5, k=0)),
    ("eye_1", lambda s: xp.eye(5, k=1, chunks=(2, 2), spec=s), lambda: np.eye(5, k=1)),
    ("ones", lambda s: xp.ones((3, 3), chunks=(2, 2), spec=s), lambda: np.ones((3, 3))),
    ("ones_like", lambda s: xp.ones_like(xp.ones((3, 3), chunks=(2, 2), spec=s)), lambda: np.ones((3, 3))),
    *[(f"tril_{k}", (lambda k: lambda s: xp.tril(xp.ones((4, 5), chunks=(2, 2), spec=s), k=k))(k),
       (lambda k: lambda: np.tril(np.ones((4, 5)), k))(k)) for k in (-1, 0, 1)],
    *[(f"triu_{k}", (lambda k: lambda s: xp.triu(xp.ones((4, 5), chunks=(2, 2), spec=s), k=k))(k),
       (lambda k: lambda: np.triu(np.ones((4, 5)), k))(k)) for k in (-1, 0, 1)],
    # data types
    ("astype_int32", lambda s: xp.astype(a3(s), xp.int32), lambda: np.array(M3, dtype=np.int32)),
    # elementwise
    ("add", lambda s: xp.add(a3(s), xp.asarray(np.ones((3, 3), int), chunks=(2, 2), spec=s)),
     lambda: np.array(M3) + 1),
    ("add_misaligned_chunks", lambda s: xp.add(xp.ones((10, 10), chunks=(10, 2), spec=s),
                                               xp.ones((10, 10), chunks=(2, 10), spec=s)),
     lambda: np.full((10, 10), 2.0)),
    ("equal", lambda s: xp.equal(a3(s), a3(s)), lambda: np.full((3, 3), True)),
    ("negative", lambda s: xp.negative(a3(s)), lambda: -np.array(M3)),
    # linear algebra
    ("matmul_int", lambda s: xp.matmul(a4(s), a4(s)), lambda: np.array(M4) @ np.array(M4)),
    ("outer", lambda s: xp.outer(xp.asarray([0, 1, 2], chunks=2, spec=s),
                                 xp.asarray([10, 50, 100], chunks=2, spec=s)),
     lambda: np.outer([0, 1, 2], [10, 50, 100])),
    *[(f"tensordot_{ax}", (lambda ax: lambda s: xp.tensordot(
        xp.asarray(np.arange(400).reshape(20, 20), chunks=(5, 4), spec=s),
        xp.asarray(np.arange(200).reshape(20, 10), chunks=(4, 5), spec=s), axes=ax))(ax),
       (lambda ax: lambda: np.tensordot(np.arange(400).reshape(20, 20), np.arange(200).reshape(20, 10),
                                        axes=ax))(ax)) for ax in (1, (1, 0))],
    # manipulation
    ("expand_dims", lambda s: xp.expand_dims(xp.asarray([1, 2, 3], chunks=(2,), spec=s), axis=0),
     lambda: np.expand_dims([1, 2, 3], 0)),
    ("moveaxis", lambda s: xp.moveaxis(a3(s), [0, -1], [-1, 0]), lambda: np.moveaxis(np.array(M3), [0, -1], [-1, 0])),
    ("permute_dims", lambda s: xp.permute_dims(a3(s), (1, 0)), lambda: np.array(M3).T),
    ("squeeze_1d", lambda s: xp.squeeze(xp.asarray([[1, 2, 3]], chunks=(1, 2), spec=s), 0),
     lambda: np.array([1, 2, 3])),
    ("squeeze_2d", lambda s: xp.squeeze(xp.asarray([[[1], [2], [3]]], chunks=(1, 2, 1), spec=s), (0, 2)),
     lambda: np.array([1, 2, 3])),
    ("reshape_chunks", lambda s: reshape_chunks(xp.arange(12, chunks=4, spec=s), (2, 6), (2, 2)),
     lambda: np.array([[0, 1, 4, 5, 8, 9], [2, 3, 6, 7, 10, 11]])),
    # searching
    ("argmax_all", lambda s: xp.argmax(xp.asarray(ARGM, chunks=(2, 2), spec=s)), lambda: np.array(ARGM).argmax()),
    ("argmax_0", lambda s: xp.argmax(xp.asarray(ARGM, chunks=(2, 2), spec=s), axis=0),
     lambda: np.array(ARGM).argmax(axis=0)),
    ("argmin_0", lambda s: xp.argmin(xp.asarray(ARGM, chunks=(2, 2), spec=s), axis=0),
     lambda: np.array(ARGM).argmin(axis=0)),
    # statistics
    ("mean_0", lambda s: xp.mean(a3(s, np.float64), axis=0), lambda: np.array(M3, float).mean(axis=0)),
    ("mean_0_new_impl", lambda s: xp.mean(a3(s, np.float64), axis=0, use_new_impl=True),
     lambda: np.array(M3, float).mean(axis=0)),
    ("sum_all", lambda s: xp.sum(a3(s)), lambda: np.array(M3).sum()),
    ("sum_0", lambda s: xp.sum(a3(s), axis=0), lambda: np.array([12, 15, 18])),
    # utility
    ("all_true", lambda s: xp.all(xp.asarray(np.ones((3, 3), bool), chunks=(2, 2), spec=s)), lambda: True),
    ("all_empty", lambda s: xp.all(xp.ones((0,), spec=s)), lambda: True),
]


@pytest.mark.parametrize("name, build, expect", CASES, ids=[c[0] for c in CASES])
def test_reference_behaviour(spec, name, build, expect):
    got = build(spec).compute()
    exp = np.asarray(expect())
    assert got.shape == exp.shape, (got.shape, exp.shape)
    assert np.array_equal(got, exp), (got, exp)


@pytest.mark.parametrize("ind", [6, (6, None), (None, 6), slice(None), slice(10), slice(3, None),
                                 slice(3, 10), (slice(10), None)])
def test_index_1d(spec, ind):
    assert np.array_equal(xp.arange(12, chunks=(4,), spec=spec)[ind].compute(), np.arange(12)[ind])


@pytest.mark.parametrize("ind", [(2, 3), (None, 2, 3), (slice(None), slice(2, 4)), (slice(3), slice(2, None)),
                                 (slice(1, None), slice(4)), (slice(1, 3), slice(None)),
                                 (None, slice(None), slice(2, 4)), (slice(None), None, slice(2, 4)),
                                 (slice(None), slice(2, 4), None), (slice(None), 1), (1, slice(2, 4))])
def test_index_2d(spec, ind):
    assert np.array_equal(a4(spec)[ind].compute(), np.array(M4)[ind])


@pytest.mark.parametrize("shape, chunks, ind, new_chunks", [
    (20, 4, slice(3, 14, 2), ((4, 2),)),
    (20, 5, slice(3, 14, 2), ((4, 2),)),
    (20, 8, slice(5, 18, 3), ((5,),)),
    (50, 5, slice(3, 50, 7), ((5, 2),)),
])
def test_index_1d_step(spec, shape, chunks, ind, new_chunks):
    b = xp.arange(shape, chunks=chunks, spec=spec)[ind]
    assert b.chunks == new_chunks
    assert np.array_equal(b.compute(), np.arange(shape)[ind])


def test_index_2d_step(spec):
    b = xp.ones((20, 20), chunks=(4, 4), spec=spec)[slice(3, 14, 2), slice(3, 14, 3)]
    assert b.chunks == ((4, 2), (3, 1))
    assert np.array_equal(b.compute(), np.ones((20, 20))[3:14:2, 3:14:3])
    with pytest.raises(NotImplementedError):
        xp.arange(12, chunks=(4,), spec=spec)[::-1]


@pytest.mark.parametrize("endpoint", [True, False])
def test_linspace(spec, endpoint):
    for args, n in (((6, 49), 50), ((1.4, 4.9), 13)):
        got = xp.linspace(*args, n, endpoint=endpoint, chunks=5, spec=spec).compute()
        assert np.allclose(got, np.linspace(*args, n, endpoint=endpoint))


@pytest.mark.parametrize("shape, chunks, new_shape, new_chunks, expected_chunks", [
    ((5, 1, 6), (3, 1, 3), (5, 4, 6), None, ((3, 2), (1, 1, 1, 1), (3, 3))),
    ((5, 1, 6), (3, 1, 3), (2, 5, 1, 6), None, ((1, 1), (3, 2), (1,), (3, 3))),
    ((5, 1, 6), (3, 1, 3), (5, 3, 6), (3, 3, 3), ((3, 2), (3,), (3, 3))),
])
def test_broadcast_to(spec, shape, chunks, new_shape, new_chunks, expected_chunks):
    x = np.random.default_rng(0).integers(10, size=shape)
    b = xp.broadcast_to(xp.asarray(x, chunks=chunks, spec=spec), shape=new_shape, chunks=new_chunks)
    assert b.shape == new_shape and b.chunks == expected_chunks
    assert np.array_equal(b.compute(), np.broadcast_to(x, new_shape))


def test_broadcast_arrays(spec):
    for sa, ca in (((30,), (3,)), ((1, 30), (1, 3))):
        a_b, b_b = xp.broadcast_arrays(xp.ones(sa, chunks=ca, spec=spec), xp.ones(30, chunks=(6,), spec=spec))
        assert np.array_equal(a_b.compute(), np.ones(sa)) and np.array_equal(b_b.compute(), np.ones(sa))
