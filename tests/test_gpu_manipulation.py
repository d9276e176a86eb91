"""concat / stack / reshape / flatten / take / meshgrid on the MI355X path
(``-m gpu``), with the reference's own cases (cubed/tests/test_array_api.py
:281-290 take, :422-433 concat, :460-493 reshape, :510-518 stack) plus
ragged, multi-dim, fused and empty-input cases.  Expected values are numpy's
(the reference's chunk functions are nxp.concat / expand_dims / reshape);
everything here is a byte move, so the bar is bit-exact."""

import random

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
from cubed_amd.array_api.manipulation_functions import reshape_chunks
from oracle import cubed_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spec(gpu_executor):
    return cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=gpu_executor)


def test_concat_reference_case(spec):
    # the middle output chunk reads from three input chunks
    a = xp.full((4, 5), 1, chunks=(3, 2), spec=spec)
    b = xp.full((1, 5), 2, chunks=(3, 2), spec=spec)
    c = xp.full((3, 5), 3, chunks=(3, 2), spec=spec)
    d = xp.concat([a, b, c], axis=0)
    exp = np.concatenate([np.full((4, 5), 1), np.full((1, 5), 2), np.full((3, 5), 3)], axis=0)
    assert np.array_equal(d.compute(), exp)


@pytest.mark.parametrize("axis", [0, 1, 2, -1])
def test_concat_random_ragged(spec, axis):
    random.seed(7)
    shapes = [(5, 6, 7), (5, 6, 7), (5, 6, 7)]
    shapes = [tuple(s if d != axis % 3 else n for d, s in enumerate(sh)) for sh, n in zip(shapes, (3, 1, 8))]
    xs = [crandom.random(sh, chunks=(2, 4, 3), spec=spec) for sh in shapes]
    random.seed(7)
    seeds = [random.getrandbits(128) for _ in shapes]
    npx = [R.random_array(sh, (2, 4, 3), s) for sh, s in zip(shapes, seeds)]
    got = xp.concat(xs, axis=axis).compute()
    assert np.array_equal(got, np.concatenate(npx, axis=axis))


def test_concat_fused_consumer_and_dtype(spec):
    a = xp.asarray(np.arange(10, dtype=np.int32), chunks=3, spec=spec)
    b = xp.asarray(np.arange(100, 107, dtype=np.int64), chunks=4, spec=spec)
    c = xp.negative(xp.concat([a, b]))  # in-degree 1: fused with the concat
    exp = -np.concatenate([np.arange(10), np.arange(100, 107)]).astype(np.int32)
    got = c.compute()
    assert got.dtype == np.int32 and np.array_equal(got, exp)
    assert np.array_equal(xp.sum(xp.concat([a, b])).compute(), exp.sum() * -1)


def test_concat_axis_none(spec):
    a = xp.asarray(np.arange(6).reshape(2, 3), chunks=2, spec=spec)
    b = xp.asarray(np.arange(6, 10).reshape(2, 2), chunks=2, spec=spec)
    got = xp.concat([a, b], axis=None).compute()
    assert np.array_equal(got, np.arange(10))


@pytest.mark.parametrize("axis", [0, 1, 2])
def test_stack_reference_case(spec, axis):
    arrs = [xp.full((4, 6), i + 1, chunks=(2, 3), spec=spec) for i in range(3)]
    exp = np.stack([np.full((4, 6), i + 1) for i in range(3)], axis=axis)
    assert np.array_equal(xp.stack(arrs, axis=axis).compute(), exp)


def test_stack_mixed_chunks(spec):
    a = xp.asarray(np.arange(20.0).reshape(4, 5), chunks=(2, 3), spec=spec)
    b = xp.asarray(np.arange(20.0, 40.0).reshape(4, 5), chunks=(3, 2), spec=spec)
    got = xp.mean(xp.stack([a, b], axis=0), axis=0).compute()
    exp = np.stack([np.arange(20.0).reshape(4, 5), np.arange(20.0, 40.0).reshape(4, 5)]).mean(axis=0)
    assert np.allclose(got, exp, rtol=1e-12, atol=0)


def test_reshape_reference_cases(spec):
    a = xp.arange(12, chunks=4, spec=spec)
    assert np.array_equal(xp.reshape(a, (3, 4)).compute(), np.arange(12).reshape(3, 4))
    b = reshape_chunks(a, (2, 6), (2, 2))
    assert b.chunks == ((2,), (2, 2, 2))
    assert np.array_equal(b.compute(), np.array([[0, 1, 4, 5, 8, 9], [2, 3, 6, 7, 10, 11]]))
    c = reshape_chunks(xp.arange(10, chunks=4, spec=spec), (2, 5), (2, 2))
    assert c.chunks == ((2,), (2, 2, 1))
    assert np.array_equal(c.compute(), np.array([[0, 1, 4, 5, 8], [2, 3, 6, 7, 9]]))


@pytest.mark.parametrize("src, chunks, dst", [
    ((6, 5, 4), (2, 5, 2), (3, 2, 5, 4)),
    ((6, 5, 4), (2, 2, 4), (30, 4)),
    ((24,), (5,), (2, 3, 4)),
    ((2, 3, 4), (1, 2, 3), (-1,)),
    ((4, 1, 6), (2, 1, 3), (4, 6, 1)),
])
def test_reshape_random(spec, src, chunks, dst):
    random.seed(3)
    x = crandom.random(src, chunks=chunks, spec=spec)
    random.seed(3)
    ref = R.random_array(src, chunks, random.getrandbits(128))
    got = xp.reshape(x, dst).compute()
    assert np.array_equal(got, ref.reshape(dst))


def test_reshape_irregular_rechunk_raises_like_reference(spec):
    # reshape_rechunk asks for chunks (2, 4) along dim 0; the reference's
    # rechunk(x, to_chunksize(...)) rejects irregular chunks the same way
    x = xp.ones((6, 5, 4), chunks=(3, 5, 2), spec=spec)
    with pytest.raises(ValueError, match="regular chunks"):
        xp.reshape(x, (3, 2, 5, 4))


def test_reshape_then_reduce(spec):
    a = xp.arange(24, chunks=4, spec=spec)
    got = xp.sum(xp.reshape(a, (4, 6)), axis=0).compute()
    assert np.array_equal(got, np.arange(24).reshape(4, 6).sum(axis=0))


@pytest.mark.parametrize("axis", [0, 1])
def test_take_reference_case(spec, axis):
    x = np.array([[1, 2, 3, 4], [5, 6, 7, 8], [9, 10, 11, 12], [13, 14, 15, 16]])
    a = xp.asarray(x, chunks=(2, 2), spec=spec)
    b = xp.asarray([1, 2], spec=spec)
    assert np.array_equal(xp.take(a, b, axis=axis).compute(), x.take([1, 2], axis=axis))


@pytest.mark.parametrize("indexing", ["xy", "ij"])
def test_meshgrid(spec, indexing):
    x = xp.arange(5, chunks=2, spec=spec)
    y = xp.arange(3, chunks=2, spec=spec)
    got = [g.compute() for g in xp.meshgrid(x, y, indexing=indexing)]
    exp = np.meshgrid(np.arange(5), np.arange(3), indexing=indexing)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)
