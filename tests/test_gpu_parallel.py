"""``compute_arrays_in_parallel`` on the MI355X (``-m gpu``): the ops of one
topological generation run on separate HIP streams, joined before the next
generation (``runtime/executors/python_async.py:86-114``; the reference test
``test_executor_features.py:153-171`` only checks that the flag is accepted).
Here the results are compared bit-exactly with the oracle and with the
sequential walk, and the TaskEndEvents with the reference's task counts."""

import random

import numpy as np
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
from cubed_amd.core.plan import arrays_to_plan
from cubed_amd.runtime.types import Callback
from oracle import cubed_ref as R

pytestmark = pytest.mark.gpu


class Rec(Callback):
    def __init__(self):
        self.events = []

    def on_task_end(self, event):
        self.events.append(event)


def seeds(seed, n):
    random.seed(seed)
    return [random.getrandbits(128) for _ in range(n)]


@pytest.mark.parametrize("parallel", [True, False])
def test_compute_arrays_in_parallel(gpu_executor, parallel):
    ex = gpu_executor
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    random.seed(21)
    a = crandom.random((10, 10), chunks=(5, 5), spec=spec)
    b = crandom.random((10, 10), chunks=(5, 5), spec=spec)
    c = xp.add(a, b)
    s1, s2 = seeds(21, 2)
    exp = R.random_array((10, 10), (5, 5), s1) + R.random_array((10, 10), (5, 5), s2)
    got = c.compute(executor=ex, compute_arrays_in_parallel=parallel)
    np.testing.assert_array_equal(got, exp)


def test_independent_pipelines_on_side_streams(gpu_executor):
    """Four independent materialised arrays (two Philox fills, two maps over
    them in the next generation) and a reduction of all four: every value
    bit-exact / rtol 1e-12 against the oracle, forks counted, one
    TaskEndEvent per op with its task count, ends after starts."""
    ex = gpu_executor
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    random.seed(22)
    a = crandom.random((300, 400), chunks=(100, 100), spec=spec)
    b = crandom.random((300, 400), chunks=(100, 100), spec=spec)
    s1, s2 = seeds(22, 2)
    A = R.random_array((300, 400), (100, 100), s1)
    B = R.random_array((300, 400), (100, 100), s2)
    forks = getattr(ex, "parallel_forks", 0)
    rec = Rec()
    arrays_to_plan(a, b).execute(executor=ex, array_names=[a.name, b.name], callbacks=[rec],
                                 compute_arrays_in_parallel=True)
    assert getattr(ex, "parallel_forks", 0) > forks
    assert len(rec.events) >= 2
    assert all(e.function_end_tstamp >= e.function_start_tstamp for e in rec.events)
    c = a * 3
    d = b + 2
    plan = arrays_to_plan(c, d)
    plan.execute(executor=ex, array_names=[c.name, d.name], resume=True, compute_arrays_in_parallel=True)
    np.testing.assert_array_equal(c.compute(resume=True), A * 3)
    np.testing.assert_array_equal(d.compute(resume=True), B + 2)
    m1 = xp.mean(c, axis=0)
    m2 = xp.sum(d, axis=1)
    p2 = arrays_to_plan(m1, m2)
    rec = Rec()
    p2.execute(executor=ex, array_names=[m1.name, m2.name], resume=True, callbacks=[rec],
               compute_arrays_in_parallel=True)
    p2.execute(executor=ex, array_names=[m1.name, m2.name], resume=False, compute_arrays_in_parallel=True)
    assert np.allclose(m1.compute(resume=True), np.mean(A * 3, axis=0), rtol=1e-12, atol=0)
    assert np.allclose(m2.compute(resume=True), np.sum(B + 2, axis=1), rtol=1e-12, atol=0)
    dag = p2._finalize_dag()
    tasks = {n: d["primitive_op"].num_tasks for n, d in dag.nodes(data=True) if "primitive_op" in d}
    for e in rec.events:
        if e.array_name in tasks:
            assert e.num_tasks == tasks[e.array_name]
