"""The executor's recorded launch schedules and buffer lifetimes (CPU, dry
lowering: the exact launch objects the GPU path would run, none executed).

* A repeated ``Plan.execute`` with the same plan, array names, resume flag
  and written state replays the recorded launch list instead of re-walking
  the DAG (runtime/executors/python.py:17-32 is the loop this replaces);
  a different written state re-walks it.
* Scratch gathers and split temporaries belong to the cache entry of the
  launches that use them: dropping the plan frees them.
* TaskEndEvents carry per-op start/end times and the reference's counts.
"""

import gc
import random

import numpy as np

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
from cubed_amd.core.plan import arrays_to_plan
from cubed_amd.storage import DeviceArray


def _reset(plan, keep):
    kept = {id(a.zarray) for a in keep}
    for _, d in plan._finalize_dag().nodes(data=True):
        t = d.get("target")
        if isinstance(t, DeviceArray) and id(t) not in kept:
            t.written = False


def test_repeat_execute_replays_the_recorded_launches(built, dry):
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(7)
    u = xp.astype(crandom.random((40, 30, 20), chunks=(10, 30, 20), spec=spec), xp.float32)
    v = xp.astype(crandom.random((40, 30, 20), chunks=(10, 30, 20), spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=dry, array_names=[u.name, v.name])
    m = xp.mean(u * v, axis=0)
    plan = arrays_to_plan(m)
    runs = []
    for _ in range(3):
        _reset(plan, (u, v))
        dry.launched.clear()
        before = dry.replays
        plan.execute(executor=dry, resume=True, array_names=[m.name])
        runs.append((dry.replays - before, [id(l) for l in dry.launched]))
    assert runs[0][0] == 0 and runs[1][0] == 1 and runs[2][0] == 1
    assert runs[0][1] == runs[1][1] == runs[2][1] and runs[0][1]
    # the inputs were not regenerated (resume): only the mean's launch ran
    assert len(runs[0][1]) == 1


def test_changed_written_state_rewalks_the_dag(built, dry):
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(8)
    a = crandom.random((40, 40), chunks=(10, 10), spec=spec)
    m = xp.mean((a + 1) * 2, axis=0)
    plan = arrays_to_plan(m)
    dry.launched.clear()
    plan.execute(executor=dry, resume=True, array_names=[m.name])
    assert dry.launched
    # everything is written now: resume skips every op (a new state, so the
    # DAG is walked again and the empty schedule recorded)
    dry.launched.clear()
    before = dry.replays
    plan.execute(executor=dry, resume=True, array_names=[m.name])
    assert dry.replays == before and not dry.launched
    plan.execute(executor=dry, resume=True, array_names=[m.name])
    assert dry.replays == before + 1 and not dry.launched
    # back to the first state: its recorded schedule replays
    _reset(plan, ())
    plan.execute(executor=dry, resume=True, array_names=[m.name])
    assert dry.replays == before + 2 and dry.launched


def test_released_array_invalidates_the_schedule(built, dry):
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(9)
    a = crandom.random((40, 40), chunks=(10, 10), spec=spec)
    arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
    m = xp.sum(a, axis=0)
    plan = arrays_to_plan(m)
    plan.execute(executor=dry, resume=True, array_names=[m.name])
    _reset(plan, (a,))
    m.zarray.release()
    before = dry.replays
    plan.execute(executor=dry, resume=True, array_names=[m.name])
    assert dry.replays == before


def test_split_temporaries_are_freed_with_their_plan(built, dry):
    """split temporaries lived as long as the executor.  They
    now belong to the cached launches of their pipeline."""
    from cubed_amd.core.optimization import fuse_all_optimize_dag

    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    gc.collect()
    base = dry.owned_bytes()
    for seed in range(3):
        random.seed(seed)
        u = crandom.random((50, 1, 98, 192), chunks=(10, 1, -1, -1), spec=spec)
        v = crandom.random((50, 1, 98, 192), chunks=(10, 1, -1, -1), spec=spec)
        m = xp.mean(u * v, axis=0)
        arrays_to_plan(m).execute(executor=dry, array_names=[m.name],
                                  optimize_function=fuse_all_optimize_dag)
        # one materialised random stream: 50 x 98 x 192 f64
        assert dry.owned_bytes() - base >= 50 * 98 * 192 * 8
        del u, v, m
        gc.collect()
        assert dry.owned_bytes() == base
    assert not [k for k in dry._cache if dry._cache[k][0]() is None]


def test_split_temporary_checked_against_hbm(built, dry, monkeypatch):
    import pytest

    import cubed_amd.runtime.executors.gpu as g
    from cubed_amd.core.optimization import fuse_all_optimize_dag

    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(3)
    u = crandom.random((50, 1, 98, 192), chunks=(10, 1, -1, -1), spec=spec)
    v = crandom.random((50, 1, 98, 192), chunks=(10, 1, -1, -1), spec=spec)
    m = xp.mean(u * v, axis=0)
    monkeypatch.setattr(g, "HBM_BYTES_PER_GPU", 50 * 98 * 192 * 8)
    with pytest.raises(MemoryError, match="split temporary"):
        arrays_to_plan(m).execute(executor=dry, array_names=[m.name],
                                  optimize_function=fuse_all_optimize_dag)


def test_task_end_events_per_op_with_times(built, dry):
    from cubed_amd.runtime.types import Callback

    class Rec(Callback):
        def __init__(self):
            self.events = []

        def on_task_end(self, event):
            self.events.append(event)

    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(10)
    a = crandom.random((40, 40), chunks=(10, 10), spec=spec)
    m = xp.mean(a, axis=0)
    plan = arrays_to_plan(m)
    for _ in range(2):  # recorded, then replayed: same events
        rec = Rec()
        _reset(plan, ())
        plan.execute(executor=dry, callbacks=[rec], resume=True, array_names=[m.name])
        names = [e.array_name for e in rec.events]
        assert len(names) == len(set(names))
        assert all(e.function_end_tstamp >= e.function_start_tstamp for e in rec.events)
        ends = [e.function_end_tstamp for e in rec.events]
        assert ends == sorted(ends)
        tasks = {e.array_name: e.num_tasks for e in rec.events}
        dag = plan._finalize_dag()
        for name, d in dag.nodes(data=True):
            if name in tasks and "primitive_op" in d:
                assert tasks[name] == d["primitive_op"].num_tasks
    assert np.isfinite(ends[-1])


def test_compute_arrays_in_parallel_groups_generations(built, dry):
    """``compute_arrays_in_parallel`` (python_async.py:86-114): the schedule
    is grouped by topological generation -- the two independent random
    arrays' ops share one group (each on its own stream on a GPU), a later
    op sits in a later group -- and the launches are the sequential walk's."""
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(12)
    a = crandom.random((40, 40), chunks=(10, 10), spec=spec)
    b = crandom.random((40, 40), chunks=(10, 10), spec=spec)
    plan = arrays_to_plan(a, b)
    dag = plan._finalize_dag()
    op_a = next(iter(dag.predecessors(a.name)))
    op_b = next(iter(dag.predecessors(b.name)))

    dry.launched.clear()
    plan.execute(executor=dry, compute_arrays_in_parallel=True, array_names=[a.name, b.name])
    sched = dry.last_schedule
    assert sched.parallel
    groups = [[sched.steps[i][0] for i in g] for g in sched.groups]
    (both,) = [g for g in groups if op_a in g]
    assert op_b in both
    i_a = [st[0] for st in sched.steps].index(op_a)
    i_b = [st[0] for st in sched.steps].index(op_b)
    assert sched.forkable[i_a] and sched.forkable[i_b]
    par = [type(l).__name__ for l in dry.launched]

    for t in (a.zarray, b.zarray):
        t.written = False
    dry.launched.clear()
    plan.execute(executor=dry, array_names=[a.name, b.name])
    assert not dry.last_schedule.parallel
    assert all(len(g) == 1 for g in dry.last_schedule.groups)
    assert sorted(par) == sorted(type(l).__name__ for l in dry.launched)


def test_parallel_chain_runs_with_its_last_member(built, dry):
    """A fused reduction chain's one launch reads what every member reads,
    so in a generation walk it is placed in its last member's generation."""
    spec = cubed.Spec(allowed_mem="2GB", executor=dry)
    random.seed(13)
    a = crandom.random((40, 40), chunks=(10, 10), spec=spec)
    arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
    m = xp.mean(a * 2, axis=0)
    s = xp.sum(a + 1, axis=1)
    plan = arrays_to_plan(m, s)
    plan.execute(executor=dry, compute_arrays_in_parallel=True, resume=True, array_names=[m.name, s.name])
    sched = dry.last_schedule
    gens = [st[4] for st in sched.steps]
    assert gens == sorted(gens)
    chains, _ = dry.chains_of(dry.exec_dag(plan._finalize_dag(), [m.name, s.name]), [m.name, s.name])
    assert chains
    import networkx as nx

    exec_dag = dry.exec_dag(plan._finalize_dag(), [m.name, s.name])
    gen_of = {n: g for g, names in enumerate(nx.topological_generations(exec_dag)) for n in names}
    for head, ch in chains.items():
        (st,) = [st for st in sched.steps if st[0] == head]
        assert st[4] == max(gen_of[n] for n in ch.nodes)


def test_lowering_failure_runs_the_lowered_prefix(built, dry):
    """a plan whose later op cannot be lowered (an untraceable
    chunk function) raises LoweringError after running the ops lowered
    before it -- they are marked written, as the reference's op-by-op
    executor would have completed them, so a resume picks up after them."""
    import numpy as np
    import pytest

    import cubed_amd as cubed
    from cubed_amd.core.ops import map_blocks
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.lowering import LoweringError

    spec = cubed.Spec(allowed_mem="1GB", executor=dry)
    a = cubed.from_array(np.arange(16.0).reshape(4, 4), chunks=(2, 2), spec=spec)
    b = a + 1

    def opaque(x):
        return np.asarray(sorted(x.ravel())).reshape(x.shape)  # not traceable

    c = map_blocks(opaque, b, dtype=b.dtype)
    plan = arrays_to_plan(c)
    dry.launched.clear()
    with pytest.raises(LoweringError):
        plan.execute(executor=dry, array_names=[c.name], optimize_graph=False)
    assert dry.launched  # b's op ran
    assert b.zarray.written and not c.zarray.written
