"""Benchmark: effective input GB/s of Cubed's hot path on MI355X.

Headline (``value``) = BASELINE.json configs[1], "quad-means": u, v float32
(1000, 720, 1440) per GPU, chunks (10, 720, 1440), ``xp.mean(u * v, axis=0)``
(fused elementwise + mean), Spec(allowed_mem="2GB", reserved_mem="100MB") as
in the reference's own quad-means test (cubed/tests/test_core.py:527-538).
Inputs are generated on the GPU (bit-exact numpy Philox) and resident in HBM
before timing; a step is one ``plan.execute(executor, resume=True)`` of the
mean's plan (every kernel and collective of the reduction), bracketed by
barrier + synchronize.  value = input bytes of all ranks / time.

``extra`` (same JSON line; each with its own ``roofline`` where one kernel
dominates):
* ``rechunk`` -- configs[2]: 50000^2 f32 row chunks (1000, 50000) -> column
  chunks (50000, 1000), materialised, under the reference-shaped plan
  (``allowed_mem=2GB``: read -> intermediate -> write, 625 + 25 tasks,
  primitive/rechunk.py:23-98) and the 288 GB plan (one copy op); bit-exact
  spot check of target chunks; its own CPU baseline (oracle restatement of
  copy_read_to_write over the same plan);
* ``rechunk_mean`` -- mean(x.rechunk(cols), axis=0) twice: "rechunk elided"
  (the executor reads the rechunk through) and "materialised" (the copy runs,
  then the mean);
* ``config1`` -- (a+1)*2 -> mean(axis=0) on random((20000,20000), (5000,5000));
* ``vorticity`` -- configs[3]: mean(a[1:]*x + b[1:]*y), (1000,900,800) f64;
* ``matmul_f32`` / ``matmul_bf16`` -- configs[4]: xp.matmul of two
  40000^2 arrays in (5000, 5000) chunks (the chunk products and the k-sum as
  one chained-GEMM launch), TFLOP/s against the dense MFMA peak.

Multi-GPU: ``python bench.py --gpus N`` (no torchrun around it) re-launches
itself as N ranks under torch.distributed.run before touching the GPU; under
torchrun, WORLD_SIZE must equal --gpus.  Quad-means weak-scales (each GPU
holds 100 time chunks of u and v: one streaming launch + one RCCL reduce of
the f64 totals, the count host-provided); the rechunk extras strong-scale (50000^2 total: pack -> one
all_to_all over xGMI -> unpack; rechunk+mean reduces before the exchange).

CPU baseline (rank 0, N=1 only): the oracle's restatement of the reference's
executors (oracle/cubed_ref.py) on the SAME inputs copied back from HBM --
sequential (PythonDagExecutor, runtime/executors/python.py:14-32) and
threaded (AsyncPythonDagExecutor's ThreadPoolExecutor, min(32, ncpu + 4)
workers, python_async.py:91,121-142), warm-up excluded, BLAS pinned to one
thread; Zarr/Blosc I/O is not modelled (optimistic for the reference).
"""

from __future__ import annotations

import argparse
import json
import os
import random
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MFMA_PEAK_TFS = {"f32": 157.3, "bf16": 2500.0}  # dense MFMA peaks (MI355X_MICROARCH.md)
EXTRAS = ("rechunk", "rechunk_mean", "rechunk_mean_share", "rechunk_mean_rehearsal", "config1", "vorticity",
          "matmul_f32", "matmul_bf16")
# RCCL all-reduce of the rehearsed ranks' group partials (50000 f64 totals =
# 400 KB, + 50 int64 counts) over 8 GPUs: NOT measured here (one GPU per box);
# an allowance added to the rehearsed per-rank step for the 8-GPU prediction
RCCL_ALLOWANCE_US = 40.0


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--t-length", type=int, default=1000, help="time steps per GPU (quad-means)")
    p.add_argument("--no-extra", action="store_true", help="headline only")
    p.add_argument("--only", default="", help="comma list of extras to run (default: all)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-matmul", action="store_true", help="skip the matmul extras")
    p.add_argument("--matmul-n", type=int, default=40000)
    p.add_argument("--backend", default="nccl",
                   help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to rehearse "
                        "several ranks on one GPU or on CPU)")
    p.add_argument("--rehearse-world", type=int, default=8,
                   help="rechunk_mean_rehearsal: the world size whose ranks are rehearsed on one GPU")
    p.add_argument("--rehearse-rank", default="all",
                   help="rechunk_mean_rehearsal: comma list of ranks to rehearse (default: all)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="per-launch HBM bytes from rocprofv3 PMC (see profiles/README.md)")
    return p.parse_args(argv)


# --------------------------------------------------------------------------- launch


def launcher_command(args_list, gpus, port):
    """The child command that runs this script as ``gpus`` ranks (one process
    per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(args_list)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def maybe_relaunch(args, argv):
    """--gpus N > 1 outside torchrun: run N ranks as a child (before any GPU
    call) and exit with its status.  Under torchrun WORLD_SIZE must agree."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus > 1:
            rc = subprocess.call(launcher_command(argv, args.gpus, free_port()))
            sys.exit(rc)
        return
    if int(world) != args.gpus:
        sys.stderr.write(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}\n")
        sys.exit(2)


def setup_dist(args):
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        dev = local % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group(args.backend)
    else:
        torch.cuda.set_device(0)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def sync():
    import torch

    torch.cuda.synchronize()


def max_over_ranks(dt, world):
    if world > 1:
        import torch
        import torch.distributed as dist

        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


HOST_US = []  # host seconds of each call inside the last timed region


def timed(fn, steps, world):
    """Mean seconds per call over ``steps`` calls, barrier + synchronize on
    both sides, max over ranks.  The host time of each call (the enqueue:
    nothing synchronises inside a step) is kept in HOST_US."""
    sync()
    barrier(world)
    HOST_US.clear()
    t0 = time.perf_counter()
    for _ in range(steps):
        h0 = time.perf_counter()
        fn()
        HOST_US.append(time.perf_counter() - h0)
    sync()
    barrier(world)
    return max_over_ranks((time.perf_counter() - t0) / steps, world)


def timed_launches(ex, fn, steps, world):
    """(seconds per call, {launch key: (count, mean ms)}).  Two passes of
    ``steps`` calls: the step time comes from the plain pass (what a user's
    compute runs: no instrumentation between the launches), the per-launch
    times from a second pass with the executor's HIP events around every
    launch (each event pair adds a few µs to the GPU timeline, which would
    otherwise be charged to the step)."""
    from cubed_amd.runtime.executors.gpu import LaunchTimer

    global INSTR_DT
    dt = timed(fn, steps, world)
    host = list(HOST_US)
    ex.timing = LaunchTimer()
    INSTR_DT = timed(fn, steps, world)
    timer, ex.timing = ex.timing, None
    HOST_US[:] = host
    return dt, timer.summary()


INSTR_DT = None  # step time of the instrumented pass (overhead())


def overhead(dt, summ, steps):
    """Per-step time outside the kernels: ``host_overhead_us`` = step time -
    sum of the step's launch times (HIP events); ``host_enqueue_us`` = the
    median host time of one step call (DAG walk or schedule replay + launch
    calls; it overlaps the previous step's kernels)."""
    launched = sum(c * ms for c, ms in summ.values()) / max(1, steps)
    # against the instrumented pass the launch times come from (its event
    # pairs stretch every launch by a few us; the plain pass's step is shorter)
    idt = INSTR_DT if INSTR_DT is not None else dt
    return {"host_overhead_us": round((idt * 1e3 - launched) * 1e3, 1),
            "host_enqueue_us": round(float(np.median(HOST_US)) * 1e6, 1) if HOST_US else None}


def fmt_launches(summ):
    return {f"{k[0]}#{k[1]}:{k[2]}": round(v[1], 4) for k, v in summ.items()}


def plan_targets(plan, keep):
    """Every array of the plan except ``keep``: marking them unwritten makes
    the next ``execute(resume=True)`` re-run every op (inputs stay resident)."""
    from cubed_amd.storage import DeviceArray

    keep = keep if isinstance(keep, (tuple, list)) else (keep,)
    kept = {id(a.zarray) for a in keep}
    return [d["target"] for _, d in plan._finalize_dag().nodes(data=True)
            if isinstance(d.get("target"), DeviceArray) and id(d["target"]) not in kept]


def step_fn(plan, ex, outs, keep):
    names = [o.name for o in outs]
    targets = plan_targets(plan, keep)

    def step():
        for t in targets:
            t.written = False
        plan.execute(executor=ex, resume=True, array_names=names)
    return step


def load_traffic(path, key):
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    v = d.get(key)
    if isinstance(v, dict):
        return v.get("bytes")
    return v


def roofline_hbm(algo_bytes, ms, traffic_key, args, kernel):
    achieved = algo_bytes / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(args.traffic_json, traffic_key),
            "algo_bytes": algo_bytes, "kernel": kernel}


def free_gpu():
    """Drop the finished extra's arrays.  Their HBM stays in torch's cache for
    the next extra (as in any long-running executor process): handing it back
    to the driver (empty_cache) and re-allocating made the next large array
    slower to stream -- the read-through rechunk + mean 1.58-1.64 vs 1.505 ms
    after the rechunk extra, profiles/r03_alloc_reuse.log."""
    import gc

    gc.collect()


# --------------------------------------------------------------------------- value checks
# Full-size checks of every benchmarked output against a host-side numpy
# restatement of the reference's arithmetic (f64 sums over the same resident
# inputs, copied back chunk by chunk).  A failed check makes bench.py exit 1.

CHECKS = []


def check_close(got, exp, rtol, what):
    got = np.asarray(got, dtype=np.float64)
    exp = np.asarray(exp, dtype=np.float64)
    rel = np.abs(got - exp) / np.maximum(np.abs(exp), 1e-300)
    return {"kind": "oracle", "pass": bool(np.all(rel <= rtol)), "rtol": rtol,
            "max_rel_err": float(np.max(rel)) if rel.size else 0.0, "what": what}


def column_means_f64(arr):
    """f64 mean over axis 0 of a resident 2-d array, chunk rows at a time."""
    import itertools

    acc = np.zeros(arr.shape[1], dtype=np.float64)
    for i, j in itertools.product(range(arr.numblocks[0]), range(arr.numblocks[1])):
        c0 = arr.chunk_start((i, j))[1]
        blk = arr.read_chunk((i, j))
        acc[c0:c0 + blk.shape[1]] += np.sum(blk, axis=0, dtype=np.float64)
    return acc / arr.shape[0]


def device_chunk(arr, coords):
    """torch view (on the device) of one resident chunk, in its dtype."""
    import torch

    tdt = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}
    ext = arr.chunk_extent(coords)
    dt = np.dtype(arr.dtype)
    nb = int(np.prod(ext)) * dt.itemsize
    start = arr.local_slot(coords) * arr.slot_bytes(None)
    raw = arr.slabs[None][start:start + nb]
    return raw.view(tdt.get(dt, torch.bfloat16)).reshape(ext)


# --------------------------------------------------------------------------- workloads


def quad_means(args, rank, world, ex):
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    T = args.t_length * world  # weak scaling: 1000 time steps per GPU
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)
    random.seed(1000)  # same plan (and root seeds) on every rank
    u = xp.astype(crandom.random((T, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    v = xp.astype(crandom.random((T, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=ex, array_names=[u.name, v.name])  # inputs in HBM (untimed)
    sync()
    m = xp.mean(u * v, axis=0)
    plan = arrays_to_plan(m)
    step = step_fn(plan, ex, [m], (u, v))
    for _ in range(args.warmup):
        step()
    dt, summ = timed_launches(ex, step, args.steps, world)
    return dict(in_bytes=u.nbytes + v.nbytes, dt=dt, summ=summ, m=m, u=u, v=v)


def dominant(summ, kind):
    keys = [k for k in summ if k[2] == kind] or list(summ)
    key = max(keys, key=lambda k: summ[k][0] * summ[k][1])
    return key, summ[key][1]


def rechunk_extra(args, ex, rank, world):
    """configs[2]: rechunk 50000^2 f32 rows -> columns, materialised.  The
    2 GB plan is the reference's own (read (2000, 50000) -> int (2000, 2000)
    -> write (50000, 2000): two copy ops); the 288 GB plan is one op."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    N = 50000
    res = {}
    for mem in ("2GB", "288GB"):
        # x carries its Spec: rechunk plans with x.spec.allowed_mem
        spec = cubed.Spec(allowed_mem=mem, executor=ex)
        random.seed(2000)
        x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
        arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
        sync()
        y = x.rechunk((N, 1000))
        plan = arrays_to_plan(y)
        dag = plan._finalize_dag()
        ops = [d for _, d in dag.nodes(data=True) if d.get("op_name") == "rechunk"]
        ntasks = [d["primitive_op"].num_tasks for d in ops]
        step = step_fn(plan, ex, [y], x)
        step()
        dt, summ = timed_launches(ex, step, 10, world)
        copies = {k: v for k, v in summ.items() if k[2] in ("CopyLaunch", "RechunkLaunch")}
        per_op_ms = [v[1] for v in copies.values()]
        r = dict(metric="rechunk effective input GB/s", value=round(x.nbytes / dt / 1e9, 1),
                 ms=round(dt * 1e3, 4), allowed_mem=mem, ops=len(ops), tasks=ntasks,
                 launches_ms=fmt_launches(summ), **overhead(dt, summ, 10))
        if world == 1 and copies:
            key, ms = max(copies.items(), key=lambda kv: kv[1][1])[0], max(per_op_ms)
            # algorithmic bytes of one copy launch: every element read once + written once
            r["roofline"] = roofline_hbm(2 * x.nbytes, ms, "rechunk_copy", args,
                                         f"{key[0]}#{key[1]} ({key[2]}), mean {ms:.4f} ms/launch")
        r["check"] = _rechunk_spot_check(x, y, ex, rank, world)
        CHECKS.append((f"rechunk {mem}", r["check"]))
        res[f"plan_{mem}"] = r
        if mem == "288GB" and rank == 0 and world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_rechunk_baseline(x, ex)
        del x, y, plan
        free_gpu()
    return res


def _rechunk_spot_check(x, y, ex, rank, world):
    """Bit-exact check of the first and last target column chunks (and one
    in the middle) against the source slices they must hold."""
    if world > 1:
        return {"kind": "skipped", "pass": True, "what": "distributed: covered by tests/test_gpu_dist.py"}
    X, Y = x.zarray, y.zarray
    nb = Y.numblocks[1]
    ok = True
    for j in sorted({0, nb // 2, nb - 1}):
        got = Y.read_chunk((0, j))
        c0 = Y.chunk_start((0, j))[1]
        w = got.shape[1]
        for i in (0, X.numblocks[0] // 2, X.numblocks[0] - 1):
            src = X.read_chunk((i, 0))[:, c0:c0 + w]
            r0 = X.chunk_start((i, 0))[0]
            ok &= bool(np.array_equal(got[r0:r0 + src.shape[0]].view(np.uint32), src.view(np.uint32)))
    return {"kind": "oracle", "pass": ok, "what": "bit-exact: 3 target column chunks x 3 source row bands"}


def rechunk_mean_extra(args, ex, rank, world):
    """configs[2] "rechunk+reduce": mean(x.rechunk(columns), axis=0).
    elided: the rechunk feeds only the mean, so the executor reads it
    through (rewrites.elide_rechunks) -- no byte moves, row-chunk pieces
    reduce in place (with N GPUs only partials cross xGMI).  materialised:
    the rechunk copy runs (all_to_all with N GPUs), then the mean."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    N = 50000
    spec = cubed.Spec(allowed_mem="288GB", executor=ex)
    random.seed(2000)
    x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
    arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
    out = {}
    exp = None
    for mode in ("rechunk elided", "materialised"):
        ex.elide_rechunks = mode == "rechunk elided"
        m = xp.mean(x.rechunk((N, 1000)), axis=0)
        plan = arrays_to_plan(m)
        step = step_fn(plan, ex, [m], x)
        step()
        dt, summ = timed_launches(ex, step, 10, world)
        r = dict(metric=f"rechunk+mean effective input GB/s ({mode})", value=round(x.nbytes / dt / 1e9, 1),
                 ms=round(dt * 1e3, 4), launches_ms=fmt_launches(summ), **overhead(dt, summ, 10))
        if world == 1:
            key, ms = dominant(summ, "FusedLaunch")
            if mode.startswith("rechunk"):
                # one read of x (the 50000 f32 means written are 0.002 % more)
                r["roofline"] = roofline_hbm(x.nbytes, ms, "rechunk_mean_stream", args,
                                             f"{key[0]}#{key[1]} ({key[2]}), mean {ms:.4f} ms/launch")
            if exp is None:
                exp = column_means_f64(x.zarray).astype(np.float32)
            got = m.compute(resume=True)
            r["check"] = check_close(got, exp, 1e-6, "oracle: f64 column means of the resident input")
            CHECKS.append((f"rechunk_mean {mode}", r["check"]))
        out["elided" if mode.startswith("rechunk") else "materialised"] = r
        del m, plan
        ex._exec_dags.clear()
    ex.elide_rechunks = True
    return out


def rechunk_mean_share_extra(args, ex, rank, world):
    """The per-rank share of config 3's rechunk+mean on 8 GPUs, timed on one:
    mean(x.rechunk(columns), axis=0) over 6250 of the 50000 source rows
    (row chunks of 1000: 6 full + one of 250), rechunk elided.  With the
    block-cyclic layout the busiest of 8 ranks holds 7 of the 50 row chunks
    (7000 rows); DESIGN.md (e) predicts the 8-GPU step from this piece, the
    per-rank partials (50000 x {n, total}) and one RCCL reduce."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    out = {}
    for rows in (6250, 7000):
        N = 50000
        spec = cubed.Spec(allowed_mem="288GB", executor=ex)
        random.seed(2001)
        x = xp.astype(crandom.random((rows, N), chunks=(1000, N), spec=spec), xp.float32)
        arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
        m = xp.mean(x.rechunk((rows, 1000)), axis=0)
        plan = arrays_to_plan(m)
        step = step_fn(plan, ex, [m], x)
        step()
        step()
        dt, summ = timed_launches(ex, step, 20, world)
        r = dict(metric=f"rechunk+mean share ({rows} of 50000 rows) effective input GB/s",
                 value=round(x.nbytes / dt / 1e9, 1), ms=round(dt * 1e3, 4),
                 launches_ms=fmt_launches(summ), **overhead(dt, summ, 20))
        if world == 1:
            got = m.compute(resume=True)
            exp = column_means_f64(x.zarray).astype(np.float32)
            r["check"] = check_close(got, exp, 1e-6, "oracle: f64 column means of the resident input")
            CHECKS.append((f"rechunk_mean_share {rows}", r["check"]))
        out[f"rows_{rows}"] = r
        del x, m, plan
        free_gpu()
    return out


def rechunk_mean_rehearsal_extra(args, rank, world, t1_ms=None):
    """Config 3's rechunk+reduce as rank r of an N-rank job, rehearsed on this
    one GPU (runtime.comm.LoopbackComm): the executor allocates rank r's
    block-cyclic share of x (50000^2 f32, row chunks of 1000), lowers
    mean(x.rechunk(columns), axis=0) with the rechunk read through exactly as
    on N GPUs (DistPiecesLaunch: this rank's pieces -> SoA partials per output
    group -> collective -> finish of its own output blocks), and every
    collective is a local copy of the same bytes.  The step time is what rank
    r's GPU spends outside xGMI; the 8-GPU prediction adds a stated RCCL
    allowance (RCCL_ALLOWANCE_US, not measured) to the busiest rank."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.comm import LoopbackComm
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    W = args.rehearse_world
    ranks = list(range(W)) if args.rehearse_rank == "all" else [int(r) for r in args.rehearse_rank.split(",")]
    N = 50000
    out = {"world": W, "ranks": {}}
    for r in ranks:
        ex = GpuDagExecutor(comm=LoopbackComm(r, W))
        spec = cubed.Spec(allowed_mem="288GB", executor=ex)
        random.seed(2000)
        x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
        arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
        m = xp.mean(x.rechunk((N, 1000)), axis=0)
        plan = arrays_to_plan(m)
        step = step_fn(plan, ex, [m], x)
        step()
        step()
        dt, summ = timed_launches(ex, step, 20, 1)
        nchunks = len([c for c in range(x.numblocks[0]) if c % W == r])
        out["ranks"][r] = dict(ms=round(dt * 1e3, 4), row_chunks=nchunks,
                               input_gbs=round(nchunks * 1000 * N * 4 / dt / 1e9, 1),
                               launches_ms=fmt_launches(summ), **overhead(dt, summ, 20))
        del x, m, plan, ex
        free_gpu()
    busiest = max(v["ms"] for v in out["ranks"].values())
    out["busiest_ms"] = busiest
    out["rccl_allowance_us"] = RCCL_ALLOWANCE_US
    out["predicted_step_ms"] = round(busiest + RCCL_ALLOWANCE_US / 1e3, 4)
    if t1_ms:
        out["one_gpu_step_ms"] = t1_ms
        out["predicted_speedup"] = round(t1_ms / out["predicted_step_ms"], 2)
    return out


def config1_extra(args, ex, rank, world):
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    random.seed(3000)
    a = crandom.random((20000, 20000), chunks=(5000, 5000), spec=spec)
    arrays_to_plan(a).execute(executor=ex, array_names=[a.name])
    sync()
    m = xp.mean((a + 1) * 2, axis=0)
    plan = arrays_to_plan(m)
    step = step_fn(plan, ex, [m], a)
    for _ in range(2):
        step()
    dt, summ = timed_launches(ex, step, 10, world)
    r = dict(metric="config1 (a+1)*2 -> mean(axis=0) effective input GB/s",
             value=round(a.nbytes / dt / 1e9, 1), ms=round(dt * 1e3, 4), launches_ms=fmt_launches(summ),
             **overhead(dt, summ, 10))
    if world == 1:
        key, ms = dominant(summ, "FusedLaunch")
        r["roofline"] = roofline_hbm(a.nbytes, ms, "config1_stream", args,
                                     f"{key[0]}#{key[1]} ({key[2]}), mean {ms:.4f} ms/launch")
        import itertools

        A = a.zarray
        acc = np.zeros(A.shape[1], dtype=np.float64)
        for i, j in itertools.product(range(A.numblocks[0]), range(A.numblocks[1])):
            c0 = A.chunk_start((i, j))[1]
            blk = A.read_chunk((i, j))
            acc[c0:c0 + blk.shape[1]] += np.sum((blk + 1) * 2, axis=0, dtype=np.float64)
        r["check"] = check_close(m.compute(resume=True), acc / A.shape[0], 1e-12,
                                 "oracle: f64 column sums of (a+1)*2 over the resident 20000^2 input")
        CHECKS.append(("config1", r["check"]))
        if rank == 0 and not args.no_cpu_baseline:
            r["cpu_baseline"] = cpu_config1_baseline(a, acc / A.shape[0])
    return r


def cpu_config1_baseline(a, gpu_exp, row_blocks=2):
    """BASELINE config 1 as the reference runs it: the sequential
    PythonDagExecutor over the finalized plan (add; multiply + _mean_func;
    merge + combine + aggregate) with every intermediate in a LOCAL ZARR
    WORK_DIR (this repo's Zarr v2 writer/reader, blosc-lz4 with byte shuffle:
    numcodecs' default compressor).  ``a`` (the random op's output) is first
    written to the work_dir from HBM (untimed, as its generation is untimed
    on the GPU); the timed sample is the first ``row_blocks`` row bands of
    chunks (all four column chunks), bounded to ~10-30 s."""
    import shutil
    import tempfile

    from oracle import cubed_ref as R
    from cubed_amd.zarr_io import ZarrV2Array, write_device_array

    A = a.zarray
    work = tempfile.mkdtemp(prefix="cubed_cpu_work_")
    try:
        src = ZarrV2Array.create(os.path.join(work, "a"), A.shape, A.dtype, A.chunks)
        write_device_array(A, src)
        t0 = time.perf_counter()
        got = R.config1_python_zarr(src, work, row_blocks=row_blocks)
        dt = time.perf_counter() - t0
        # the sample's mean over its rows, checked against the resident input
        rows = row_blocks * A.chunks[0]
        import itertools

        acc = np.zeros(A.shape[1], dtype=np.float64)
        for i, j in itertools.product(range(row_blocks), range(A.numblocks[1])):
            c0 = A.chunk_start((i, j))[1]
            blk = A.read_chunk((i, j))
            acc[c0:c0 + blk.shape[1]] += np.sum((blk + 1) * 2, axis=0, dtype=np.float64)
        ok = bool(np.allclose(got, acc / rows, rtol=1e-12, atol=0))
    finally:
        shutil.rmtree(work, ignore_errors=True)
    nbytes = rows * A.shape[1] * A.dtype.itemsize
    return {"value": round(nbytes / dt / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{row_blocks} of {A.numblocks[0]} row bands of config 1 ({rows}x{A.shape[1]} f64, "
                      f"{row_blocks * A.numblocks[1]} chunk tasks per op): oracle restatement of the "
                      f"sequential PythonDagExecutor over the reference's finalized plan (add; multiply + "
                      f"_mean_func; merge + combine + aggregate), every intermediate written to and read "
                      f"from a local Zarr v2 work_dir (blosc-lz4 + byte shuffle, this repo's host codec, "
                      f"{{n, total}} partials as two arrays); input a already in the work_dir (untimed); "
                      f"one timed pass; {_cpu_info(1)}",
            "seconds": round(dt, 3), "values_match": ok}


def vorticity_extra(args, ex, rank, world, T=1000):
    """configs[3]: the pangeo-vorticity expression of the reference example
    (examples/pangeo-vorticity.ipynb cell 2) -- mean(a[1:] * x + b[1:] * y)
    with a, b (1000, 900, 800) f64 and x, y (900, 800) f64, chunks 100."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    random.seed(5000)
    a = crandom.random((T, 900, 800), chunks=100, spec=spec)
    b = crandom.random((T, 900, 800), chunks=100, spec=spec)
    x = crandom.random((900, 800), chunks=100, spec=spec)
    y = crandom.random((900, 800), chunks=100, spec=spec)
    arrays_to_plan(a, b, x, y).execute(executor=ex, array_names=[a.name, b.name, x.name, y.name])
    m = xp.mean(a[1:] * x + b[1:] * y)
    plan = arrays_to_plan(m)
    step = step_fn(plan, ex, [m], (a, b, x, y))
    step()
    dt, summ = timed_launches(ex, step, 10, world)
    in_bytes = a.nbytes + b.nbytes + x.nbytes + y.nbytes
    r = dict(metric="vorticity mean(a[1:]*x + b[1:]*y) effective input GB/s",
             value=round(in_bytes / dt / 1e9, 1), ms=round(dt * 1e3, 4), launches_ms=fmt_launches(summ),
             **overhead(dt, summ, 10))
    if world == 1:
        key, ms = dominant(summ, "FusedLaunch")
        # the dominant launch reads a[1:] and b[1:] (x, y broadcast: L2-resident)
        algo = 2 * (T - 1) * 900 * 800 * 8 + 2 * 900 * 800 * 8
        r["roofline"] = roofline_hbm(algo, ms, "vorticity_pieces", args,
                                     f"{key[0]}#{key[1]} ({key[2]}), mean {ms:.4f} ms/launch")
        import itertools

        A, B, X, Y = a.zarray, b.zarray, x.zarray, y.zarray
        xs = {c: X.read_chunk(c) for c in itertools.product(*[range(n) for n in X.numblocks])}
        ys = {c: Y.read_chunk(c) for c in itertools.product(*[range(n) for n in Y.numblocks])}
        total = 0.0
        for c in itertools.product(*[range(n) for n in A.numblocks]):
            ca, cb = A.read_chunk(c), B.read_chunk(c)
            if c[0] == 0:  # a[1:]: the first time row is not read
                ca, cb = ca[1:], cb[1:]
            total += float(np.sum(ca * xs[c[1:]] + cb * ys[c[1:]], dtype=np.float64))
        exp = total / ((T - 1) * 900 * 800)
        r["check"] = check_close(m.compute(resume=True), exp, 1e-12,
                                 "oracle: chunked f64 sum over the resident (1000,900,800) inputs")
        CHECKS.append(("vorticity", r["check"]))
        if rank == 0 and not args.no_cpu_baseline:
            r["cpu_baseline"] = cpu_vorticity_baseline(A, B, X, Y)
    return r


def cpu_vorticity_baseline(A, B, X, Y, t_blocks=2):
    """BASELINE config 4 on the reference's finalized plan (map_direct a[1:],
    b[1:]; multiply by x, y; add + _mean_func; combine + aggregate) restated
    chunk by chunk with in-memory intermediates (no Zarr: optimistic), the
    sequential and the threaded executor; sample = the first ``t_blocks``
    time blocks of a[1:] (all 72 spatial chunks each)."""
    import itertools

    from threadpoolctl import threadpool_limits

    from oracle import cubed_ref as R

    c = A.chunks[0]
    nrows = min(A.shape[0], (t_blocks + 1) * c)

    def host(Z, rows):
        out = np.empty((rows,) + tuple(Z.shape[1:]), dtype=Z.dtype)
        for key in itertools.product(*[range(n) for n in Z.numblocks]):
            st = Z.chunk_start(key)
            if st[0] >= rows:
                continue
            blk = Z.read_chunk(key)
            out[tuple(slice(s, s + e) for s, e in zip(st, blk.shape))] = blk[:rows - st[0]]
        return out

    a, b = host(A, nrows), host(B, nrows)
    x, y = X.to_numpy(), Y.to_numpy()
    threads = min(32, (os.cpu_count() or 1) + 4)
    res = {}
    with threadpool_limits(1):
        for name, th in (("sequential", 1), ("threads", threads)):
            R.vorticity_python(a, b, x, y, c, t_blocks=1, threads=th)  # warm-up
            t0 = time.perf_counter()
            got = R.vorticity_python(a, b, x, y, c, t_blocks=t_blocks, threads=th)
            res[name] = time.perf_counter() - t0
    exp = float(np.mean(a[1:1 + t_blocks * c] * x + b[1:1 + t_blocks * c] * y, dtype=np.float64))
    nbytes = 2 * t_blocks * c * x.size * 8 + 2 * x.size * 8
    return {"value": round(nbytes / res["threads"] / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{t_blocks} of {-(-(A.shape[0] - 1) // c)} time blocks of a[1:], b[1:] "
                      f"({t_blocks * 72} chunk tasks per op): oracle restatement of the reference's finalized "
                      f"plan (index a[1:], b[1:]; * x, * y; add + _mean_func; combine + aggregate) on the "
                      f"threaded executor, in-memory intermediates (no Zarr/Blosc: optimistic), one timed "
                      f"pass after a warm-up; {_cpu_info(threads)}",
            "sequential": {"value": round(nbytes / res["sequential"] / 1e9, 3), "cores": 1},
            "values_match": bool(abs(got - exp) <= 1e-12 * abs(exp))}


def matmul_extra(args, ex, rank, world, dt_name):
    """configs[4]: xp.matmul of two (n, n) arrays in (5000, 5000) chunks,
    f32 or bf16 (inputs Philox f64 -> astype), one chained-GEMM launch."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    n, c = args.matmul_n, 5000
    spec = cubed.Spec(allowed_mem="288GB", executor=ex)
    random.seed(4000)
    xdt = xp.bfloat16 if dt_name == "bf16" else xp.float32
    A = xp.astype(crandom.random((n, n), chunks=(c, c), spec=spec), xdt)
    B = xp.astype(crandom.random((n, n), chunks=(c, c), spec=spec), xdt)
    arrays_to_plan(A, B).execute(executor=ex, array_names=[A.name, B.name])
    m = xp.matmul(A, B)
    plan = arrays_to_plan(m)
    step = step_fn(plan, ex, [m], (A, B))
    step()  # records the launch schedule
    step()  # first replay (one-off host costs) stays out of the two timed steps
    dt, summ = timed_launches(ex, step, 2, world)
    flop = 2.0 * n ** 3
    gemm = [v for k, v in summ.items() if k[2] == "GemmLaunch"]
    r = dict(metric=f"matmul {dt_name} TFLOP/s (whole plan)", value=round(flop / dt / 1e12, 1),
             ms=round(dt * 1e3, 3), n=n, chunk=c, launches_ms=fmt_launches(summ), **overhead(dt, summ, 2))
    if gemm and world == 1:
        gms = gemm[0][1]
        tf = flop / (gms * 1e-3) / 1e12
        r["roofline"] = {"bound": "mfma", "achieved": round(tf, 1), "peak": MFMA_PEAK_TFS[dt_name],
                         "unit": "TFLOP/s", "frac": round(tf / MFMA_PEAK_TFS[dt_name], 4),
                         "traffic": load_traffic(args.traffic_json, f"matmul_{dt_name}"),
                         "algo_flops": flop, "kernel": f"GemmLaunch, mean {gms:.3f} ms/launch"}
    if world == 1:
        r["check"] = matmul_check(A.zarray, B.zarray, m.zarray, n, c, dt_name == "bf16")
        CHECKS.append((f"matmul_{dt_name}", r["check"]))
    return r


def matmul_check(A, B, C, n, c, bf16):
    """64 output entries (8 rows x 8 columns, seeded) against f64 dot products
    of the copied-back operand rows / columns.  Bound (tests/test_gpu_matmul.py):
    8 sqrt(K) 2^-24 sum|a||b| (+ 2^-8 |C| for a bf16 output)."""
    import torch

    rng = np.random.default_rng(5)
    rows = np.sort(rng.choice(n, 8, replace=False))
    cols = np.sort(rng.choice(n, 8, replace=False))
    nk = -(-n // c)
    Ar = torch.stack([torch.cat([device_chunk(A, (i // c, kk))[i % c] for kk in range(nk)])
                      for i in rows]).double().cpu().numpy()
    Bc = torch.stack([torch.cat([device_chunk(B, (kk, j // c))[:, j % c] for kk in range(nk)])
                      for j in cols], dim=1).double().cpu().numpy()
    got = np.array([[float(device_chunk(C, (i // c, j // c))[i % c, j % c].double()) for j in cols]
                    for i in rows])
    exp = Ar @ Bc
    bound = 8.0 * np.sqrt(n) * 2.0 ** -24 * (np.abs(Ar) @ np.abs(Bc))
    if bf16:
        bound = bound + 2.0 ** -8 * np.abs(exp)
    err = np.abs(got - exp)
    return {"kind": "bound", "pass": bool(np.all(err <= bound)), "entries": int(got.size),
            "max_err_over_bound": float(np.max(err / bound)),
            "what": "64 sampled entries vs f64 products of the resident rounded operands"}


# --------------------------------------------------------------------------- CPU baselines


def _cpu_info(threads):
    return (f"numpy {np.__version__}, host cpus {os.cpu_count()}, affinity "
            f"{len(os.sched_getaffinity(0))}, worker threads {threads}, BLAS threads 1")


def cpu_baseline(res, ex):
    """The oracle's restatement of the reference's executors on config 2's
    full inputs (copied back from HBM: the same bytes the GPU read),
    sequential and threaded, warm-up excluded; also checks the GPU mean
    against the oracle's at full size (rtol 1e-6, f32 output)."""
    from threadpoolctl import threadpool_limits

    from oracle import cubed_ref as R

    u = res["u"].zarray.to_numpy()
    v = res["v"].zarray.to_numpy()
    threads = min(32, (os.cpu_count() or 1) + 4)
    out = {}
    with threadpool_limits(1):
        for name, th, reps in (("sequential", 1, 2), ("threads", threads, 3)):
            R.quad_means_cpu(u, v, 10, 2_000_000_000, 100_000_000, threads=th)  # warm-up
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                exp = R.quad_means_cpu(u, v, 10, 2_000_000_000, 100_000_000, threads=th)
                ts.append(time.perf_counter() - t0)
            out[name] = (float(np.median(ts)), th)
    got = res["m"].compute()
    parity = bool(np.allclose(got, exp, rtol=1e-6, atol=0))
    nbytes = u.nbytes + v.nbytes
    dt, th = out["threads"]
    return {"value": round(nbytes / dt / 1e9, 3), "unit": "GB/s", "cores": th, "kind": "port",
            "sample": f"full config 2: quad-means ({u.shape[0]},720,1440) f32 u,v, chunks (10,720,1440), "
                      f"oracle restatement of the reference threads executor (AsyncPythonDagExecutor "
                      f"ThreadPoolExecutor), median of 3 after a warm-up; {_cpu_info(th)}; excludes "
                      f"Zarr/Blosc I/O (optimistic)",
            "sequential": {"value": round(nbytes / out["sequential"][0] / 1e9, 3), "cores": 1,
                           "sample": "same inputs, PythonDagExecutor restatement, median of 2"},
            "gpu_matches_oracle_full_size": parity}


def cpu_rechunk_baseline(x, ex):
    """copy_read_to_write (primitive/rechunk.py:187-192) over the reference's
    2 GB plan (read -> intermediate -> write chunks) restated on numpy
    arrays in memory, on the same 50000^2 f32 input; sequential and threaded
    (one task per target chunk, as the threads executor maps them)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import cubed_ref as R

    X = x.zarray.to_numpy()
    N = X.shape[0]
    read, inter, write = R.rechunking_plan(X.shape, (1000, N), (N, 1000), 4, (2_000_000_000 - 100_000_000) // 4)
    threads = min(32, (os.cpu_count() or 1) + 4)

    def copy_op(src, dst, chunks, pool):
        keys = [(i, j) for i in range(-(-N // chunks[0])) for j in range(-(-N // chunks[1]))]

        def task(k):
            sl = tuple(slice(k[d] * chunks[d], min(N, (k[d] + 1) * chunks[d])) for d in range(2))
            dst[sl] = src[sl]
        if pool is None:
            for k in keys:
                task(k)
        else:
            list(pool.map(task, keys))

    I = np.empty_like(X)
    Y = np.empty_like(X)
    out = {}
    for name, th in (("sequential", 1), ("threads", threads)):
        pool = ThreadPoolExecutor(th) if th > 1 else None
        copy_op(X, I, inter, pool)  # warm-up (page faults of I, Y)
        copy_op(I, Y, write, pool)
        t0 = time.perf_counter()
        copy_op(X, I, inter, pool)
        copy_op(I, Y, write, pool)
        out[name] = time.perf_counter() - t0
        if pool:
            pool.shutdown()
    ok = bool(np.array_equal(Y.view(np.uint32), X.view(np.uint32)))
    return {"value": round(X.nbytes / out["threads"] / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"full config 3: 50000^2 f32, reference 2 GB plan read {read} -> int {inter} -> "
                      f"write {write}, in-memory numpy region copies (no Zarr/Blosc: optimistic), one "
                      f"timed pass after a warm-up; {_cpu_info(threads)}",
            "sequential": {"value": round(X.nbytes / out["sequential"] / 1e9, 3), "cores": 1},
            "values_unchanged": ok}


# --------------------------------------------------------------------------- main


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    maybe_relaunch(args, argv)
    rank, world, local = setup_dist(args)
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    ex = GpuDagExecutor()
    res = quad_means(args, rank, world, ex)
    dt = res["dt"]
    in_bytes = res["in_bytes"]
    value = in_bytes / dt / 1e9  # global input bytes: all ranks
    key, ms = dominant(res["summ"], "FusedLaunch")
    # algorithmic bytes of the dominant launch: the fused u*v -> mean kernel
    # reads this rank's u and v once (2 x 4.147e9 B at T=1000)
    algo = in_bytes // world
    extra = {"launches_ms": fmt_launches(res["summ"]), **overhead(dt, res["summ"], args.steps)}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(res, ex)
        CHECKS.append(("quad-means", {"pass": cpu["gpu_matches_oracle_full_size"]}))
    del res
    free_gpu()
    wanted = [e for e in EXTRAS if not args.only or e in args.only.split(",")]
    if args.no_extra:
        wanted = []
    if args.no_matmul:
        wanted = [e for e in wanted if not e.startswith("matmul")]
    for name in wanted:
        try:
            if name == "rechunk":
                extra[name] = rechunk_extra(args, ex, rank, world)
            elif name == "rechunk_mean":
                extra[name] = rechunk_mean_extra(args, ex, rank, world)
            elif name == "rechunk_mean_share":
                extra[name] = rechunk_mean_share_extra(args, ex, rank, world)
            elif name == "rechunk_mean_rehearsal":
                if world == 1:
                    t1 = extra.get("rechunk_mean", {}).get("elided", {}).get("ms")
                    extra[name] = rechunk_mean_rehearsal_extra(args, rank, world, t1)
            elif name == "config1":
                extra[name] = config1_extra(args, ex, rank, world)
            elif name == "vorticity":
                extra[name] = vorticity_extra(args, ex, rank, world)
            elif name.startswith("matmul"):
                extra[name] = matmul_extra(args, ex, rank, world, name.split("_")[1])
        except Exception as e:  # pragma: no cover - reported, then fails the run
            extra[name] = {"error": repr(e)}
            CHECKS.append((name, {"pass": False, "error": repr(e)}))
        free_gpu()
    line = {
        "metric": "effective input GB/s (node) for fused elementwise+mean (quad-means)",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (on-GPU numpy-Philox U[0,1) inputs, bit-exact with cubed.random)",
        "backend": args.backend if world > 1 else None,
        "config": {"workload": "quad-means: mean(u*v, axis=0), u,v (1000,720,1440) f32 per GPU, "
                               "chunks (10,720,1440), Spec(allowed_mem=2GB, reserved_mem=100MB)",
                   "t_length_per_gpu": args.t_length, "parallelism": f"block-cyclic dp{world}",
                   "extras_scaling": "strong: every extra keeps its total size as N grows (rechunk and "
                                     "rechunk+mean 50000^2, config 1 20000^2, vorticity T=1000, matmul "
                                     "40000^2); only the headline quad-means weak-scales"},
        "roofline": roofline_hbm(algo, ms, "quad_means_fused", args,
                                 f"{key[0]}#{key[1]} ({key[2]}), mean {ms:.4f} ms/launch"),
        "extra": extra,
    }
    if cpu is not None:
        line["cpu_baseline"] = cpu
    failed = [name for name, c in CHECKS if not c.get("pass", False)]
    line["checks_failed"] = failed
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    if failed:
        sys.stderr.write(f"bench.py: value checks failed: {failed}\n")
        sys.exit(1)


if __name__ == "__main__":
    main()
