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
EXTRAS = ("rechunk", "rechunk_rehearsal", "rechunk_mean", "rechunk_mean_share", "rechunk_mean_rehearsal",
          "config1", "vorticity", "var", "matmul_f32", "matmul_bf16", "matmul_rehearsal")
# RCCL all-reduce of the rehearsed ranks' group partials (50000 f64 totals =
# 400 KB, + 50 int64 counts) over 8 GPUs: NOT measured here (one GPU per box);
# an allowance added to the rehearsed per-rank step for the 8-GPU prediction
RCCL_ALLOWANCE_US = 40.0
# ... and for a REDUCE-SCATTER of the same partials (several owners of the
# output blocks, dist.ScatterCombine): a ring reduce-scatter is the first
# half of a ring all-reduce -- (W-1) of its 2(W-1) latency-bound steps, on
# 1/W of the bytes per step -- so half the allowance (same assumption)
RCCL_SCATTER_ALLOWANCE_US = RCCL_ALLOWANCE_US / 2
# xGMI: 7 links per MI355X, one to each peer of an 8-GPU node, ~153 GB/s per
# direction each (task statement / SURVEY.md §5; not measured here): the
# rechunk_rehearsal prediction of the per-pair transfers
XGMI_LINK_GBS = 153.0


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


EVENT_MS = []  # GPU ms per call of the last timed region (HIP events around it)


def timed(fn, steps, world):
    """Mean seconds per call over ``steps`` calls, barrier + synchronize on
    both sides, max over ranks.  The host time of each call (the enqueue:
    nothing synchronises inside a step) is kept in HOST_US; HIP events on the
    current stream (the executor's) bracket the timed region, and the GPU
    time per call they measure is kept in EVENT_MS."""
    import torch

    sync()
    barrier(world)
    HOST_US.clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        h0 = time.perf_counter()
        fn()
        HOST_US.append(time.perf_counter() - h0)
    e1.record()
    sync()
    barrier(world)
    EVENT_MS[:] = [e0.elapsed_time(e1) / steps]
    return max_over_ranks((time.perf_counter() - t0) / steps, world)


def timed_launches(ex, fn, steps, world):
    """(seconds per call, {launch key: (count, mean ms)}).  Two passes of
    ``steps`` calls: the step time comes from the plain pass (what a user's
    compute runs: no instrumentation between the launches), the per-launch
    times from a second pass with the executor's HIP events around every
    launch (each event pair adds a few µs to the GPU timeline, which would
    otherwise be charged to the step)."""
    from cubed_amd.runtime.executors.gpu import LaunchTimer

    global INSTR_DT, PLAIN_EVENT_MS
    dt = timed(fn, steps, world)
    PLAIN_EVENT_MS = EVENT_MS[0]
    host = list(HOST_US)
    ex.timing = LaunchTimer()
    INSTR_DT = timed(fn, steps, world)
    timer, ex.timing = ex.timing, None
    HOST_US[:] = host
    return dt, timer.summary()


INSTR_DT = None  # step time of the instrumented pass (overhead())
PLAIN_EVENT_MS = None  # GPU ms per step of the plain pass (HIP events around the timed region)


def launch_symbols(ex, kind="FusedLaunch"):
    """Kernel symbols of the executor's cached launches of ``kind`` (the JIT
    kernels carry a per-program digest, so a rocprof row names one program)."""
    import re

    from cubed_amd import _native as nat

    out = []
    for v in ex._cache.values():
        for l in v[1]:
            h = getattr(l, "handle", None)
            if type(l).__name__ == kind and h is not None:
                m = re.search(r"void (cubed_\w+)\(", nat.program_source(h))
                if m:
                    out.append(m.group(1))
    return out


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


def roofline_step(algo_bytes, dt):
    """With several ranks: one rank's algorithmic HBM bytes over the WHOLE
    per-rank step (kernels + collectives + finish), max over ranks.  No PMC
    pass exists per rank, so ``traffic`` is null."""
    achieved = algo_bytes / dt / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "algo_bytes": int(algo_bytes),
            "kernel": "whole per-rank step (every launch and collective), max over ranks"}


def free_gpu():
    """Drop the finished extra's arrays.  Their HBM stays in torch's cache for
    the next extra (as in any long-running executor process): handing it back
    to the driver (empty_cache) and re-allocating made the next large array
    slower to stream -- the read-through rechunk + mean 1.58-1.64 vs 1.505 ms
    after the rechunk extra, profiles/r03_alloc_reuse.log."""
    import gc

    gc.collect()


# --------------------------------------------------------------------------- value checks
# Full-size checks of every benchmarked output, at every world size: every
# output position of the reductions (the rechunk: 3 x 3 bands bit for bit,
# the matmul: 64 entries against f64 dot products).  The
# expected values are restated with torch f64 arithmetic over the SAME
# resident inputs (independent of this repo's kernels): each rank reduces
# the chunks it owns, one f64 all-reduce sums the ranks' shares (each output
# element's computed value is contributed by its one owner, zeros elsewhere),
# and every rank then compares the same numbers -- so an N-GPU line can only
# report checks that combined every rank's data.  Rechunk targets are
# compared bit for bit with a local regeneration of the Philox source.  A
# failed check makes bench.py exit 1 (``finish``).

CHECKS = []


def _dist():
    """torch.distributed when it runs with > 1 rank, else None."""
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist
    return None


def allreduce_(t, op="sum"):
    """In-place all-reduce over the world (a no-op on one rank); gloo stages
    device tensors through the host."""
    dist = _dist()
    if dist is None:
        return t
    o = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}[op]
    if str(dist.get_backend()).lower() == "gloo" and t.device.type != "cpu":
        h = t.cpu()
        dist.all_reduce(h, op=o)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=o)
    return t


def check_close(got, exp, rtol, what):
    got = np.asarray(got, dtype=np.float64)
    exp = np.asarray(exp, dtype=np.float64)
    rel = np.abs(got - exp) / np.maximum(np.abs(exp), 1e-300)
    return {"kind": "oracle", "pass": bool(np.all(rel <= rtol)), "rtol": rtol,
            "max_rel_err": float(np.max(rel)) if rel.size else 0.0, "what": what}


def sampled_check(exp_part, got_part, denom, rtol, what):
    """``exp_part``: this rank's share (f64) of the expected sums at k sampled
    outputs; ``got_part``: the computed outputs at the sampled positions this
    rank owns (0 elsewhere).  Both are summed over the ranks; every rank then
    compares got with exp / denom at ``rtol`` -- the same verdict everywhere."""
    import torch

    buf = torch.stack([exp_part.reshape(-1).double(), got_part.reshape(-1).double()])
    allreduce_(buf)
    exp, got = (buf[0] / denom).cpu().numpy(), buf[1].cpu().numpy()
    r = check_close(got, exp, rtol, what)
    r.update(kind="sampled", entries=int(exp.size), world=world_size())
    return r


def agreed(ok: bool) -> bool:
    """True iff every rank's ``ok`` is True."""
    import torch

    dist = _dist()
    if dist is None:
        return bool(ok)
    dev = "cpu" if str(dist.get_backend()).lower() == "gloo" else "cuda"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    allreduce_(t, "min")
    return bool(t.item())


def world_size() -> int:
    dist = _dist()
    return dist.get_world_size() if dist is not None else 1


def device_chunk(arr, coords):
    """torch view (on the device) of one resident chunk this rank owns, in
    its dtype."""
    import torch

    tdt = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}
    ext = arr.chunk_extent(coords)
    dt = np.dtype(arr.dtype)
    nb = int(np.prod(ext)) * dt.itemsize
    start = arr.local_slot(coords) * arr.slot_bytes(None)
    raw = arr.slabs[None][start:start + nb]
    return raw.view(tdt.get(dt, torch.bfloat16)).reshape(ext)


def owned_chunks(arr):
    import itertools

    for coords in itertools.product(*[range(n) for n in arr.numblocks]):
        if arr.owner(coords) == arr.rank:
            yield coords


def sample_columns(shape, k, seed):
    """k distinct multi-indices into ``shape`` (seeded, sorted)."""
    rng = np.random.default_rng(seed)
    size = int(np.prod(shape))
    flat = np.sort(rng.choice(size, min(k, size), replace=False))
    return np.stack(np.unravel_index(flat, shape), axis=1) if shape else np.zeros((1, 0), np.int64)


def owned_axis0_sums(arrs, fn, center=None):
    """f64 sums over axis 0 of ``fn(*chunks)`` at EVERY output position, over
    the chunks of ``arrs`` (equal chunking) this rank owns (0 elsewhere).
    ``fn`` gets the chunks in their own dtype (numpy's arithmetic: f32 * f32
    stays f32) and its result is summed in f64 (statistical_functions.py:57,
    ``dtype=float64``).  ``center`` (the output's shape): sum the squared
    deviations from it instead (a two-pass variance)."""
    import torch

    A = arrs[0]
    acc = torch.zeros(A.shape[1:], dtype=torch.float64, device=A.device)
    for coords in owned_chunks(A):
        st, ext = A.chunk_start(coords)[1:], A.chunk_extent(coords)[1:]
        sl = tuple(slice(a, a + e) for a, e in zip(st, ext))
        val = fn(*[device_chunk(a, coords) for a in arrs]).double()
        if center is not None:
            val = (val - center[sl]) ** 2
        acc[sl] += val.sum(0)
    return acc


def owned_output_full(M):
    """Every computed output of ``M`` this rank owns (f64, 0 elsewhere)."""
    import torch

    got = torch.zeros(M.shape, dtype=torch.float64, device=M.device)
    for coords in owned_chunks(M):
        st, ext = M.chunk_start(coords), M.chunk_extent(coords)
        got[tuple(slice(a, a + e) for a, e in zip(st, ext))] = device_chunk(M, coords).double()
    return got


def owned_output_values(M, cols):
    """The computed outputs of ``M`` at ``cols`` (k, M.ndim) this rank owns
    (f64, 0 elsewhere)."""
    import torch

    got = torch.zeros(len(cols), dtype=torch.float64, device=M.device)
    for n, idx in enumerate(cols):
        coords = tuple(M.chunk_of(d, int(i)) for d, i in enumerate(idx))
        if M.owner(coords) != M.rank:
            continue
        st = M.chunk_start(coords)
        ch = device_chunk(M, coords)
        got[n] = ch[tuple(int(i) - s for i, s in zip(idx, st))].double()
    return got


def column_mean_check(inputs, out, fn, rtol, what):
    """mean over axis 0 of fn(*inputs), checked at EVERY output position on
    every world size: each rank sums its own input chunks and fills its own
    output chunks, one f64 all-reduce of the two output-sized vectors."""
    M = out.zarray
    exp = owned_axis0_sums([a.zarray for a in inputs], fn)
    got = owned_output_full(M)
    r = sampled_check(exp, got, inputs[0].shape[0], rtol, what)
    r["kind"] = "full"
    return r


def full_host(arr):
    """Every chunk of a (small) resident array on the host, on every rank."""
    if arr.world == 1:
        return arr.to_numpy()
    from cubed_amd.runtime.executors.dist import gather_distributed

    return gather_distributed(arr)


def rank_info(backend):
    """What this rank's process group is (recorded in the line per rank)."""
    import torch

    dist = _dist()
    info = {"world_size": dist.get_world_size() if dist is not None else 1,
            "backend": str(dist.get_backend()) if dist is not None else None,
            "device": torch.cuda.current_device() if torch.cuda.is_available() else None}
    try:
        v = torch.cuda.nccl.version()
        info["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception as e:  # noqa: BLE001 -- reported, not fatal
        info["rccl_version"] = f"unavailable ({type(e).__name__})"
    if dist is None:
        return [dict(info, rank=0)]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, dict(info, rank=dist.get_rank()))
    return out


def finish(line, checks, rank, world):
    """Agree on the failed checks over all ranks, print the line on rank 0;
    the exit status (1 when any rank saw a failed check)."""
    failed = [name for name, c in checks if not c.get("pass", False)]
    ok = agreed(not failed)
    if not ok and not failed:
        failed = ["(another rank)"]
    line["checks_failed"] = failed
    line["checks_run"] = len(checks)
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0 if ok else 1


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
    return dict(in_bytes=u.nbytes + v.nbytes, dt=dt, summ=summ, m=m, u=u, v=v, plain_event_ms=PLAIN_EVENT_MS,
                symbols=launch_symbols(ex))


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
    xl = regenerate_source((N, N), (1000, N), 2000)  # the checks' source (every rank, whole)
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
        elif world > 1:
            # per rank: its source rows read once + its target columns written once
            r["roofline"] = roofline_step(2 * x.nbytes // world, dt)
        r["check"] = rechunk_check(xl, y)
        CHECKS.append((f"rechunk {mem}", r["check"]))
        res[f"plan_{mem}"] = r
        if mem == "288GB" and rank == 0 and world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_rechunk_baseline(x, ex)
        del x, y, plan
        free_gpu()
    del xl
    free_gpu()
    return res


def regenerate_source(shape, chunks, seed):
    """The rechunk source x = astype(random(shape, chunks), f32) rebuilt
    WHOLE on this rank by a single-GPU executor (same root seed, same block
    offsets: cubed/random.py:31-36), so every rank can check its target
    chunks without any peer data."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    local = GpuDagExecutor(comm=None)
    spec = cubed.Spec(allowed_mem="288GB", executor=local)
    random.seed(seed)
    xl = xp.astype(crandom.random(shape, chunks=chunks, spec=spec), xp.float32)
    arrays_to_plan(xl).execute(executor=local, array_names=[xl.name])
    sync()
    return xl


def rechunk_check(xl, y):
    """Bit-exact check of EVERY target chunk this rank owns against the
    regenerated source ``xl`` (row chunks) -- then agreed over the ranks."""
    import torch

    X, Y = xl.zarray, y.zarray
    ok, nchunks, nbytes = True, 0, 0
    for tc in owned_chunks(Y):
        got = device_chunk(Y, tc)
        t0 = Y.chunk_start(tc)
        te = Y.chunk_extent(tc)
        for i in range(X.numblocks[0]):
            r0, rows = X.chunk_start((i, 0))[0], X.chunk_extent((i, 0))[0]
            lo, hi = max(r0, t0[0]), min(r0 + rows, t0[0] + te[0])
            if lo >= hi:
                continue
            src = device_chunk(X, (i, 0))[lo - r0:hi - r0, t0[1]:t0[1] + te[1]]
            ok &= bool(torch.equal(got[lo - t0[0]:hi - t0[0]].view(torch.int32), src.view(torch.int32)))
        nchunks += 1
        nbytes += got.numel() * 4
    sync()
    return {"kind": "bit-exact", "pass": agreed(ok), "world": world_size(),
            "what": f"every target chunk vs a local Philox regeneration of the source; this rank "
                    f"{nchunks} chunks, {nbytes} B"}


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
        elif mode.startswith("rechunk"):
            r["roofline"] = roofline_step(x.nbytes // world, dt)
        r["check"] = column_mean_check([x], m, lambda c: c, 1e-6,
                                       "every column mean vs f64 sums of the resident input")
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
        r["check"] = column_mean_check([x], m, lambda c: c, 1e-6,
                                       "every column mean vs f64 sums of the resident input")
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
    collective is a local copy of the same bytes.  The step timed again with
    the collectives skipped (LoopbackComm.skip_collectives) is what rank r's
    GPU spends outside the collective; the 8-GPU prediction adds a stated RCCL allowance
    (RCCL_SCATTER_ALLOWANCE_US / RCCL_ALLOWANCE_US, not measured) to the
    busiest rank."""
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
        from cubed_amd.runtime.executors.dist import DistPiecesLaunch

        dps = [l for v in ex._cache.values() for l in v[1] if isinstance(l, DistPiecesLaunch)]
        scatter = bool(dps) and dps[0].scatter is not None
        # the loopback collective is a local copy standing in for RCCL's: the
        # step is timed again with the collectives skipped (the allowance
        # below replaces them)
        ex.comm.skip_collectives = True
        step()
        dt0, _ = timed_launches(ex, step, 20, 1)
        ex.comm.skip_collectives = False
        stand_in = (dt - dt0) * 1e3
        out["ranks"][r] = dict(ms=round(dt * 1e3, 4), row_chunks=nchunks,
                               input_gbs=round(nchunks * 1000 * N * 4 / dt / 1e9, 1),
                               collective="reduce_scatter" if scatter else "all_reduce",
                               stand_in_ms=round(stand_in, 4), ms_outside_collective=round(dt0 * 1e3, 4),
                               launches_ms=fmt_launches(summ), **overhead(dt, summ, 20))
        del x, m, plan, ex
        free_gpu()
    busiest = max(v["ms_outside_collective"] for v in out["ranks"].values())
    scatter = all(v["collective"] == "reduce_scatter" for v in out["ranks"].values())
    allowance = RCCL_SCATTER_ALLOWANCE_US if scatter else RCCL_ALLOWANCE_US
    out["busiest_ms"] = busiest
    out["busiest"] = "the largest per-rank step timed with the loopback collectives skipped"
    out["rccl_allowance_us"] = allowance
    out["rccl_allowance"] = ("reduce-scatter of the f64 totals (owner-major, 1/W per rank): half the 40 us "
                             "all-reduce allowance (W-1 of its 2(W-1) ring steps); assumed, not measured"
                             if scatter else "all-reduce of the f64 totals: assumed, not measured")
    out["predicted_step_ms"] = round(busiest + allowance / 1e3, 4)
    if t1_ms:
        out["one_gpu_step_ms"] = t1_ms
        out["predicted_speedup"] = round(t1_ms / out["predicted_step_ms"], 2)
    return out


def rechunk_rehearsal_extra(args, rank, world, t1_ms=None):
    """Config 3's MATERIALISED rechunk (50000^2 f32 rows -> (50000, 1000)
    columns) as each rank of an N-rank job, rehearsed on this one GPU: all N
    rehearsed ranks (LoopbackComm over one LoopbackMesh) allocate their
    block-cyclic shares and run RechunkLaunch for real -- pack of the strided
    source pieces, local copies, and the receive side of every peer transfer
    written into the target slots from the peer's recorded send (matched by
    pair and order, so the targets hold the right bytes and are checked bit
    for bit).  Per rank: the HIP-event time of each phase and the bytes it
    sends over xGMI.  The 8-GPU prediction adds the transfer time at a
    STATED link rate (XGMI_LINK_GBS per direction on the dedicated link of
    each peer pair, not measured: one GPU per box) -- serial (pack + local
    copies + unpack, then every transfer) and overlapped (the first slice's
    pack, then the transfers, with the later packs and local copies behind
    them: RechunkLaunch's slicing) bounds.  The rehearsal's slot writes
    stand in for RCCL's receive-side writes and are reported, not charged."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.comm import LoopbackComm, LoopbackMesh
    from cubed_amd.runtime.executors.dist import RechunkLaunch
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    W = args.rehearse_world
    N = 50000
    mesh = LoopbackMesh(W)
    ranks = []
    for r in range(W):
        ex = GpuDagExecutor(comm=LoopbackComm(r, W, mesh=mesh))
        spec = cubed.Spec(allowed_mem="288GB", executor=ex)
        random.seed(2000)
        x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
        arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
        y = x.rechunk((N, 1000))
        plan = arrays_to_plan(y)
        step = step_fn(plan, ex, [y], x)
        step()  # record phase: this rank's sends go to the mesh
        ranks.append((ex, x, y, step))
    sync()
    mesh.phase = "replay"
    xl = regenerate_source((N, N), (1000, N), 2000)
    out = {"world": W, "xgmi_link_gbs_assumed": XGMI_LINK_GBS, "ranks": {}}
    ok = True
    for r, (ex, x, y, step) in enumerate(ranks):
        step()
        dt, summ = timed_launches(ex, step, 5, 1)
        rl = [l for v in ex._cache.values() for l in v[1] if isinstance(l, RechunkLaunch)][0]
        plan = rl.plan
        phases = {k[2]: round(c * ms / 5, 4) for k, (c, ms) in summ.items() if k[0] == "rechunk"}
        per_peer = [sum(x_.nbytes for x_ in lst) for lst in plan.send]
        xgmi_ms = max(max(per_peer), max(sum(x_.nbytes for x_ in lst) for lst in plan.recv)) / \
            (XGMI_LINK_GBS * 1e9) * 1e3
        # the rank's own stream work: pack, local copies, unpack.  The
        # slot writes are the loopback's stand-in for RCCL writing the
        # arriving bytes (part of the transfer on a real rank, not charged)
        local_ms = sum(phases.get(p, 0.0) for p in ("pack", "local_copies", "unpack"))
        first_pack = phases.get("pack", 0.0) / max(1, len(rl.slices))
        chk = rechunk_check(xl, y)
        ok &= chk["pass"]
        out["ranks"][r] = dict(ms=round(dt * 1e3, 4), phases_ms=phases, slices=len(rl.slices),
                               stream_work_ms=round(local_ms, 4),
                               bytes_out=plan.send_bytes, bytes_in=plan.recv_bytes,
                               max_bytes_per_peer=max(per_peer), xgmi_ms_assumed=round(xgmi_ms, 4),
                               predicted_serial_ms=round(local_ms + xgmi_ms, 4),
                               predicted_overlapped_ms=round(max(local_ms, first_pack + xgmi_ms), 4),
                               check=chk["pass"])
    busiest = max(out["ranks"].values(), key=lambda v: v["predicted_serial_ms"])
    out["predicted_step_ms"] = {"serial": busiest["predicted_serial_ms"],
                                "overlapped": max(v["predicted_overlapped_ms"] for v in out["ranks"].values())}
    if t1_ms:
        out["one_gpu_step_ms"] = t1_ms
        out["predicted_speedup"] = {k: round(t1_ms / v, 2) for k, v in out["predicted_step_ms"].items()}
    out["check"] = {"kind": "bit-exact", "pass": bool(ok), "what": f"every target chunk of all {W} rehearsed "
                    f"ranks vs a local Philox regeneration of the source"}
    CHECKS.append(("rechunk_rehearsal", out["check"]))
    del ranks, xl
    free_gpu()
    return out


def var_extra(args, ex, rank, world):
    """north_star's var at config 2's size: xp.var(u * v, axis=0) and
    xp.std(u * v, axis=0), u, v (1000, 720, 1440) f32 in (10, 720, 1440)
    chunks -- the mean's reduction pattern (statistical_functions.py:28-100)
    over a {n, mu, M2} intermediate, one fused pass.  No reference var
    exists in v0.12.0 (api_status.md:72,74): checked against a two-pass f64
    var of the resident inputs (numpy's definition)."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    T = args.t_length * world
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)
    random.seed(1000)
    u = xp.astype(crandom.random((T, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    v = xp.astype(crandom.random((T, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=ex, array_names=[u.name, v.name])
    sync()
    out = {}
    for fname in ("var", "std"):
        m = getattr(xp, fname)(u * v, axis=0)
        plan = arrays_to_plan(m)
        step = step_fn(plan, ex, [m], (u, v))
        # var's first ~15 steps run up to 20 % slower than its steady state
        # (tools/var_timing_probe.py: 5 steps 1.43 ms, then 1.204 ms = mean's
        # step) -- warm 15 steps, time 20
        for _ in range(15):
            step()
        dt, summ = timed_launches(ex, step, 20, world)
        r = dict(metric=f"{fname}(u*v, axis=0) effective input GB/s", value=round((u.nbytes + v.nbytes) / dt / 1e9, 1),
                 ms=round(dt * 1e3, 4), launches_ms=fmt_launches(summ), **overhead(dt, summ, 20))
        if world == 1:
            key, ms = dominant(summ, "FusedLaunch")
            r["roofline"] = roofline_hbm(u.nbytes + v.nbytes, ms, f"{fname}_stream", args,
                                         f"{key[0]}#{key[1]} ({key[2]}), mean {ms:.4f} ms/launch")
        else:
            r["roofline"] = roofline_step((u.nbytes + v.nbytes) // world, dt)
        r["check"] = column_var_check(u, v, m, fname == "std")
        CHECKS.append((fname, r["check"]))
        out[fname] = r
        del m, plan
    return out


def column_var_check(u, v, m, sqrt):
    """Two-pass f64 var over axis 0 of u*v (f32 products) at every output
    position: every rank sums its chunks, one all-reduce for the sums, one
    for the squared deviations from the mean; rtol 1e-6 (f32 output)."""
    import torch

    M = m.zarray
    U, V = u.zarray, v.zarray
    n = u.shape[0]
    s1 = allreduce_(owned_axis0_sums([U, V], lambda a, b: a * b))
    s2 = allreduce_(owned_axis0_sums([U, V], lambda a, b: a * b, center=s1 / n))
    exp = s2 / n
    if sqrt:
        exp = torch.sqrt(exp)
    got = allreduce_(owned_output_full(M))
    r = check_close(got.cpu().numpy(), exp.cpu().numpy(), 1e-6,
                    f"every {'std' if sqrt else 'var'} output vs a two-pass f64 var of the resident inputs")
    r.update(kind="full", entries=int(got.numel()), world=world_size())
    return r


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
    else:
        r["roofline"] = roofline_step(a.nbytes // world, dt)
    r["check"] = column_mean_check([a], m, lambda c: (c + 1) * 2, 1e-12,
                                   "every column mean vs f64 sums of (a+1)*2 over the resident input")
    CHECKS.append(("config1", r["check"]))
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        r["cpu_baseline"] = cpu_config1_baseline(a)
    return r


def cpu_config1_baseline(a, row_blocks=None):
    """BASELINE config 1 as the reference runs it: the sequential
    PythonDagExecutor over the finalized plan (add; multiply + _mean_func;
    merge + combine + aggregate) with every intermediate in a LOCAL ZARR
    WORK_DIR (this repo's Zarr v2 writer/reader, blosc-lz4 with byte shuffle:
    numcodecs' default compressor).  ``a`` (the random op's output) is first
    written to the work_dir from HBM (untimed, as its generation is untimed
    on the GPU); the timed sample is the first ``row_blocks`` row bands of
    chunks (all four column chunks; default: every band), median of CPU_REPS runs after a
    warm-up."""
    import shutil
    import tempfile

    from oracle import cubed_ref as R
    from cubed_amd.zarr_io import ZarrV2Array, write_device_array

    A = a.zarray
    row_blocks = A.numblocks[0] if row_blocks is None else row_blocks
    work = tempfile.mkdtemp(prefix="cubed_cpu_work_")
    try:
        src = ZarrV2Array.create(os.path.join(work, "a"), A.shape, A.dtype, A.chunks)
        write_device_array(A, src)
        run_dir = os.path.join(work, "run")

        def fresh():  # every run writes its intermediates into an empty work_dir
            shutil.rmtree(run_dir, ignore_errors=True)
            os.makedirs(run_dir)

        dt, runs, got = median_run(lambda: R.config1_python_zarr(src, run_dir, row_blocks=row_blocks), setup=fresh)
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
                      f"median of {CPU_REPS} timed passes after a warm-up; {_cpu_info(1)}",
            "seconds": round(dt, 3), "runs_s": runs, "values_match": ok}


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
    else:
        r["roofline"] = roofline_step(in_bytes // world, dt)
    r["check"] = vorticity_check(a, b, x, y, m)
    CHECKS.append(("vorticity", r["check"]))
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        r["cpu_baseline"] = cpu_vorticity_baseline(a.zarray, b.zarray, x.zarray, y.zarray)
    return r


def vorticity_check(a, b, x, y, m):
    """f64 sum of a[1:]*x + b[1:]*y over the (a, b) chunks this rank owns (x,
    y gathered whole: 5.8 MB each), summed over the ranks, against the
    computed scalar mean at rtol 1e-12."""
    import torch

    A, B = a.zarray, b.zarray
    X = torch.as_tensor(full_host(x.zarray), device=A.device)
    Y = torch.as_tensor(full_host(y.zarray), device=A.device)
    total = torch.zeros(1, dtype=torch.float64, device=A.device)
    for c in owned_chunks(A):
        ca, cb = device_chunk(A, c), device_chunk(B, c)
        if c[0] == 0:  # a[1:]: the first time row is not read
            ca, cb = ca[1:], cb[1:]
        (j0, k0), (je, ke) = A.chunk_start(c)[1:], A.chunk_extent(c)[1:]
        total += (ca * X[j0:j0 + je, k0:k0 + ke] + cb * Y[j0:j0 + je, k0:k0 + ke]).sum()
    got = owned_output_values(m.zarray, np.zeros((1, 0), np.int64))
    return sampled_check(total, got, (a.shape[0] - 1) * a.shape[1] * a.shape[2], 1e-12,
                         "f64 sum over every resident chunk of a[1:], b[1:] (x, y gathered) vs the mean")


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
    res, runs = {}, {}
    with threadpool_limits(1):
        for name, th in (("sequential", 1), ("threads", threads)):
            res[name], runs[name], got = median_run(
                lambda: R.vorticity_python(a, b, x, y, c, t_blocks=t_blocks, threads=th))
    exp = float(np.mean(a[1:1 + t_blocks * c] * x + b[1:1 + t_blocks * c] * y, dtype=np.float64))
    nbytes = 2 * t_blocks * c * x.size * 8 + 2 * x.size * 8
    return {"value": round(nbytes / res["threads"] / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{t_blocks} of {-(-(A.shape[0] - 1) // c)} time blocks of a[1:], b[1:] "
                      f"({t_blocks * 72} chunk tasks per op): oracle restatement of the reference's finalized "
                      f"plan (index a[1:], b[1:]; * x, * y; add + _mean_func; combine + aggregate) on the "
                      f"threaded executor, in-memory intermediates (no Zarr/Blosc: optimistic), median "
                      f"of {CPU_REPS} timed passes after a warm-up; {_cpu_info(threads)}",
            "runs_s": runs["threads"],
            "sequential": {"value": round(nbytes / res["sequential"] / 1e9, 3), "cores": 1,
                           "runs_s": runs["sequential"]},
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
    r["check"] = matmul_check(A.zarray, B.zarray, m.zarray, n, c, dt_name == "bf16")
    CHECKS.append((f"matmul_{dt_name}", r["check"]))
    return r


def matmul_rehearsal_extra(args, dt_name, t1_ms=None):
    """Config 5 on N GPUs, every rank rehearsed on this one GPU through ONE
    LoopbackMesh (dist.DistGemmLaunch): each rank allocates its block-cyclic
    share of A and B (40000^2 in 5000^2 chunks: rank r owns A's k chunk
    column r, B's and C's chunk column r), receives the halo columns of the
    next k chunk, packs its k blocks into the k-major A image, sends them to
    every peer (the mesh writes each receive from the peer's recorded send),
    packs its B^T and runs the packed GEMM over its C columns.  After a
    record pass and two replay passes every rank holds its true C columns:
    64 sampled entries of C are checked against f64 dot products of the
    resident operands (the matmul bound).  Per rank: HIP-event time of each
    phase, bytes in / out.  Predicted N-GPU step (busiest rank) = halo +
    pack A + max(transfers at a STATED link rate -- XGMI_LINK_GBS per
    direction on each peer pair's own link, not measured --, pack B) + GEMM;
    the mesh's slot writes stand in for RCCL's receive-side writes and are
    reported, not charged."""
    import torch

    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.comm import LoopbackComm, LoopbackMesh
    from cubed_amd.runtime.executors.dist import DistGemmLaunch
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    W = args.rehearse_world
    n, c = args.matmul_n, 5000
    xdt = xp.bfloat16 if dt_name == "bf16" else xp.float32
    mesh = LoopbackMesh(W)
    ranks = []
    for r in range(W):
        ex = GpuDagExecutor(comm=LoopbackComm(r, W, mesh=mesh))
        spec = cubed.Spec(allowed_mem="288GB", executor=ex)
        random.seed(4000)
        A = xp.astype(crandom.random((n, n), chunks=(c, c), spec=spec), xdt)
        B = xp.astype(crandom.random((n, n), chunks=(c, c), spec=spec), xdt)
        arrays_to_plan(A, B).execute(executor=ex, array_names=[A.name, B.name])
        m = xp.matmul(A, B)
        step = step_fn(arrays_to_plan(m), ex, [m], (A, B))
        step()  # record pass
        ranks.append((ex, A, B, m, step))
    sync()
    mesh.phase = "replay"
    for _ in range(2):  # halos, then the blocks packed from them, reach every rank
        for ex, A, B, m, step in ranks:
            step()
        sync()
    out = {"world": W, "dtype": dt_name, "n": n, "chunk": c, "xgmi_link_gbs_assumed": XGMI_LINK_GBS, "ranks": {}}
    for r, (ex, A, B, m, step) in enumerate(ranks):
        dt, summ = timed_launches(ex, step, 2, 1)
        dg = [l for v in ex._cache.values() for l in v[1] if isinstance(l, DistGemmLaunch)]
        if len(dg) != 1:
            raise RuntimeError(f"rank {r}: {len(dg)} DistGemmLaunch")
        d = dg[0]
        ph = {k[2]: round(cnt * ms / 2, 4) for k, (cnt, ms) in summ.items() if k[0] == "matmul"}
        xfer = d.predicted_xfer_ms(XGMI_LINK_GBS)
        pred = ph.get("halo", 0) + ph.get("pack_a", 0) + max(xfer, ph.get("pack_b", 0)) + ph.get("gemm", 0)
        gtf = d.flops / (ph["gemm"] * 1e-3) / 1e12 if ph.get("gemm") else None
        out["ranks"][r] = dict(ms=round(dt * 1e3, 4), phases_ms=ph, bytes_out=d.bytes_out, bytes_in=d.bytes_in,
                               halo_cols=[d.halo_w[q] for q in d.owned], xgmi_ms_assumed=round(xfer, 4),
                               gemm_tflops=round(gtf, 1) if gtf else None,
                               predicted_ms=round(pred, 4))
    busiest = max(v["predicted_ms"] for v in out["ranks"].values())
    out["predicted_step_ms"] = busiest
    out["predicted"] = ("busiest rank: halo + pack A + max(xGMI transfers at the assumed link rate, pack B) + "
                        "GEMM; the mesh's slot writes are not charged")
    if t1_ms:
        out["one_gpu_step_ms"] = t1_ms
        out["predicted_speedup"] = round(t1_ms / busiest, 2)
    # 64 sampled entries of the rehearsed C against f64 products of the
    # operands, each chunk read from the rank that owns it
    rng = np.random.default_rng(5)
    rows = np.sort(rng.choice(n, 8, replace=False))
    cols = np.sort(rng.choice(n, 8, replace=False))
    nk = -(-n // c)

    def chunk(i_arr, coords):
        return device_chunk(ranks[ranks[0][i_arr].zarray.chunk_offset(coords) % W][i_arr].zarray, coords)

    Ar = np.stack([np.concatenate([chunk(1, (i // c, q))[i % c].double().cpu().numpy() for q in range(nk)])
                   for i in rows])
    Bc = np.stack([np.concatenate([chunk(2, (q, j // c))[:, j % c].double().cpu().numpy() for q in range(nk)])
                   for j in cols], axis=1)
    got = np.array([[chunk(3, (i // c, j // c))[i % c, j % c].double().item() for j in cols] for i in rows])
    exp = Ar @ Bc
    bound = 8.0 * np.sqrt(n) * 2.0 ** -24 * (np.abs(Ar) @ np.abs(Bc))
    if dt_name == "bf16":
        bound = bound + 2.0 ** -8 * np.abs(exp)
    err = np.abs(got - exp)
    out["check"] = {"kind": "bound", "pass": bool(np.all(err <= bound)), "entries": int(got.size),
                    "max_err_over_bound": float(np.max(err / bound)),
                    "what": f"64 sampled entries of C assembled from {W} rehearsed ranks vs f64 products"}
    CHECKS.append((f"matmul_rehearsal_{dt_name}", out["check"]))
    del ranks
    torch.cuda.synchronize()
    free_gpu()
    return out


def matmul_check(A, B, C, n, c, bf16):
    """64 output entries (8 rows x 8 columns, seeded) against f64 dot products
    of the copied-back operand rows / columns.  Bound (tests/test_gpu_matmul.py):
    8 sqrt(K) 2^-24 sum|a||b| (+ 2^-8 |C| for a bf16 output)."""
    import torch

    rng = np.random.default_rng(5)
    rows = np.sort(rng.choice(n, 8, replace=False))
    cols = np.sort(rng.choice(n, 8, replace=False))
    nk = -(-n // c)
    # each rank fills the slices of the sampled A rows / B columns / C
    # entries held by the chunks it owns (zeros elsewhere); one f64 sum over
    # the ranks assembles them whole on every rank
    dev = A.device
    Ar = torch.zeros(len(rows), n, dtype=torch.float64, device=dev)
    Bc = torch.zeros(n, len(cols), dtype=torch.float64, device=dev)
    Cs = torch.zeros(len(rows), len(cols), dtype=torch.float64, device=dev)
    for a, i in enumerate(rows):
        for kk in range(nk):
            if A.owner((i // c, kk)) == A.rank:
                Ar[a, kk * c:(kk + 1) * c] = device_chunk(A, (i // c, kk))[i % c].double()
    for b, j in enumerate(cols):
        for kk in range(nk):
            if B.owner((kk, j // c)) == B.rank:
                Bc[kk * c:(kk + 1) * c, b] = device_chunk(B, (kk, j // c))[:, j % c].double()
    for a, i in enumerate(rows):
        for b, j in enumerate(cols):
            if C.owner((i // c, j // c)) == C.rank:
                Cs[a, b] = device_chunk(C, (i // c, j // c))[i % c, j % c].double()
    flat = allreduce_(torch.cat([Ar.reshape(-1), Bc.reshape(-1), Cs.reshape(-1)]))
    Ar = flat[:Ar.numel()].reshape(Ar.shape).cpu().numpy()
    Bc = flat[Ar.size:Ar.size + Bc.numel()].reshape(Bc.shape).cpu().numpy()
    got = flat[Ar.size + Bc.size:].reshape(Cs.shape).cpu().numpy()
    exp = Ar @ Bc
    bound = 8.0 * np.sqrt(n) * 2.0 ** -24 * (np.abs(Ar) @ np.abs(Bc))
    if bf16:
        bound = bound + 2.0 ** -8 * np.abs(exp)
    err = np.abs(got - exp)
    return {"kind": "bound", "pass": bool(np.all(err <= bound)), "entries": int(got.size), "world": world_size(),
            "max_err_over_bound": float(np.max(err / bound)),
            "what": "64 sampled entries vs f64 products of the resident rounded operands"}


# --------------------------------------------------------------------------- CPU baselines


CPU_REPS = 5  # BASELINE.md's protocol: median of >= 5 timed runs after a warm-up


def median_run(fn, reps=CPU_REPS, warmup=True, setup=None):
    """(median seconds, every run's seconds, the last result) of ``fn()``
    over ``reps`` timed runs after one untimed warm-up run; ``setup()`` runs
    untimed before every run."""
    if warmup:
        if setup:
            setup()
        fn()
    ts, out = [], None
    for _ in range(reps):
        if setup:
            setup()
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), [round(t, 4) for t in ts], out


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
        for name, th in (("sequential", 1), ("threads", threads)):
            med, runs, exp = median_run(lambda: R.quad_means_cpu(u, v, 10, 2_000_000_000, 100_000_000, threads=th))
            out[name] = (med, th, runs)
    got = res["m"].compute()
    parity = bool(np.allclose(got, exp, rtol=1e-6, atol=0))
    nbytes = u.nbytes + v.nbytes
    dt, th, runs = out["threads"]
    return {"value": round(nbytes / dt / 1e9, 3), "unit": "GB/s", "cores": th, "kind": "port",
            "sample": f"full config 2: quad-means ({u.shape[0]},720,1440) f32 u,v, chunks (10,720,1440), "
                      f"oracle restatement of the reference threads executor (AsyncPythonDagExecutor "
                      f"ThreadPoolExecutor), median of {CPU_REPS} after a warm-up; {_cpu_info(th)}; excludes "
                      f"Zarr/Blosc I/O (optimistic)",
            "runs_s": runs,
            "sequential": {"value": round(nbytes / out["sequential"][0] / 1e9, 3), "cores": 1,
                           "sample": f"same inputs, PythonDagExecutor restatement, median of {CPU_REPS} after a "
                                     f"warm-up", "runs_s": out["sequential"][2]},
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
    out, runs = {}, {}
    for name, th in (("sequential", 1), ("threads", threads)):
        pool = ThreadPoolExecutor(th) if th > 1 else None
        out[name], runs[name], _ = median_run(lambda: (copy_op(X, I, inter, pool), copy_op(I, Y, write, pool)))
        if pool:
            pool.shutdown()
    ok = bool(np.array_equal(Y.view(np.uint32), X.view(np.uint32)))
    return {"value": round(X.nbytes / out["threads"] / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"full config 3: 50000^2 f32, reference 2 GB plan read {read} -> int {inter} -> "
                      f"write {write}, in-memory numpy region copies (no Zarr/Blosc: optimistic), median "
                      f"of {CPU_REPS} timed passes after a warm-up; {_cpu_info(threads)}",
            "runs_s": runs["threads"],
            "sequential": {"value": round(X.nbytes / out["sequential"] / 1e9, 3), "cores": 1,
                           "runs_s": runs["sequential"]},
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
    key, ms_instr = dominant(res["summ"], "FusedLaunch")
    kernels = [k for k in res["summ"] if k[2] not in ("_Alloc", "_Upload")]  # (host-only steps launch nothing)
    one_launch = kernels == [key] and res["summ"][key][0] == args.steps
    # the step is ONE launch: its duration is the GPU time per step of the
    # plain (timed) pass, HIP events around that region on the executor's
    # stream; the per-launch events of the instrumented pass are reported
    # beside it
    ms = res["plain_event_ms"] if one_launch else ms_instr
    # algorithmic bytes of the dominant launch: the fused u*v -> mean kernel
    # reads this rank's u and v once (2 x 4.147e9 B at T=1000)
    algo = in_bytes // world
    symbols = [x for x in res["symbols"] if not x.startswith("cubed_map_")]  # the reduction's kernel, not the inputs' astype
    extra = {"launches_ms": fmt_launches(res["summ"]), **overhead(dt, res["summ"], args.steps)}
    # every world size: every output vs f64 sums of u*v over every rank's chunks
    extra["check"] = column_mean_check([res["u"], res["v"]], res["m"], lambda a, b: a * b, 1e-6,
                                       "every mean vs f64 sums of u*v (f32 products) over the resident inputs")
    CHECKS.append(("quad-means sampled", extra["check"]))
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
            elif name == "rechunk_rehearsal":
                if world == 1:
                    t1 = extra.get("rechunk", {}).get("plan_288GB", {}).get("ms")
                    extra[name] = rechunk_rehearsal_extra(args, rank, world, t1)
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
            elif name == "var":
                extra[name] = var_extra(args, ex, rank, world)
            elif name == "vorticity":
                extra[name] = vorticity_extra(args, ex, rank, world)
            elif name == "matmul_rehearsal":
                if world == 1:
                    extra[name] = {}
                    for dn in ("bf16", "f32"):
                        t1 = extra.get(f"matmul_{dn}", {}).get("ms")
                        extra[name][dn] = matmul_rehearsal_extra(args, dn, t1)
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
        "roofline": (roofline_hbm(algo, ms, "quad_means_fused", args,
                                  f"{key[0]}#{key[1]} ({key[2]}: {', '.join(symbols)}), "
                                  + (f"{ms:.4f} ms per launch from HIP events around the timed (plain) pass of "
                                     f"{args.steps} one-launch steps; per-launch events of the instrumented pass "
                                     f"{ms_instr:.4f} ms" if one_launch else
                                     f"mean {ms:.4f} ms/launch (per-launch HIP events, instrumented pass)"))
                     if world == 1 else roofline_step(algo, dt)),
        "extra": extra,
        "ranks": rank_info(args.backend),
    }
    if cpu is not None:
        line["cpu_baseline"] = cpu
    rc = finish(line, CHECKS, rank, world)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    if rc:
        sys.stderr.write(f"bench.py: value checks failed: {line['checks_failed']}\n")
        sys.exit(rc)


if __name__ == "__main__":
    main()
