"""Benchmark: effective input GB/s of Cubed's hot path on MI355X.

Default workload = BASELINE.json configs[1], "quad-means": u, v float32
(1000, 720, 1440) per GPU, chunks (10, 720, 1440), ``xp.mean(u * v, axis=0)``
(fused elementwise + mean), Spec(allowed_mem="2GB", reserved_mem="100MB") as
in the reference's own quad-means test (cubed/tests/test_core.py:527-538).
Inputs are generated on the GPU (bit-exact numpy Philox) and are resident in
HBM before timing; a step is one ``plan.execute(executor, resume=True)`` of
the mean's plan (every kernel and collective of the reduction), bracketed by
barrier + synchronize.  value = input bytes of all ranks / time.

Also reported in the same JSON line (``extra``): rechunk 50000x50000 f32
row-chunks -> column-chunks (configs[2]) and config 1 ((a+1)*2 -> mean).

Multi-GPU (torchrun, one process per GPU, RCCL): weak scaling -- the arrays
grow to (1000 * N, 720, 1440) and their chunks are spread block-cyclically
over the N GPUs by the distributed GpuDagExecutor (chunk offset mod N), so
every GPU holds 100 time chunks of u and v.  Each GPU reduces its own chunks
to (n, total) partials in one streaming launch, one RCCL reduce per field
combines them on the output block's owner, which runs the aggregate
(cubed_fused_finish).  No other data-path collective runs.

CPU baseline (rank 0, N=1 only): the oracle's restatement of the
reference's numpy executor (oracle/cubed_ref.py quad_means_cpu), 1 thread,
on a bounded sample (300 of the 1000 time steps), Zarr/Blosc I/O excluded.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--t-length", type=int, default=1000, help="time steps per GPU (quad-means)")
    p.add_argument("--no-extra", action="store_true", help="skip the rechunk/config-1 extras")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-matmul", action="store_true", help="skip the matmul extra")
    p.add_argument("--cpu-sample", type=int, default=300)
    p.add_argument("--backend", default="nccl",
                   help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to rehearse "
                        "several ranks on one GPU)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="per-launch HBM bytes from rocprofv3 PMC (see profiles/README.md)")
    return p.parse_args()


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


def run_plan(plan, ex, names, resume):
    plan.execute(executor=ex, resume=resume, array_names=names)


def quad_means(args, rank, world, ex):
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.executors.gpu import LaunchTimer

    T = args.t_length * world  # weak scaling: 1000 time steps per GPU
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)
    random.seed(1000)  # same plan (and root seeds) on every rank
    u = xp.astype(crandom.random((T, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    v = xp.astype(crandom.random((T, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    # materialise the inputs in HBM (untimed)
    arrays_to_plan(u, v).execute(executor=ex, array_names=[u.name, v.name])
    sync()
    m = xp.mean(u * v, axis=0)
    plan = arrays_to_plan(m)
    in_bytes = u.nbytes + v.nbytes

    keep = (u, v)

    def step():
        # every op of the mean's plan runs each step; only u, v stay resident
        _reset_targets(plan, keep)
        run_plan(plan, ex, [m.name], resume=True)

    for _ in range(args.warmup):
        step()
    sync()
    barrier(world)
    ex.timing = LaunchTimer()
    sync()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    barrier(world)
    t1 = time.perf_counter()
    timer, ex.timing = ex.timing, None
    dt = t1 - t0
    if world > 1:
        import torch
        import torch.distributed as dist

        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dict(in_bytes=in_bytes, dt=dt, timer=timer, m=m, u=u, v=v)


def timed_launches(ex, fn, steps, world):
    """(seconds per call, {launch: mean ms}) -- the executor's per-launch HIP
    events recorded during the timed calls."""
    from cubed_amd.runtime.executors.gpu import LaunchTimer

    ex.timing = LaunchTimer()
    dt = timed(fn, steps, world)
    timer, ex.timing = ex.timing, None
    return dt, {f"{k[0]}#{k[1]}:{k[2]}": round(v[1], 4) for k, v in timer.summary().items()}


def timed(fn, steps, world):
    """Mean seconds per call of fn over `steps` calls, barrier + synchronize
    on both sides, max over ranks."""
    sync()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    barrier(world)
    dt = (time.perf_counter() - t0) / steps
    if world > 1:
        import torch
        import torch.distributed as dist

        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def dominant(timer, algo_bytes_by_key):
    """The kernel launch with the largest total time (collectives excluded:
    the roofline is the fused kernel's)."""
    summ = timer.summary()
    kern = [k for k in summ if k[2] == "FusedLaunch"] or list(summ)
    key = max(kern, key=lambda k: summ[k][0] * summ[k][1])
    count, ms = summ[key]
    return key, ms, summ


def rechunk_extra(ex, rank):
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    N = 50000
    spec = cubed.Spec(allowed_mem="288GB", executor=ex)
    random.seed(2000)
    x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
    arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
    sync()
    y = x.rechunk((N, 1000))
    plan = arrays_to_plan(y)
    for _ in range(2):
        _exec_only(plan, ex, y, x)
    dt, launches = timed_launches(ex, lambda: _exec_only(plan, ex, y, x), 5, ex.world)
    nops = sum(1 for _, d in plan._finalize_dag().nodes(data=True)
               if d.get("op_name") == "rechunk")
    # correctness spot check: a few columns
    return dict(metric="rechunk effective input GB/s", value=x.nbytes / dt / 1e9,
                ms=dt * 1e3, ops=nops, bytes_moved_per_op=2 * x.nbytes, launches_ms=launches)


def rechunk_mean_extra(ex, rank):
    """configs[2] "rechunk+reduce": mean(x.rechunk(columns), axis=0) with x
    50000^2 f32 in row chunks.  The rechunk feeds only the mean, so the
    executor reads it through (rewrites.elide_rechunks): each GPU reduces the
    row-chunk pieces it holds; with N GPUs the partials are combined over
    RCCL.  value = x bytes / time."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan

    N = 50000
    spec = cubed.Spec(allowed_mem="288GB", executor=ex)
    random.seed(2000)
    x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
    arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
    m = xp.mean(x.rechunk((N, 1000)), axis=0)
    plan = arrays_to_plan(m)

    def step():
        _reset_targets(plan, x)
        plan.execute(executor=ex, resume=True, array_names=[m.name])

    step()
    dt, launches = timed_launches(ex, step, 5, ex.world)
    return dict(metric="rechunk+mean effective input GB/s", value=x.nbytes / dt / 1e9,
                ms=dt * 1e3, launches_ms=launches)


def _exec_only(plan, ex, y, x):
    # re-run every rechunk op (x stays resident)
    from cubed_amd.storage import DeviceArray

    for _, d in plan._finalize_dag().nodes(data=True):
        t = d.get("target")
        if isinstance(t, DeviceArray) and t is not x.zarray:
            t.written = False
    plan.execute(executor=ex, resume=True, array_names=[y.name])


def config1_extra(ex, rank):
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
    def step():
        _reset_targets(plan, a)
        plan.execute(executor=ex, resume=True, array_names=[m.name])

    for _ in range(2):
        step()
    dt, launches = timed_launches(ex, step, 5, ex.world)
    return dict(metric="config1 (a+1)*2 -> mean(axis=0) effective input GB/s",
                value=a.nbytes / dt / 1e9, ms=dt * 1e3, launches_ms=launches)


def matmul_extra(ex, rank, n=20000, c=5000):
    """configs[4] shape of work, scaled to one GPU: xp.matmul of two f32
    (n, n) arrays in (c, c) chunks -- (n/c)^3 chunk GEMMs on MFMA, then the
    k-sum reduction.  Reports the whole plan's TFLOP/s and the GEMM launch's
    own rate (HIP events on the executor stream)."""
    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.executors.gpu import LaunchTimer

    spec = cubed.Spec(allowed_mem="288GB", executor=ex)
    random.seed(4000)
    A = xp.astype(crandom.random((n, n), chunks=(c, c), spec=spec), xp.float32)
    B = xp.astype(crandom.random((n, n), chunks=(c, c), spec=spec), xp.float32)
    arrays_to_plan(A, B).execute(executor=ex, array_names=[A.name, B.name])
    m = xp.matmul(A, B)
    plan = arrays_to_plan(m)

    def step():
        _reset_targets(plan, (A, B))
        plan.execute(executor=ex, resume=True, array_names=[m.name])

    step()
    ex.timing = LaunchTimer()
    dt = timed(step, 2, ex.world)
    timer, ex.timing = ex.timing, None
    summ = timer.summary()
    gemm = [v for k, v in summ.items() if k[2] == "GemmLaunch"]
    flop = 2.0 * n ** 3
    out = dict(metric="matmul f32 TFLOP/s (whole plan)", value=flop / dt / 1e12, ms=dt * 1e3,
               n=n, chunk=c)
    if gemm:
        out["gemm_launch_ms"] = gemm[0][1]
        out["gemm_tflops"] = flop / (gemm[0][1] * 1e-3) / 1e12 / ex.world
        out["mfma_util_vs_157TF"] = out["gemm_tflops"] / 157.3
    return out


def vorticity_extra(ex, rank, T=1000):
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

    def step():
        _reset_targets(plan, (a, b, x, y))
        plan.execute(executor=ex, resume=True, array_names=[m.name])

    step()
    dt, launches = timed_launches(ex, step, 3, ex.world)
    in_bytes = a.nbytes + b.nbytes + x.nbytes + y.nbytes
    return dict(metric="vorticity mean(a[1:]*x + b[1:]*y) effective input GB/s",
                value=in_bytes / dt / 1e9, ms=dt * 1e3, launches_ms=launches)


def _reset_targets(plan, keep):
    from cubed_amd.storage import DeviceArray

    keep = keep if isinstance(keep, tuple) else (keep,)
    kept = {id(a.zarray) for a in keep}
    for _, d in plan._finalize_dag().nodes(data=True):
        t = d.get("target")
        if isinstance(t, DeviceArray) and id(t) not in kept:
            t.written = False


def cpu_baseline(args):
    from oracle import cubed_ref as R

    T = args.cpu_sample
    rs1, rs2 = R.root_seed_after(11), R.root_seed_after(12)
    u = R.random_array((T, 720, 1440), (10, 720, 1440), rs1).astype(np.float32)
    v = R.random_array((T, 720, 1440), (10, 720, 1440), rs2).astype(np.float32)
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        R.quad_means_cpu(u, v, 10, 2_000_000_000, 100_000_000, threads=1)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    return {"value": round((u.nbytes + v.nbytes) / dt / 1e9, 3), "unit": "GB/s", "cores": 1,
            "kind": "port",
            "sample": f"quad-means ({T},720,1440) f32 u,v, chunks (10,720,1440), oracle "
                      f"restatement of the reference python executor, median of 5, numpy "
                      f"{np.__version__}, host cpus {os.cpu_count()}, affinity "
                      f"{len(os.sched_getaffinity(0))}; excludes Zarr/Blosc I/O (optimistic)"}


def load_traffic(path, key_name):
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(key_name)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    rank, world, local = setup_dist(args)
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    ex = GpuDagExecutor()
    res = quad_means(args, rank, world, ex)
    dt = res["dt"]
    in_bytes = res["in_bytes"]
    value = in_bytes / (dt / args.steps) / 1e9  # global input bytes: all ranks
    key, ms, summ = dominant(res["timer"], {})
    # algorithmic bytes of the dominant launch: the fused u*v -> mean kernel
    # reads u and v once (8.294e9 B at T=1000) and writes the (n, total)
    # partials / final mean (2 x 4.147e9 B read)
    algo = in_bytes // world  # this rank's share of u and v, read once by the fused launch
    achieved = algo / (ms * 1e-3) / 1e9
    extra = {"launches_ms": {f"{k[0]}#{k[1]}:{k[2]}": round(v[1], 4) for k, v in summ.items()}}
    if not args.no_extra:
        try:
            extra["rechunk"] = rechunk_extra(ex, rank)
        except Exception as e:  # pragma: no cover - reported, not fatal
            extra["rechunk"] = {"error": repr(e)}
        try:
            extra["rechunk_mean"] = rechunk_mean_extra(ex, rank)
        except Exception as e:  # pragma: no cover
            extra["rechunk_mean"] = {"error": repr(e)}
        try:
            extra["config1"] = config1_extra(ex, rank)
        except Exception as e:  # pragma: no cover
            extra["config1"] = {"error": repr(e)}
        try:
            extra["vorticity"] = vorticity_extra(ex, rank)
        except Exception as e:  # pragma: no cover
            extra["vorticity"] = {"error": repr(e)}
        if not args.no_matmul:
            try:
                extra["matmul"] = matmul_extra(ex, rank)
            except Exception as e:  # pragma: no cover
                extra["matmul"] = {"error": repr(e)}
    line = {
        "metric": "effective input GB/s (node) for fused elementwise+mean (quad-means)",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (on-GPU numpy-Philox U[0,1) inputs, bit-exact with cubed.random)",
        "backend": args.backend if world > 1 else None,
        "config": {"workload": "quad-means: mean(u*v, axis=0), u,v (1000,720,1440) f32 per GPU, "
                               "chunks (10,720,1440), Spec(allowed_mem=2GB, reserved_mem=100MB)",
                   "t_length_per_gpu": args.t_length, "parallelism": f"block-partition dp{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": load_traffic(args.traffic_json, "quad_means_fused"),
                     "kernel": f"{key[0]}#{key[1]} ({key[2]}), mean {ms:.4f} ms/launch"},
        "extra": extra,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
