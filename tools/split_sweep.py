"""Sweep the streaming split target (cubed_stream_split_target) over the
split-reduction workloads: the per-rank share of config 3's rechunk + mean
(7000 rows, one GPU plan and the rehearsed rank 0 of 8), config 1 and the
elided full rechunk + mean.  One process, one box: every target times the
same resident inputs with HIP events (bench.py's timed_launches).

    python tools/split_sweep.py [targets...]
"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    import torch

    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd import _native as nat
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.comm import LoopbackComm
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor

    torch.cuda.set_device(0)
    targets = [int(t) for t in sys.argv[1:]] or [512, 1024, 1536, 2048, 3072]
    L = nat.lib()
    out = {}

    def run(name, ex, build, steps=20):
        x, m = build(ex)
        plan = arrays_to_plan(m)
        step = bench.step_fn(plan, ex, [m], x)
        step()
        step()
        dt, summ = bench.timed_launches(ex, step, steps, 1)
        out.setdefault(name, {})[tgt] = {"ms": round(dt * 1e3, 4), "launches_ms": bench.fmt_launches(summ)}
        print(name, tgt, out[name][tgt], flush=True)
        del x, m, plan
        bench.free_gpu()

    def share(rows, N=50000):
        def build(ex):
            spec = cubed.Spec(allowed_mem="288GB", executor=ex)
            random.seed(2001)
            x = xp.astype(crandom.random((rows, N), chunks=(1000, N), spec=spec), xp.float32)
            arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
            return x, xp.mean(x.rechunk((rows, 1000)), axis=0)
        return build

    def config1(ex):
        spec = cubed.Spec(allowed_mem="2GB", executor=ex)
        random.seed(3000)
        a = crandom.random((20000, 20000), chunks=(5000, 5000), spec=spec)
        arrays_to_plan(a).execute(executor=ex, array_names=[a.name])
        return a, xp.mean((a + 1) * 2, axis=0)

    def quad(ex):
        spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)
        random.seed(1000)
        u = xp.astype(crandom.random((1000, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
        v = xp.astype(crandom.random((1000, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
        arrays_to_plan(u, v).execute(executor=ex, array_names=[u.name, v.name])
        return (u, v), xp.mean(u * v, axis=0)

    if os.environ.get("SWEEP_QUAD_W"):
        import cubed_amd.lowering as Lw

        for w in (1, 2, 4):
            tgt = f"W{w}"
            Lw.FORCE_STREAM_W = w
            run("quad_means", GpuDagExecutor("cuda:0"), quad)
        Lw.FORCE_STREAM_W = None

    if os.environ.get("SWEEP_QUAD_SPLIT"):
        # quad-means (grid already fills the chip: unsplit by default) with
        # its time range forced into 2-4 splits folded in-kernel, at W = 1 / 2
        import cubed_amd.lowering as Lw

        for rep in range(2):
            for w in (2, 1):
                for ns in (0, 2, 3, 4):
                    tgt = f"W{w}_split{ns}_{rep}"
                    Lw.FORCE_STREAM_W = w
                    L.cubed_stream_force_split(ns)
                    run("quad_means", GpuDagExecutor("cuda:0"), quad)
        L.cubed_stream_force_split(0)
        Lw.FORCE_STREAM_W = None
        targets = []
    if os.environ.get("SWEEP_EVEN_AB"):
        # balanced split (CUBED_MODE_STREAM_EVEN) against the uniform split,
        # interleaved twice, at the default target
        import cubed_amd.lowering as Lw

        for rep in range(2):
            for even in (False, True):
                tgt = f"{'even' if even else 'uniform'}{rep}"
                Lw.STREAM_EVEN = even
                run("share7000", GpuDagExecutor("cuda:0"), share(7000))
                run("rehearsed_rank0_of_8", GpuDagExecutor("cuda:0", comm=LoopbackComm(0, 8)), share(50000))
                run("config1", GpuDagExecutor("cuda:0"), config1, steps=10)
                run("elided_full", GpuDagExecutor("cuda:0"), share(50000), steps=10)
        Lw.STREAM_EVEN = False
        targets = [t for t in targets if os.environ.get("SWEEP_TARGETS")]
    for tgt in targets:
        L.cubed_stream_split_target(tgt)
        run("share7000", GpuDagExecutor("cuda:0"), share(7000))
        run("rehearsed_rank0_of_8", GpuDagExecutor("cuda:0", comm=LoopbackComm(0, 8)), share(50000))
        run("config1", GpuDagExecutor("cuda:0"), config1, steps=10)
        run("elided_full", GpuDagExecutor("cuda:0"), share(50000), steps=10)
    L.cubed_stream_split_target(256)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
