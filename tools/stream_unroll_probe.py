"""Development probe (not part of the library): rows in flight per lane of
the JIT streaming kernels (cubed_stream_force_unroll, jit.hip) on the
vorticity reduction (configs[3], f64, two streamed + two broadcast leaves),
the headline quad-means (f32, two leaves), the 7000-row per-rank share of
config 3's rechunk + mean (f32, one leaf) and config 1 (f64, one leaf), each
U in its own plan, all in one process, alternating.

    python tools/stream_unroll_probe.py [rounds] [U[wW],...] [workload,...]   (U 0 = the library's choice)
"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import cubed_amd as cubed  # noqa: E402
import cubed_amd.array_api as xp  # noqa: E402
import cubed_amd.random as crandom  # noqa: E402
from cubed_amd import _native as nat  # noqa: E402
from cubed_amd.core.plan import arrays_to_plan  # noqa: E402
from cubed_amd.runtime.executors.gpu import GpuDagExecutor  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    L = nat.lib()
    import ctypes

    L.cubed_stream_force_unroll.argtypes = [ctypes.c_int]
    L.cubed_stream_force_unroll.restype = ctypes.c_int
    ex = GpuDagExecutor("cuda:0")
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    random.seed(5000)
    a = crandom.random((1000, 900, 800), chunks=100, spec=spec)
    b = crandom.random((1000, 900, 800), chunks=100, spec=spec)
    x = crandom.random((900, 800), chunks=100, spec=spec)
    y = crandom.random((900, 800), chunks=100, spec=spec)
    u = xp.astype(crandom.random((1000, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    v = xp.astype(crandom.random((1000, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    spec2 = cubed.Spec(allowed_mem="288GB", executor=ex)
    s7 = xp.astype(crandom.random((7000, 50000), chunks=(1000, 50000), spec=spec2), xp.float32)
    c1 = crandom.random((20000, 20000), chunks=(5000, 5000), spec=spec)
    arrays_to_plan(a, b, x, y, u, v, c1).execute(
        executor=ex, array_names=[a.name, b.name, x.name, y.name, u.name, v.name, c1.name])
    arrays_to_plan(s7).execute(executor=ex, array_names=[s7.name])
    work = {  # name: (bytes, plan builder)
        "vorticity": (2 * 999 * 900 * 800 * 8, lambda: (xp.mean(a[1:] * x + b[1:] * y), (a, b, x, y))),
        "quad-means": (2 * 1000 * 720 * 1440 * 4, lambda: (xp.mean(u * v, axis=0), (u, v))),
        "share-7000": (7000 * 50000 * 4, lambda: (xp.mean(s7.rechunk((7000, 1000)), axis=0), s7)),
        "config1": (20000 * 20000 * 8, lambda: (xp.mean((c1 + 1) * 2, axis=0), c1)),
    }
    # entries "U" or "UwW" (W: kept groups per lane, lowering.FORCE_STREAM_W)
    us = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "4", "8", "16"]
    if len(sys.argv) > 3:  # workloads to run (comma list of names)
        keep_names = sys.argv[3].split(",")
        work = {k: v for k, v in work.items() if k in keep_names}
    import cubed_amd.lowering as Lw

    steps = {}  # (position in the U list, workload): a plan of its own (its own buffers) per entry
    for ui, tag in enumerate(us):
        U, _, W = tag.partition("w")
        L.cubed_stream_force_unroll(int(U))
        Lw.FORCE_STREAM_W = int(W) if W else None
        for name, (_, build) in work.items():
            m, keep = build()
            st = bench.step_fn(arrays_to_plan(m), ex, [m], keep)
            st()  # lowering + JIT compile with this U
            steps[(ui, name)] = st
    L.cubed_stream_force_unroll(0)
    Lw.FORCE_STREAM_W = None
    for r in range(rounds):
        for ui, U in enumerate(us):
            line = []
            for name, (nbytes, _) in work.items():
                st = steps[(ui, name)]
                for _ in range(3):
                    st()
                d = bench.timed(st, 10, 1)
                line.append(f"{name} {d * 1e3:.4f} ms ({nbytes / d / 8e12:.4f})")
            print(f"round {r} plan {ui} U {U if U != '0' else 'default'}: " + "  ".join(line), flush=True)


if __name__ == "__main__":
    main()
