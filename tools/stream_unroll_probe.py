"""Development probe (not part of the library): rows in flight per lane of
the JIT streaming kernels (cubed_stream_force_unroll, jit.hip) on the
vorticity reduction (configs[3], f64, two streamed + two broadcast leaves)
and the headline quad-means (f32, two leaves), each U in its own plan, all in
one process, alternating.

    python tools/stream_unroll_probe.py [rounds]
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
    arrays_to_plan(a, b, x, y, u, v).execute(executor=ex, array_names=[a.name, b.name, x.name, y.name, u.name, v.name])
    vort_bytes = 2 * 999 * 900 * 800 * 8
    qm_bytes = 2 * 1000 * 720 * 1440 * 4
    steps = {}
    for U in (0, 4, 8, 3):
        L.cubed_stream_force_unroll(U)
        mv = xp.mean(a[1:] * x + b[1:] * y)
        mq = xp.mean(u * v, axis=0)
        steps[U] = (bench.step_fn(arrays_to_plan(mv), ex, [mv], (a, b, x, y)),
                    bench.step_fn(arrays_to_plan(mq), ex, [mq], (u, v)))
        for s in steps[U]:
            s()  # lowering + JIT compile with this U
    L.cubed_stream_force_unroll(0)
    for r in range(rounds):
        for U, (sv, sq) in steps.items():
            for _ in range(3):
                sv()
                sq()
            dv = bench.timed(sv, 10, 1)
            dq = bench.timed(sq, 10, 1)
            print(f"round {r} U {U or 'default'}: vorticity {dv * 1e3:.4f} ms ({vort_bytes / dv / 8e12:.4f} of 8 TB/s)"
                  f"  quad-means {dq * 1e3:.4f} ms ({qm_bytes / dq / 8e12:.4f})", flush=True)


if __name__ == "__main__":
    main()
