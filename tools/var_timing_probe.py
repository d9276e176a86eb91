"""Development probe: why var's plain-pass step time (bench.py var extra)
sits ~0.1 ms above its launch time.  Times the same step over several step
counts, back to back, with the bench's own timed()."""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
import cubed_amd as cubed  # noqa: E402
import cubed_amd.array_api as xp  # noqa: E402
import cubed_amd.random as crandom  # noqa: E402
from cubed_amd.core.plan import arrays_to_plan  # noqa: E402
from cubed_amd.runtime.executors.gpu import GpuDagExecutor  # noqa: E402


def main():
    ex = GpuDagExecutor()
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=ex)
    random.seed(1000)
    u = xp.astype(crandom.random((1000, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    v = xp.astype(crandom.random((1000, 720, 1440), chunks=(10, 720, 1440), spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=ex, array_names=[u.name, v.name])
    bench.sync()
    for fname in ("mean", "var"):
        m = getattr(xp, fname)(u * v, axis=0)
        plan = arrays_to_plan(m)
        step = bench.step_fn(plan, ex, [m], (u, v))
        step()
        step()
        for n in (5, 5, 5, 5, 10, 10, 10, 20, 40, 80):
            dt = bench.timed(step, n, 1)
            print(f"{fname} steps={n:3d}: {dt * 1e3:.4f} ms/step, host enqueue median "
                  f"{sorted(bench.HOST_US)[len(bench.HOST_US) // 2] * 1e6:.1f} us, max {max(bench.HOST_US) * 1e6:.1f} us",
                  flush=True)
        del m, plan


if __name__ == "__main__":
    main()
