"""Host time of one matmul step (config 5 shape, smaller n): where the
enqueue goes (cProfile of a replayed step).  Development aid."""
import cProfile
import os
import pstats
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
from cubed_amd.core.plan import arrays_to_plan
from cubed_amd.runtime.executors.gpu import GpuDagExecutor
from cubed_amd.storage import DeviceArray

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
ex = GpuDagExecutor("cuda:0")
spec = cubed.Spec(allowed_mem="288GB", executor=ex)
random.seed(1)
A = xp.astype(crandom.random((n, n), chunks=(5000, 5000), spec=spec), xp.bfloat16)
B = xp.astype(crandom.random((n, n), chunks=(5000, 5000), spec=spec), xp.bfloat16)
arrays_to_plan(A, B).execute(executor=ex, array_names=[A.name, B.name])
m = xp.matmul(A, B)
plan = arrays_to_plan(m)
keep = {id(A.zarray), id(B.zarray)}
targets = [d["target"] for _, d in plan._finalize_dag().nodes(data=True)
           if isinstance(d.get("target"), DeviceArray) and id(d["target"]) not in keep]


def step():
    for t in targets:
        t.written = False
    plan.execute(executor=ex, resume=True, array_names=[m.name])


step()
torch.cuda.synchronize()
for i in range(3):
    t0 = time.perf_counter()
    step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"step {i}: host {1e6 * (t1 - t0):.1f} us, total {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
step()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("cumulative").print_stats(18)
