import sys, os, json, random, time
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import torch
import bench
import cubed_amd as cubed, cubed_amd.array_api as xp, cubed_amd.random as crandom
from cubed_amd.core.plan import arrays_to_plan
from cubed_amd.runtime.executors.gpu import GpuDagExecutor
ex = GpuDagExecutor()
spec = cubed.Spec(allowed_mem="2GB", executor=ex)
random.seed(1)
a = crandom.random((1000, 900, 800), chunks=100, spec=spec)
arrays_to_plan(a).execute(executor=ex, array_names=[a.name])
m = xp.mean(a)
plan = arrays_to_plan(m)
def step():
    bench._reset_targets(plan, a)
    plan.execute(executor=ex, resume=True, array_names=[m.name])
step()
dt, l = bench.timed_launches(ex, step, 3, 1)
print(json.dumps({"lift": os.environ.get("CUBED_AMD_LIFT", "1"), "fullmean_ms": dt * 1e3, "launches": l}))
print(json.dumps({"vort": bench.vorticity_extra(ex, 0)}))
