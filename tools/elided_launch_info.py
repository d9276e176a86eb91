"""Print the launch the GPU executor builds for the elided rechunk + mean
(BASELINE config 3 "rechunk+reduce") and dump its JIT source and task table
(development aid for tools/stream_jit_probe.hip)."""
import os
import random
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.lowering as L
import cubed_amd.random as crandom
from cubed_amd import _native as nat
from cubed_amd.core.plan import arrays_to_plan
from cubed_amd.runtime.executors.gpu import GpuDagExecutor

N = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
ex = GpuDagExecutor("cuda:0")
spec = cubed.Spec(allowed_mem="288GB", executor=ex)
random.seed(2000)
x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
m = xp.mean(x.rechunk((N, 1000)), axis=0)
plan = arrays_to_plan(m)
plan.execute(executor=ex, array_names=[m.name], resume=True)
fl = [l for v in ex._cache.values() for l in v[1] if isinstance(l, L.FusedLaunch)]
for f in fl:
    p = f.prog
    print("mode", p.mode, "nred", p.nred, "nleaves", p.nleaves, "nfields", p.nfields, "ntasks", f.ntasks,
          "max_kept", f.max_kept, "max_red", f.max_red, "ws", f.ws_bytes, "groups", f.groups is not None,
          "fold", f.fold is not None)
    tab = f.table.cpu().numpy().view(np.uint8).reshape(f.ntasks, -1)
    print("task0 int64 words", tab[0].view(np.int64)[:24].tolist())
    open("gpurun_out/elided_jit.hip", "w").write(nat.program_source(f.handle))
