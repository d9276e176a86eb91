"""Run bench.py's extra workloads by name (development / profiling tool):
    python tools/extras.py rechunk config1 vorticity matmul
prints one JSON object per workload."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from cubed_amd.runtime.executors.gpu import GpuDagExecutor  # noqa: E402

FUNCS = {"rechunk": bench.rechunk_extra, "rechunk_mean": bench.rechunk_mean_extra, "config1": bench.config1_extra,
         "vorticity": bench.vorticity_extra, "matmul": bench.matmul_extra}

if __name__ == "__main__":
    torch.cuda.set_device(0)
    ex = GpuDagExecutor()
    for name in sys.argv[1:] or list(FUNCS):
        print(json.dumps({name: FUNCS[name](ex, 0)}), flush=True)
