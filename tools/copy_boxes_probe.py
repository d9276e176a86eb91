"""Development probe (not part of the library): the box tables of the config 3
rechunk copy under the reference's 2 GB plan (two ops composed into one copy)
and the 288 GB plan (one op), with each launch's time.  Run on the GPU box:
    python tools/copy_boxes_probe.py [N] [plans, e.g. 288GB,2GB] [untimed launches before the 5 timed]
"""
import collections
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
import cubed_amd as cubed  # noqa: E402
import cubed_amd.array_api as xp  # noqa: E402
import cubed_amd.random as crandom  # noqa: E402
from cubed_amd.core.plan import arrays_to_plan  # noqa: E402
from cubed_amd.lowering import CopyLaunch  # noqa: E402
from cubed_amd.runtime.executors.gpu import GpuDagExecutor  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
    ex = GpuDagExecutor()
    pre = float(os.environ.get("PRE_ALLOC_GB", "0"))
    if pre:  # allocate + free a dummy buffer first (placement diagnosis)
        d = torch.empty(int(pre * 2**30), dtype=torch.uint8, device="cuda")
        d.fill_(1)
        torch.cuda.synchronize()
        del d
        if os.environ.get("PRE_EMPTY"):
            torch.cuda.empty_cache()
    for mem in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("2GB", "288GB")):
        spec = cubed.Spec(allowed_mem=mem, executor=ex)
        random.seed(2000)
        x = xp.astype(crandom.random((N, N), chunks=(1000, N), spec=spec), xp.float32)
        arrays_to_plan(x).execute(executor=ex, array_names=[x.name])
        torch.cuda.synchronize()
        y = x.rechunk((N, 1000))
        plan = arrays_to_plan(y)
        step = bench.step_fn(plan, ex, [y], x)
        step()
        torch.cuda.synchronize()
        for name, launches, *_ in ex.last_schedule.steps:
            for L in launches:
                if not isinstance(L, CopyLaunch) or L.nboxes == 0:
                    continue
                shapes = collections.Counter((tuple(b.extent), tuple(b.sstride), tuple(b.dstride))
                                             for b in L.boxes)
                src = sorted(b.src for b in L.boxes)
                print(f"{mem} {name}: nboxes {L.nboxes} path {L.path} lane {L.lane} work {L.work} "
                      f"row_bytes {L.row_bytes}", flush=True)
                for k, c in shapes.most_common(4):
                    print(f"    {c} x extent {k[0]} sstride {k[1]} dstride {k[2]}")
                b0 = L.boxes[:3]
                for b in b0:
                    print(f"    box src +{b.src - src[0]} dst {b.dst:#x}")
                s = torch.cuda.Stream()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                warm = int(sys.argv[3]) if len(sys.argv) > 3 else 1
                with torch.cuda.stream(s):
                    for r in range(warm + 5):
                        if r == warm:
                            e0.record(s)
                        L.run(s.cuda_stream)
                    e1.record(s)
                torch.cuda.synchronize()
                print(f"    {e0.elapsed_time(e1) / 5:.4f} ms per launch (5 back to back)", flush=True)
        del x, y, plan, step
        bench.free_gpu()
        time.sleep(0.5)


if __name__ == "__main__":
    main()
