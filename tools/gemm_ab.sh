#!/bin/bash
# A/B of the bf16 GEMM tilings on config 5 (bench.py --only matmul_bf16), on
# one box, alternating so clock drift shows:  bash tools/gemm_ab.sh [rounds] [bf16|f32]
#   packed: default (operands packed, then whole-matrix tiles: gemm_bf16_w4p.h)
#   chunk : GemmLaunch.PACKED off (the per-chunk w4l kernel)
#   grid  : PACKED off, GRID_INPUTS widened to bf16 (w4l's whole-matrix form)
#   (f32: chunk and grid both run the unpacked grid kernel, k_gemm_f32_chain<.., GRID>)
# (the library reads no environment; the switch is made in-process here)
set -e
R=${1:-2}
DT=${2:-bf16}
mkdir -p gpurun_out
for r in $(seq $R); do
  for v in packed chunk grid; do
    timeout -k 10 240 python -u - "$v" "$DT" > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err <<'PY'
import runpy, sys
import numpy as np
sys.path.insert(0, ".")
from cubed_amd import ir
from cubed_amd.lowering import GemmLaunch
if sys.argv[1] != "packed":
    GemmLaunch.PACKED = False
if sys.argv[1] == "grid":
    GemmLaunch.GRID_INPUTS = GemmLaunch.GRID_INPUTS | {ir.dtype_code(ir.bfloat16)}
sys.argv = ["bench.py", "--only", "matmul_" + sys.argv[2], "--no-cpu-baseline"]
runpy.run_path("bench.py", run_name="__main__")
PY
    python - "$v" "$DT" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/ab_{sys.argv[1]}.json") if l.startswith("{")][-1])
m = d["extra"]["matmul_" + sys.argv[2]]
print(f"{sys.argv[1]:6s} {m['value']:8.1f} TF  {m['ms']:8.3f} ms  check {m['check']['pass']}", flush=True)
PY
  done
done
