#!/bin/bash
# A/B of the streaming split target (CUBED_STREAM_TARGET at build time) on the
# bench workloads that split: libraries tools/var/lib_t*.so built from the same
# sources with -DCUBED_STREAM_TARGET=N, swapped in for each run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
cp cubed_amd/libcubed_amd.so gpurun_out/lib_base.so
for v in base t2048 t4096 base; do
  if [ "$v" = base ]; then cp gpurun_out/lib_base.so cubed_amd/libcubed_amd.so; else cp tools/var/lib_$v.so cubed_amd/libcubed_amd.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --only rechunk_mean,rechunk_mean_share,config1,vorticity > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_$v.err; cp gpurun_out/lib_base.so cubed_amd/libcubed_amd.so; exit 1; }
  python - "$v" gpurun_out/ab_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
e = d["extra"]
print(sys.argv[1], "quad", d["ms_per_step"], "elided", e["rechunk_mean"]["elided"]["ms"],
      "share6250", e["rechunk_mean_share"]["rows_6250"]["ms"], "share7000", e["rechunk_mean_share"]["rows_7000"]["ms"],
      "config1", e["config1"]["ms"], "vort", e["vorticity"]["ms"], "fails", d.get("checks_failed"))
PY
done
cp gpurun_out/lib_base.so cubed_amd/libcubed_amd.so
