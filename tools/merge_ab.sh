#!/bin/bash
# GPU parity tests, then merge on/off A/B of the bench workloads it touches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -8 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit 1; fi
fi
for v in ${ARMS:-off on off on}; do
  timeout -k 10 300 python tools/merge_ab.py $v --no-cpu-baseline --steps 20 --warmup 3 --only ${ONLY:-rechunk_mean,rechunk_mean_share,config1,vorticity} > gpurun_out/mab_$v.json 2> gpurun_out/mab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/mab_$v.err; exit 1; }
  python - "$v" gpurun_out/mab_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
e = d["extra"]
print(sys.argv[1], "quad", d["ms_per_step"], "elided", e["rechunk_mean"]["elided"]["ms"], e["rechunk_mean"]["elided"]["launches_ms"],
      "share6250", e["rechunk_mean_share"]["rows_6250"]["ms"], "share7000", e["rechunk_mean_share"]["rows_7000"]["ms"],
      "config1", e["config1"]["ms"], "vort", e["vorticity"]["ms"], e["vorticity"]["launches_ms"], "fails", d.get("checks_failed"), flush=True)
PY
done
