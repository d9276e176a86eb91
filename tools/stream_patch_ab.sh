#!/bin/bash
# Streaming kernels' load form A/B (tools/stream_patch_ab.py), alternated arms, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
for v in ${ARMS:-base xcd base xcd}; do
  timeout -k 10 300 python tools/stream_patch_ab.py $v --no-cpu-baseline --steps 20 --warmup 3 --only ${ONLY:-rechunk_mean,rechunk_mean_share,config1,vorticity} > gpurun_out/spab_$v.json 2> gpurun_out/spab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/spab_$v.err; exit 1; }
  python - "$v" gpurun_out/spab_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
e = d["extra"]
rm = e["rechunk_mean"]
print(sys.argv[1], "quad", d["ms_per_step"], "elided", rm["elided"]["ms"], "mat", rm["materialised"]["launches_ms"],
      "share6250", e["rechunk_mean_share"]["rows_6250"]["ms"], "share7000", e["rechunk_mean_share"]["rows_7000"]["ms"],
      "config1", e["config1"]["ms"], "vort", e["vorticity"]["ms"], "fails", d.get("checks_failed"), flush=True)
PY
done
