#!/bin/bash
# A/B of the streaming kernel's row batching (development): quad-means headline,
# config 1 and vorticity per variant, one bench process each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
run() {
  echo "== $1" >> gpurun_out/stream_ab.log
  env $2 timeout -k 10 180 python bench.py --only config1,vorticity --no-cpu-baseline --steps 20 > gpurun_out/ab.json 2>> gpurun_out/stream_ab.err || exit 1
  python - >> gpurun_out/stream_ab.log <<'PY'
import json
d = json.loads(open("gpurun_out/ab.json").read().strip().splitlines()[-1])
e = d["extra"]
print("  quad-means %.4f ms/step, kernel %s" % (d["ms_per_step"], d["roofline"]["kernel"]))
for k in ("config1", "vorticity"):
    print("  %s %.4f ms, %s" % (k, e[k]["ms"], e[k]["roofline"]["kernel"]))
PY
}
run default ""
run U8 "CUBED_AMD_STREAM_U=8"
run dbuf "CUBED_AMD_JIT_DEFS=-DCUBED_STREAM_DBUF=1"
run dbuf_U2 "CUBED_AMD_JIT_DEFS=-DCUBED_STREAM_DBUF=1 CUBED_AMD_STREAM_U=2"
run dbuf_U8 "CUBED_AMD_JIT_DEFS=-DCUBED_STREAM_DBUF=1 CUBED_AMD_STREAM_U=8"
run default2 ""
cat gpurun_out/stream_ab.log
