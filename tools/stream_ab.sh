#!/bin/bash
# A/B of the streaming kernel's launch shape (development): kept groups per
# thread (CUBED_AMD_STREAM_W) and the workgroup target before a time split
# (CUBED_AMD_STREAM_TARGET); quad-means headline, config 1, vorticity and the
# elided rechunk+mean per variant, one bench process each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
run() {
  echo "== $1" >> gpurun_out/stream_ab.log
  env $2 timeout -k 10 240 python bench.py --only ${ONLY:-config1,vorticity,rechunk_mean} --no-cpu-baseline --steps 20 > gpurun_out/ab.json 2>> gpurun_out/stream_ab.err || exit 1
  python - >> gpurun_out/stream_ab.log <<'PY'
import json
d = json.loads(open("gpurun_out/ab.json").read().strip().splitlines()[-1])
e = d["extra"]
print("  quad-means %.4f ms/step (%.0f GB/s), kernel %s" % (d["ms_per_step"], d["value"], d["roofline"]["kernel"]))
for k in ("config1", "vorticity"):
    if k in e:
        print("  %s %.4f ms, %s" % (k, e[k]["ms"], e[k]["roofline"]["kernel"]))
if "rechunk_mean" in e:
    print("  rechunk_mean elided %.4f ms, materialised %.4f ms" % (e["rechunk_mean"]["elided"]["ms"], e["rechunk_mean"]["materialised"]["ms"]))
if "rechunk" in e:
    for p in ("plan_2GB", "plan_288GB"):
        r = e["rechunk"][p]
        print("  rechunk %s %.4f ms, %s (%s)" % (p, r["ms"], r["roofline"]["kernel"], r["check"]))
PY
}
for v in ${VARIANTS:-"default:" "W1_T2048:CUBED_AMD_STREAM_W=1 CUBED_AMD_STREAM_TARGET=2048" "W1_T256:CUBED_AMD_STREAM_W=1" "W4:CUBED_AMD_STREAM_W=4" "W2_T512:CUBED_AMD_STREAM_W=2 CUBED_AMD_STREAM_TARGET=512" "W2_T1024:CUBED_AMD_STREAM_W=2 CUBED_AMD_STREAM_TARGET=1024" "default2:"}; do
  run "${v%%:*}" "${v#*:}"
done
cat gpurun_out/stream_ab.log
