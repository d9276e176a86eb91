#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over ONE bench extra (bench.py --only $ONLY),
# so kernels that share a name with other extras' kernels (e.g. the elided
# rechunk + mean and the per-rank share: both cubed_stream_f32_l1_r1) get their
# own per-launch traffic.  Usage: ONLY=rechunk_mean KERNELS="key=kernel ..." bash tools/gpu_pmc_only.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --only $ONLY"
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmco_fetch" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmco_fetch.log" 2>&1 || { echo pmc fetch failed; tail -20 "$R/gpurun_out/pmco_fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmco_write" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmco_write.log" 2>&1 || { echo pmc write failed; tail -20 "$R/gpurun_out/pmco_write.log"; exit 1; }
cd "$R" && python tools/traffic.py gpurun_out/pmco_fetch gpurun_out/pmco_write $KERNELS > gpurun_out/traffic_only.json && cat gpurun_out/traffic_only.json
