#!/bin/bash
# Round-end profile refresh on a 1-GPU MI355X box: kernel-trace stats of the
# whole bench (every extra), FETCH_SIZE / WRITE_SIZE passes -> per-kernel
# traffic.json, then the bench line itself reading that traffic.  Each step
# has its own time limit; any failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof.log" 2>&1 || { echo prof failed; tail -20 "$R/gpurun_out/prof.log"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_fetch.log" 2>&1 || { echo pmc fetch failed; tail -20 "$R/gpurun_out/pmc_fetch.log"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_write.log" 2>&1 || { echo pmc write failed; tail -20 "$R/gpurun_out/pmc_write.log"; exit 1; }
cd "$R"
python tools/traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write $TRAFFIC_KERNELS > gpurun_out/traffic.json || exit 1
cat gpurun_out/traffic.json
cp gpurun_out/traffic.json profiles/traffic.json
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
tail -c 600 gpurun_out/bench.json
echo all-done
