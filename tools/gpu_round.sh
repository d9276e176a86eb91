#!/bin/bash
# One GPU session: smoke, parity smoke, bench, kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1" >> gpurun_out/steps.log; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
step parity
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest-gpu failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
step bench
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; exit 1; }
step prof
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { echo prof failed; exit 1; }
echo all-done
