#!/bin/bash
# GPU parity tests of the fused/stream paths, then the bench's streaming
# extras (quad-means headline, rechunk+mean, per-rank share, config 1,
# vorticity) with a one-line summary.  Every GPU step has its own limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_api_cases.py tests/test_gpu_core_cases.py -p no:cacheprovider \
  > gpurun_out/par.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/par.log; exit 1; }
tail -2 gpurun_out/par.log
timeout -k 10 400 python bench.py --no-cpu-baseline --only rechunk_mean,rechunk_mean_share,config1,vorticity \
  > gpurun_out/b2.json 2> gpurun_out/b2.err || { echo "bench failed"; tail -20 gpurun_out/b2.err; exit 1; }
python tools/extras_summary.py gpurun_out/b2.json
