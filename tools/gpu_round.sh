#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, kernel-trace profile.
# Every GPU step has its own time limit; a crash/abort/timeout ends the session
# (test *failures* -- pytest exit 1 -- do not, so the bench still runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >> gpurun_out/steps.log; }
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
step pytest
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
if fatal $rc; then echo "pytest-gpu crashed rc=$rc"; exit 1; fi
step bench
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
step prof
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
if [ -z "${NO_PMC}" ]; then
  step pmc
  R=$GRAFT_REPO_ROOT
  cd /tmp && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline > $R/gpurun_out/pmc_fetch.log 2>&1 || { echo pmc fetch failed; tail -20 $R/gpurun_out/pmc_fetch.log; exit 1; }
  cd /tmp && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline > $R/gpurun_out/pmc_write.log 2>&1 || { echo pmc write failed; tail -20 $R/gpurun_out/pmc_write.log; exit 1; }
  cd $R && python tools/traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write cubed_stream_f32_l2_r1 > gpurun_out/traffic.json && cat gpurun_out/traffic.json
fi
echo all-done
