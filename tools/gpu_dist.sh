#!/bin/bash
# GPU session for the distributed executor: 2/3 ranks sharing the box's one
# GPU (gloo-staged collectives), the whole -m gpu suite, and a 2-rank bench
# rehearsal.  Each GPU step has its own limit; a crash ends the session.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/dist.log 2>&1
rc=$?; tail -30 gpurun_out/dist.log; if fatal $rc; then echo "dist crashed rc=$rc"; exit 1; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread --ignore=tests/test_gpu_dist.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; if fatal $rc; then echo "pytest-gpu crashed rc=$rc"; exit 1; fi
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --backend gloo --t-length 100 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo bench2 failed; tail -30 gpurun_out/bench2.err; exit 1; }
cat gpurun_out/bench2.json
echo all-done
