#!/bin/bash
# PMC passes over the bench (no CPU baseline): FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 runs (kernel-trace only), then per-kernel HBM bytes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}"
cd /tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_fetch.log" 2>&1 || { echo pmc fetch failed; tail -20 "$R/gpurun_out/pmc_fetch.log"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_write.log" 2>&1 || { echo pmc write failed; tail -20 "$R/gpurun_out/pmc_write.log"; exit 1; }
cd "$R" && python tools/traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write \
  quad_means_fused=cubed_stream_f32_l2_r1 rechunk_copy=k_copy_flat config1_stream=cubed_stream_f64_l1_r2_split \
  vorticity_pieces=cubed_stream_f64_l4_r2_partials_split matmul_f32=k_gemm_f32_chain matmul_bf16=k_gemm_bf16_chain \
  rechunk_mean_stream=cubed_stream_f32_l1_r1_split@65536 \
  > gpurun_out/traffic.json && cat gpurun_out/traffic.json
