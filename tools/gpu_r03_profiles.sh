#!/bin/bash
# Round-3 profile session on a 1-GPU MI355X box: kernel-trace stats of the
# whole bench, FETCH_SIZE / WRITE_SIZE passes -> per-kernel traffic.json,
# an MFMA-utilisation counter pass over the two GEMM extras, the pieces
# probe, then the bench line itself reading the new traffic.  Every step has
# its own time limit and any failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline"
KERNELS="quad_means_fused=cubed_stream_f32_l2_r1 rechunk_copy=k_copy_flat config1_stream=cubed_stream_f64_l1_r2 \
vorticity_pieces=cubed_stream_f64_l4_r2_partials matmul_f32=k_gemm_f32_chain matmul_bf16=k_gemm_bf16_chain \
rechunk_mean_stream=cubed_stream_f32_l1_r1"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof.log" 2>&1 || { echo prof failed; tail -20 "$R/gpurun_out/prof.log"; exit 1; }
echo prof-done
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_fetch.log" 2>&1 || { echo pmc fetch failed; tail -20 "$R/gpurun_out/pmc_fetch.log"; exit 1; }
echo fetch-done
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_write.log" 2>&1 || { echo pmc write failed; tail -20 "$R/gpurun_out/pmc_write.log"; exit 1; }
echo write-done
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_mfma" -o run -- python3 "$R/bench.py" --only matmul_f32,matmul_bf16 --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc_mfma.log" 2>&1 || { echo pmc mfma failed; tail -20 "$R/gpurun_out/pmc_mfma.log"; exit 1; }
echo mfma-done
cd "$R"
python tools/traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write $KERNELS > gpurun_out/traffic.json || exit 1
# the elided rechunk + mean shares its kernel name with the per-rank share and
# the materialised mean: its own pass, told apart by grid size
ONLY=rechunk_mean KERNELS="rechunk_mean_stream=cubed_stream_f32_l1_r1@239616 rechunk_mean_materialised=cubed_stream_f32_l1_r1@243712" \
  bash tools/gpu_pmc_only.sh > /dev/null || { echo pmc only failed; exit 1; }
python - <<'PY' || exit 1
import json
t = json.load(open("gpurun_out/traffic.json"))
t.update(json.load(open("gpurun_out/traffic_only.json")))
json.dump(t, open("gpurun_out/traffic.json", "w"), indent=1)
PY
cp gpurun_out/traffic.json profiles/traffic.json
timeout -k 10 180 tools/pieces_probe 5 > gpurun_out/pieces_probe.log 2>&1 || { echo probe failed; tail -5 gpurun_out/pieces_probe.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
tail -c 300 gpurun_out/bench.json
echo all-done
