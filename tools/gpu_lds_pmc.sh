#!/bin/bash
# LDS / issue counters of the chained bf16 GEMM (BASELINE config 5), one
# rocprofv3 --pmc pass per counter set (kernel trace only), over
# tools/matmul_probe.py (two timed launches after a warm-up).  Writes the
# per-dispatch CSVs under gpurun_out/lds_pmc_*; tools/pmc_summary.py folds
# them per kernel.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
DT="${DT:-bf16}"
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/rocprof_counters.txt" 2>&1 || true
i=0
for SET in \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d "$R/gpurun_out/lds_pmc_$i" -o run -- \
    python3 "$R/tools/matmul_probe.py" --dtypes "$DT" --reps 2 > "$R/gpurun_out/lds_pmc_$i.log" 2>&1 \
    || { echo "pmc pass $i failed"; tail -20 "$R/gpurun_out/lds_pmc_$i.log"; exit 1; }
done
cd "$R" && python tools/pmc_summary.py gpurun_out/lds_pmc_1 gpurun_out/lds_pmc_2 k_gemm_ > gpurun_out/lds_pmc.json && cat gpurun_out/lds_pmc.json
