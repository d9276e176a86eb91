#!/bin/bash
# Round-6 profile session (as rounds 4-5) on a 1-GPU MI355X box: kernel-trace stats of the
# whole bench, then FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel
# trace only) whose per-dispatch CSVs come back under gpurun_out/ and are
# folded per kernel by tools/traffic.py on the host, then the default bench
# line (with the CPU baseline).  Every step has its own time limit and any
# failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline"
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof.log" 2>&1 || { echo prof failed; tail -20 "$R/gpurun_out/prof.log"; exit 1; }
echo prof-done
if [ -z "$SKIP_PMC" ]; then
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_fetch.log" 2>&1 || { echo pmc fetch failed; tail -20 "$R/gpurun_out/pmc_fetch.log"; exit 1; }
echo fetch-done
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_write.log" 2>&1 || { echo pmc write failed; tail -20 "$R/gpurun_out/pmc_write.log"; exit 1; }
echo write-done
fi
cd "$R"
# fold the PMC passes here (their CSVs can exceed what a call brings back) and
# keep the kernel stats; the per-dispatch traces stay on the box
python3 tools/traffic.py --compact gpurun_out/pmc_fetch FETCH_SIZE > gpurun_out/pmc_fetch.json &&
python3 tools/traffic.py --compact gpurun_out/pmc_write WRITE_SIZE > gpurun_out/pmc_write.json || { echo fold failed; exit 1; }
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/r06_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof/run_kernel_trace.csv")))
with open("gpurun_out/r06_kernel_sequence.txt", "w") as f:
    for r in rows:
        n = r["Kernel_Name"][:100]
        f.write(f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:10.2f} {r.get('Grid_Size', r.get('Grid_Size_X', ''))} {n}\n")
PY
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
[ -n "$SKIP_BENCH" ] && { echo all-done; exit 0; }
timeout -k 10 420 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
tail -c 300 gpurun_out/bench.json
echo all-done
