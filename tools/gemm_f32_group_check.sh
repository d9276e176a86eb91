set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --only matmul_f32 > gpurun_out/gm8.json 2> gpurun_out/gm8.err || { tail -5 gpurun_out/gm8.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/gm8.json').read().strip().splitlines()[-1]); e=d['extra']['matmul_f32']; print('gm8', e['ms'], e['value'], e['check']['pass'])"
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/gm8_fetch" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --only matmul_f32 > "$R/gpurun_out/gm8_fetch.log" 2>&1 || { tail -5 "$R/gpurun_out/gm8_fetch.log"; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/gm8_write" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --only matmul_f32 > "$R/gpurun_out/gm8_write.log" 2>&1 || { tail -5 "$R/gpurun_out/gm8_write.log"; exit 1; }
cd "$R" && python tools/traffic.py gpurun_out/gm8_fetch gpurun_out/gm8_write matmul_f32=k_gemm_f32_chain
