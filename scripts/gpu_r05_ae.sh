# Round 5, call ae: checkpoint cells written key-major then transposed through LDS; range GPU tests, config 3
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_ae}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ranges.py tests/test_gpu_resident.py tests/test_gpu_shards.py tests/test_gpu_accept.py > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for i in 1 2; do
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu > "$O/bench_c3.$i.json" 2> "$O/bench_c3.$i.err" || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c3.$i.json'));print('config 3', round(d['ms_per_step'],4), round(d['stage_ms']['count'],3), d['count_stage_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace_c3" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 3 --warmup 1 --no-cpu > "$O/prof_trace_c3.log" 2>&1 || exit 1
