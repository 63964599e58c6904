# Round 5, call ac: levelling with the staged resolver only (knobs pruned); WaitingOn GPU tests, config 5
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_ac}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_waiting_on.py tests/test_ready.py > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu > "$O/bench_c5.json" 2> "$O/bench_c5.err" || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c5.json'));print('config 5', round(d['ms_per_step'],3), round(d['stage_ms']['wo_level'],3))"
