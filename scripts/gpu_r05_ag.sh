# Round 5, call ag: final build -- the GPU suite and config 3
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_ag}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu > "$O/bench_c3.json" 2> "$O/bench_c3.err" || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('config 3', round(d['ms_per_step'],4), d['count_stage_ms'])"
