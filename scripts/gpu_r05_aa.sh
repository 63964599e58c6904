# Round 5, call aa: bench timed without profiling events (stage split from a profiled pass); profile switch test
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_aa}"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_keydeps.py tests/test_abi.py > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for c in 2 2; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu > "$O/bench_c$c.json" 2> "$O/bench_c$c.err" || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_c$c.json'));print('config $c', round(d['ms_per_step'],4), round(d['stage_ms']['total'],4), round(d['stage_ms']['fill'],4), round(d['roofline']['frac'],3))"
done
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu > "$O/bench_c3.json" 2> "$O/bench_c3.err" || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('config 3', round(d['ms_per_step'],4), round(d['stage_ms']['total'],4))"
