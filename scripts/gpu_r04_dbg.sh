# round-4 debug: executesAtLeast difference of the rf=0.1 schedule, then the readiness / keydeps tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04_dbg"; mkdir -p "$O"
timeout -k 10 300 python3 -u scripts/dbg_eal.py > "$O/dbg.txt" 2>&1; echo "dbg rc=$?"; tail -60 "$O/dbg.txt"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_ready.py tests/test_waiting_on_init.py tests/test_redundant_before.py \
  tests/test_gpu_keydeps.py tests/test_gpu_ranges.py > "$O/pytest_gpu.log" 2>&1; echo "pytest rc=$?"; tail -8 "$O/pytest_gpu.log"
for c in 2 3; do
  timeout -k 10 120 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > "$O/c$c.json" 2>"$O/c$c.err" || exit 1
  python3 -c "import json;d=json.loads(open('$O/c$c.json').read().strip().splitlines()[-1]);print('c$c', round(d['ms_per_step'],4), d['stage_ms'], d['count_stage_ms'])"
done
