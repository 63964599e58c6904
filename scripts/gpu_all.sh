# All GPU tests + config-2/5 bench lines (no CPU baseline), optional stamp run.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-all}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > "$O/bench.json" 2> "$O/bench.err" && \
timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu > "$O/bench_c5.json" 2> "$O/bench_c5.err"
rc=$?; echo "rc=$rc"; tail -2 "$O/pytest_gpu.log"
python - "$O" <<'PY'
import json, sys
for f in ("bench.json", "bench_c5.json"):
    try:
        d = json.load(open(f"{sys.argv[1]}/{f}"))
        print(f, "ms/step %.3f" % d["ms_per_step"], {k: round(v, 3) for k, v in d["stage_ms"].items() if v})
    except Exception as e:
        print(f, "n/a", e)
PY
exit $rc
