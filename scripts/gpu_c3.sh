# Range path iteration: range GPU tests (incl. config 3 full), then a config-3 bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-c3}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${FILES:-tests/test_gpu_ranges.py} > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu > "$O/bench_c3.json" 2> "$O/bench_c3.err" || { tail -5 "$O/bench_c3.err"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c3.json'));print(d['ms_per_step'], d['stage_ms'])"
