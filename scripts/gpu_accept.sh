# Accept-batch GPU parity + PreAccept regressions + config-2 bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-accept}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_accept.py tests/test_gpu_ranges.py tests/test_gpu_keydeps.py > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stage_ms'])"
