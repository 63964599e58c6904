# Round 5, call e: register-resident levelling resolver -- waiting-on tests, config-5 bench with the 1-core levelling leg
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_e}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_waiting_on.py > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 600 python -u bench.py --config 5 --steps 3 --warmup 1 --cpu-budget 10 > "$O/bench_c5.json" 2> "$O/bench_c5.err" || { tail -20 "$O/bench_c5.err"; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench_c5.json') if l.startswith('{')][-1])
print(d['ms_per_step'], {k: round(v,3) for k,v in d['stage_ms'].items() if v}); print(d['cpu_baseline'].get('levelling_1core')); print(d.get('waiting_on'))"
