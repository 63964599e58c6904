# Round 5, call y: speculative check inside the sizes scan, key flags / RedundantBefore status zeroed by the init launch, registered join queued inside the compute
# by the init launch; GPU suite, registered leg, config 2
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_y}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python scripts/ready_latency.py --registered --batches 64 --batch 1024 > "$O/reg_lat.json" 2> "$O/reg_lat.err" || exit 1
python3 -c "import json;d=json.load(open('$O/reg_lat.json'));r=d['registered'];t=d['status_at_time_W'];print('registered dev/wall', round(r['device_ms_per_batch'],4), round(r['compute_wall_ms_per_batch'],4), 'sat dev/wall', round(t['device_ms_per_batch'],4), round(t['compute_wall_ms_per_batch'],4))"
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > "$O/bench.json" 2> "$O/bench.err" || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print('config2', round(d['ms_per_step'],4), round(d['stage_ms']['total'],4), round(d['stage_ms']['fill'],4))"
