# Round 5, calls av..: GPU suite, registered leg, kernel statistics of the registered leg
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_av}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python scripts/ready_latency.py --registered --batches 64 --batch 1024 > "$O/reg_lat.json" 2> "$O/reg_lat.err" || exit 1
python3 -c "import json;d=json.load(open('$O/reg_lat.json'));r=d['registered'];t=d['status_at_time_W'];print('registered dev/wall/sort', round(r['device_ms_per_batch'],4), round(r['compute_wall_ms_per_batch'],4), round(r['sort_ms_per_batch'],4), 'sat dev/wall', round(t['device_ms_per_batch'],4), round(t['compute_wall_ms_per_batch'],4))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/reg_k" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --registered --batches 32 --batch 1024 > "$O/reg_k.log" 2>&1 || exit 1
