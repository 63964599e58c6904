# Round 5, calls ax..: readiness tests, readiness latency, kernel statistics of the readiness calls
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_ax}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ready.py tests/test_gpu_status_events.py > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python scripts/ready_latency.py > "$O/ready_lat.json" 2> "$O/ready_lat.err" || exit 1
python3 -c "import json;d=json.load(open('$O/ready_lat.json'));print('ready ms/call', round(d['update_ms_per_call'],4), d['update_calls'], d['released'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/ready_k" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --batches 4 > "$O/ready_k.log" 2>&1 || exit 1
