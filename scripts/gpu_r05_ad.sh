# Round 5, call ad: readiness evaluation fused into the filter launch; readiness GPU tests, latency, trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_ad}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ready.py tests/test_gpu_waiting_on.py tests/test_gpu_status_events.py > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for i in 1 2; do
timeout -k 10 300 python scripts/ready_latency.py > "$O/ready_lat.$i.json" 2> "$O/ready_lat.$i.err" || exit 1
python3 -c "import json;d=json.load(open('$O/ready_lat.$i.json'));print('ready ms/call', round(d['update_ms_per_call'],4), d['update_calls'], d['released'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/ready_trace" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --batches 4 > "$O/ready_trace.log" 2>&1 || exit 1
