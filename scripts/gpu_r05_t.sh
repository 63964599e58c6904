# Round 5, call t: readiness results through the host buffer (last block of the last evaluation) and
# unfiltered evaluation of small launches; readiness GPU tests, call latency (filter on / off), trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_t}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ready.py tests/test_gpu_waiting_on.py tests/test_gpu_status_events.py > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
ACCORD_READY_FILTER_MIN=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ready.py > "$O/pytest_gpu_f0.log" 2>&1 || { tail -30 "$O/pytest_gpu_f0.log"; exit 1; }
tail -1 "$O/pytest_gpu_f0.log"
for f in 0 16384 65536 0 16384 65536; do
  ACCORD_READY_FILTER_MIN=$f timeout -k 10 300 python scripts/ready_latency.py > "$O/ready_lat_$f.json" 2> "$O/ready_lat_$f.err" || exit 1
  python3 -c "import json;d=json.load(open('$O/ready_lat_$f.json'));print('filter_min $f', round(d['update_ms_per_call'],4), d['update_calls'], d['released'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/ready_trace" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --batches 2 > "$O/ready_trace.log" 2>&1 || exit 1
cd "$R"
timeout -k 10 300 python scripts/ready_latency.py --registered --batches 64 --batch 1024 > "$O/reg_lat.json" 2> "$O/reg_lat.err" || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/reg_trace" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --registered --batches 16 --batch 1024 > "$O/reg_trace.log" 2>&1 || exit 1
