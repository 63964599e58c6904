# Round 5, call aj: HIP API + kernel timelines of the current registered batch and readiness call
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_aj}"; mkdir -p "$O"
timeout -k 10 300 python scripts/ready_latency.py > "$O/ready_lat.json" 2> "$O/ready_lat.err" || exit 1
python3 -c "import json;d=json.load(open('$O/ready_lat.json'));print('ready ms/call', round(d['update_ms_per_call'],4), d['update_calls'], d['released'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -d "$O/ready_api" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --batches 4 > "$O/ready_api.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -d "$O/reg_api" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --registered --batches 16 --batch 1024 > "$O/reg_api.log" 2>&1 || exit 1
