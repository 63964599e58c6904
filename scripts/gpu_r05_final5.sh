# Round 5, final small-batch measurement after the RedundantBefore / upload / registration changes:
# registered + readiness bench line, readiness latency, registered leg, kernel statistics
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_final5}"; mkdir -p "$O"
timeout -k 10 300 python bench.py --registered --ready --steps 3 --warmup 1 --no-cpu > "$O/bench_config2_registered.json" 2> "$O/bench_config2_registered.err" || exit 1
timeout -k 10 300 python bench.py --resident --steps 3 --warmup 1 --no-cpu > "$O/bench_config2_resident.json" 2> "$O/bench_config2_resident.err" || exit 1
timeout -k 10 300 python scripts/ready_latency.py > "$O/ready_lat.json" 2> "$O/ready_lat.err" || exit 1
timeout -k 10 300 python scripts/ready_latency.py --registered --batches 64 --batch 1024 > "$O/reg_lat.json" 2> "$O/reg_lat.err" || exit 1
python3 -c "import json;d=json.load(open('$O/reg_lat.json'));r=d['registered'];print({k:round(v,4) for k,v in r.items() if 'wall' in k or 'device' in k})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kreg" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --registered --batches 32 --batch 1024 > "$O/kreg.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -d "$O/reg_api" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --registered --batches 16 --batch 1024 > "$O/reg_api.log" 2>&1 || exit 1
echo done
