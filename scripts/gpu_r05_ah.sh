# Round 5, calls ah/ai: RedundantBefore entries in one pinned copy + one scatter launch, truncation bounds
# looked up on the device; GPU suite, registered leg
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_ah}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python scripts/ready_latency.py --registered --batches 64 --batch 1024 > "$O/reg_lat.json" 2> "$O/reg_lat.err" || exit 1
python3 -c "import json;d=json.load(open('$O/reg_lat.json'));r=d['registered'];print('registered dev/wall/register/rb', round(r['device_ms_per_batch'],4), round(r['compute_wall_ms_per_batch'],4), round(r['register_wall_ms_per_batch'],4), round(r['rb_wall_ms_per_batch'],4))"
