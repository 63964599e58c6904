# Round 5, call s: speculative fill (v2 = HEAD + speculative fill) vs HEAD (v0) on configs 2 and 5;
# bucket union of range txns (config 3, ACCORD_RK_UNION=sort for the bitonic union); the GPU suite;
# readiness call latency and its kernel / copy trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_s}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_keydeps.py tests/test_gpu_ranges.py > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for round in 1 2; do for u in bucket sort; do
  ACCORD_RK_UNION=$u timeout -k 10 200 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu > "$O/c3_$u.$round.json" 2> "$O/c3_$u.$round.err" || { tail -5 "$O/c3_$u.$round.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$u.$round.json'));s=d['stage_ms'];print('$u', round(d['ms_per_step'],3), {k:round(x,3) for k,x in s.items() if x})"
done; done
TAG=r05_s2 BENCH_ARGS="--config 2" bash scripts/ab_libs.sh || exit 1
TAG=r05_s25 BENCH_ARGS="--config 5" bash scripts/ab_libs.sh || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu_all.log" 2>&1 || { tail -30 "$O/pytest_gpu_all.log"; exit 1; }
tail -1 "$O/pytest_gpu_all.log"
timeout -k 10 300 python scripts/ready_latency.py > "$O/ready_lat.json" 2> "$O/ready_lat.err" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/ready_trace" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --batches 2 > "$O/ready_trace.log" 2>&1 || exit 1
python3 "$R/scripts/ready_latency.py" --analyse "$O/ready_trace" > "$O/ready_trace_summary.json"
