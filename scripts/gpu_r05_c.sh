# Round 5, call c: gapped KeyDeps txnIds (no compaction in the compute): whole GPU suite, config-2 bench + kernel trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_c}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
tail -1 "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace" -o run -- python3 "$R/bench.py" --no-cpu --steps 10 --warmup 2 > "$O/bench_trace.json" 2>&1 || exit 1
find "$O/prof_trace" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats_config2.csv" \;
