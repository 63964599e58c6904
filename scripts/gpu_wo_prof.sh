# WaitingOn levelling profile: kernel trace of a config-5 bench (per-kernel durations).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-wo}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_waiting_on.py > "$O/pytest_wo.log" 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --config 5 --steps 2 --warmup 1 --no-cpu > "$O/prof.log" 2>&1
rc=$?; echo "rc=$rc"; tail -2 "$O/pytest_wo.log"; cut -d, -f1-4 "$O/prof/run_kernel_stats.csv" | head -30; exit $rc
