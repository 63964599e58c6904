# GPU check with the range path: all gpu tests, config-2 and config-3 bench lines, kernel traces.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
TAG=${TAG:-check}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/$TAG/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --range-frac 0.2 --seed 3 --no-cpu > gpurun_out/$TAG/bench_c3.json 2> gpurun_out/$TAG/bench_c3.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG/prof_trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$R/gpurun_out/$TAG/prof_trace.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG/prof_trace_c3" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --range-frac 0.2 --seed 3 > "$R/gpurun_out/$TAG/prof_trace_c3.log" 2>&1
rc=$?
echo "rc=$rc"
tail -3 "$R/gpurun_out/$TAG/pytest_gpu.log"
exit $rc
