# GPU check: parity tests, then bench, then a rocprofv3 kernel trace.  Every step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
TAG=${TAG:-check}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/$TAG/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG/prof_trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS} > "$R/gpurun_out/$TAG/prof_trace.log" 2>&1
rc=$?
echo "rc=$rc"
tail -3 "$R/gpurun_out/$TAG/pytest_gpu.log"
exit $rc
