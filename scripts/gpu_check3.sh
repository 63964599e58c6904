# GPU check with WaitingOn levelling: all gpu tests, config-2 and config-5 bench lines, config-5 trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
TAG=${TAG:-check}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/$TAG/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 400 python bench.py --config 5 --steps 3 --warmup 1 > gpurun_out/$TAG/bench_c5.json 2> gpurun_out/$TAG/bench_c5.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG/prof_trace_c5" -o run --output-format csv -- python3 "$R/bench.py" --config 5 --steps 2 --warmup 1 --no-cpu > "$R/gpurun_out/$TAG/prof_trace_c5.log" 2>&1
rc=$?
echo "rc=$rc"
tail -3 "$R/gpurun_out/$TAG/pytest_gpu.log"
exit $rc
