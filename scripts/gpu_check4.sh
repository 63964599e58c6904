# Full GPU check: all gpu tests, config-2/5 bench lines, kernel traces for both, then PMC passes
# (one counter group per pass, kernel trace only) on config 2.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
TAG=${TAG:-check}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
timeout -k 10 900 python -m pytest tests -x -q -m gpu > "$O/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$O/bench.json" 2> "$O/bench.err" && \
timeout -k 10 400 python bench.py --config 5 --steps 3 --warmup 1 > "$O/bench_c5.json" 2> "$O/bench_c5.err" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$O/prof_trace.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace_c5" -o run --output-format csv -- python3 "$R/bench.py" --config 5 --steps 2 --warmup 1 --no-cpu > "$O/prof_trace_c5.log" 2>&1 && \
i=0 && \
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d "$O/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu > "$O/pmc$i.log" 2>&1 || { echo "pmc$i failed"; exit 1; }
done
rc=$?
echo "rc=$rc"
tail -3 "$O/pytest_gpu.log"
exit $rc
