# PMC passes (one counter group per pass, kernel trace only, no sys/runtime trace).
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=${TAG:-pmc}
mkdir -p "$R/gpurun_out/$TAG"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/$TAG/counters.txt" 2>&1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d "$R/gpurun_out/$TAG/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS} > "$R/gpurun_out/$TAG/pmc$i.log" 2>&1 || { echo "pmc$i failed"; exit 1; }
done
echo done
