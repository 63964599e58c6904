# Config-3 PMC passes (SQ stall breakdown) + the counter list, for the range kernels.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-c3pmc}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$O/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 1 --warmup 0 --no-cpu > "$O/pmc$i.log" 2>&1 || { echo "pmc$i failed"; exit 1; }
done
echo done
