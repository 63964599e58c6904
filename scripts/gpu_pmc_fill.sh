# Address/data-path counters of the config-2 pipeline (fill kernel focus): list the gfx950 counters,
# then one pass per group (kernel trace only).  TAG=... bash scripts/gpu_pmc_fill.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
i=0
for grp in "TA_TA_BUSY TA_BUFFER_READ_WAVEFRONTS" "TD_TD_BUSY TD_TC_STALL" "TCP_TCP_TA_DATA_STALL_CYCLES TCP_PENDING_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d "$O/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu > "$O/pmc$i.log" 2>&1 || echo "pmc$i failed ($grp)"
done
cd "$R"; for d in "$O"/pmc[0-9]*/; do echo "== $d"; python3 scripts/pmc_table.py "$d/run_counter_collection.csv" 2>&1 | grep -E "fast|history2|compact|downsweep|upsweep|Name|^ *[A-Z]" | head -30; done
