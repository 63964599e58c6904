# Config-3 PMC passes (FETCH_SIZE, WRITE_SIZE, SQ busy/wait) over a short run, one group per pass.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${TAG:-c3pmc}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$O/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 1 --warmup 0 --no-cpu > "$O/pmc$i.log" 2>&1 || { echo "pmc$i failed"; exit 1; }
done
cd "$R"
for d in "$O"/pmc[0-9]*/; do python3 scripts/pmc_table.py "$d/run_counter_collection.csv" range; done
