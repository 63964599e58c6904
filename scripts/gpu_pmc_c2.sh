# PMC passes (one counter group per run, kernel trace only) on the config-2 bench: TAG=... bash scripts/gpu_pmc_c2.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-pmc}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$O/prof_trace.log" 2>&1 || { echo "trace failed"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$O/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu > "$O/pmc$i.log" 2>&1 || { echo "pmc$i failed"; exit 1; }
done
cd "$R"
python3 scripts/pmc_table.py "$O"/pmc1 "$O"/pmc2 "$O"/pmc3 "$O"/pmc4 "$O"/pmc5 > "$O/pmc_table.txt"
python3 scripts/traffic_json.py "$O/pmc1" "$O/pmc2" "txnrec_kernel,keydeps_fast_kernel<,keydeps_kernel<" "profiles/$TAG" "$O/traffic_config2.json" > /dev/null
echo done
