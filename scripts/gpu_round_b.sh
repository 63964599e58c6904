# Round check, part B: kernel traces of configs 2/5/3, PMC passes on config 2 (one counter group
# per pass, kernel trace only) and the per-launch traffic of the roofline kernels
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-round}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$O/prof_trace.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace_c5" -o run --output-format csv -- python3 "$R/bench.py" --config 5 --steps 2 --warmup 1 --no-cpu > "$O/prof_trace_c5.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace_c3" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 3 --warmup 1 --no-cpu > "$O/prof_trace_c3.log" 2>&1 && \
i=0 && \
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC" "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$O/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu > "$O/pmc$i.log" 2>&1 || { echo "pmc$i failed"; exit 1; }
done
rc=$?
cd "$R"
[ $rc -eq 0 ] && python3 scripts/traffic_json.py "$O/pmc1" "$O/pmc2" "txnrec_kernel,keydeps_fast_kernel<,keydeps_kernel<" "profiles/$TAG" "$O/traffic_config2.json" "$O/pmc6"
echo "rc=$rc"
exit $rc
