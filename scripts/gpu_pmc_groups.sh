# PMC passes over the config-2 bench, one counter group per pass ($PMC_GROUPS separated by ';').
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=${TAG:-pmcg}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra GS <<< "$PMC_GROUPS"
for grp in "${GS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$O/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS} > "$O/pmc$i.log" 2>&1 || { echo "pmc$i failed"; tail -5 "$O/pmc$i.log"; exit 1; }
done
python3 "$R/scripts/pmc_table.py" "$O"/pmc*/ | grep -A40 "${KERNEL:-keydeps_kernel}" | head -45
