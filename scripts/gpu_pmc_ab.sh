# PMC groups ($PMC_GROUPS, ';'-separated) for every measurement build; table for kernels matching $KERNEL.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra GS <<< "$PMC_GROUPS"
for f in "$R"/cassandra-accord_amd/libaccord_deps_v*.so; do
  v=$(basename $f .so); i=0
  for grp in "${GS[@]}"; do
    i=$((i+1))
    ACCORD_LIB=$f timeout -s KILL 120 rocprofv3 --pmc $grp -d "$O/$v/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS} > "$O/$v.pmc$i.log" 2>&1 || { echo "$v pmc$i failed"; tail -5 "$O/$v.pmc$i.log"; exit 1; }
  done
  echo "== $v"
  for c in $(find "$O/$v" -name "*counter_collection.csv" | sort); do python3 "$R/scripts/pmc_table.py" "$c" "${KERNEL:-keydeps}"; done
done
