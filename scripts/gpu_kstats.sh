# Per-kernel stats of each measurement build: TAG=... BENCH_ARGS=... bash scripts/gpu_kstats.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for f in "$R"/cassandra-accord_amd/libaccord_deps_v*.so; do
  v=$(basename $f .so)
  ACCORD_FILL_STATS=1 ACCORD_LIB=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS} > "$O/$v.log" 2>&1 || { echo "$v failed"; tail -5 "$O/$v.log"; exit 1; }
  grep "took the general" "$O/$v.log" | tail -1
  f2=$(find "$O/$v" -name "*kernel_stats.csv" | head -1)
  python3 - "$f2" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'  {r["Name"][:60]:60s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"])/1e3:9.1f}')
PY
done
