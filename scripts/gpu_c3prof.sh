# Kernel trace of the config-3 (20% range txns) pipeline.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-c3}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 3 --warmup 1 --no-cpu > "$O/prof.log" 2>&1
rc=$?
python3 - "$(find "$O/prof" -name '*kernel_stats.csv' | head -n 1)" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print("%-60s %6s %10.1f us %5s%%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"]))
PY
exit $rc
