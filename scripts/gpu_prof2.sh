# Kernel trace of the default bench command (config 2, one batch size), plus the bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-p2}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$O/bench.json" 2> "$O/prof.log"
rc=$?
python3 - "$(find "$O/prof" -name '*kernel_stats.csv' | head -n 1)" "$O/bench.json" <<'PY'
import csv, sys, json
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print("%-60s %6s %10.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(d["ms_per_step"], {k: round(v, 3) for k, v in d["stage_ms"].items() if v})
PY
exit $rc
