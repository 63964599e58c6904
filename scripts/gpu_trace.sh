# Kernel trace of one bench config (dev aid): per-kernel average durations.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/${TAG:-trace}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" ${BENCH_ARGS} --steps 2 --warmup 1 --no-cpu > "$O/prof.log" 2>&1 || { tail -5 "$O/prof.log"; exit 1; }
python3 - "$O/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:28]:
    print("%-60s %4s %10.1f us" % (r["Name"][:60].replace("accord::(anonymous namespace)::", ""), r["Calls"], float(r["AverageNs"]) / 1e3))
PY
