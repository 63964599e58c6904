# Copy a gpu_round_a.sh + gpu_round_b.sh result (gpurun_out/$TAG) into profiles/$TAG: bench lines, kernel-trace stats,
# PMC table (all passes), the pytest log, and refresh profiles/traffic_config2.json.
set -e
TAG=${1:?tag}; O=gpurun_out/$TAG; P=profiles/$TAG
mkdir -p "$P"
cp "$O/bench.json" "$P/bench_config2.json"
cp "$O/bench_c5.json" "$P/bench_config5.json"
cp "$O/bench_c3.json" "$P/bench_config3.json"
[ -f "$O/bench_resident.json" ] && cp "$O/bench_resident.json" "$P/bench_config2_resident.json"
[ -f "$O/bench_registered.json" ] && cp "$O/bench_registered.json" "$P/bench_config2_registered.json"
[ -f "$O/prof_trace_c3/run_kernel_stats.csv" ] && cp "$O/prof_trace_c3/run_kernel_stats.csv" "$P/kernel_stats_config3.csv"
cp "$O/prof_trace/run_kernel_stats.csv" "$P/kernel_stats_config2.csv"
cp "$O/prof_trace_c5/run_kernel_stats.csv" "$P/kernel_stats_config5.csv"
cp "$O/pytest_gpu.log" "$P/pytest_gpu.log"
{ echo "rocprofv3 --pmc, one counter group per pass (FETCH_SIZE / WRITE_SIZE separately), config 2;"
  echo "sums over all dispatches of the run. gfx950 FETCH_SIZE reports ~1/2 of wide coalesced reads (MI355X_MICROARCH.md)"
  for d in "$O"/pmc[0-9]*/; do echo "== $d"; python3 scripts/pmc_table.py "$d/run_counter_collection.csv"; done; } > "$P/pmc_config2.txt"
cp "$O/traffic_config2.json" profiles/traffic_config2.json
python3 - "$P" <<'PY'
import json, sys
for c in (2, 3, 5):
    d = json.loads([l for l in open(f"{sys.argv[1]}/bench_config{c}.json") if l.startswith("{")][-1])
    print(c, "%.3f ms/step" % d["ms_per_step"], "%.1fM txns/s" % (d["value"] / 1e6),
          "roofline frac %.3f" % d["roofline"]["frac"], "cpu", (d["cpu_baseline"] or {}).get("value"),
          d.get("boundary_inclusive"))
    print("   ", {k: round(v, 3) for k, v in d["stage_ms"].items() if v})
PY
