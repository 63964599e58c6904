# kernel trace of one bench config: TAG=... CFG=3 bash scripts/gpu_prof_cfg.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 300 python bench.py --config ${CFG:-3} --steps 3 --warmup 1 --no-cpu > "$O/bench_c${CFG:-3}.json" 2> "$O/bench.err" || { echo bench failed; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --config ${CFG:-3} --steps 2 --warmup 1 --no-cpu > "$O/prof.log" 2>&1 || { echo prof failed; exit 1; }
cd "$R"; python3 - "$O" <<'PY'
import csv, sys, json
d = json.loads([l for l in open(sys.argv[1] + "/bench_c" + __import__("os").environ.get("CFG", "3") + ".json") if l.startswith("{")][-1])
print("ms/step", round(d["ms_per_step"], 3), {k: round(v, 3) for k, v in d["stage_ms"].items() if v})
rows = list(csv.DictReader(open(sys.argv[1] + "/prof/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f'{float(r["TotalDurationNs"])/1e6/ int(r["Calls"]) * 1e3:9.1f} us x{r["Calls"]:>4}  {r["Name"][:90]}')
PY
