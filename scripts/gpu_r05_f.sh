# Round 5, call f: levelling resolver cycle breakdown (LV_PROF build) + kernel trace of config 5
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_f}"; mkdir -p "$O"
ACCORD_LV_PROF=1 ACCORD_LIB=$R/cassandra-accord_amd/libaccord_deps_vprof.so timeout -k 10 300 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu > "$O/prof.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
grep lv_prof "$O/prof.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o c5 -- python3 "$R/bench.py" --config 5 --steps 2 --warmup 1 --no-cpu > "$O/kt.log" 2>&1 || { tail -20 "$O/kt.log"; exit 1; }
f=$(ls "$O"/kt/*/c5_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find "$O/kt" -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3),'ms')"
