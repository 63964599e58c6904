# Round 5, call l: 4-wave resolver ablations (solo, no exchange, no fetch) and 2 / 1 resolver waves
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_l}"; mkdir -p "$O"
true

for v in cassandra-accord_amd/libaccord_deps_v*.so; do
ACCORD_LV_PROF=1 ACCORD_LIB=$R/$v timeout -k 10 300 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu > "$O/prof.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
echo $v; grep lv_prof "$O/prof.err" | tail -1
python3 -c "import json;d=json.load(open('$O/prof.json'));print(d['stage_ms']['wo_level'])"
done
timeout -k 10 300 python -u scripts/rank_sim.py 8 1 > "$O/rank1.log" 2>&1 || { tail -5 "$O/rank1.log"; exit 1; }
tail -3 "$O/rank1.log"
