# Round 5, call j: ablations of the resolver step (solo)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_j}"; mkdir -p "$O"
true

for v in cassandra-accord_amd/libaccord_deps_v*.so; do
ACCORD_LV_PROF=1 ACCORD_LIB=$R/$v timeout -k 10 300 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu > "$O/prof.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
echo $v; grep lv_prof "$O/prof.err" | tail -1
python3 -c "import json;d=json.load(open('$O/prof.json'));print(d['stage_ms']['wo_level'])"
done
