# Round 5, call g: levelling resolver step breakdown (LV_PROF build, finer split)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_g}"; mkdir -p "$O"
for v in cassandra-accord_amd/libaccord_deps_v*.so; do
ACCORD_LV_PROF=1 ACCORD_LIB=$R/$v timeout -k 10 300 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu > "$O/prof.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
echo $v; grep lv_prof "$O/prof.err" | tail -1
python3 -c "import json;d=json.load(open('$O/prof.json'));print(d['stage_ms']['wo_level'])"
done
timeout -k 10 600 python -u scripts/config4_local.py --out "$O/config4_local.json" > "$O/config4.log" 2>&1 || { tail -20 "$O/config4.log"; exit 1; }
tail -1 "$O/config4.log" | cut -c1-600
