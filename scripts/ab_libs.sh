# A/B timing of measurement builds (libaccord_deps_v*.so): TAG=... bash scripts/ab_libs.sh
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
for f in cassandra-accord_amd/libaccord_deps_v*.so; do
  v=$(basename $f .so)
  ACCORD_LIB=$R/$f timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > "$O/$v.json" 2>"$O/$v.err" || { echo "$v failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$v.json'));print('$v', round(d['stage_ms']['fill'],3), round(d['stage_ms']['total'],3))"
done
