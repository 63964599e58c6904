# A/B timing of measurement builds (libaccord_deps_v*.so), two interleaved rounds:
#   TAG=... BENCH_ARGS="--config 2" bash scripts/ab_libs.sh
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
for round in 1 2; do
for f in cassandra-accord_amd/libaccord_deps_v*.so; do
  v=$(basename $f .so)
  ACCORD_LIB=$R/$f timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS} > "$O/$v.$round.json" 2>"$O/$v.$round.err" || { echo "$v failed"; tail -5 "$O/$v.$round.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$v.$round.json'));s=d['stage_ms'];print('$v', d['ms_per_step'], {k:round(x,3) for k,x in s.items() if x}, [(r['batches'], round(r['device_ratio'], 3), round(r['device_ms'], 3)) for r in d.get('resident_batches') or []])"
done
done
