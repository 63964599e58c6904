R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
for v in vA vB; do
  ACCORD_LIB=$R/cassandra-accord_amd/libaccord_deps_$v.so timeout -k 10 300 python bench.py --ready --ready-events --steps 2 --warmup 1 --no-cpu --ready-cpu-batch 0 > "$O/ev_$v.json" 2> "$O/ev_$v.err" || { echo "$v failed"; tail -5 "$O/ev_$v.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ev_$v.json'));r=d['readiness'];e=r['events_mode'];print('$v poll', round(r['update_ms_per_call'],4), round(r['per_call_ms_update_plus_register'],4), 'events', round(e['update_ms_per_call'],4), round(e['per_call_ms_update_plus_register'],4), round(e['register_stable_ms_per_batch'],3))"
done
