# A/B of library variants on the config-5 levelling time (dev aid): LIBS="a.so b.so" (in cassandra-accord_amd/).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-abc5}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
for v in default $LIBS; do
  if [ $v != default ]; then export ACCORD_LIB="$R/cassandra-accord_amd/$v"; fi
  timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu > "$O/bench_$v.json" 2> "$O/bench_$v.err" || { echo "$v failed"; tail -3 "$O/bench_$v.err"; exit 1; }
  echo "$v $(grep -o '"wo_level": [0-9.]*' "$O/bench_$v.json")"
done
