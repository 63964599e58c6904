# Fill-kernel occupancy sweep (dev aid): config-2 fill ms per ACCORD_KD_MINW.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/${TAG:-kdminw}"; mkdir -p "$O"
for w in ${MINWS:-8 7 6 4}; do
  ACCORD_KD_MINW=$w timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > "$O/bench_$w.json" 2> "$O/bench_$w.err" || { echo "minw $w failed"; exit 1; }
  echo "minw=$w $(grep -o '"fill": [0-9.]*' "$O/bench_$w.json")"
done
