# Levelling resolve-pass stamps (dev aid): config-5 bench with ACCORD_LV_DEBUG, then analysis,
# for each ACCORD_LV_WAVES in $WAVES.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-lvdbg}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
for nw in ${WAVES:-8}; do
  ACCORD_LV_WAVES=$nw ACCORD_LV_DEBUG="$O/stamps$nw.bin" timeout -k 10 300 python bench.py --config 5 --steps 1 --warmup 0 --no-cpu > "$O/bench_c5_$nw.json" 2> "$O/bench_c5.err" || exit 1
  echo "waves=$nw"; python scripts/lv_stamps.py "$O/stamps$nw.bin" || exit 1
  ACCORD_LV_WAVES=$nw timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu > "$O/bench_c5_$nw.json" 2> "$O/bench_c5.err" || exit 1
  grep -o '"wo_level": [0-9.]*' "$O/bench_c5_$nw.json"
done
