# Fill-kernel ablation (dev aid): config-2 bench per ACCORD_KD_MODE (results invalid for mode != 0).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-kdmodes}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
for m in ${MODES:-0 1 2 3 4}; do export ACCORD_KD_MINW=${MINW:-8};
  ACCORD_KD_MODE=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > "$O/bench_$m.json" 2> "$O/bench_$m.err" || { echo "mode $m failed"; tail -3 "$O/bench_$m.err"; }
  echo "mode=$m $(grep -o '"fill": [0-9.]*' "$O/bench_$m.json")"
done
