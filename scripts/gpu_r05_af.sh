# Round 5, call af2: cold-key checkpoint walk: v096 (no prefetch, 96) vs vp096 / vp256 (prefetching walk); range tests with vp096 (default)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_af}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ranges.py > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for round in 1 2; do
for f in cassandra-accord_amd/libaccord_deps_v*.so; do
  v=$(basename $f .so)
  ACCORD_LIB=$R/$f timeout -k 10 200 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu > "$O/$v.$round.json" 2>"$O/$v.$round.err" || { echo "$v failed"; tail -5 "$O/$v.$round.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$v.$round.json'));print('$v', round(d['ms_per_step'],4), round(d['count_stage_ms']['rk_checkpoints'],4))"
done
done
