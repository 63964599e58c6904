# round-4 check: readiness / keydeps GPU tests, A/B of the measurement builds, fill grid sizes, stamps
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04_cv"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_ready.py tests/test_waiting_on_init.py tests/test_registered_schedule.py tests/test_redundant_before.py \
  tests/test_gpu_keydeps.py tests/test_gpu_ranges.py > "$O/pytest_gpu.log" 2>&1; echo "pytest rc=$?"; tail -3 "$O/pytest_gpu.log"
TAG=r04_cv bash scripts/ab_libs.sh
for b in 4096 2048 1024 4096 2048 1024; do
  ACCORD_FK_BLOCKS=$b timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > "$O/blk$b.json" 2>"$O/blk$b.err" || exit 1
  python3 -c "import json;d=json.loads(open('$O/blk$b.json').read().strip().splitlines()[-1]);s=d['stage_ms'];print('blocks $b', round(d['ms_per_step'],4), 'fill', round(s['fill'],4))"
done
ACCORD_LIB=$R/cassandra-accord_amd/libaccord_deps_stamps.so timeout -k 10 120 python3 scripts/fk_stamps.py > "$O/stamps.txt" 2>&1; cat "$O/stamps.txt"
for x in 0 1 0 1; do
  ACCORD_RK_XCD=$x timeout -k 10 120 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu > "$O/c3_xcd$x.json" 2>"$O/c3_xcd$x.err" || exit 1
  python3 -c "import json;d=json.loads(open('$O/c3_xcd$x.json').read().strip().splitlines()[-1]);s=d['stage_ms'];print('c3 rk_xcd $x', round(d['ms_per_step'],4), {k:round(v,3) for k,v in s.items() if v}, d['count_stage_ms'])"
done
