# round-4 check: readiness / keydeps / ranges GPU tests, A/B of the measurement builds (configs 2, 3),
# fill grid sizes, sizes-kernel and rangekeys XCD-order A/Bs, fill stamps, kernel traces of configs 2, 3
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04_cv"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_ready.py tests/test_waiting_on_init.py tests/test_redundant_before.py \
  tests/test_gpu_keydeps.py tests/test_gpu_ranges.py > "$O/pytest_gpu.log" 2>&1; echo "pytest rc=$?"; tail -3 "$O/pytest_gpu.log"
TAG=r04_cv bash scripts/ab_libs.sh
TAG=r04_cv3 BENCH_ARGS="--config 3 --steps 5 --warmup 2" bash scripts/ab_libs.sh
for b in 4096 2048 1024; do
  ACCORD_FK_BLOCKS=$b timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > "$O/blk$b.json" 2>"$O/blk$b.err" || exit 1
  python3 -c "import json;d=json.loads(open('$O/blk$b.json').read().strip().splitlines()[-1]);s=d['stage_ms'];print('blocks $b', round(d['ms_per_step'],4), 'fill', round(s['fill'],4))"
done
for v in "ACCORD_SIZES_TXN=1" "ACCORD_X=0"; do
  env $v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > "$O/sz.json" 2>"$O/sz.err" || exit 1
  python3 -c "import json;d=json.loads(open('$O/sz.json').read().strip().splitlines()[-1]);s=d['stage_ms'];print('$v', round(d['ms_per_step'],4), d['count_stage_ms'])"
done
for x in 0 1; do
  ACCORD_RK_XCD=$x timeout -k 10 120 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu > "$O/c3_xcd$x.json" 2>"$O/c3_xcd$x.err" || exit 1
  python3 -c "import json;d=json.loads(open('$O/c3_xcd$x.json').read().strip().splitlines()[-1]);s=d['stage_ms'];print('c3 rk_xcd $x', round(d['ms_per_step'],4), d['count_stage_ms'])"
done
ACCORD_LIB=$R/cassandra-accord_amd/libaccord_deps_stamps.so timeout -k 10 120 python3 scripts/fk_stamps.py > "$O/stamps.txt" 2>&1; cat "$O/stamps.txt"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 3 --warmup 1 --no-cpu > "$O/prof_c3.log" 2>&1; echo "prof c3 rc=$?"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$O/prof_c2.log" 2>&1; echo "prof c2 rc=$?"
