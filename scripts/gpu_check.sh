# Round check: GPU tests, default bench line, --resident and --registered legs, then (AB=1) an A/B
# of the measurement builds cassandra-accord_amd/libaccord_deps_v*.so.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-check}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${FILES:-tests} > "$O/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${CPU:---no-cpu} > "$O/bench.json" 2> "$O/bench.err" && \
{ [ -z "$AB" ] || TAG=$TAG bash scripts/ab_libs.sh; } && \
{ [ -z "$LEGS" ] || { timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --resident > "$O/bench_resident.json" 2> "$O/bench_resident.err" && \
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --registered --ready > "$O/bench_registered.json" 2> "$O/bench_registered.err"; }; }
rc=$?; echo "rc=$rc"; tail -3 "$O/pytest_gpu.log"; exit $rc
