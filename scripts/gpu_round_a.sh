# Round check, part A (one MI355X): all GPU tests and the bench lines of configs 2/3/5 and the
# drop-in legs (gpu_round_b.sh: kernel traces and PMC passes)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-round}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$O/bench.json" 2> "$O/bench.err" && \
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 > "$O/bench_c5.json" 2> "$O/bench_c5.err" && \
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu > "$O/bench_c3.json" 2> "$O/bench_c3.err" && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --resident > "$O/bench_resident.json" 2> "$O/bench_resident.err" && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --registered --ready > "$O/bench_registered.json" 2> "$O/bench_registered.err"
rc=$?; echo "rc=$rc"; tail -2 "$O/pytest_gpu.log"; exit $rc
