# Round 5, call ab: direct (register-resident) single-pass scan (v1) vs LDS-staged (v0), config 2;
# GPU suite with v1 (the default build)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_ab}"; mkdir -p "$O"
TAG=r05_ab BENCH_ARGS="--config 2" bash scripts/ab_libs.sh || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$O/prof_trace.log" 2>&1 || exit 1
