# GPU tests (FILES, default all) then an A/B of the measurement builds: TAG=... BENCH_ARGS=... bash scripts/gpu_ab.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${FILES:-tests} > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
fi
TAG=$TAG bash scripts/ab_libs.sh
