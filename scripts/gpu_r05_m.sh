# Round 5, call m: packed-verdict fill (v1) vs HEAD (v0) on config 2; config-4 one-GPU record; fill-path GPU tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_m}"; mkdir -p "$O"
TAG=r05_m BENCH_ARGS="--config 2" bash scripts/ab_libs.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_keydeps.py tests/test_gpu_big_txns.py tests/test_gpu_exchange.py > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 600 python -u scripts/config4_local.py --out "$O/config4_local.json" > "$O/config4.log" 2>&1 || { tail -20 "$O/config4.log"; exit 1; }
tail -1 "$O/config4.log" | cut -c1-300
