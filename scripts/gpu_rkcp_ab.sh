# config 3: checkpoint table by cells (default) vs by positions (ACCORD_RK_CP_CELLS=0), after the range parity tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=r04_rkcp ENV_A="ACCORD_RK_CP_CELLS=0" ENV_B="ACCORD_RK_CP_CELLS=1" FILES="tests/test_gpu_ranges.py tests/test_gpu_resident.py tests/test_gpu_shards.py" BENCH_ARGS="--config 3" bash scripts/gpu_env_ab.sh
