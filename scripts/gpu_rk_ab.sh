# config 3: rangekeys grid cap (ACCORD_RK_BLOCKS) A/B after the range parity tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=r04_rk1 ENV_A="ACCORD_RK_BLOCKS=4096" ENV_B="ACCORD_RK_BLOCKS=16384" FILES="tests/test_gpu_ranges.py" BENCH_ARGS="--config 3" bash scripts/gpu_env_ab.sh && \
TAG=r04_rk2 ENV_A="ACCORD_RK_BLOCKS=4096" ENV_B="ACCORD_RK_BLOCKS=65536" BENCH_ARGS="--config 3" bash scripts/gpu_env_ab.sh
