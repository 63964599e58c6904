set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ready.py -k "injection or initialise" > gpurun_out/inj.log 2>&1; echo "inj rc=$?"; tail -2 gpurun_out/inj.log
TAG=r04_rs1 ENV_A="ACCORD_X=0" ENV_B="ACCORD_RS_LOWFIRST=1" FILES="tests/test_gpu_keydeps.py" bash scripts/gpu_env_ab.sh && \
TAG=r04_rs2 ENV_A="ACCORD_X=0" ENV_B="ACCORD_RS_PASSES=3" bash scripts/gpu_env_ab.sh
