# segment-stage probe (ACCORD_H2_COMB) and compaction block size (ACCORD_CV_OUT) A/Bs on config 2,
# after the parity tests of the default build
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=r04_h2 ENV_A="ACCORD_H2_COMB=0" ENV_B="ACCORD_H2_COMB=1" FILES="tests/test_gpu_keydeps.py tests/test_gpu_resident.py tests/test_gpu_accept.py" bash scripts/gpu_env_ab.sh && \
TAG=r04_cv1 ENV_A="ACCORD_CV_OUT=4096" ENV_B="ACCORD_CV_OUT=8192" bash scripts/gpu_env_ab.sh && \
TAG=r04_cv2 ENV_A="ACCORD_CV_OUT=4096" ENV_B="ACCORD_CV_OUT=2048" bash scripts/gpu_env_ab.sh
