# Round 5, call d: fill-path tests with the header kernel, A/B v0 (HEAD fill) vs v1 (kd_header_kernel), vmem micro-benchmark
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_d}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_keydeps.py tests/test_gpu_ranges.py tests/test_gpu_accept.py tests/test_gpu_status_events.py tests/test_gpu_resident.py tests/test_gpu_big_txns.py tests/test_gpu_shards.py > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
TAG=${TAG:-r05_d} bash scripts/ab_libs.sh || exit 1
hipcc --offload-arch=gfx950 -O3 -o /tmp/vmem_patterns scripts/micro/vmem_patterns.hip && timeout -k 10 120 /tmp/vmem_patterns > "$O/vmem_patterns.txt" 2>&1; cat "$O/vmem_patterns.txt"
hipcc --offload-arch=gfx950 -O3 -o /tmp/lv_product scripts/micro/lv_product.hip 2>/dev/null && timeout -k 10 60 /tmp/lv_product > "$O/lv_product.txt" 2>&1; cat "$O/lv_product.txt"
