# round-4: wo-init eal debug; levelling stats; resident/registered tests with the merge join; registered trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04_lv2"; mkdir -p "$O"
timeout -k 10 300 python3 -u scripts/dbg_eal.py > "$O/dbg.txt" 2>&1; echo "dbg rc=$?"; grep -m 12 "wo-init-dbg\|MISMATCH" "$O/dbg.txt"
ACCORD_LV_STATS=1 timeout -k 10 200 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu > "$O/c5.json" 2>"$O/c5.err" || { tail -5 "$O/c5.err"; exit 1; }
grep "lv stats" "$O/c5.err" | tail -2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resident.py tests/test_registered_schedule.py tests/test_ready.py tests/test_waiting_on_init.py > "$O/pytest.log" 2>&1; echo "pytest rc=$?"; tail -4 "$O/pytest.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/registered" -o run --output-format csv -- python3 "$R/scripts/reg_trace.py" registered > "$O/registered.log" 2>&1; echo "trace rc=$?"; tail -c 1200 "$O/registered.log"
