set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$R/gpurun_out/prof_trace.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/prof_fetch" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu > "$R/gpurun_out/prof_fetch.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/prof_write" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu > "$R/gpurun_out/prof_write.log" 2>&1
echo "rc=$?"
