# Round 5, final measurement: GPU suite, bench lines (config 2 with the CPU baseline, registered +
# readiness, resident, config 3, config 5), kernel statistics of config 2 / 3 and the registered leg
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_final4}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python bench.py > "$O/bench_config2.json" 2> "$O/bench_config2.err" || exit 1
python3 -c "import json;d=json.load(open('$O/bench_config2.json'));print('config2', round(d['ms_per_step'],4), d['roofline']['frac'])"
timeout -k 10 300 python bench.py --registered --ready --steps 3 --warmup 1 --no-cpu > "$O/bench_config2_registered.json" 2> "$O/bench_config2_registered.err" || exit 1
timeout -k 10 300 python bench.py --resident --steps 3 --warmup 1 --no-cpu > "$O/bench_config2_resident.json" 2> "$O/bench_config2_resident.err" || exit 1
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu > "$O/bench_config3.json" 2> "$O/bench_config3.err" || exit 1
python3 -c "import json;d=json.load(open('$O/bench_config3.json'));print('config3', round(d['ms_per_step'],4))"
timeout -k 10 400 python bench.py --config 5 --steps 3 --warmup 1 > "$O/bench_config5.json" 2> "$O/bench_config5.err" || exit 1
python3 -c "import json;d=json.load(open('$O/bench_config5.json'));print('config5', round(d['ms_per_step'],4))"
timeout -k 10 300 python scripts/ready_latency.py > "$O/ready_lat.json" 2> "$O/ready_lat.err" || exit 1
timeout -k 10 300 python scripts/ready_latency.py --registered --batches 64 --batch 1024 > "$O/reg_lat.json" 2> "$O/reg_lat.err" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/k2" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu > "$O/k2.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/k3" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 5 --warmup 2 --no-cpu > "$O/k3.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kreg" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --registered --batches 32 --batch 1024 > "$O/kreg.log" 2>&1 || exit 1
echo done
