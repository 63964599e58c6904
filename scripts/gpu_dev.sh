# Dev loop on one MI355X: all GPU tests, config-2 bench line, resident 8-batch kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-dev}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${FILES:-tests} > "$O/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > "$O/bench.json" 2> "$O/bench.err" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof8" -o run --output-format csv -- python3 "$R/scripts/resident_run.py" 8 3 > "$O/prof8.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof1" -o run --output-format csv -- python3 "$R/scripts/resident_run.py" 1 3 > "$O/prof1.log" 2>&1
rc=$?; cd "$R"; echo "rc=$rc"; tail -3 "$O/pytest_gpu.log"; grep rep "$O/prof8.log" "$O/prof1.log"
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'], {k:round(v,3) for k,v in d['stage_ms'].items() if v}, d.get('resident_batches'))"
exit $rc
