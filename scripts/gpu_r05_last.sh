# Round 5, last check of the committed tree: GPU suite, smoke, default bench line
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_last}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print('config2', round(d['ms_per_step'],4), round(d['value']/1e6,1), d['roofline']['frac'], d['cpu_baseline']['value'])"
