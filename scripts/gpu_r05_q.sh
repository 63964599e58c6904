# Round 5, call q: readiness per-call timeline (kernel trace of the --ready leg, small sample) + the leg's numbers
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_q}"; mkdir -p "$O"
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --ready --ready-batches 4 > "$O/ready.json" 2> "$O/ready.err" || { tail -20 "$O/ready.err"; exit 1; }
python3 -c "import json;d=json.loads([l for l in open('$O/ready.json') if l.startswith('{')][-1]);r=d['readiness'];print({k:r[k] for k in r if 'ms' in k or 'calls' in k})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$O/kt" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --ready --ready-batches 2 > "$O/kt.log" 2>&1 || { tail -20 "$O/kt.log"; exit 1; }
ls "$O/kt"
