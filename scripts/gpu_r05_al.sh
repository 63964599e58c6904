# Round 5, call al: kernel statistics of the registered leg (merge join of resident batches)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_al}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/reg_k" -o run --output-format csv -- python3 "$R/scripts/ready_latency.py" --registered --batches 32 --batch 1024 > "$O/reg_k.log" 2>&1 || exit 1
