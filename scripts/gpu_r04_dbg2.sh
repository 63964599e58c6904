set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04_dbg2"; mkdir -p "$O"
timeout -k 10 300 python3 -u scripts/dbg_eal.py > "$O/dbg.txt" 2>&1; echo "dbg rc=$?"; grep -B3 -A3 "MISMATCH" "$O/dbg.txt" | head; grep -c trace "$O/dbg.txt"
bash scripts/gpu_r04_trace.sh
