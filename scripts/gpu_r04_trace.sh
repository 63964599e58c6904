# round-4: kernel traces of the drop-in legs (registered, resident, ready)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04_trace"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for leg in registered resident ready; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$leg" -o run --output-format csv -- python3 "$R/scripts/reg_trace.py" $leg > "$O/$leg.log" 2>&1 || { echo "$leg failed"; tail -5 "$O/$leg.log"; exit 1; }
  echo "$leg ok"; tail -c 1500 "$O/$leg.log"
done
