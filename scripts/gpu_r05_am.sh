# Round 5, call am: one-workgroup batch sort micro-benchmark (phase stamps)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_am}"; mkdir -p "$O"
hipcc --offload-arch=gfx950 -O3 -I cassandra-accord_amd/csrc scripts/micro/batch_sort.hip -o /tmp/batch_sort 2>/dev/null && timeout -k 10 60 /tmp/batch_sort > "$O/batch_sort.txt" 2>&1; cat "$O/batch_sort.txt"
