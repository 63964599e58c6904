# Round 5, call z: launch cost of a kernel chain -- direct launches vs stream capture + graph update vs replay
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_z}"; mkdir -p "$O"
for k in 8 32; do timeout -k 10 120 ./scripts/micro/graph_launch $k 300 | tee -a "$O/graph_launch.json" || exit 1; done
