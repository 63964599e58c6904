# Round 5, call r: fast fill kernel segment shares (ACCORD_FK_STAMPS build), config 2
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_r}"; mkdir -p "$O"
ACCORD_LIB=$R/cassandra-accord_amd/libaccord_deps_vstamps.so timeout -k 10 300 python -u scripts/fk_stamps.py > "$O/fk_stamps.txt" 2>&1 || { tail -20 "$O/fk_stamps.txt"; exit 1; }
cat "$O/fk_stamps.txt"
