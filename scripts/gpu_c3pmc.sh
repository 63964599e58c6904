# One PMC pass over the config-3 pipeline (instruction mix / LDS behaviour per kernel).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-c3pmc}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD} -d "$O/pmc" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 1 --warmup 0 --no-cpu > "$O/pmc.log" 2>&1
rc=$?
python3 - "$O/pmc/run_counter_collection.csv" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "rangekeys" in r["Kernel_Name"]:
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print(k, {a: "%.3g" % b for a, b in v.items()})
PY
exit $rc
