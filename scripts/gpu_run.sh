# The one GPU recipe: TAG=<gpurun_out subdir> STEPS="<step> ..." bash scripts/gpu_run.sh
# Every step runs under its own time limit; the first failing step ends the run (no retries).
#   tests          pytest -m gpu (FILES="tests/x.py ..." narrows it)
#   smoke          __graft_entry__.smoke()
#   bench2         python bench.py (config 2, CPU baseline included)         -> bench_config2.json
#   bench3|bench5  config 3 / config 5 lines                                 -> bench_config{3,5}.json
#   registered     bench --registered --ready; resident: bench --resident; events: bench --ready --ready-events
#   seg4           scripts/config4_local.py --check (config 4, per-rank record) -> config4_segments.json
#   rehearse       bench.py --gpus 2 --one-device (the multi-rank code path on one GPU, gloo)
#   prof2|prof3|prof5|prof4  rocprofv3 --kernel-trace --stats of bench config 2 / 3 / 5 / config4_local
#   pmc2           FETCH_SIZE, WRITE_SIZE and request-size passes of config 2 (separate runs) -> traffic_config2.json
#   py:<script args>  any python script under scripts/ (e.g. py:ready_latency.py --registered)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
TAG=${TAG:-run}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
export TMPDIR=/tmp
run() {  # run <seconds> <log> <cmd...>
    local t=$1 log=$2; shift 2
    echo "== $(date +%T) $*" | tee -a "$O/steps.log"
    timeout -k 10 "$t" "$@" > "$O/$log" 2> "$O/$log.err"
    local rc=$?
    echo "   rc=$rc" | tee -a "$O/steps.log"
    if [ $rc -ne 0 ]; then tail -25 "$O/$log" "$O/$log.err"; exit $rc; fi
}
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],4), 'ms/step', d.get('roofline',{}).get('frac'))" "$1"; }
for step in ${STEPS:-tests bench2}; do
  case "$step" in
    tests) run 1500 pytest_gpu.log python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu ${FILES:-tests}
           tail -1 "$O/pytest_gpu.log";;
    smoke) run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()";;
    bench2) run 400 bench_config2.json python bench.py; line "$O/bench_config2.json";;
    bench3) run 300 bench_config3.json python bench.py --config 3 --steps 5 --warmup 2 --no-cpu; line "$O/bench_config3.json";;
    bench5) run 500 bench_config5.json python bench.py --config 5 --steps 3 --warmup 1; line "$O/bench_config5.json";;
    registered) run 400 bench_config2_registered.json python bench.py --registered --ready --steps 3 --warmup 1 --no-cpu;;
    events) run 600 bench_ready_events.json python bench.py --ready --ready-events --steps 3 --warmup 1 --no-cpu;;
    resident) run 300 bench_config2_resident.json python bench.py --resident --steps 3 --warmup 1 --no-cpu;;
    seg4) run 600 config4_segments.json python -u scripts/config4_local.py --check --out "$O/config4_segments.line.json";;
    rehearse) run 400 rehearse_g2.json python bench.py --gpus 2 --one-device --steps 5 --warmup 2 --no-cpu;;
    prof2) (cd /tmp && run 300 k2.log rocprofv3 --kernel-trace --stats -d "$O/k2" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu) || exit 1;;
    prof3) (cd /tmp && run 300 k3.log rocprofv3 --kernel-trace --stats -d "$O/k3" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 5 --warmup 2 --no-cpu) || exit 1;;
    prof5) (cd /tmp && run 500 k5.log rocprofv3 --kernel-trace --stats -d "$O/k5" -o run --output-format csv -- python3 "$R/bench.py" --config 5 --steps 2 --warmup 1 --no-cpu) || exit 1;;
    prof4) (cd /tmp && run 600 k4.log rocprofv3 --kernel-trace --stats -d "$O/k4" -o run --output-format csv -- python3 "$R/scripts/config4_local.py" --reps 3) || exit 1;;
    pmc2) for c in FETCH_SIZE WRITE_SIZE; do
            (cd /tmp && run 120 "pmc_$c.log" timeout -s KILL 100 rocprofv3 --pmc "$c" --kernel-trace -d "$O/pmc_$c" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu) || exit 1
          done
          (cd /tmp && run 120 pmc_RDREQ.log timeout -s KILL 100 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --kernel-trace -d "$O/pmc_RDREQ" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu) || exit 1
          python3 scripts/traffic_json.py "$O/pmc_FETCH_SIZE" "$O/pmc_WRITE_SIZE" "txnrec_kernel,keydeps_fast_kernel<,keydeps_kernel<" "profiles/$TAG" "$O/traffic_config2.json" "$O/pmc_RDREQ" > /dev/null;;
    py:*) a="${step#py:}"; a="${a//,/ }"; run 600 "$(echo "${a%% *}" | tr -c 'a-z0-9_\n' '_').log" python -u scripts/$a;;
    *) echo "unknown step $step"; exit 2;;
  esac
done
echo done
