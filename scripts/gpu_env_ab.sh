# GPU tests with an env setting (ENV="A=1"), then bench A/B of two env settings, interleaved:
#   TAG=... ENV_A="X=0" ENV_B="X=1" FILES="tests/..." BENCH_ARGS="..." bash scripts/gpu_env_ab.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
if [ -n "$FILES" ]; then
  env $ENV_B timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $FILES > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
  tail -2 "$O/pytest_gpu.log"
fi
for round in 1 2; do
  for v in A B; do
    eval e=\$ENV_$v
    env $e timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS} > "$O/$v.$round.json" 2>"$O/$v.$round.err" || { echo "$v failed"; tail -5 "$O/$v.$round.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/$v.$round.json').read().strip().splitlines()[-1]);s=d['stage_ms'];print('$v $e', round(d['ms_per_step'],4), {k:round(x,3) for k,x in s.items() if x})"
  done
done
