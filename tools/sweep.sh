#!/bin/bash
# Env-var sweep of bench.py on the GPU box: each argument is one "VAR=x VAR2=y" setting.
# Prints value + breakdown per setting; stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BARGS="${BENCH_ARGS:---no-cpu --steps 600}"
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python3 bench.py $BARGS > gpurun_out/sweep.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "sweep [$cfg] rc=$rc"; tail -5 gpurun_out/sweep.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '|', d['value'], d['ms_per_step'], d['breakdown_ms'].get('step_observe'), d['breakdown_ms']['split'], d['roofline']['frac'])" gpurun_out/sweep.log "$cfg"
done
