#!/bin/bash
# Rollout-path timing of diagnostic builds: one bench line per library in LIBS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${LIBS:-libmapf}; do
  MAPF_LIB=primal-ppo_amd/lib/$lib.so timeout -k 10 100 python3 bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/diag.log 2>&1 || { tail -5 gpurun_out/diag.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/diag.log').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('%-22s %.3e  rollout %.2f us/step  per-step launch %.2f us' % (sys.argv[1], d['value'], 1e3*(b['rollout_per_step'] or 0), 1e3*b['step_observe_launch']))" $lib
done
