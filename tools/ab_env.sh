#!/bin/bash
# A/B of environment switches on ONE box, interleaved ('+' joins several in one variant):  VARIANTS="MAPF_WIDE_PRIO=0 MAPF_WIDE_PRIO=1" CFGS=c4 bash tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in ${ROUNDS:-1 2}; do
  for c in ${CFGS:-c4}; do
    for v in ${VARIANTS:-MAPF_WIDE_PRIO=0 MAPF_WIDE_PRIO=1}; do
      env ${v//+/ } timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-paths --steps ${BSTEPS:-512} --warmup 16 ${BARGS:-} \
        > gpurun_out/abenv.log 2>&1 || { rc=$?; tail -5 gpurun_out/abenv.log; exit $rc; }
      python3 -c "
import json,sys
d=json.loads(open('gpurun_out/abenv.log').read().strip().splitlines()[-1]); b=d['breakdown_ms']
print(sys.argv[1], sys.argv[2], sys.argv[3], 'per_step_us %.3f'%(b['rollout_per_step']*1e3), 'frac', d['roofline']['frac'], 'value %.4g'%d['value'])" $round $c "$v"
    done
  done
done
