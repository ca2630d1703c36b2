#!/bin/bash
# A/B of launch forms (mapf_tuning fields, include/mapf.h) on ONE box, interleaved; each variant is a
# bench.py --tune string ("-" = the defaults):
#   VARIANTS="wide_prio=0 wide_prio=1" CFGS=c4 bash tools/ab_tune.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in ${ROUNDS:-1 2}; do
  for c in ${CFGS:-c4}; do
    for v in ${VARIANTS:-wide_prio=0 wide_prio=1}; do
      t=$v; [ "$t" = "-" ] && t=""
      timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-paths --steps ${BSTEPS:-512} --warmup 16 --tune "$t" ${BARGS:-} \
        > gpurun_out/abtune.log 2>&1 || { rc=$?; tail -5 gpurun_out/abtune.log; exit $rc; }
      python3 -c "
import json,sys
d=json.loads(open('gpurun_out/abtune.log').read().strip().splitlines()[-1]); b=d['breakdown_ms']
print(sys.argv[1], sys.argv[2], sys.argv[3], 'per_step_us %.3f'%(b['rollout_per_step']*1e3), 'frac', d['roofline']['frac'], 'value %.4g'%d['value'])" $round $c "$v"
    done
  done
done
