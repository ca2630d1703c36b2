#!/bin/bash
# A/B of library builds on ONE box, interleaved: per-step time of the roofline kernel per config.
#   LIBS="libmapf.so libmapf_argptr.so" CFGS="c2 c4" bash tools/ab_libs.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in ${ROUNDS:-1 2}; do
  for c in ${CFGS:-c2 c4}; do
    for lib in ${LIBS:-libmapf.so libmapf_argptr.so}; do
      MAPF_LIB=primal-ppo_amd/lib/$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-paths --steps ${BSTEPS:-512} \
        --warmup 16 ${BARGS:-} > gpurun_out/ablib.log 2>&1 || { rc=$?; tail -5 gpurun_out/ablib.log; exit $rc; }
      python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ablib.log').read().strip().splitlines()[-1]); b=d['breakdown_ms']
print(sys.argv[1], sys.argv[2], sys.argv[3], 'per_step_us %.3f'%(b['rollout_per_step']*1e3), 'frac', d['roofline']['frac'], 'value %.4g'%d['value'], 'ctr', d['device_counters'][:3])" $round $c $lib
    done
  done
done
