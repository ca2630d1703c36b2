#!/bin/bash
# Round-3 wide-kernel check on the GPU box: GPU suite (optional), c4/c5 bench lines, c4 stamps.
#   STEPS="pytest bench stamps" bash tools/r3_wide_check.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
summ() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d['roofline']; b=d['breakdown_ms']
print(sys.argv[2], 'value %.4g'%d['value'], 'per_step_us %.3f'%(b['rollout_per_step']*1e3 if b.get('rollout_per_step') else -1), 'frac', r['frac'], 'counters', d['device_counters'], 'paths', {k:v['frac'] for k,v in d.get('paths',{}).items()})
" "$1" "$2"; }
for s in ${STEPS:-pytest bench stamps}; do
  case "$s" in
    pytest)
      timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc ;;
    bench)
      for c in ${CFGS:-c4 c5}; do
        timeout -k 10 300 python3 bench.py --config $c --no-cpu --steps ${BSTEPS:-512} --warmup 16 > gpurun_out/bench_$c.log 2>&1 || { rc=$?; tail -5 gpurun_out/bench_$c.log; exit $rc; }
        summ gpurun_out/bench_$c.log $c
      done ;;
    stamps)
      for c in ${SCFGS:-c4}; do
        MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so CFG=$c timeout -k 10 120 python3 tools/stamps_wide.py > gpurun_out/stamps_$c.log 2>&1 || { rc=$?; tail -5 gpurun_out/stamps_$c.log; exit $rc; }
        grep -v amdgpu.ids gpurun_out/stamps_$c.log
      done ;;
  esac
done
