#!/bin/bash
# After a kernel change, on one box: the whole GPU suite, then bench lines for CFGS and the
# wide-kernel stamps of c5.  Any GPU failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_check.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_check.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-c5 c4 c2}; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu > gpurun_out/bench_check_$c.log 2>&1 || { tail -5 gpurun_out/bench_check_$c.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4e'%d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])" gpurun_out/bench_check_$c.log $c
done
MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so CFG=c5 timeout -k 10 150 python3 tools/stamps_wide.py > gpurun_out/stamps_check_c5.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamps_check_c5.log | grep -v "XCD x"
