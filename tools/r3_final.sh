#!/bin/bash
# Round-3 record on one box: GPU suite, smoke, the driver's bench line (--steps 20) and the
# default one, per-config bench + rocprofv3 kernel stats + PMC passes (tools/c45_profile.sh),
# c4 phase stamps, the c3 policy-in-the-loop rollout + PPO update.  Any GPU failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20.log 2>&1 || { tail -5 gpurun_out/bench_k20.log; exit 1; }
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
for f in bench_k20 bench_default; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4e'%d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/$f.log $f
done
CONFIGS="${CONFIGS:-c2 c4 c5}" bash tools/c45_profile.sh || exit 1
if [ -f primal-ppo_amd/lib/libmapf_stamps.so ]; then
  MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so CFG=c4 timeout -k 10 120 python3 tools/stamps_wide.py > gpurun_out/stamps_c4.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/stamps_c4.log | tail -10
fi
timeout -k 10 600 python3 tools/bench_rollout.py --envs 4096 --agents 8 --size 20 --steps 16 --train > gpurun_out/rollout_c3.log 2>&1 || { tail -5 gpurun_out/rollout_c3.log; exit 1; }
grep phase gpurun_out/rollout_c3.log | cut -c1-200
