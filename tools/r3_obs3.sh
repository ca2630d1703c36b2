#!/bin/bash
# Three waves per env (c4: a stepper and two observers taking alternate steps): the wide
# rollout's parity tests, an interleaved A/B against one observer, c4 stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "rollout_random_matches or wide or full_size_rollout" > gpurun_out/pytest_obs3.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_obs3.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="MAPF_WIDE_OBS=1 MAPF_WIDE_BFSOBS=0 MAPF_WIDE_BFSOBS=1" CFGS=c4 BSTEPS=512 bash tools/ab_env.sh || exit 1
VARIANTS="MAPF_WIDE_BFSOBS=0 MAPF_WIDE_BFSOBS=1" CFGS=c4 ROUNDS=1 BSTEPS=256 BARGS=--slots bash tools/ab_env.sh || exit 1
MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so CFG=c4 T=256 timeout -k 10 150 python3 tools/stamps_wide.py > gpurun_out/stamps_c4_obs3.log 2>&1 || { tail -5 gpurun_out/stamps_c4_obs3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_c4_obs3.log | head -24
