#!/bin/bash
# CU-group pair rollout: parity, per-wave stamps, then A/B in place and slots (c2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "cu_groups or rollout_random_matches or full_size_rollout" > gpurun_out/pytest_group.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_group.log; [ $rc -eq 0 ] || exit $rc
for v in MAPF_ROLL_GROUP=0 MAPF_ROLL_GROUP=1; do for s in 0 1; do
  env $v SLOTS=$s MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so timeout -k 10 150 python3 tools/stamps_pairs.py > gpurun_out/stamps_pairs.log 2>&1 || { tail -5 gpurun_out/stamps_pairs.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/stamps_pairs.log
done; done
VARIANTS="MAPF_ROLL_GROUP=0 MAPF_ROLL_SLACK=1 MAPF_ROLL_SLACK=2 MAPF_ROLL_SLACK=4 MAPF_ROLL_SLACK=-1" CFGS=c2 BSTEPS=256 bash tools/ab_env.sh || exit 1
VARIANTS="MAPF_ROLL_GROUP=0 MAPF_ROLL_SLACK=1 MAPF_ROLL_SLACK=4" CFGS=c2 BSTEPS=256 BARGS=--slots bash tools/ab_env.sh || exit 1
