#!/bin/bash
# Issue priority by progress (c2 in place default, slots / c5 candidates): parity of the grouped
# rollouts, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "cu_groups or fair or env_groups or full_size_rollout or c2_full_size" > gpurun_out/pytest_fair.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fair.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="MAPF_ROLL_FAIR=0 MAPF_ROLL_FAIR=4 MAPF_ROLL_FAIR=8" CFGS=c2 ROUNDS=1 BSTEPS=512 bash tools/ab_env.sh || exit 1
VARIANTS="MAPF_ROLL_FAIR=0 MAPF_ROLL_FAIR=2 MAPF_ROLL_FAIR=4" CFGS=c2 ROUNDS=1 BSTEPS=256 BARGS=--slots bash tools/ab_env.sh || exit 1
VARIANTS="MAPF_WIDE_FAIR=0 MAPF_WIDE_FAIR=1 MAPF_WIDE_FAIR=2 MAPF_WIDE_FAIR=4" CFGS=c5 ROUNDS=1 BSTEPS=128 bash tools/ab_env.sh || exit 1
