#!/bin/bash
# Envs-per-workgroup check on one box: the wide-kernel parity tests, then A/B of the group
# form against one env per workgroup (c4, c5), then stamps of the group form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "wide or full_size_rollout or split_path" > gpurun_out/pytest_epw.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_epw.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="${VARIANTS:-MAPF_WIDE_EPW=1 MAPF_WIDE_SLACK=-1 MAPF_WIDE_SLACK=4 MAPF_WIDE_PAIR=1}" CFGS="${CFGS:-c4 c5}" \
  BSTEPS=256 bash tools/ab_env.sh || exit 1
for c in c4 c5; do
  MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so CFG=$c timeout -k 10 150 python3 tools/stamps_wide.py > gpurun_out/stamps_epw_$c.log 2>&1 || exit 1
  grep -h -A9 "start us" gpurun_out/stamps_epw_$c.log | grep -v slowest; grep launch gpurun_out/stamps_epw_$c.log
done
