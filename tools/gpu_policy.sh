#!/bin/bash
# Policy-forward profile on the gpurun box (tools/profile_policy.py), output in gpurun_out/pp.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/profile_policy.py ${POLICY_ARGS:-} > gpurun_out/pp.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/pp.log | cut -c1-220 | head -45
exit $rc
