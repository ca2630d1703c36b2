#!/bin/bash
# c4 diagnosis: phase stamps with per-XCD / per-CU / SIMD-sharing spreads at T = 256, and the
# launch length sweep (time = a + b T).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so CFG=c4 T=256 timeout -k 10 150 python3 tools/stamps_wide.py > gpurun_out/stamps_c4.log 2>&1 || { tail -5 gpurun_out/stamps_c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_c4.log
CFG=c4 timeout -k 10 150 python3 tools/launch_len.py > gpurun_out/launch_len_c4.log 2>&1 || { tail -5 gpurun_out/launch_len_c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/launch_len_c4.log
