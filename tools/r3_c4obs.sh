#!/bin/bash
# c4 observer diagnosis: stamps with the observer's store loop off (EXP=2) and with the
# bit-stream build off (EXP=3), then the store-only ceilings of c4's pattern (1,024 waves,
# one per SIMD, 32 KiB each, in place) against more waves with the same bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for x in 0 2 3; do
  MAPF_WIDE_EXP=$x MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so CFG=c4 T=256 timeout -k 10 150 python3 tools/stamps_wide.py > gpurun_out/stamps_c4_x$x.log 2>&1 || { tail -5 gpurun_out/stamps_c4_x$x.log; exit 1; }
  echo "== EXP=$x"; grep -v amdgpu.ids gpurun_out/stamps_c4_x$x.log | head -16
done
hipcc -O3 --offload-arch=gfx950 tools/store_pattern.hip -o gpurun_out/store_pattern 2> /dev/null || exit 1
for a in "1024 32 256 1 1" "1024 32 256 1 4" "2048 16 256 1 2" "4096 8 256 1 4" "4096 23 256 1 4" "8192 4 256 1 8" "1024 32 64 0 1"; do
  timeout -k 10 60 gpurun_out/store_pattern $a || exit 1
done
