#!/bin/bash
# PC sampling of one rollout config (rocprofv3, beta): which instructions the waves sit on.
#   CFG=c4 METHOD=stochastic UNIT=cycles INTERVAL=1048576 bash tools/pc_sample.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 -L) > "$OUT/rocprof_list.log" 2>&1
grep -i -A12 "pc.sampl" "$OUT/rocprof_list.log" | head -40
rm -rf "$OUT/pcs_${CFG:-c4}"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} \
  --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${INTERVAL:-1048576} --output-format csv -d "$OUT/pcs_${CFG:-c4}" -o run \
  -- python3 "$ROOT/bench.py" --config ${CFG:-c4} --no-cpu --no-paths --steps 256 --warmup 8) > "$OUT/pcs_${CFG:-c4}.log" 2>&1
rc=$?; echo "pc sampling rc=$rc"; tail -5 "$OUT/pcs_${CFG:-c4}.log"; find "$OUT/pcs_${CFG:-c4}" -type f | head
exit $rc
