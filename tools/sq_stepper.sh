#!/bin/bash
# SQ counters of the c4 wide rollout kernel with the observation switched off (stamps build,
# TUNE=diag_exp=1): what the stepping wave's instructions are and where its cycles go.
#   bash tools/sq_stepper.sh   (on the GPU box; writes gpurun_out/sq_stepper_*)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export CFG=${CFG:-c4} TUNE=${TUNE:-diag_exp=1}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
    -d "$OUT/sq_stepper_$i" -o run -- python3 "$ROOT/tools/stamps_wide.py") > "$OUT/sq_stepper_$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
