#!/bin/bash
# SQ counters (MFMA busy, waits, LDS conflicts, clock) of the c3 acting forward's GEMM-shaped kernels:
# the 512-linears (tools/bench_lin_impl.py) and the implicit-GEMM convolutions (tools/bench_conv_impl.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; ROOT=$(pwd); OUT=$ROOT/gpurun_out/${TAG:-r05}_sq; mkdir -p $OUT
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for tool in bench_lin_impl bench_conv_impl; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv \
     -d $OUT/$tool -o run -- python3 $ROOT/tools/$tool.py --iters 2 --rounds 1) > $OUT/$tool.log 2>&1
  rc=$?; echo "$tool rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/sq_table.py $OUT/bench_lin_impl $OUT/bench_conv_impl --match linear512_kernel conv_img_kernel conv_igemm32 \
  > $OUT/table.txt && cat $OUT/table.txt
