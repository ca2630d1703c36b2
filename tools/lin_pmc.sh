#!/bin/bash
# Counters of the 512-linear's GEMM core (libmapf_lindbg1.so: plain fp16 store epilogue), GELU form,
# 2-stage ring, 128- and 64-row workgroups: L2 hit rate, TA busy, SQ waits / MFMA busy.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; ROOT=$(pwd); OUT=$ROOT/gpurun_out/${TAG:-r05l}; mkdir -p $OUT
export MAPF_LIB=$ROOT/primal-ppo_amd/lib/libmapf_lindbg${DBG:-1}.so
pass() {
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
     -d $OUT/$name -o run -- python3 $ROOT/tools/bench_lin_impl.py --iters 2 --rounds 1 --stages 2 --only gelu_dropout) \
     > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; return $rc
}
pass tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit 1
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE || exit 1
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE || echo "(tcp pass failed)"
pass ta TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE || echo "(ta pass failed)"
python3 tools/sq_table.py $OUT/tcc $OUT/sq $OUT/tcp $OUT/ta --match linear512_kernel > $OUT/table.txt; cat $OUT/table.txt
