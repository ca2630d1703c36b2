#!/bin/bash
# conv experiment builds (primal-ppo_amd/lib/convx/*.so) timed side by side; PMC=<lib.so> adds an SQ
# counter pass (wait / issue / LDS / MFMA cycles) over that build
cd "${GRAFT_REPO_ROOT:-/root/repo}"; ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; L=primal-ppo_amd/lib/convx
timeout -k 10 300 python3 tools/bench_conv.py $L/*.so > $OUT/${TAG:-r04j}_conv.log 2>&1 || exit 1
grep "{" $OUT/${TAG:-r04j}_conv.log
[ -z "$PMC" ] || (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/${TAG:-r04j}_pmc -o run -- python3 $ROOT/tools/bench_conv.py $ROOT/$L/$PMC --iters 2 --agents 8192) > $OUT/${TAG:-r04j}_pmc.log 2>&1
