#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run per group) of bench.py's fused
# launch, for each library given in LIBS (default: the product build and the
# no-step diagnostic build), then a table per library (tools/pmc_table.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
LIBS="${LIBS:-libmapf libmapf_nostep}"
GROUPS_1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH"
GROUPS_2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS"
for lib in $LIBS; do
  i=0
  dirs=""
  for grp in "$GROUPS_1" "$GROUPS_2"; do
    i=$((i+1))
    d="$OUT/sq_${lib}_$i"
    (cd /tmp && export TMPDIR=/tmp && MAPF_LIB="$ROOT/primal-ppo_amd/lib/$lib.so" timeout -s KILL 120 rocprofv3 --pmc $grp \
      --kernel-trace --output-format csv -d "$d" -o run -- python3 "$ROOT/bench.py" --steps 64 --warmup 10 --no-cpu \
      --graph-steps 0 --rollout-steps 32 --kernel-launches 4 ${BENCH_ARGS:-}) > "$OUT/sq_${lib}_$i.log" 2>&1
    rc=$?; echo "sq $lib $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/sq_${lib}_$i.log"; exit $rc; fi
    dirs="$dirs $d"
  done
  python3 tools/pmc_table.py $dirs --kernel ${KERNEL:-rollout_random_kernel}
done
