#!/bin/bash
# WRITE_SIZE / FETCH_SIZE passes (one rocprofv3 --pmc run per counter, kernel-trace only) of the
# rollout kernels, 32-step launches:  PASSES="c2 c2inplace c4 c5" bash tools/pmc_passes.sh
# -> gpurun_out/pmc_<pass>_<COUNTER>/ ; tools/pmc_report.py turns them into profiles/*.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
# (bench.py's default rollout writes [T]-slot buffers; the *inplace passes re-write [B] buffers)
for p in ${PASSES:-c2 c2inplace c4 c4inplace c5 c5inplace}; do
  case "$p" in
    *inplace) args="--config ${p%inplace} --inplace" ;;
    *) args="--config $p" ;;
  esac
  for ctr in WRITE_SIZE FETCH_SIZE; do
    rm -rf "$OUT/pmc_${p}_$ctr"
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d "$OUT/pmc_${p}_$ctr" -o run -- python3 "$ROOT/bench.py" $args --steps 64 --warmup 4 --no-cpu --no-paths \
      --rollout-steps 32 --kernel-launches 4) > "$OUT/pmc_${p}_$ctr.log" 2>&1
    rc=$?; echo "pmc $p $ctr rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_${p}_$ctr.log"; exit $rc; }
  done
done
