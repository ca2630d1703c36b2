#!/bin/bash
# round 5, third GPU pass: distributed update test, replay-hazard bisection, FETCH_SIZE calibration
# of the BFS-window reads, c5 bench after the VGPR cut, c3 rollout timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r5c_$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-4} "gpurun_out/r5c_$name.log"
  echo "== $name rc=$rc"
  [ $rc -le 1 ] && return 0
  return $rc
}
run pytest_dist 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_distributed_update.py &&
TAILN=8 run diag7 600 python -u tools/diag_graph7.py &&
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
   -d $ROOT/gpurun_out/r5c_fetch -o run -- $ROOT/tools/fetch_calib > $ROOT/gpurun_out/r5c_fetch.log 2>&1); echo "fetch rc=$?" &&
tail -2 gpurun_out/r5c_fetch.log &&
run bench_c5 300 python -u bench.py --config c5 --steps 64 --warmup 8 --no-cpu --no-paths &&
run rollout_c3 600 python -u tools/bench_rollout.py --envs 4096 --agents 8 --size 20 --steps 16 --train
