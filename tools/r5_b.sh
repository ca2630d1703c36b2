#!/bin/bash
# round 5, second GPU pass: the new distributed-update / capture-slot tests, the replay-hazard
# diagnosis, the multi-rank bench rehearsal, then the image-resident conv (tests + A/B timing)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r5b_$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/r5b_$name.log"
  echo "== $name rc=$rc"
  # a failed assertion (1) lets the next step run; a crash, abort or time limit stops the script
  [ $rc -le 1 ] && return 0
  return $rc
}
run pytest_dist 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_distributed_update.py &&
run diag6 400 python -u tools/diag_graph6.py churn trace &&
run pytest_conv 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_policy.py -k "conv" &&
run conv_ab 300 python -u tools/bench_conv_impl.py &&
run pytest_lin 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_policy.py -k "linear512" &&
run lin_ab 300 python -u tools/bench_lin_impl.py
