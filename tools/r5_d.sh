#!/bin/bash
# round 5, fourth GPU pass: foreach-metadata hypothesis for the replay hazard; distributed test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r5d_$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-4} "gpurun_out/r5d_$name.log"
  echo "== $name rc=$rc"
  [ $rc -le 1 ] && return 0
  return $rc
}
TAILN=14 run diag8 300 python -u tools/diag_graph8.py &&
run pytest_dist 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_distributed_update.py
