#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_policy.py -k "linear512" > gpurun_out/r5j_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5j_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_lin_impl.py --rounds 2 > gpurun_out/r5j_lin.jsonl 2>&1; rc=$?; cat gpurun_out/r5j_lin.jsonl | cut -c1-200; exit $rc
