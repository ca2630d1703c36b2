#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_policy.py -k "linear512" > gpurun_out/r5l_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5l_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_lin_impl.py --rounds 1 --only gelu_dropout,rows_x17,tokens > gpurun_out/r5l_lin.jsonl 2>&1 || exit 1
MAPF_LIB=$PWD/primal-ppo_amd/lib/libmapf_lindbg1.so timeout -k 10 300 python -u tools/bench_lin_impl.py --rounds 1 --only gelu_dropout > gpurun_out/r5l_lin_dbg1.jsonl 2>&1 || exit 1
grep -h '^{' gpurun_out/r5l_lin.jsonl gpurun_out/r5l_lin_dbg1.jsonl | cut -c1-200
