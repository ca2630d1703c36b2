#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_train_linear.py tests/test_gpu_update_graph.py tests/test_gpu_ppo_loss.py tests/test_gpu_distributed_update.py > gpurun_out/r5n_pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|rel diff|passed|failed|Error" gpurun_out/r5n_pytest.log | tail -20 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/profile_update.py --no-profile > gpurun_out/r5n_upd.log 2>&1 && tail -1 gpurun_out/r5n_upd.log
