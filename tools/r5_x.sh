#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_linear.py tests/test_gpu_policy.py tests/test_gpu_update_graph.py tests/test_gpu_ppo_loss.py tests/test_gpu_distributed_update.py > gpurun_out/r5x_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5x_pytest.log | cut -c1-300; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r5x_pytest.log | head -20 | cut -c1-300; exit $rc; }
timeout -k 10 300 python -u tools/profile_update.py --updates 10 > gpurun_out/r5x_update_profile.txt 2>&1 && sed -n 5,5p gpurun_out/r5x_update_profile.txt
