#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_linear.py > gpurun_out/r5r_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5r_pytest.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/profile_update.py --updates 10 > gpurun_out/r5r_update_profile.txt 2>&1 && sed -n 5,5p gpurun_out/r5r_update_profile.txt && grep -E "ln_bwd_colsum|layernorm_bwd" gpurun_out/r5r_update_profile.txt | cut -c1-50,180-300
