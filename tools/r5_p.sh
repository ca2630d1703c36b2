#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_policy.py -k "attention" tests/test_gpu_update_graph.py > gpurun_out/r5p_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5p_pytest.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/profile_update.py --updates 10 > gpurun_out/r5p_update_profile.txt 2>&1 && sed -n 2,5p gpurun_out/r5p_update_profile.txt && grep attention_bwd gpurun_out/r5p_update_profile.txt | cut -c1-60,150-260
