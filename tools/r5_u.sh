#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python3 -c "
import sys; sys.path.insert(0, 'primal-ppo_amd')
import torch
from mapf_amd.gemm_tuning import use_tuned_gemms
print('tuned gemms in use:', use_tuned_gemms(), torch.cuda.tunable.is_enabled(), torch.cuda.tunable.tuning_is_enabled())"
timeout -k 10 400 python3 -u tools/bench_rollout.py --train > gpurun_out/r5u_c3.jsonl 2>&1 || exit 1
grep '^{' gpurun_out/r5u_c3.jsonl | cut -c1-200
timeout -k 10 400 python3 -u tools/bench_rollout.py --envs 1024 --agents 16 --size 40 --train > gpurun_out/r5u_c4.jsonl 2>&1 || exit 1
grep '^{' gpurun_out/r5u_c4.jsonl | cut -c1-200
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_linear.py tests/test_gpu_policy.py tests/test_gpu_update_graph.py tests/test_gpu_ppo_loss.py tests/test_gpu_distributed_update.py tests/test_gpu_rollout.py > gpurun_out/r5u_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5u_pytest.log | cut -c1-300; exit $rc
