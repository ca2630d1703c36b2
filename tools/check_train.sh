#!/bin/bash
# The training path's GPU tests and the c3 / c4 rollout + update timings, one gpurun call
# (from the repo root): TAG=x bash tools/check_train.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-train}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_linear.py \
  tests/test_gpu_update_graph.py tests/test_gpu_ppo_loss.py tests/test_gpu_distributed_update.py tests/test_gpu_policy.py \
  > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${T}_pytest.log | head -20 | cut -c1-300; exit $rc; }
timeout -k 10 400 python3 -u tools/bench_rollout.py --train > gpurun_out/${T}_c3.jsonl 2>&1 || exit 1
grep '^{' gpurun_out/${T}_c3.jsonl | cut -c1-160
timeout -k 10 400 python3 -u tools/bench_rollout.py --envs 1024 --agents 16 --size 40 --train > gpurun_out/${T}_c4.jsonl 2>&1 || exit 1
grep '^{' gpurun_out/${T}_c4.jsonl | cut -c1-160
