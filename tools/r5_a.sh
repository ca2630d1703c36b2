#!/bin/bash
# round 5, first GPU pass: the new distributed-update / capture-slot tests, the replay-hazard
# diagnosis and the multi-rank bench rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_distributed_update.py tests/test_gpu_update_graph.py tests/test_gpu_zcapture.py \
  > gpurun_out/r5a_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5a_pytest.log; exit 1; }
tail -3 gpurun_out/r5a_pytest.log
timeout -k 10 400 python -u tools/diag_graph5.py base twin_stream rocblas nomiopen > gpurun_out/r5a_diag5.log 2>&1
echo "diag exit $?"
MAPF_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 64 --warmup 8 --no-paths --no-cpu \
  > gpurun_out/r5a_bench_gloo2.log 2>&1
echo "bench exit $?"
tail -2 gpurun_out/r5a_bench_gloo2.log
