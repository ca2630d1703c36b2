#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_graph_capture_mode.py tests/test_gpu_update_graph.py tests/test_gpu_zcapture.py > gpurun_out/r5i_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r5i_pytest.log | tail -20 | cut -c1-250
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/profile_update.py --no-profile > gpurun_out/r5i_upd.log 2>&1 && tail -4 gpurun_out/r5i_upd.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5i_bench0.log 2>&1 && tail -1 gpurun_out/r5i_bench0.log | cut -c1-400
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 300 python -u bench.py > gpurun_out/r5i_bench1.log 2>&1 && tail -1 gpurun_out/r5i_bench1.log | cut -c1-400
