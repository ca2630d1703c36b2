#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_graph17.py > gpurun_out/r5g_diag17.log 2>&1; echo "rc=$?"; tail -7 gpurun_out/r5g_diag17.log | cut -c1-400
