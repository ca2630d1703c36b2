#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_graph19.py > gpurun_out/r5h_diag19.log 2>&1; echo "rc=$?"; tail -8 gpurun_out/r5h_diag19.log | cut -c1-600
