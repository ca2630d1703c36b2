#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/diag_graph12.py > gpurun_out/r5e_diag12.log 2>&1; echo "rc=$?"; tail -32 gpurun_out/r5e_diag12.log
