#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_graph20.py > gpurun_out/r5h_diag20.log 2>&1; echo "rc=$?"; tail -9 gpurun_out/r5h_diag20.log | cut -c1-300
echo "== DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python -u tools/diag_graph20.py > gpurun_out/r5h_diag20b.log 2>&1; echo "rc=$?"; tail -9 gpurun_out/r5h_diag20b.log | cut -c1-300
