#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
t() { echo "== $*"; timeout -k 10 200 env "$@" python -u tools/diag_graph14.py bwd > gpurun_out/r5f_ws.log 2>&1; echo "rc=$?"; tail -1 gpurun_out/r5f_ws.log | cut -c1-300; }
t A=1
t HIPBLASLT_WORKSPACE_SIZE=0 CUBLASLT_WORKSPACE_SIZE=0
t HIPBLAS_WORKSPACE_CONFIG=:0:0 CUBLAS_WORKSPACE_CONFIG=:0:0
t HIPBLASLT_WORKSPACE_SIZE=0 CUBLASLT_WORKSPACE_SIZE=0 HIPBLAS_WORKSPACE_CONFIG=:0:0 CUBLAS_WORKSPACE_CONFIG=:0:0
bash tools/gemm_sq.sh 2>&1 | tail -60
