#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5t
for m in default rocblas tunable; do
  TUNE_DIR=$PWD/gpurun_out/r5t timeout -k 10 400 python -u tools/bench_gemm_backends.py --mode $m > gpurun_out/r5t/$m.jsonl 2>&1 || { tail -5 gpurun_out/r5t/$m.jsonl; exit 1; }
  grep '^{' gpurun_out/r5t/$m.jsonl
done
