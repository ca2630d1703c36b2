#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for d in 0 1 2; do
MAPF_LIN_DEBUG=$d timeout -k 10 200 python -u tools/bench_lin_impl.py --rounds 1 --stages 2 > gpurun_out/r5k_lin$d.jsonl 2>&1 || exit 1
grep '^{' gpurun_out/r5k_lin$d.jsonl | cut -c1-200
done
