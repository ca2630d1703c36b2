#!/bin/bash
# TunableOp tuning pass for SCRIMPNet's GEMM shapes on the gpurun box (from the repo root): the c3
# rollout + its 256 x 8-row updates, then the c4-shaped rollout + updates, with every GEMM's candidate
# solutions benchmarked on first use; results -> gpurun_out/tune/tunableop_results.csv, to be copied
# to primal-ppo_amd/mapf_amd/tunableop_gfx950.csv (mapf_amd/gemm_tuning.py loads it with tuning off).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tune/tunableop_results.csv
# KEEP=1: start from the shipped results, so only shapes missing from them are benchmarked
# (TunableOp appends the device ordinal to the file name: results0.csv on device 0)
if [ -n "${KEEP:-}" ]; then cp primal-ppo_amd/mapf_amd/tunableop_gfx950.csv "${PYTORCH_TUNABLEOP_FILENAME%.csv}0.csv"; fi
timeout -k 10 500 python3 -u tools/bench_rollout.py --train --updates 4 --update-warmup 3 > gpurun_out/tune/c3.log 2>&1 \
  || { echo "c3 rc=$?"; tail -5 gpurun_out/tune/c3.log; exit 1; }
timeout -k 10 500 python3 -u tools/bench_rollout.py --envs 1024 --agents 16 --size 40 --train --updates 4 --update-warmup 3 \
  > gpurun_out/tune/c4.log 2>&1 || { echo "c4 rc=$?"; tail -5 gpurun_out/tune/c4.log; exit 1; }
[ -n "${KEEP:-}" ] || timeout -k 10 300 python3 -u tools/bench_gemm_backends.py --mode default > gpurun_out/tune/backends.log 2>&1 \
  || exit 1
wc -l gpurun_out/tune/tunableop_results.csv
