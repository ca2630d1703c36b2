#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tune2
cp primal-ppo_amd/mapf_amd/tunableop_gfx950.csv gpurun_out/tune2/res0.csv
cp primal-ppo_amd/mapf_amd/tunableop_gfx950.csv gpurun_out/tune2/res.csv
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tune2/res.csv
timeout -k 10 300 python3 -u tools/profile_policy.py --unfused-linear --no-profile 2>&1 | grep model.step
timeout -k 10 300 python3 -u tools/profile_policy.py --no-profile 2>&1 | grep model.step
timeout -k 10 300 python3 -u tools/profile_policy.py --unfused-linear --no-profile 2>&1 | grep model.step
ls -la gpurun_out/tune2
