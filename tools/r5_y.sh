#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tune3
cp primal-ppo_amd/mapf_amd/tunableop_gfx950.csv gpurun_out/tune3/res0.csv
cp primal-ppo_amd/mapf_amd/tunableop_gfx950.csv gpurun_out/tune3/res.csv
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tune3/res.csv
for a in "--fp16-partials" "" "--fp16-partials --split 8" "--split 8"; do
  timeout -k 10 300 python3 -u tools/profile_update.py --no-profile $a > gpurun_out/tune3/upd.log 2>&1 || exit 1
  echo "$a: $(tail -1 gpurun_out/tune3/upd.log)"
done
