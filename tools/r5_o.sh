#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for s in 4 16 8; do
timeout -k 10 300 python -u tools/profile_update.py --no-profile --split $s > gpurun_out/r5o_upd_$s.log 2>&1 || exit 1; echo "split $s: $(tail -1 gpurun_out/r5o_upd_$s.log)"
done
timeout -k 10 300 python -u tools/profile_update.py --updates 10 > gpurun_out/r5o_update_profile.txt 2>&1 || exit 1
