#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/profile_update.py --updates 10 > gpurun_out/r5m_update_profile.txt 2>&1; rc=$?; head -5 gpurun_out/r5m_update_profile.txt; exit $rc
