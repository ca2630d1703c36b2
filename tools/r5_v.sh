#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for f in none cast ln split cast+ln+split; do timeout -k 10 120 python3 tools/diag_peak.py $f 2>&1 | grep '^{' || exit 1; done
PYTORCH_TUNABLEOP_ENABLED=0 timeout -k 10 120 python3 tools/diag_peak.py cast+ln+split 2>&1 | grep '^{'
