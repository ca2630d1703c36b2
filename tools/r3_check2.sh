#!/bin/bash
# After the CU-group change: whole GPU suite, c2 slot-path PMC passes, slot-buffer A/B of the
# wide kernel's env groups (c4 pipelined, c5), bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_check2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_check2.log; [ $rc -eq 0 ] || exit $rc
PASSES="c2slots" bash tools/r3_pmc.sh || exit 1
VARIANTS="MAPF_WIDE_EPW=1 MAPF_WIDE_EPW=4" CFGS=c4 BSTEPS=256 BARGS=--slots bash tools/ab_env.sh || exit 1
VARIANTS="MAPF_WIDE_EPW=1 MAPF_WIDE_EPW=8" CFGS=c5 ROUNDS=1 BSTEPS=128 BARGS=--slots bash tools/ab_env.sh || exit 1
for c in c2 c4 c5; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu > gpurun_out/bench_check2_$c.log 2>&1 || { tail -5 gpurun_out/bench_check2_$c.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4e'%d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v for k, v in d.get('breakdown_ms', {}).items() if 'slot' in k or 'per_step' in k})" gpurun_out/bench_check2_$c.log $c
done
