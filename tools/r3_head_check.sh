#!/bin/bash
# HEAD check on one box: the GPU suite, then the default bench line and c4 / c5 / c2-slots
# lines (no profiles).  Any GPU failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_head.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_head.log; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4e'%d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (v['ms_per_step'], v['frac']) for k, v in d.get('paths', {}).items()})" "$1" "$2"; }
timeout -k 10 400 python3 bench.py > gpurun_out/bench_head_default.log 2>&1 || { tail -5 gpurun_out/bench_head_default.log; exit 1; }
line gpurun_out/bench_head_default.log default
for c in c4 c5; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu > gpurun_out/bench_head_$c.log 2>&1 || { tail -5 gpurun_out/bench_head_$c.log; exit 1; }
  line gpurun_out/bench_head_$c.log $c
done
