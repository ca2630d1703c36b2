#!/bin/bash
# Last record of round 3 (after the c2 in-place priority change): GPU suite, smoke, the driver's
# bench line and the default one, c2 rocprofv3 kernel stats + PMC passes, c4 / c5 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final3.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_final3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1 || { tail -5 gpurun_out/smoke3.log; exit 1; }
tail -1 gpurun_out/smoke3.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench3_k20.log 2>&1 || { tail -5 gpurun_out/bench3_k20.log; exit 1; }
timeout -k 10 400 python3 bench.py > gpurun_out/bench3_default.log 2>&1 || { tail -5 gpurun_out/bench3_default.log; exit 1; }
for f in bench3_k20 bench3_default; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4e'%d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], (d.get('cpu_baseline') or {}).get('value'), {k: (v['ms_per_step'], v['frac']) for k, v in d.get('paths', {}).items()})" gpurun_out/$f.log $f
done
CONFIGS="c2" bash tools/c45_profile.sh || exit 1
NO_PROF=1 CONFIGS="c4 c5" bash tools/c45_profile.sh || exit 1
