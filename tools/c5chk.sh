set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in c5 c4; do
  timeout -k 10 120 python3 bench.py --no-cpu --config $c --steps 200 --warmup 20 > gpurun_out/$c.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], '%.3e'%d['value'], d['ms_per_step'], d['breakdown_ms']['split'], d['roofline']['frac'], d['device_counters'])" gpurun_out/$c.log $c
done
