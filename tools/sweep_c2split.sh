set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for oe in 1 2 4 8; do
  MAPF_OBS_ENVS=$oe timeout -k 10 120 python3 bench.py --no-cpu --steps 300 --warmup 20 --path split > gpurun_out/sw.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sw.log') if l.startswith('{')][-1]); print('c2 split obs_envs', sys.argv[1], d['breakdown_ms']['split'])" $oe
done
timeout -k 10 120 python3 bench.py --no-cpu --config c4 --steps 300 --warmup 20 > gpurun_out/c4_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/c4_bench.log | cut -c1-300
