set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in c1 c4 c5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 300 --warmup 20 --cpu-seconds 8 > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed rc=$?"; tail -20 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log
done
timeout -k 10 600 python3 tools/bench_rollout.py --envs 4096 --agents 8 --size 20 --steps 16 --train > gpurun_out/rollout_c3.log 2>&1 || { echo "rollout failed"; tail -20 gpurun_out/rollout_c3.log; exit 1; }
grep phase gpurun_out/rollout_c3.log
