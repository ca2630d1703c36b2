#!/bin/bash
# A/B of the PPO minibatch update between this tree and an older one checked out at ./_r01
# (git worktree add _r01 <commit>; built in place), on ONE box, interleaved A B A B, then the
# torch-profiler kernel table of each (tools/profile_update.py).  Writes gpurun_out/ab_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OLD=${OLD:-_r01}
for round in 1 2; do
  for tree in . "$OLD"; do
    tag=$([ "$tree" = . ] && echo head || echo old)
    timeout -k 10 300 python3 "$tree/tools/bench_rollout.py" --envs 4096 --agents 8 --size 20 --steps 16 --train \
      --updates 30 > "gpurun_out/ab_${tag}_${round}.log" 2>&1 || { rc=$?; tail -5 "gpurun_out/ab_${tag}_${round}.log"; exit $rc; }
    echo "$tag $round: $(grep -h 'phase' "gpurun_out/ab_${tag}_${round}.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['phase'][:12], d.get('ms_per_step') or d.get('ms_per_update'), d.get('ms_median',''), end=' | ')")"
  done
done
for tree in . "$OLD"; do
  tag=$([ "$tree" = . ] && echo head || echo old)
  timeout -k 10 300 python3 "$tree/tools/profile_update.py" --updates 10 > "gpurun_out/ab_prof_${tag}.log" 2>&1 || { rc=$?; tail -5 "gpurun_out/ab_prof_${tag}.log"; exit $rc; }
  grep "update:" "gpurun_out/ab_prof_${tag}.log"
done
