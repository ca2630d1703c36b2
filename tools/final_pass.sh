#!/bin/bash
# One full measurement pass on the gpurun box (from the repo root), logs under gpurun_out/${TAG}_*:
#   GPU parity suite -> smoke -> the driver's bench line (--steps 20) and the default one ->
#   per config (c2 c4 c5): bench line, rocprofv3 kernel stats, WRITE_SIZE / FETCH_SIZE passes
#   (tools/c45_profile.sh); the c3 / c4 rollouts; the c3 kernel breakdown; the PPO update timing.
#   STEPS selects a subset: STEPS="pytest bench" TAG=r04a bash tools/final_pass.sh
# Every GPU step has its own limit and any failure ends the script (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r04}
for st in ${STEPS:-pytest smoke bench profile rollout}; do
  case "$st" in
    pytest)
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v ${PYTEST_ARGS:-} --timeout 300 --timeout-method thread \
        > gpurun_out/${TAG}_pytest_gpu.log 2>&1
      rc=$?; grep -E "passed|failed|error" gpurun_out/${TAG}_pytest_gpu.log | tail -3; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
        || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -1 gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.log 2>&1 \
        || { tail -5 gpurun_out/${TAG}_bench_k20.log; exit 1; }
      timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 \
        || { tail -5 gpurun_out/${TAG}_bench_default.log; exit 1; }
      for f in bench_k20 bench_default; do
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], '%.4e'%d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['traffic'], (d.get('cpu_baseline') or {}).get('value'), {k: (v['ms_per_step'], v['frac']) for k, v in d.get('paths', {}).items()})" gpurun_out/${TAG}_$f.log $f
      done ;;
    profile)
      CONFIGS="${CONFIGS:-c2 c4 c5}" STEPS=${BENCH_STEPS:-1024} bash tools/c45_profile.sh || exit 1 ;;
    rollout)   # c3: policy in the loop (4096 x 8, FOV 9) + PPO updates; c4-shaped updates (1024 x 16, 40x40)
      timeout -k 10 400 python3 tools/bench_rollout.py --train > gpurun_out/${TAG}_rollout_c3.jsonl 2>&1 \
        || { tail -5 gpurun_out/${TAG}_rollout_c3.jsonl; exit 1; }
      grep '^{' gpurun_out/${TAG}_rollout_c3.jsonl | cut -c1-300
      timeout -k 10 400 python3 tools/bench_rollout.py --envs 1024 --agents 16 --size 40 --train \
        > gpurun_out/${TAG}_rollout_c4.jsonl 2>&1 || { tail -5 gpurun_out/${TAG}_rollout_c4.jsonl; exit 1; }
      grep '^{' gpurun_out/${TAG}_rollout_c4.jsonl | cut -c1-300 ;;
    c3prof)    # rocprofv3 kernel trace of the c3 rollout, summarised per acting step (one conv_first launch)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OLDPWD/gpurun_out/${TAG}_c3prof" \
        -o c3 -- python3 "$OLDPWD/tools/bench_rollout.py" --steps 16 > "$OLDPWD/gpurun_out/${TAG}_c3prof.log" 2>&1) \
        || { tail -5 gpurun_out/${TAG}_c3prof.log; exit 1; }
      python3 tools/rocpd_summary.py gpurun_out/${TAG}_c3prof/c3_results.db --per conv_first_kernel --top 45 \
        > gpurun_out/${TAG}_c3_breakdown.txt && head -12 gpurun_out/${TAG}_c3_breakdown.txt | cut -c1-160 ;;
    update)    # the PPO minibatch update, 256 x 8 rows: captured graph vs eager (medians)
      timeout -k 10 300 python3 tools/profile_update.py --no-profile > gpurun_out/${TAG}_update.log 2>&1 \
        || { tail -5 gpurun_out/${TAG}_update.log; exit 1; }
      tail -1 gpurun_out/${TAG}_update.log ;;
  esac
done
