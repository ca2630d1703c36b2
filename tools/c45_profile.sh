#!/bin/bash
# c4 / c5 measurement on the gpurun box, from the repo root:
#   bench line -> rocprofv3 kernel stats -> WRITE_SIZE and FETCH_SIZE passes (one counter
#   per pass) of the rollout kernel, for each config in $CONFIGS.
# Every GPU step has its own limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for c in ${CONFIGS:-c5 c4}; do
  timeout -k 10 200 python3 bench.py --no-cpu --config $c --steps ${STEPS:-1024} --warmup 20 ${BENCH_ARGS:-} > "$OUT/bench_$c.log" 2>&1 \
    || { echo "bench $c rc=$?"; tail -20 "$OUT/bench_$c.log"; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], '%.3e'%d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['device_counters'], {k: (v['ms_per_step'], v['frac']) for k, v in d.get('paths', {}).items()})" "$OUT/bench_$c.log" $c
  [ -n "${NO_PROF:-}" ] && continue
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_$c" -o run -- python3 "$ROOT/bench.py" --no-cpu --no-paths --config $c --steps 512 --warmup 10) \
    > "$OUT/prof_$c.log" 2>&1 || { echo "prof $c rc=$?"; tail -20 "$OUT/prof_$c.log"; exit 1; }
  for ctr in WRITE_SIZE FETCH_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d "$OUT/pmc_${c}_$ctr" -o run -- python3 "$ROOT/bench.py" --no-cpu --no-paths --config $c --steps 64 \
      --warmup 5 --rollout-steps 32 --kernel-launches 4) \
      > "$OUT/pmc_${c}_$ctr.log" 2>&1 || { echo "pmc $c $ctr rc=$?"; tail -20 "$OUT/pmc_${c}_$ctr.log"; exit 1; }
  done
  echo "$c done"
done
