#!/bin/bash
# GPU validation pass, run on the gpurun box from the repo root:
#   smoke -> GPU parity tests -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault, abort, segfault or time
# limit ends the script (no further GPU work in this call).  A plain test
# failure (pytest rc 1) still lets the bench and the profile run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1

stop_if_fatal() {   # $1 = rc, $2 = step name
  case "$1" in
    0|1) return 0 ;;
    *) echo "FATAL: $2 exited with $1 -- stopping GPU work"; exit "$1" ;;
  esac
}

STEPS="${STEPS:-smoke pytest bench prof}"
for s in $STEPS; do
  case "$s" in
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; stop_if_fatal $rc smoke ;;
    pytest)
      timeout -k 10 1000 python3 -m pytest ${PYTEST_ARGS:-tests} -m gpu -q > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"; stop_if_fatal $rc pytest ;;
    bench)
      timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
      rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.log"; stop_if_fatal $rc bench ;;
    sweep)
      for cfg in ${SWEEP:-"search_blocks=32" "search_blocks=64" "search_blocks=128"}; do
        timeout -k 10 200 python3 bench.py --no-cpu --steps 2000 --path split --tune "$cfg" > "$OUT/sweep.log" 2>&1
        rc=$?; echo "sweep $cfg rc=$rc $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['breakdown_ms'])" "$OUT/sweep.log" 2>/dev/null)"
        stop_if_fatal $rc sweep
      done ;;
    stamps)
      timeout -k 10 200 python3 tools/stamps.py > "$OUT/stamps.log" 2>&1
      rc=$?; echo "stamps rc=$rc"; cat "$OUT/stamps.log" | grep -v amdgpu.ids; stop_if_fatal $rc stamps ;;
    timeline)
      timeout -k 10 200 python3 tools/timeline.py > "$OUT/timeline.log" 2>&1
      rc=$?; echo "timeline rc=$rc"; grep -v amdgpu.ids "$OUT/timeline.log"; stop_if_fatal $rc timeline ;;
    rollout)
      timeout -k 10 600 python3 tools/bench_rollout.py --train ${ROLLOUT_ARGS:-} > "$OUT/rollout.log" 2>&1
      rc=$?; echo "rollout rc=$rc"; grep phase "$OUT/rollout.log"; tail -2 "$OUT/rollout.log"; stop_if_fatal $rc rollout ;;
    pmc)
      for ctr in WRITE_SIZE FETCH_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
          -d "$OUT/pmc_$ctr" -o run -- python3 "$ROOT/bench.py" --steps 64 --warmup 10 --no-cpu --graph-steps 0 \
          --rollout-steps 32 --kernel-launches 4 ${PMC_ARGS:-}) > "$OUT/pmc_$ctr.log" 2>&1
        rc=$?; echo "pmc $ctr rc=$rc"; stop_if_fatal $rc pmc
      done
      find "$OUT" -path "*pmc_*" -name "*.csv" | head ;;
    sq)   # instruction mix of every kernel (SQ counters), one pass per counter group
      i=0
      for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH" ${SQ_EXTRA:-}; do
        i=$((i+1))
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
          -d "$OUT/sq_$i" -o run -- python3 "$ROOT/bench.py" --steps 64 --warmup 10 --no-cpu --graph-steps 0 \
          --rollout-steps 32 --kernel-launches 4) > "$OUT/sq_$i.log" 2>&1
        rc=$?; echo "sq $i ($grp) rc=$rc"; stop_if_fatal $rc sq
      done ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --no-cpu ${PROF_ARGS:-}) > "$OUT/prof.log" 2>&1
      rc=$?; echo "prof rc=$rc"; tail -3 "$OUT/prof.log"; stop_if_fatal $rc prof
      find "$OUT/prof" -name "*stats*" | head ;;
  esac
done
