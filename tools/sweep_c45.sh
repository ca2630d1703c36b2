set -u
cd "$GRAFT_REPO_ROOT"
run() {  # $1 = label, rest = command
  local lab=$1; shift
  "$@" > gpurun_out/sw.log 2>&1 || { echo "$lab FAILED rc=$?"; tail -3 gpurun_out/sw.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sw.log') if l.startswith('{')][-1]); b=d['breakdown_ms']; print(sys.argv[1], '%.3e'%d['value'], d['ms_per_step'], b['split'], d['roofline']['frac'])" "$lab"
}
B="timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 --path split"
for oe in 1 2 4 8; do run "c4 obs_envs=$oe" $B --config c4 --tune obs_envs=$oe; done
for oe in 1 2; do run "c5 obs_envs=$oe" $B --config c5 --tune obs_envs=$oe; done
for sb in 32 128 256; do run "c5 search_blocks=$sb" $B --config c5 --tune search_blocks=$sb; done
for sb in 32 128; do run "c4 search_blocks=$sb" $B --config c4 --tune search_blocks=$sb; done
