set -u
VARIANTS="MAPF_WIDE_EPW=1 MAPF_WIDE_PAIR=1+MAPF_WIDE_SLACK=-1 MAPF_WIDE_PAIR=1+MAPF_WIDE_SLACK=16 MAPF_WIDE_PAIR=1+MAPF_WIDE_SLACK=-1+MAPF_WIDE_PRIO=0 MAPF_WIDE_PAIR=0+MAPF_WIDE_SLACK=-1" CFGS=c4 BSTEPS=256 bash tools/ab_env.sh || exit 1
VARIANTS="MAPF_WIDE_SLACK=1 MAPF_WIDE_SLACK=2 MAPF_WIDE_SLACK=4 MAPF_WIDE_SLACK=8" CFGS=c5 BSTEPS=256 bash tools/ab_env.sh || exit 1
for v in "MAPF_WIDE_EPW=1" "MAPF_WIDE_PAIR=1 MAPF_WIDE_SLACK=-1"; do
  env $v MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so CFG=c4 timeout -k 10 150 python3 tools/stamps_wide.py > gpurun_out/stamps_epw2_c4.log 2>&1 || exit 1
  echo "== $v"; grep -A12 "SIMD sharing" gpurun_out/stamps_epw2_c4.log; grep -h "by dispatch\|launch" gpurun_out/stamps_epw2_c4.log
done
