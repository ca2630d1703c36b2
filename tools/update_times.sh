#!/bin/bash
# One definition of the PPO update time (tools/bench_rollout.py --train: median of 20 Model.train calls
# through driver.py's call shape) for the one-rank captured update and the distributed form (two graph
# segments around a 1-rank RCCL all-reduce), at the 256 x 8 (c3) and 256 x 16 (c4) minibatch shapes.
#   tools/update_times.sh <tag>   -> gpurun_out/<tag>_update_{c3,c4}{,_dist}.jsonl
set -u
tag=${1:-r06}
mkdir -p gpurun_out
run() {   # name, args...: stop at a fault / abort / time limit (no further GPU step after one)
    local name=$1; shift
    timeout -k 10 240 python -u tools/bench_rollout.py "$@" > gpurun_out/${tag}_update_${name}.jsonl 2> gpurun_out/${tag}_update_${name}.err
    local rc=$?
    echo "update ${name}: rc=${rc}"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
run c3 --envs 4096 --agents 8 --size 20 --fov 9 --steps 16 --train --minibatch 256
run c3_dist --envs 4096 --agents 8 --size 20 --fov 9 --steps 16 --train --minibatch 256 --distributed-path
run c4 --envs 1024 --agents 16 --size 40 --fov 9 --steps 16 --train --minibatch 256
run c4_dist --envs 1024 --agents 16 --size 40 --fov 9 --steps 16 --train --minibatch 256 --distributed-path
