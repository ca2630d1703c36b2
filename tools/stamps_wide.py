"""Phase breakdown of rollout_wide_kernel from the MAPF_STAMPS diagnostic build.

    make -C primal-ppo_amd/csrc stamps
    MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so CFG=c4 python tools/stamps_wide.py

Per env: s_memtime cycles (100 MHz) of each phase summed over one launch of T steps;
prints the mean per step over envs.  Phases: step, BFS maps, observe staging, observe
emit (bit-stream + float4 stores issued), human path search."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]
os.environ.setdefault("MAPF_LIB", os.path.join(ROOT, "primal-ppo_amd", "lib", "libmapf_stamps.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mapf_amd.config import make_config  # noqa: E402
from mapf_amd.env import BatchedMapfGym  # noqa: E402

cfg = os.environ.get("CFG", "c4")
T = int(os.environ.get("T", "128"))
p = bench.PRESETS[cfg]
B, N, H, F, C = p["envs"], p["agents"], p["size"], p["fov"], p["channels"]
world, shared = bench.make_maps(p["maps"], B, H, H, 0)
env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                 goal_mode="random", fix_choice=1, seed=1234, shared_map=shared))
env.reset_seeded(world)
assert env.rollout_kernel == 2, "not a wide-kernel config"
env.rollout_random(16)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
env.rollout_random(T)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b)
tl = env.timeline(min(2 * B, 8192)).astype(np.float64)
assert (tl[:B, 7] == 1).all(), "no stamps: MAPF_LIB is not the stamps build"
names = ["step", "bfs + snapshot", "human path", "observe"]
print(f"{cfg}: launch {ms * 1e3 / T:.2f} us/step (stamps build)")
# rows B.. hold the observing waves of the pipelined form
for who, rows in (("first wave (steps)", tl[:B]), ("observing wave", tl[B:2 * B][tl[B:2 * B, 7] == 1])):
    if not len(rows):
        continue
    us = rows[:, :4] / 100.0 / T          # s_memrealtime ticks at 100 MHz -> us per step
    print(f" {who}: per-env phase us/step, mean / p99 over envs:")
    for k, nm in enumerate(names):
        print(f"  {nm:14s} {us[:, k].mean():7.2f} {np.percentile(us[:, k], 99):7.2f}")
    print(f"  {'total':14s} {us.sum(1).mean():7.2f} {np.percentile(us.sum(1), 99):7.2f}")

# step_group's own phases (STAMP 0-6, shader-clock cycles) of the LAST step of the launch,
# per stepping wave (pipelined form: waves 2b; else b)
wp = env.wave_profile(min(65536, 2 * B)).astype(np.float64)
rows = wp[wp[:, 7] == 1][:, :7]
PHASES = ["loads+masks", "conflicts(j-loop)", "status+reward+outputs", "fixActions", "move+goals", "human",
          "final outputs"]
if len(rows):
    print(f"step_group phases, last step, {len(rows)} stepping waves (cycles): mean / p90")
    for k, nm in enumerate(PHASES):
        print(f"  {nm:24s} {rows[:, k].mean():9.0f} {np.percentile(rows[:, k], 90):9.0f}")
    print(f"  {'total':24s} {rows.sum(1).mean():9.0f}")
