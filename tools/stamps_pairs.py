"""Per-wave timing of the pair-lane rollout kernel (c2) from the MAPF_STAMPS build: each env
wave's start / end and its CU, SIMD and wave slot -- does the launch wait for some waves?

    make -C primal-ppo_amd/csrc stamps
    MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so python tools/stamps_pairs.py"""
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

cfg = os.environ.get("CFG", "c2")
T = int(os.environ.get("T", "256"))
slots = int(os.environ.get("SLOTS", "0"))
p = bench.PRESETS[cfg]
B, N, H, F, C = p["envs"], p["agents"], p["size"], p["fov"], p["channels"]
world, shared = bench.make_maps(p["maps"], B, H, H, 0)
env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                 goal_mode="random", fix_choice=1, seed=1234, shared_map=shared), tuning=os.environ.get("TUNE", ""))
env.reset_seeded(world)
assert env.rollout_kernel == 1, "not a pair-lane rollout config"
kw = {}
if slots:
    dev = env.device
    kw = dict(slots=True, actions=torch.zeros(T, B, N, dtype=torch.int32, device=dev),
              obs=torch.empty(T, B, N, C, F, F, device=dev), vec=torch.empty(T, B, N, 4, device=dev),
              out={k: torch.empty((T,) + tuple(v.shape), dtype=v.dtype, device=dev) for k, v in env.out.items()})
env.rollout_random(T, **kw)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
env.rollout_random(T, **kw)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b)
r = env.wave_profile(32768 + B)[32768:].astype(np.uint64)
assert (r[:, 7] == 1).all(), "no stamps: MAPF_LIB is not the stamps build"
st, en = r[:, 4].astype(np.float64), r[:, 5].astype(np.float64)
hw = r[:, 6]
xcc = (hw >> np.uint64(32)).astype(np.int64)
h = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
slot, simd = h & 15, (h >> 4) & 3
cukey = ((xcc * 8 + ((h >> 13) & 7)) * 2 + ((h >> 12) & 1)) * 16 + ((h >> 8) & 15)
dur = (en - st) / 100.0 / T            # us per step, each wave's own loop
print(f"{cfg}{' slots' if slots else ''}: launch {ms * 1e3 / T:.2f} us/step; per-wave loop us/step mean "
      f"{dur.mean():.2f} p50 {np.median(dur):.2f} p99 {np.percentile(dur, 99):.2f} max {dur.max():.2f}")
xs = sorted(set(xcc.tolist()))
print(" per XCD mean/max: " + "  ".join(f"{x}:{dur[xcc == x].mean():.2f}/{dur[xcc == x].max():.2f}" for x in xs))
print(" per XCD wall us/step: " + "  ".join(
    f"{x}:{(en[xcc == x].max() - st[xcc == x].min()) / 100.0 / T:.2f}" for x in xs))
print(" per wave slot: " + "  ".join(f"{k}:{dur[slot == k].mean():.2f}({(slot == k).sum()})" for k in range(16)
                                    if (slot == k).any()))
print(" per SIMD: " + "  ".join(f"{k}:{dur[simd == k].mean():.2f}" for k in range(4)))
u, inv, cnt = np.unique(cukey, return_inverse=True, return_counts=True)
cu_mean = np.bincount(inv, dur) / cnt
cu_max = np.array([dur[inv == k].max() for k in range(len(u))])
print(f" {len(u)} CUs, waves per CU {sorted(set(cnt.tolist()))}; per-CU mean min {cu_mean.min():.2f} p50 "
      f"{np.median(cu_mean):.2f} max {cu_mean.max():.2f}; per-CU max wave p50 {np.median(cu_max):.2f} max {cu_max.max():.2f}")
# start skew within an XCD (its counters agree)
sk = np.concatenate([(st[xcc == x] - st[xcc == x].min()) / 100.0 for x in xs])
print(f" start skew within XCD us: mean {sk.mean():.2f} max {sk.max():.2f}")
