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
                                 goal_mode="random", fix_choice=1, seed=1234, shared_map=shared), tuning=os.environ.get("TUNE", ""))
env.reset_seeded(world)
assert env.rollout_kernel == 2, "not a wide-kernel config"
env.rollout_random(16)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
env.rollout_random(T)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b)
tl = env.timeline(min(3 * B, 8192)).astype(np.float64)
assert (tl[:B, 7] == 1).all(), "no stamps: MAPF_LIB is not the stamps build"
names = ["step", "bfs + snapshot", "human path", "observe"]
print(f"{cfg}: launch {ms * 1e3 / T:.2f} us/step (stamps build)")
# rows B.. hold the observing waves of the pipelined form (2B..: the second observer of the
# three-wave form)
for who, rows in (("first wave (steps)", tl[:B]), ("observing wave", tl[B:2 * B][tl[B:2 * B, 7] == 1]),
                  ("second observing wave", tl[2 * B:3 * B][tl[2 * B:3 * B, 7] == 1])):
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

# where the slow envs are: each wave's start / end on the realtime counter and its CU
# (slot 6 = HW_ID | XCC_ID << 32), grouped by XCD and by CU
raw = env.timeline(min(3 * B, 8192))
rows_all = [("first wave", np.arange(B))]
if (raw[B:2 * B, 7] == 1).any():
    rows_all.append(("observing wave", np.arange(B, 2 * B)))
if len(raw) >= 3 * B and (raw[2 * B:3 * B, 7] == 1).any():
    rows_all.append(("second observing wave", np.arange(2 * B, 3 * B)))
t0 = raw[:3 * B][raw[:3 * B, 7] == 1, 4].min()
for who, idx in rows_all:
    r = raw[idx]
    ok = r[:, 7] == 1
    r, idx = r[ok], idx[ok]
    st = (r[:, 4] - t0) / 100.0
    en = (r[:, 5] - t0) / 100.0
    hw = r[:, 6].astype(np.uint64)
    xcc = (hw >> np.uint64(32)).astype(np.int64)
    h = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
    simd = (h >> 4) & 3
    cu = (h >> 8) & 15
    sh = (h >> 12) & 1
    se = (h >> 13) & 7
    cukey = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    tot = (r[:, :4].sum(1)) / 100.0 / T
    print(f" {who}: start us mean {st.mean():.2f} max {st.max():.2f}; end us mean {en.mean():.1f} "
          f"p50 {np.percentile(en, 50):.1f} p99 {np.percentile(en, 99):.1f} max {en.max():.1f}")
    xs = sorted(set(xcc.tolist()))
    print("  per XCD: " + "  ".join(f"{x}:{tot[xcc == x].mean():.2f}/{tot[xcc == x].max():.2f}" for x in xs))
    # the realtime counters of different XCDs are not aligned: wall per XCD from its own first start
    print("  per XCD wall us/step: " + "  ".join(
        f"{x}:{(r[xcc == x, 5].max() - r[xcc == x, 4].min()) / 100.0 / T:.2f}" for x in xs))
    print("  per SIMD: " + "  ".join(f"{k}:{tot[simd == k].mean():.2f}" for k in range(4) if (simd == k).any()))
    u, inv, cnt = np.unique(cukey, return_inverse=True, return_counts=True)
    cu_mean = np.bincount(inv, tot) / cnt
    print(f"  {len(u)} CUs, waves per CU {np.bincount(cnt).nonzero()[0].tolist()}; per-CU mean total "
          f"min {cu_mean.min():.2f} p50 {np.median(cu_mean):.2f} max {cu_mean.max():.2f}; "
          f"within-CU spread mean {np.mean([tot[inv == k].max() - tot[inv == k].min() for k in range(len(u))]):.2f}")
    wslot = h & 15
    print("  per wave slot: " + "  ".join(f"{k}:{tot[wslot == k].mean():.2f}({(wslot == k).sum()})"
                                          for k in range(16) if (wslot == k).any()))
    # dispatch order within the CU (workgroup id; with the XCD remap env b runs as
    # workgroup (b % (B/8)) * 8 + b // (B/8))
    bb = idx % B
    wg = (bb % (B // 8)) * 8 + bb // (B // 8) if B % 8 == 0 else bb
    rank = np.zeros(len(tot), np.int64)
    for k in range(len(u)):
        m = np.nonzero(inv == k)[0]
        rank[m[np.argsort(wg[m])]] = np.arange(len(m))
    print("  by dispatch rank in CU: " + "  ".join(f"{k}:{tot[rank == k].mean():.2f}" for k in range(rank.max() + 1)))
    print("  XCD x wave slot: " + "  ".join(
        f"{x}/{k}:{tot[(xcc == x) & (wslot == k)].mean():.2f}({((xcc == x) & (wslot == k)).sum()})"
        for x in xs for k in range(4) if ((xcc == x) & (wslot == k)).any()))
    print("  XCD x rank: " + "  ".join(
        f"{x}/{k}:{tot[(xcc == x) & (rank == k)].mean():.2f}" for x in xs for k in range(rank.max() + 1)))
    slow = np.argsort(tot)[-8:]
    print("  slowest: " + "  ".join(f"b{idx[k] % B}:{tot[k]:.2f}(x{xcc[k]} cu{cukey[k] % 256} s{simd[k]})" for k in slow))

# SIMD sharing: which roles share each SIMD (two waves per SIMD), and each role's mean total by
# the role of the other wave on its SIMD and by its own wave slot
if len(rows_all) >= 2:
    recs = []
    for role, (who, idx) in enumerate(rows_all):
        r = raw[idx]
        ok = r[:, 7] == 1
        r = r[ok]
        hw = r[:, 6].astype(np.uint64)
        xcc = (hw >> np.uint64(32)).astype(np.int64)
        h = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
        key = ((((xcc * 8 + ((h >> 13) & 7)) * 2 + ((h >> 12) & 1)) * 16 + ((h >> 8) & 15)) * 4 + ((h >> 4) & 3))
        tot = r[:, :4].sum(1) / 100.0 / T
        for q in range(len(r)):
            recs.append((int(key[q]), min(role, 1), int(h[q] & 15), float(tot[q])))
    by = {}
    for k_, role, slot, tt in recs:
        by.setdefault(k_, []).append((role, slot, tt))
    comp = {}
    for k_, lst in by.items():
        for i, (role, slot, tt) in enumerate(lst):
            others = "".join(sorted("SO"[o[0]] for j, o in enumerate(lst) if j != i))
            comp.setdefault(("SO"[role], others, slot), []).append(tt)
    print(" SIMD sharing (own role | other roles on the SIMD | own slot): mean total, count")
    for kk in sorted(comp):
        print(f"  {kk[0]} | {kk[1] or '-':3s} | slot {kk[2]}: {np.mean(comp[kk]):.2f} ({len(comp[kk])})")
