"""GPU: makeBfsMap (mapf_gym.py:211-244) on every row type of the device search, against
the oracle's BFS (oracle/mapf_oracle.c: oc_bfs_map), bit-exact.

The device keeps a BFS map's distances as bit planes in registers and decodes them
straight into the 8x8 tiles; maps deeper than the planes hold (serpentine mazes, distances
past 511 on u64 / two-u64 rows) take the LDS-image path.  Both are covered here, on u32
rows (W <= 32), u64 rows (W <= 64), two-u64 rows (W <= 128), one and two rows per lane
(H above 64), ragged tile edges (H, W not multiples of 8) and goals on every kind of cell.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")


def serpentine(H, W):
    """Walls on every other row, one gap alternating between the ends: one corridor of ~H*W/2 cells."""
    w = np.zeros((H, W), np.int8)
    for r in range(1, H, 2):
        w[r, :] = -1
        w[r, W - 1 if (r // 2) % 2 == 0 else 0] = 0
    return w


def random_map(H, W, p, seed):
    rng = np.random.default_rng(seed)
    return -(rng.random((H, W)) < p).astype(np.int8)


CASES = {
    "u32_20x20_rand": (lambda: random_map(20, 20, 0.25, 1)),
    "u32_19x27_serp": (lambda: serpentine(19, 27)),
    "u64_40x40_rand": (lambda: random_map(40, 40, 0.25, 2)),
    "u64_40x40_serp": (lambda: serpentine(40, 40)),       # distances past 511: the LDS-image path
    "u64_37x45_serp": (lambda: serpentine(37, 45)),
    "u64_70x50_rand": (lambda: random_map(70, 50, 0.2, 3)),
    "u64_70x50_serp": (lambda: serpentine(70, 50)),
    "row2_80x80_rand": (lambda: random_map(80, 80, 0.3, 4)),
    "row2_80x80_serp": (lambda: serpentine(80, 80)),
    "row2_30x100_rand": (lambda: random_map(30, 100, 0.2, 5)),
    "row2_30x100_serp": (lambda: serpentine(30, 100)),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_bfs_maps_match_oracle(name):
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    world = CASES[name]()
    H, W = world.shape
    free = np.argwhere(world == 0)
    rng = np.random.default_rng(sum(name.encode()))
    # goals: corners of the free region, the far end of a corridor, random free cells
    goals = [free[0], free[-1], free[len(free) // 2]] + [free[k] for k in rng.choice(len(free), 9, replace=False)]
    B = len(goals)
    env = BatchedMapfGym(make_config(B, H, W, num_agents=1, fov=3, num_channel=5, human_mode="looping",
                                     goal_mode="sequence", fix_choice=0, max_seq=2))
    starts = [free[1] if not np.array_equal(free[1], g) else free[2] for g in goals]
    env.reset_fixed(world, [[[s, g]] for s, g in zip(starts, goals)], [free[3]] * B, [free[4]] * B)
    bfs = env.bfs().cpu().numpy()
    deep = 0
    for b, g in enumerate(goals):
        want = O.bfs_map(world, g)
        deep += int(want.max() >= 512)
        np.testing.assert_array_equal(bfs[b, 0], want, err_msg=f"{name}: goal {tuple(g)}")
    if "serp" in name and H * W >= 1600:
        assert deep > 0, "no case reached the LDS-image path"
    env.close()
