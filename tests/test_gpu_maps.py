"""Obstacle maps generated on the GPU (mapf_reset_generated), against the
oracle's restatement of the same Philox spec and the reference's own warehouses
(g7_warehouses.npz), and the seeded reset / steps on them against the oracle."""
import numpy as np
import pytest
import torch

from golden_io import load
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")


def mk(B, H, W, N=8, shared=False, offset=0, seed=77, C=6, fov=9):
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    return BatchedMapfGym(make_config(B, H, W, num_agents=N, fov=fov, num_channel=C, human_mode="random",
                                      goal_mode="random", fix_choice=1, seed=seed, shared_map=shared,
                                      env_offset=offset))


def test_device_warehouses_are_the_references():
    """MapfGym()'s map per env: a length in WORLD_SIZE = [10, 40] (Philox), generateWarehouse
    of that length at the top-left of the 40 x 60 stack -- bit-exact vs the reference's map of
    that length, and vs the oracle's draw of it."""
    z = load("g7_warehouses")
    B = 620
    env = mk(B, 40, 60, offset=11)
    maps = env.reset_generated("warehouse", 10, 40, epoch=5, seed=99, return_maps=True).cpu().numpy()
    seen = set()
    for b in range(B):
        want, L = O.gen_map(0, 40, 60, 11 + b, epoch=5, seed=99)
        np.testing.assert_array_equal(maps[b], want, err_msg=f"env {b}")
        ref = z[f"L{L}"]
        np.testing.assert_array_equal(maps[b][:ref.shape[0], :ref.shape[1]], ref)
        seen.add(L)
    assert len(seen) == 31
    # the reset on them: agents and humans on each env's own warehouse, steps run clean
    for _ in range(20):
        env.step_random()
        env.observe()
    st = env.get_state()
    for b in range(B):
        assert (maps[b][st["pos"][b][:, 0], st["pos"][b][:, 1]] == 0).all()
    assert not env.counters()[:8].any()


def test_device_random_maps_largest_component():
    """c5's maps on the device: -(rand < 0.3) over 80 x 80, then only the largest 4-connected
    free component kept -- bit-exact vs the oracle's map through maps.keep_largest_component
    (scipy.ndimage labels); then the seeded reset and 30 steps bit-exact vs the oracle."""
    from mapf_amd.maps import keep_largest_component
    B, N, H, W = 64, 16, 80, 80
    env = mk(B, H, W, N=N, offset=3, seed=1234, C=7, fov=11)
    maps = env.reset_generated("random", density=0.3, largest=True, epoch=2, return_maps=True).cpu().numpy()
    cfg = O.make_config(H, W, N, 11, 7, human_mode=1, goal_mode=1, fix_choice=1, seed=1234)
    oracles = []
    for b in range(B):
        raw, _ = O.gen_map(1, H, W, 3 + b, epoch=2, seed=1234, density=0.3)
        want = keep_largest_component(raw)
        np.testing.assert_array_equal(maps[b], want, err_msg=f"env {b}")
        oe = O.OracleEnv(cfg, env_id=3 + b)
        oe.reset_random(want)
        oracles.append(oe)
    for t in range(30):
        acts = env.random_actions()
        a = acts.cpu().numpy()
        out = {k: v.cpu().numpy() for k, v in env.step(acts).items()}
        obs = env.observe()[0]
        for b in range(0, B, 7):
            r = oracles[b].step(a[b])
            np.testing.assert_array_equal(out["status"][b], r["status"], err_msg=f"t={t} b={b}")
            np.testing.assert_array_equal(out["actions_fixed"][b], r["fixed"], err_msg=f"t={t} b={b}")
            if t % 10 == 9:
                np.testing.assert_array_equal(obs[b].cpu().numpy(), oracles[b].observe()[0])
        for b in range(B):
            if b % 7:
                oracles[b].step(a[b])


def test_uploaded_maps_build_the_same_bitmaps():
    """mapf_reset (host maps, bitmaps built on the device) and mapf_reset_generated give the
    same env: identical observations after the same steps."""
    B, H, W = 32, 40, 60
    gen = mk(B, H, W, seed=5)
    maps = gen.reset_generated("warehouse", 10, 40, epoch=1, return_maps=True)
    up = mk(B, H, W, seed=5)
    up.reset_seeded(maps.cpu().numpy())
    for _ in range(10):
        for e in (gen, up):
            e.step_random()
            e.observe()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gen.obs.cpu().numpy(), up.obs.cpu().numpy())


def test_device_runner_with_device_maps():
    """DeviceRunner(new_maps=DeviceMaps()): a fresh device-generated MapfGym() per rollout."""
    from mapf_amd.model import Model
    from mapf_amd.runner import DeviceMaps, DeviceRunner
    B, N, T = 16, 8, 4
    env = mk(B, 40, 60, N=N)
    model = Model(0, "cuda", global_model=False, numChannel=6, num_agents=N, fov=9)
    runner = DeviceRunner(env, model, n_steps=T, seed=2, new_maps=DeviceMaps())
    firsts = []
    for r in range(2):
        mb, _ = runner.run()
        firsts.append(mb.observations[::T].cpu().numpy())
    assert not np.array_equal(firsts[0], firsts[1])
    assert not env.counters()[:8].any()
