"""Guard: every rollout-kernel instantiation a BASELINE preset launches by default -- in place
and into slot buffers, at the preset's full per-GPU size, as bench.py runs it -- has been run by
an oracle-compared case of this session (tests/kernel_registry.py).  Runs after
test_gpu_parity.py (file order) and before test_gpu_zcapture.py.

The default form depends on the launch size (nontemporal stores above 128 MB, one workgroup
per CU at four workgroups per CU, three waves per env where they fit), so the instantiation is
asked of the library for the preset's own handle (mapf_rollout_plan), not assumed."""
import pytest
import torch

from kernel_registry import COVERED

pytestmark = pytest.mark.gpu


def preset_env(cfg):
    import bench
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    p = bench.PRESETS[cfg]
    return BatchedMapfGym(make_config(p["envs"], p["size"], p["size"], num_agents=p["agents"], fov=p["fov"],
                                      num_channel=p["channels"], human_mode="random", goal_mode="random", fix_choice=1,
                                      seed=1, shared_map=p["maps"] == "warehouse"))


@pytest.mark.parametrize("cfg", ["c1", "c2", "c4", "c5"])
def test_default_rollout_kernels_are_oracle_covered(cfg):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    if not COVERED:
        pytest.skip("no oracle-compared rollout case ran in this session (tests/test_gpu_parity.py deselected)")
    env = preset_env(cfg)
    try:
        assert env.rollout_fused, cfg
        for slots in (False, True):
            name = env.rollout_kernel_name(slots)
            assert name in COVERED, (f"{cfg} slots={slots}: {env.rollout_plan(slots)} is launched by default but "
                                     f"no oracle-compared case ran it; covered: {sorted(COVERED)}")
    finally:
        env.close()
