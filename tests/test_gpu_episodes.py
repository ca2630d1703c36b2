"""Batched evaluation over the reference's fixed episodes (evaluate.py:169-256)
on the device env, against the OneEpPerformance sums the reference's own
evaluate loop produced on the same files with the same recorded actions
(tests/golden/make_golden.py g6; fixActions' random.choice = rotating rule)."""
import os

import numpy as np
import pytest
import torch

from mapf_amd.episodes import METRIC_KEYS, evaluate_fixed_episodes, load_fixed_episode_infos

G6 = os.path.join(os.path.dirname(__file__), "golden", "g6_episodes")


@pytest.mark.gpu
@pytest.mark.parametrize("mtype,da_hp", [(0, False), (1, True)])
def test_fixed_episodes_match_reference_evaluate(mtype, da_hp):
    infos = load_fixed_episode_infos(G6)
    exp = np.load(os.path.join(G6, "expected.npz"))
    acts = exp[f"actions_type{mtype}"]
    want = exp[f"metrics_type{mtype}"]
    steps = acts.shape[1]

    def replay(obs, vec, env, t):
        return torch.from_numpy(np.ascontiguousarray(acts[env.episodes, t])).to(torch.int32).cuda()

    got = evaluate_fixed_episodes(infos, replay, num_channel=6, fov=9, use_da=da_hp, use_hp=da_hp,
                                  human_movement_type=mtype, max_steps=steps, fix_choice=0)
    for k, key in enumerate(METRIC_KEYS):
        if key in ("episodeReward", "episodeCostReward"):   # the reference accumulates in float32
            np.testing.assert_allclose(got[key], want[:, k], rtol=1e-5, atol=1e-3, err_msg=key)
        else:
            np.testing.assert_array_equal(got[key], want[:, k], err_msg=key)
