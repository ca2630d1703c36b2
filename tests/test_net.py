"""Policy network and PPO update vs the reference (CPU, fp32, dropout off).

tests/golden/g5_net.npz holds the reference's SCRIMPNet outputs (net.py:101-155)
and one Model.train update (model.py:78-199) for deterministic weights derived
from the parameter names (det_weights, shared with make_golden.py)."""
import json
import zlib

import numpy as np
import pytest
import torch

from golden_io import load


def det_weights(state_dict):
    out = {}
    for k, v in state_dict.items():
        n = v.numel()
        phase = (zlib.crc32(k.encode()) % 1000) / 1000.0
        x = np.sin(np.arange(n, dtype=np.float64) * 0.37 + phase * 6.283) * 0.05
        out[k] = torch.from_numpy(x.reshape(tuple(v.shape)).astype(np.float32))
    return out


@pytest.fixture(scope="module")
def z():
    return load("g5_net")


def make_net():
    from mapf_amd.net import SCRIMPNet
    net = SCRIMPNet(numChannel=6, num_agents=2, fov=9)
    net.load_state_dict(det_weights(net.state_dict()))
    return net.eval()


def test_state_dict_keys_and_shapes_match_reference(z):
    from mapf_amd.net import SCRIMPNet
    sd = SCRIMPNet(numChannel=6).state_dict()
    keys = sorted(sd.keys())
    assert keys == [str(k) for k in z["keys"]]
    assert [list(sd[k].shape) for k in keys] == json.loads(str(z["shapes"]))
    assert sum(v.numel() for v in sd.values()) == 8230840


def test_forward_matches_reference(z):
    net = make_net()
    with torch.no_grad():
        outs = net(torch.from_numpy(z["obs"]), torch.from_numpy(z["vec"]))
    for name, o in zip(["policy", "value", "blocking", "policy_sig", "x", "logits", "cost_value"], outs):
        np.testing.assert_allclose(o.numpy(), z[f"out_{name}"], rtol=1e-4, atol=1e-5, err_msg=name)


def test_ppo_update_matches_reference(z):
    from mapf_amd.config import EnvParameters
    from mapf_amd.model import Model
    old = EnvParameters.N_AGENTS
    EnvParameters.N_AGENTS = 2
    try:
        m = Model(0, "cpu", global_model=True, numChannel=6, num_agents=2, fov=9)
        m.network.load_state_dict(det_weights(m.network.state_dict()))
        m.network.eval()
        g = lambda k: z["train_" + k]
        stats = m.train(g("observation"), g("vector"), g("returns"), g("cost_returns"), g("old_v"), g("old_cv"),
                        g("action"), g("old_ps"), None, g("train_valid"), 3.0)
    finally:
        EnvParameters.N_AGENTS = old
    got = np.array([float(np.asarray(x)) for x in stats])
    np.testing.assert_allclose(got, z["train_stats"], rtol=2e-4, atol=2e-6)
    sd = m.network.state_dict()
    for k in ["conv1.weight", "fully_connected_2.bias", "transformer.layers.1.0.fn.fn.to_qkv.weight",
              "policy_layer.weight"]:
        np.testing.assert_allclose(sd[k].numpy().reshape(-1)[:2048], z["after_" + k.replace(".", "_")],
                                   rtol=1e-5, atol=1e-7, err_msg=k)
