"""world_size-2 gloo tests of the only exchange step on the path: the PPO
gradient all-reduce (and the global advantage statistics / Lagrangian cost it
needs), SURVEY.md §8(e).  Two ranks training on the two halves of a
minibatch must end where one process training on the whole minibatch ends."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from golden_io import load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train_once(batch, world=1, rank=0):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd"), os.path.join(ROOT, "tests")]
    from mapf_amd.config import EnvParameters
    from mapf_amd.model import Model
    from test_net import det_weights
    EnvParameters.N_AGENTS = 2
    m = Model(0, "cpu", global_model=True, numChannel=6, num_agents=2, fov=9)
    m.network.load_state_dict(det_weights(m.network.state_dict()))
    m.network.eval()
    sl = slice(rank * len(batch["returns"]) // world, (rank + 1) * len(batch["returns"]) // world)
    g = lambda k: batch[k][sl]
    stats = m.train(g("observation"), g("vector"), g("returns"), g("cost_returns"), g("old_v"), g("old_cv"),
                    g("action"), g("old_ps"), None, g("train_valid"), 3.0)
    return {k: v.clone() for k, v in m.network.state_dict().items()}, stats


def _worker(rank, world, port, batch, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sd, stats = _train_once(batch, world, rank)
        q.put((rank, {k: v.numpy() for k, v in sd.items() if k in KEYS}, float(np.asarray(stats[8]))))
    finally:
        dist.destroy_process_group()


KEYS = ["conv1.weight", "fully_connected_2.weight", "transformer.layers.0.0.fn.fn.to_qkv.weight", "policy_layer.weight",
        "value_layer.bias"]


def test_two_rank_ppo_update_equals_single_process():
    z = load("g5_net")
    batch = {k[len("train_"):]: z[k] for k in z.files if k.startswith("train_") and k != "train_stats"}
    ref_sd, ref_stats = _train_once(batch)
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda x: x[0])
    for k in KEYS:
        # both ranks hold identical weights after the all-reduced step ...
        np.testing.assert_array_equal(res[0][1][k], res[1][1][k])
        # ... equal to one process on the whole minibatch (global advantage statistics)
        np.testing.assert_allclose(res[0][1][k], ref_sd[k].numpy(), rtol=1e-5, atol=1e-8, err_msg=k)
    assert abs(res[0][2] - float(np.asarray(ref_stats[8]))) < 1e-3 * max(1.0, abs(float(np.asarray(ref_stats[8]))))


def _seeded_worker(rank, world, port, batch, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd"), os.path.join(ROOT, "tests")]
        from mapf_amd.config import EnvParameters
        from mapf_amd.model import Model
        EnvParameters.N_AGENTS = 2
        torch.manual_seed(100 + rank)              # every rank draws different initial weights ...
        m = Model(0, "cpu", global_model=True, numChannel=6, num_agents=2, fov=9)
        init = {k: v.numpy().copy() for k, v in m.network.state_dict().items()}
        sl = slice(rank * len(batch["returns"]) // world, (rank + 1) * len(batch["returns"]) // world)
        g = lambda k: batch[k][sl]
        m.train(g("observation"), g("vector"), g("returns"), g("cost_returns"), g("old_v"), g("old_cv"),
                g("action"), g("old_ps"), None, g("train_valid"), 3.0)
        after = {k: v.numpy().copy() for k, v in m.network.state_dict().items()}
        q.put((rank, init, after))
    finally:
        dist.destroy_process_group()


def test_ranks_with_different_seeds_share_rank0_weights():
    """SURVEY.md §8(e) "weights broadcast at init": ranks that construct their global Model from
    different seeds hold rank 0's weights after construction (Model.broadcast_weights) and
    identical weights after one all-reduced update (dropout active, masks differ per rank)."""
    sys.path[:0] = [os.path.join(ROOT, "primal-ppo_amd")]
    from mapf_amd.config import EnvParameters
    from mapf_amd.model import Model
    z = load("g5_net")
    batch = {k[len("train_"):]: z[k] for k in z.files if k.startswith("train_") and k != "train_stats"}
    n_agents = EnvParameters.N_AGENTS
    EnvParameters.N_AGENTS = 2
    try:
        torch.manual_seed(100)
        rank0_alone = {k: v.numpy().copy() for k, v in
                       Model(0, "cpu", global_model=True, numChannel=6, num_agents=2, fov=9).network.state_dict().items()}
        torch.manual_seed(101)
        rank1_alone = Model(0, "cpu", global_model=True, numChannel=6, num_agents=2, fov=9).network.state_dict()
    finally:
        EnvParameters.N_AGENTS = n_agents
    assert not np.array_equal(rank0_alone["conv1.weight"], rank1_alone["conv1.weight"].numpy())
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_seeded_worker, args=(r, 2, port, batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda x: x[0])
    (_, init0, after0), (_, init1, after1) = res
    assert set(init0) == set(rank0_alone)
    for k in init0:
        np.testing.assert_array_equal(init0[k], rank0_alone[k], err_msg=k)
        np.testing.assert_array_equal(init1[k], rank0_alone[k], err_msg=k)
        np.testing.assert_array_equal(after0[k], after1[k], err_msg=k)
    assert any(not np.array_equal(after0[k], init0[k]) for k in KEYS)
