"""Fixed evaluation episodes (evaluate.py:32-137): the on-disk format, CPU side.

tests/golden/g6_episodes/ was written by the reference's own
generateFixedEpisodeInfos + saveFixedEpisodeInfos (tests/golden/make_golden.py g6)."""
import json
import os

import numpy as np

from mapf_amd.episodes import (generate_fixed_episode_infos, load_fixed_episode_infos,
                               save_fixed_episode_infos)

G6 = os.path.join(os.path.dirname(__file__), "golden", "g6_episodes")


def test_load_reference_written_folder():
    infos = load_fixed_episode_infos(G6)
    js = json.load(open(os.path.join(G6, "infos.json")))
    assert infos["numEpisodes"] == js["numEpisodes"] == 4
    for i in range(4):
        m = infos["obstacleMap"][i]
        assert m.dtype == np.int64 and set(np.unique(m)) <= {0, -1}
        seqs = infos["agentsSequence"][i]
        assert len(seqs) == 2 and all(isinstance(c, tuple) for s in seqs for c in s)
        for s in seqs:                       # every start / goal is a free cell
            assert all(m[c] == 0 for c in s)
        hs = infos["humanSequence"][i]
        assert hs[0] == infos["humanStart"][i] and (hs[0][0] == 0 or hs[0][1] == 0)
        assert infos["humanGoal"][i] == hs[-1]


def test_save_round_trip_matches_reference_bytes(tmp_path):
    """Our writer reproduces the reference's infos.json byte for byte and the same .npy maps."""
    infos = load_fixed_episode_infos(G6)
    save_fixed_episode_infos(infos, str(tmp_path))
    assert open(tmp_path / "infos.json").read() == open(os.path.join(G6, "infos.json")).read()
    for i in range(4):
        a = np.load(tmp_path / f"obstacleMap{i}.npy")
        b = np.load(os.path.join(G6, f"obstacleMap{i}.npy"))
        assert a.dtype == b.dtype and np.array_equal(a, b)
    again = load_fixed_episode_infos(str(tmp_path))
    for k in ("agentsSequence", "humanSequence", "humanStart", "humanGoal", "numEpisodes"):
        assert again[k] == infos[k]


def test_generator_follows_reference_protocol():
    infos = generate_fixed_episode_infos(6, 3, 40, world_size=(10, 14), rng=np.random.default_rng(3))
    assert infos["numEpisodes"] == 6
    for i in range(6):
        m = infos["obstacleMap"][i]
        L = m.shape[0]
        assert 10 <= L <= 14 and m.shape[1] == int(L / (2 / 3))
        hs = infos["humanSequence"][i]
        assert hs[0][0] == 0 or hs[0][1] == 0
        assert sum(abs(a[0] - b[0]) + abs(a[1] - b[1]) for a, b in zip(hs, hs[1:])) > 40
        starts = [s[0] for s in infos["agentsSequence"][i]]
        assert len(set(starts)) == 3 and hs[0] not in starts
        for s in infos["agentsSequence"][i]:
            assert sum(abs(a[0] - b[0]) + abs(a[1] - b[1]) for a, b in zip(s, s[1:])) > 40
            assert all(m[c] == 0 for c in s)


def test_random_warehouse_batch_pads_with_obstacles():
    """MapfGym() maps for a batch: random lengths in WORLD_SIZE, each warehouse at the
    top-left of one [B, 40, 60] stack, the rest obstacles (maps.random_warehouse_batch)."""
    from mapf_amd.maps import generate_warehouse, random_warehouse_batch
    m = random_warehouse_batch(np.random.default_rng(0), 64, (10, 40))
    assert m.shape == (64, 40, 60) and m.dtype == np.int8
    lengths = set()
    for b in range(64):
        free = np.argwhere(m[b] == 0)
        L = int(free[:, 0].max()) + 1
        W = int(free[:, 1].max()) + 1
        w = generate_warehouse(L)
        assert W == w.shape[1]
        np.testing.assert_array_equal(m[b, :L, :W], w)
        assert (m[b, L:, :] == -1).all() and (m[b, :, W:] == -1).all()
        lengths.add(L)
    assert len(lengths) > 10 and min(lengths) >= 10 and max(lengths) <= 40
