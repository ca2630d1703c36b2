"""Obstacle maps (CPU): the restated generators against the reference's own maps.

g7_warehouses.npz holds generateWarehouse(length=L) (map_generator.py:127-138) for
every L in WORLD_SIZE = (10, 40), written by the reference (tests/golden/make_golden.py).
Both the host restatement (maps.generate_warehouse) and the oracle's restatement of the
device generator (oc_gen_map, = mapf_maps.hip) must reproduce them bit for bit."""
import numpy as np

from golden_io import load
from oracle import oracle as O


def test_generate_warehouse_matches_reference_every_length():
    from mapf_amd.maps import generate_warehouse
    z = load("g7_warehouses")
    assert sorted(int(k[1:]) for k in z.files) == list(range(10, 41))
    for k in z.files:
        L = int(k[1:])
        np.testing.assert_array_equal(generate_warehouse(L), z[k], err_msg=k)


def test_device_generator_restatement_matches_reference():
    """oc_gen_map kind 0 (the device kernel's spec): the drawn length's map, padded with
    obstacles into the 40 x 60 stack, is the reference's map of that length."""
    z = load("g7_warehouses")
    seen = set()
    for env in range(400):
        m, L = O.gen_map(0, 40, 60, env, epoch=3)
        ref = z[f"L{L}"]
        h, w = ref.shape
        np.testing.assert_array_equal(m[:h, :w], ref)
        assert (m[h:] == -1).all() and (m[:, w:] == -1).all()
        seen.add(L)
    assert len(seen) == 31          # every length of [10, 40] drawn


def test_length_draws_are_uniform():
    counts = np.bincount([O.gen_map(0, 40, 60, env, epoch=0)[1] for env in range(6200)], minlength=41)[10:]
    chi2 = ((counts - 200.0) ** 2 / 200.0).sum()
    assert chi2 < 80, counts          # 30 dof: p ~ 1e-6 at 80


def test_random_maps_density_and_independence():
    a, _ = O.gen_map(1, 80, 80, 0, epoch=0, density=0.3)
    b, _ = O.gen_map(1, 80, 80, 1, epoch=0, density=0.3)
    c, _ = O.gen_map(1, 80, 80, 0, epoch=1, density=0.3)
    for m in (a, b, c):
        assert abs((m == -1).mean() - 0.3) < 0.02
    assert (a != b).any() and (a != c).any()
    assert (O.gen_map(1, 20, 20, 0, density=0.0)[0] == 0).all()
    assert (O.gen_map(1, 20, 20, 0, density=1.0)[0] == -1).all()
