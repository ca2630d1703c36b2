"""Obstacle maps (reset inputs), restated from the reference's generators.

generate_warehouse follows map_generator.py:127-138 (generateWarehouse):
shelves of `shelf_size` cells on every odd row 1..length-2, placed from
column freeSpace in steps of shelf_size + 1; -1 = obstacle, 0 = free.
The benchmark configs use the "generalised" warehouse with an explicit
width.  random_map follows the PRIMAL random_generator rule
-(rand < p) (map_generator.py:13-28).
"""
import numpy as np


def generate_warehouse(length, width=None, shelf_size=5, lb_ratio=2 / 3, free_space_ratio=1 / 3):
    breadth = int(length / lb_ratio) if width is None else int(width)
    world = np.zeros((length, breadth), dtype=np.int8)
    n_shelves = int((breadth * (1 - free_space_ratio)) / (shelf_size + 1))
    free_space = int((breadth - n_shelves * (shelf_size + 1)) / 2)
    for col in range(free_space, free_space + n_shelves * (shelf_size + 1), shelf_size + 1):
        world[1:length - 1:2, col:col + shelf_size] = -1
    return world


def random_warehouse(rng, world_size=(10, 40)):
    """MapfGym's map: generateWarehouse(num_block=WORLD_SIZE) -- random length in [lo, hi]."""
    length = int(rng.integers(world_size[0], world_size[1] + 1))
    return generate_warehouse(length)


def random_warehouse_batch(rng, num_envs, world_size=(10, 40)):
    """One MapfGym() map per env (random length in WORLD_SIZE, mapf_gym.py:166) in ONE
    [B, Lmax, Wmax] int8 stack: each warehouse at the top-left, padded with obstacle
    rows/columns at the bottom/right.  Equivalent for the env: off-map and padding
    cells read alike everywhere (static masks, FOV channel 0, A*/BFS passability,
    getFreeCell's rejection; the human entrance lies on row 0 / column 0, unpadded);
    tests/test_gpu_parity.py replays reference episodes on a padded map."""
    big = generate_warehouse(world_size[1])
    out = np.full((num_envs,) + big.shape, -1, dtype=np.int8)
    for b in range(num_envs):
        w = random_warehouse(rng, world_size)
        out[b, :w.shape[0], :w.shape[1]] = w
    return out


def random_map(rng, height, width, density):
    return -(rng.random((height, width)) < density).astype(np.int8)


def keep_largest_component(world):
    """Turn free cells outside the largest 4-connected free component into obstacles
    (config c5 extension: a random 0.3-density map can be disconnected, and the
    reference's astar_4 then returns a ValueError, astar_4.py:109)."""
    from scipy import ndimage
    free = world == 0
    lab, n = ndimage.label(free)
    if n <= 1:
        return world.copy()
    sizes = ndimage.sum(free, lab, index=np.arange(1, n + 1))
    keep = 1 + int(np.argmax(sizes))
    out = world.copy()
    out[(lab != keep) & free] = -1
    return out
