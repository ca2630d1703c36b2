"""renderWorld (util.py:189-232): the numpy restatement (oracle/render_oracle.py, CPU) and
the device renderer behind mapf_render (GPU, bit-exact vs the restatement), plus the GIF
writer.  cv2 -- the reference's rasteriser -- is absent from this image: the pixel rules
are this build's (inside-or-on integer polygons, dx^2 + dy^2 <= r^2 discs), parity vs cv2
unpinned; the colours, shapes' vertices and painter's order are the reference's."""
import numpy as np
import pytest
import torch

from oracle import render_oracle as R


def _warehouse(h, w):
    from mapf_amd.maps import generate_warehouse
    return generate_warehouse(h, w)


def test_oracle_frame_structure():
    world = _warehouse(10, 10)
    path = [(9, 9), (9, 8), (8, 8), (7, 8), (8, 8), (9, 8), (9, 9)]
    f = R.render_world(world, [(0, 0), (2, 3)], [(0, 1), (5, 5)], (9, 9), path, 0)
    assert f.shape == (200, 200, 3) and f.dtype == np.uint8
    assert (f[0:20, 0:20] == R.palette(2)[3]).all()                   # agent 0's whole cell
    assert (f[105:115, 110:111] == R.palette(2)[4]).all()             # agent 1's goal disc at (5, 5)
    assert (f[20 * 1 + 1, 20 * 2 + 2] == 0).all()                      # a shelf cell stays black
    # the path segment path[1:4] is drawn: arrows on (9,8) and (8,8), the star on (7,8)
    star = np.all(f[140:160, 160:180] == 127, axis=-1)
    arrow = np.all(f[180:200, 160:180] == 127, axis=-1)
    assert star.sum() > 40 and arrow.sum() > 40
    assert np.all(f[180 + 9, 180 + 10] == 127)                         # the human's triangle, mid cell


def test_oracle_palette_is_hsv():
    pal = R.palette(8)
    assert tuple(pal[3]) == (255, 0, 0) and tuple(pal[5]) == (127, 255, 0)   # hsv(1/4) * 255 truncated
    assert tuple(pal[2]) == (127, 127, 127)                                 # colours[-2] = 0.5


def test_oracle_geometry_and_colours_match_reference_g8():
    """The restatement's palette and shape vertices == the reference's init_colors /
    getArrowPoints / drawStar / getRectPoints / getCenter / getTriPoints (util.py:88-187),
    from tests/golden/g8_render.npz, over 36 cells x 6 scales x 4 directions and 9 agent
    counts.  With the device kernel bit-exact to this restatement (GPU test below), only the
    cv2 fill rule itself is unpinned."""
    import colorsys
    from golden_io import load
    z = load("g8_render")
    for n in (1, 2, 3, 4, 6, 7, 8, 16, 64):
        np.testing.assert_array_equal(R.palette(n), z[f"colors_u8_{n}"], err_msg=f"palette n={n}")
        # the float colours too (matplotlib's hsv_to_rgb vs colorsys: same float64 formula)
        f = np.array([[1, 1, 1], [0, 0, 0], [0.5, 0.5, 0.5]] +
                     [list(colorsys.hsv_to_rgb(a / float(n), 1.0, 1.0)) for a in range(n)])
        np.testing.assert_array_equal(f, z[f"colors_f_{n}"])
    for si, sc in enumerate(z["scales"]):
        sc = int(sc)
        for ci, (r, c) in enumerate(z["coords"]):
            coord = (int(r), int(c))
            for di, d in enumerate(z["dirs"]):
                np.testing.assert_array_equal(R.arrow_points(d, coord, sc), z["arrows"][si, di, ci])
            np.testing.assert_array_equal(R.star_points(coord, sc), z["stars"][si, ci])
            np.testing.assert_array_equal(R.rect_points(coord, sc), z["rects"][si, ci])
            np.testing.assert_array_equal(R.tri_points(coord, sc), z["tris"][si, ci])
            assert R.center(coord, sc) == list(z["centers"][si, ci])
    assert R.arrow_points((0, 0), (1, 1), 20) is None


def test_make_gif_roundtrip(tmp_path):
    from PIL import Image

    from mapf_amd.render import make_gif
    world = _warehouse(10, 10)
    frames = [R.render_world(world, [(0, k)], [(5, 5)], (9, 9), [(9, 9), (9, 8), (9, 9)], 0) for k in range(3)]
    out = tmp_path / "ep.gif"
    make_gif(frames, str(out))
    im = Image.open(out)
    assert im.n_frames == 3 and im.size == (200, 200)
    im.seek(1)
    assert np.array_equal(np.asarray(im.convert("RGB")), frames[1])


def _oracle_frame(st, world, b, scale):
    n = st["pos"].shape[1]
    hum = st["human"][b]
    L = int(hum[7])
    path = [tuple(int(x) for x in st["human_path"][b, k]) for k in range(L)]
    return R.render_world(world, [tuple(p) for p in st["pos"][b]], [tuple(g) for g in st["goal"][b]],
                          (int(hum[0]), int(hum[1])), path, int(hum[6]), scale=scale)


@pytest.mark.gpu
@pytest.mark.parametrize("H,n,scale,maps", [(20, 8, 20, "wh"), (12, 5, 15, "wh"), (40, 16, 8, "rand")])
def test_device_render_matches_oracle(H, n, scale, maps):
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    from mapf_amd.maps import keep_largest_component, random_map
    B = 6
    if maps == "wh":
        world, shared = _warehouse(H, H), True
    else:
        rng = np.random.default_rng(3)
        world, shared = np.stack([keep_largest_component(random_map(rng, H, H, 0.3)) for _ in range(B)]), False
    env = BatchedMapfGym(make_config(B, H, H, num_agents=n, fov=9, num_channel=6, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=11, shared_map=shared))
    env.reset_seeded(world)
    for t in range(40):
        if t % 13 == 0:
            frames = env.render([0, 5, 2], scale=scale).cpu().numpy()
            st = env.get_state()
            for k, b in enumerate([0, 5, 2]):
                want = _oracle_frame(st, world if shared else world[b], b, scale)
                np.testing.assert_array_equal(frames[k], want, err_msg=f"t={t} env {b}")
        env.step(env.random_actions())
    with pytest.raises(IndexError):
        env.render([B])
    env.close()


@pytest.mark.gpu
def test_single_env_render_and_episode_gif(tmp_path):
    from mapf_amd.mapf_gym import MapfGym
    from mapf_amd.render import episode_frames, make_gif
    g = MapfGym(num_agents=4, size=(10, 12), seed=5)
    f = g._render()
    assert f.dtype == np.uint8 and f.shape[2] == 3 and f.shape[0] % 20 == 0
    frames = episode_frames(g._env, 5)
    assert frames.shape[0] == 6
    make_gif(frames, str(tmp_path / "e.gif"))
    torch.cuda.synchronize()
