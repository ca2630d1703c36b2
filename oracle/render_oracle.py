"""CPU restatement of renderWorld (util.py:189-232) -- TEST INFRASTRUCTURE: only tests/
use it, as the checker of the device renderer (primal-ppo_amd/csrc/mapf_render.hip).

Same painter's order and colours as the reference: every cell white (0) / black (-1)
(getRectPoints, colours[0] / colours[-1]); the human's remaining path
humanPath[step+1 : half+1] (or [step+1:] past the half) as grey arrows (getArrowPoints,
:96-155) with a star on the last cell (drawStar, :157-175); agent i's cell in
hsv(i / N, 1, 1) (init_colors :88-94); agent i's goal as a disc of radius S/2 - 1 at
getCenter (:181-183); the human's triangle (getTriPoints, :185-187); then * 255 and
astype('uint8').  The reference fills with cv2 (absent here); these rules -- a pixel is
covered iff it lies inside or on the integer-vertex polygon, a disc iff dx^2 + dy^2 <= r^2
-- are this build's, so parity with cv2's rasteriser is unpinned; the device kernel is
pinned to this restatement bit-exactly.  The geometry and the colours themselves --
init_colors, getArrowPoints, drawStar, getRectPoints, getCenter, getTriPoints -- ARE pinned:
tests/golden/g8_render.npz holds the reference functions' own outputs over a grid of cells,
scales and agent counts (tests/test_render.py checks palette(), arrow_points(), star_points(),
rect_points(), center() and tri_points() against it); only cv2's fill rule stays unpinned.
"""
import colorsys
import math

import numpy as np


def palette(n):
    """init_colors (util.py:88-94) * 255 cast to uint8 (renderWorld :229-230): rows 0 = free
    cell (colours[0]), 1 = obstacle (colours[-1]), 2 = human grey (colours[-2]), 3 + i = agent
    i (colours[i + 1] = hsv(i / n, 1, 1)); n is EnvParameters.N_AGENTS in the reference."""
    pal = [(255, 255, 255), (0, 0, 0), (127, 127, 127)]
    for a in range(n):
        r, g, b = colorsys.hsv_to_rgb(a / float(n), 1.0, 1.0)
        pal.append((int(r * 255.0), int(g * 255.0), int(b * 255.0)))
    return np.array(pal, dtype=np.uint8)


def _in_polygon(vx, vy, px, py):
    """inside (crossing number) or on the boundary; px, py integer grids."""
    n = len(vx)
    inside = np.zeros(px.shape, bool)
    on = np.zeros(px.shape, bool)
    for k in range(n):
        j = (k - 1) % n
        ax, ay, bx, by = vx[j], vy[j], vx[k], vy[k]
        cr = (bx - ax) * (py - ay) - (by - ay) * (px - ax)
        on |= (cr == 0) & (px >= min(ax, bx)) & (px <= max(ax, bx)) & (py >= min(ay, by)) & (py <= max(ay, by))
        cross = (ay > py) != (by > py)
        lhs, rhs = (px - ax) * (by - ay), (py - ay) * (bx - ax)
        hit = cross & ((lhs < rhs) if by > ay else (lhs > rhs))
        inside ^= hit
    return inside | on


def arrow_points(direction, coord, scale):
    """getArrowPoints (util.py:96-155) with renderWorld's tailWidth = scale / 10 and
    headWidth = scale / 2 - 2 (:214); None for a zero direction (the reference leaves
    `arrow` unbound there and raises)."""
    half = int(scale / 2) - 1
    th, tw, hw = half - 2, scale / 10, scale / 2 - 2
    cx, cy = coord[1] * scale + half, coord[0] * scale + half
    d = tuple(int(x) for x in direction)
    if d == (0, 1):
        pts = [[cx, cy - tw], [cx - th, cy - tw], [cx - th, cy + tw], [cx, cy + tw], [cx, cy + hw], [cx + hw, cy],
               [cx, cy - hw]]
    elif d == (1, 0):
        pts = [[cx - tw, cy], [cx - tw, cy - th], [cx + tw, cy - th], [cx + tw, cy], [cx + hw, cy], [cx, cy + hw],
               [cx - hw, cy]]
    elif d == (0, -1):
        pts = [[cx, cy + tw], [cx + th, cy + tw], [cx + th, cy - tw], [cx, cy - tw], [cx, cy - hw], [cx - hw, cy],
               [cx, cy + hw]]
    elif d == (-1, 0):
        pts = [[cx + tw, cy], [cx + tw, cy + th], [cx - tw, cy + th], [cx - tw, cy], [cx - hw, cy], [cx, cy - hw],
               [cx + hw, cy]]
    else:
        return None
    return np.array(pts, dtype="int64")


def star_points(coord, scale):
    """drawStar (util.py:157-175) with diameter = scale, numPoints = 5 (:211)."""
    half = int(scale / 2) - 1
    cx, cy = coord[1] * scale + half, coord[0] * scale + half
    outer = scale // 2
    inner = int(outer * 3 / 8)
    between = 2 * math.pi / 5
    pts = []
    for i in range(5):
        pa = math.pi / 2 + i * between
        pts += [(cx + inner * math.cos(pa - between / 2), cy - inner * math.sin(pa - between / 2)),
                (cx + outer * math.cos(pa), cy - outer * math.sin(pa)),
                (cx + inner * math.cos(pa + between / 2), cy - inner * math.sin(pa + between / 2))]
    return np.array(pts, dtype="int64")


def rect_points(coord, scale):
    """getRectPoints (util.py:177-179): the cell's four corners, (x, y) = (col, row) * scale."""
    x, y = coord[1] * scale, coord[0] * scale
    return np.array([[x, y], [x + scale - 1, y], [x + scale - 1, y + scale - 1], [x, y + scale - 1]], dtype="int64")


def center(coord, scale):
    """getCenter (util.py:181-183): floor of the cell's origin + scale / 2."""
    return [int(math.floor(coord[1] * scale + scale / 2)), int(math.floor(coord[0] * scale + scale / 2))]


def tri_points(coord, scale):
    """getTriPoints (util.py:185-187): apex at the top edge's floor(x + scale / 2)."""
    x, y = coord[1] * scale, coord[0] * scale
    return np.array([[int(math.floor(x + scale / 2)), y], [x + scale - 1, y + scale - 1], [x, y + scale - 1]],
                    dtype="int64")


def render_world(world, agents, goals, human, human_path, human_step, scale=20):
    """uint8 [H*scale, W*scale, 3]; agents / goals lists of (row, col), human (row, col),
    human_path the current path as a list of (row, col), human_step its index."""
    H, W = world.shape
    n = len(agents)
    pal = palette(n)
    py, px = np.mgrid[0:H * scale, 0:W * scale]
    col = np.where(world[py // scale, px // scale] != 0, 1, 0)
    half = int(len(human_path) / 2)
    path = human_path[human_step + 1:half + 1] if human_step < half else human_path[human_step + 1:]
    for idx, val in enumerate(path):
        if idx == len(path) - 1:
            pts = star_points(val, scale)
        else:
            pts = arrow_points(np.subtract(path[idx + 1], val), val, scale)
            if pts is None:
                continue
        col = np.where(_in_polygon(pts[:, 0], pts[:, 1], px, py), 2, col)
    for i, (r, c) in enumerate(agents):
        col = np.where((py // scale == r) & (px // scale == c), 3 + i, col)
    rad = int(math.floor(scale / 2)) - 1
    for i, (r, c) in enumerate(goals):
        gx, gy = center((r, c), scale)
        disc = (px - gx) ** 2 + (py - gy) ** 2 <= rad * rad
        col = np.where(disc & (py // scale == r) & (px // scale == c), 3 + i, col)
    r, c = human
    tri = tri_points((r, c), scale)
    col = np.where(_in_polygon(tri[:, 0], tri[:, 1], px, py) & (py // scale == r) & (px // scale == c), 2, col)
    return pal[col]
