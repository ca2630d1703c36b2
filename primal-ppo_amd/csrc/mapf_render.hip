// primal-ppo_amd/csrc/mapf_render.hip -- renderWorld (util.py:189-232) for a batch of
// envs on the device: one RGB uint8 frame [H*S][W*S][3] per env, drawn from the
// env's state in HBM (obstacle bitmap, agents' cells and goals, the human's cell and
// path), for the evaluation GIFs (driver.py:232-276, util.make_gif).
//
// The reference paints with cv2 on a float64 image, in this order:
//   every cell: white (free) / black (obstacle)            getRectPoints, colours[0/-1]
//   human.path[step+1 : half+1] (or [step+1:] past the half): an arrow towards the
//     next cell (getArrowPoints), a star on the last one (drawStar), grey
//   agent i: its cell in colours[i+1] = hsv(i / N, 1, 1)     getRectPoints
//   agent i's goal: a disc of radius S/2 - 1 at the cell centre (getCenter)
//   the human: a triangle (getTriPoints), grey
// then scene * 255 cast to uint8 (truncation).  Here each pixel runs the same
// painter's sequence over the shapes that can cover it.  Rasterisation rules: a
// pixel is painted iff its integer coordinates lie inside or on the integer-vertex
// polygon; a disc covers dx^2 + dy^2 <= r^2.  cv2's own scanline and circle
// rasterisation is not available in this image (parity vs cv2 unpinned: along
// slanted edges the two can differ by a pixel); oracle/render_oracle.py states
// these rules in numpy and pins the kernel to them bit-exactly.
#include "mapf_common.h"
#include "mapf_kernels.h"

namespace mapf {

// inside or on a convex polygon of n integer vertices (either orientation)
__device__ inline bool in_convex(const int *vx, const int *vy, int n, int px, int py) {
    bool pos = false, neg = false;
    for (int k = 0; k < n; ++k) {
        const int ax = vx[k], ay = vy[k], bx = vx[(k + 1) % n], by = vy[(k + 1) % n];
        const long cr = (long)(bx - ax) * (py - ay) - (long)(by - ay) * (px - ax);
        pos |= cr > 0;
        neg |= cr < 0;
    }
    return !(pos && neg);
}

// inside (crossing number) or on the boundary of a simple polygon
__device__ inline bool in_polygon(const int *vx, const int *vy, int n, int px, int py) {
    bool in = false;
    for (int k = 0, j = n - 1; k < n; j = k++) {
        const int ax = vx[j], ay = vy[j], bx = vx[k], by = vy[k];
        const long cr = (long)(bx - ax) * (py - ay) - (long)(by - ay) * (px - ax);
        if (cr == 0 && px >= min(ax, bx) && px <= max(ax, bx) && py >= min(ay, by) && py <= max(ay, by)) return true;
        if ((ay > py) != (by > py)) {
            // px < ax + (py - ay) * (bx - ax) / (by - ay), without division
            const long lhs = (long)(px - ax) * (by - ay), rhs = (long)(py - ay) * (bx - ax);
            if (by > ay ? lhs < rhs : lhs > rhs) in = !in;
        }
    }
    return in;
}

// getArrowPoints(direction (dr, dc), coord (r, c), S, S/10, S/2 - 2) = tail rectangle
// + head triangle; vertices truncated to integers as np.array(..., 'int64') does
__device__ inline bool in_arrow(int r, int c, int ddr, int ddc, int S, int px, int py) {
    const int half = S / 2 - 1, th = half - 2;
    const double tw = S / 10.0, hw = S / 2.0 - 2.0;
    const double cx = (double)c * S + half, cy = (double)r * S + half;
    auto T = [](double v) { return (int)(long)v; };    // int64 cast: truncation (all coordinates >= 0 here)
    int vx[7], vy[7];
    if (ddr == 0 && ddc == 1) {
        const double x[7] = {cx, cx - th, cx - th, cx, cx, cx + hw, cx};
        const double y[7] = {cy - tw, cy - tw, cy + tw, cy + tw, cy + hw, cy, cy - hw};
        for (int k = 0; k < 7; ++k) { vx[k] = T(x[k]); vy[k] = T(y[k]); }
    } else if (ddr == 1 && ddc == 0) {
        const double x[7] = {cx - tw, cx - tw, cx + tw, cx + tw, cx + hw, cx, cx - hw};
        const double y[7] = {cy, cy - th, cy - th, cy, cy, cy + hw, cy};
        for (int k = 0; k < 7; ++k) { vx[k] = T(x[k]); vy[k] = T(y[k]); }
    } else if (ddr == 0 && ddc == -1) {
        const double x[7] = {cx, cx + th, cx + th, cx, cx, cx - hw, cx};
        const double y[7] = {cy + tw, cy + tw, cy - tw, cy - tw, cy - hw, cy, cy + hw};
        for (int k = 0; k < 7; ++k) { vx[k] = T(x[k]); vy[k] = T(y[k]); }
    } else if (ddr == -1 && ddc == 0) {
        const double x[7] = {cx + tw, cx + tw, cx - tw, cx - tw, cx - hw, cx, cx + hw};
        const double y[7] = {cy, cy + th, cy + th, cy, cy, cy - hw, cy};
        for (int k = 0; k < 7; ++k) { vx[k] = T(x[k]); vy[k] = T(y[k]); }
    } else {
        return false;                                   // not a unit move: the reference draws nothing
    }
    return in_polygon(vx, vy, 7, px, py);
}

__global__ __launch_bounds__(256) void render_kernel(DevEnv e, const int32_t *__restrict__ envs, RenderSpec rs,
                                                     uint8_t *__restrict__ frames) {
    const int S = rs.scale, FH = e.H * S, FW = e.W * S;
    const int f = blockIdx.y;                           // frame
    const int b = envs[f];
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= FH * FW) return;
    if (b < 0 || b >= e.B) {                            // not an env of this handle: a black frame
        uint8_t *o = frames + ((size_t)f * FH * FW + pix) * 3;
        o[0] = o[1] = o[2] = 0;
        return;
    }
    const int py = pix / FW, px = pix - py * FW;
    const int r = py / S, c = px / S;
    const uint32_t *bits = env_map(e, b);
    int col = obstacle_at(e, bits, r, c) ? 1 : 0;       // palette: 0 free, 1 obstacle, 2 grey, 3 + i agent i
    // the human's remaining path segment: arrows, a star on its last cell
    {
        const int cur = e.hcur[b], L = e.hlen[b * 2 + cur], st = e.hstep[b], half = L / 2;
        const uint32_t *p = human_path(e, b, cur);
        const int k0 = st + 1, k1 = st < half ? min(half + 1, L) : L;
        for (int k = k0; k < k1; ++k) {
            const uint32_t q = p[k];
            const int qr = prow(q), qc = pcol(q);
            if (abs(qr - r) > 1 || abs(qc - c) > 1) continue;   // shapes reach at most one cell out
            if (k == k1 - 1) {
                // drawStar: centre + r cos(a), centre - r sin(a) in float64, then int64 (truncation)
                const double cx = (double)(qc * S + (S / 2 - 1)), cy = (double)(qr * S + (S / 2 - 1));
                int vx[15], vy[15];
                for (int v = 0; v < 15; ++v) { vx[v] = (int)(long)(cx + rs.star_x[v]); vy[v] = (int)(long)(cy - rs.star_y[v]); }
                if (in_polygon(vx, vy, 15, px, py)) col = 2;
            } else {
                const uint32_t n = p[k + 1];
                if (qr == r && qc == c && in_arrow(qr, qc, prow(n) - qr, pcol(n) - qc, S, px, py)) col = 2;
            }
        }
    }
    const size_t base = (size_t)b * e.N;
    for (int i = 0; i < e.N; ++i)                       // agents: whole cells
        if (e.pos[base + i] == pack(r, c)) col = 3 + i;
    const int rad = S / 2 - 1, cxo = S / 2;             // getCenter: floor(base + S / 2)
    for (int i = 0; i < e.N; ++i) {                     // goals: discs
        const uint32_t g = e.goal[base + i];
        if (prow(g) != r || pcol(g) != c) continue;
        const int dx = px - (c * S + cxo), dy = py - (r * S + cxo);
        if (dx * dx + dy * dy <= rad * rad) col = 3 + i;
    }
    {                                                   // the human: a triangle
        const uint32_t h = e.hpos[b];
        if (prow(h) == r && pcol(h) == c) {
            const int x0 = c * S, y0 = r * S;
            const int vx[3] = {x0 + S / 2, x0 + S - 1, x0}, vy[3] = {y0, y0 + S - 1, y0 + S - 1};
            if (in_convex(vx, vy, 3, px, py)) col = 2;
        }
    }
    uint8_t *o = frames + ((size_t)f * FH * FW + pix) * 3;
    o[0] = rs.palette[col * 3];
    o[1] = rs.palette[col * 3 + 1];
    o[2] = rs.palette[col * 3 + 2];
}

void launch_render(const DevEnv &e, const int32_t *envs, int n, const RenderSpec &rs, uint8_t *frames,
                   hipStream_t s) {
    const long px = (long)e.H * rs.scale * e.W * rs.scale;
    hipLaunchKernelGGL(render_kernel, dim3((unsigned)((px + 255) / 256), (unsigned)n), dim3(256), 0, s, e, envs, rs,
                       frames);
}

}  // namespace mapf
