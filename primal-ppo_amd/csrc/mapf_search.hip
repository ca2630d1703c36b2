// primal-ppo_amd/csrc/mapf_search.hip -- BFS distance maps and human A* paths.
//
// One wave per work item, rows of the grid on the lanes (row r = lane + 64k,
// k < 2 -> H <= 128), each row a 128-bit mask (W <= 128).  A BFS level is
// one frontier dilation: horizontal neighbours by shifting the row mask,
// vertical neighbours by ds_bpermute from the lanes holding rows r-1 / r+1.
// Distances land in an LDS image and leave as one coalesced int16 sweep.
//
//  * makeBfsMap (mapf_gym.py:211-244): bfs[b][i] = copy of obstacleMap with
//    free cells -2, then level-order distance from the goal (goal = 0).
//  * astar_4 (astar_4.py:21-109) for the human (Human.getAstarPath,
//    mapf_gym.py:33-37): the heap pops in the total order of the keys
//    (f, g, row, col) (duplicate entries of one cell share their key, so the
//    parent field of the heap tuple never matters), pops are monotone under
//    the consistent Manhattan heuristic, and `parents[c]` is overwritten when
//    new_g <= g_scores[c] (:58).  Hence parent(c) is the LAST expanded
//    neighbour p with d(p) = d(c) - 1 before c is popped, i.e. the one with
//    the largest key (h(p), row, col) -- every such p has a smaller key than c
//    and is expanded before it.  So astar_4's path = BFS distances from the
//    start + a walk back from the goal choosing, at each step, the neighbour
//    with d-1 and the largest (manhattan-to-goal, row, col).  Pinned against
//    the reference's own astar_4 outputs (tests/golden/g3_search.npz) and
//    against the oracle's literal heap A* on random maps.
#include "mapf_common.h"
#include "mapf_kernels.h"

namespace mapf {

namespace {

struct Row2 { uint64_t lo, hi; };

__device__ inline uint64_t bits64_at(const uint32_t *row, int WW, int off) {
    // 64 bits starting at bit `off` of a row of WW u32 words (words past the end read as 1s)
    const int w = off >> 5, s = off & 31;
    auto word = [&](int k) -> uint64_t { return (k < WW) ? (uint64_t)row[k] : 0xFFFFFFFFull; };
    const uint64_t a = word(w) | (word(w + 1) << 32);
    const uint64_t b = word(w + 2);
    return s == 0 ? a : ((a >> s) | (b << (64 - s)));
}

// free-cell mask of row r (bit c = column c), columns >= W cleared
__device__ inline Row2 free_row(const DevEnv &e, const uint32_t *bits, int r) {
    Row2 f = {0, 0};
    if (r >= e.H) return f;
    const uint32_t *row = bits + (size_t)(r + e.P) * e.WW;
    f.lo = ~bits64_at(row, e.WW, e.P);
    f.hi = ~bits64_at(row, e.WW, e.P + 64);
    if (e.W < 64) { f.lo &= (1ull << e.W) - 1; f.hi = 0; }
    else if (e.W < 128) f.hi &= (e.W == 64) ? 0ull : ((1ull << (e.W - 64)) - 1);
    return f;
}

__device__ inline Row2 or2(Row2 a, Row2 b) { return {a.lo | b.lo, a.hi | b.hi}; }
__device__ inline Row2 and2(Row2 a, Row2 b) { return {a.lo & b.lo, a.hi & b.hi}; }
__device__ inline Row2 andn2(Row2 a, Row2 b) { return {a.lo & ~b.lo, a.hi & ~b.hi}; }
__device__ inline Row2 shl1(Row2 a) { return {a.lo << 1, (a.hi << 1) | (a.lo >> 63)}; }
__device__ inline Row2 shr1(Row2 a) { return {(a.lo >> 1) | (a.hi << 63), a.hi >> 1}; }
__device__ inline bool any2(Row2 a) { return (a.lo | a.hi) != 0; }
__device__ inline Row2 shfl2(Row2 a, int src) { return {shfl64(a.lo, src), shfl64(a.hi, src)}; }

// BFS over free cells from (sr, sc); dist (LDS, H*W int16) must be pre-filled
// with the values non-reached cells keep.  Sets dist[start] = 0.
__device__ void wave_bfs(const DevEnv &e, const uint32_t *bits, int sr, int sc, int16_t *dist) {
    const int lane = lane_id();
    const int W = e.W;
    Row2 fr[2], vis[2], fre[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int r = lane + 64 * k;
        fre[k] = free_row(e, bits, r);
        Row2 s = {0, 0};
        if (r == sr) { if (sc < 64) s.lo = 1ull << sc; else s.hi = 1ull << (sc - 64); }
        fr[k] = s; vis[k] = s;
    }
    if (lane == 0) dist[sr * W + sc] = 0;
    const int up_src = (lane + 63) & 63, dn_src = (lane + 1) & 63;
    for (int d = 1;; ++d) {
        Row2 a[2], bb[2], nw[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) { a[k] = shfl2(fr[k], up_src); bb[k] = shfl2(fr[k], dn_src); }
        bool any = false;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            Row2 up = lane > 0 ? a[k] : (k > 0 ? a[k - 1] : Row2{0, 0});
            Row2 dn = lane < 63 ? bb[k] : (k + 1 < 2 ? bb[k + 1] : Row2{0, 0});
            Row2 nb = or2(or2(shl1(fr[k]), shr1(fr[k])), or2(up, dn));
            nw[k] = andn2(and2(nb, fre[k]), vis[k]);
            any |= any2(nw[k]);
        }
        if (__ballot(any) == 0) break;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            vis[k] = or2(vis[k], nw[k]);
            fr[k] = nw[k];
            const int r = lane + 64 * k;
            uint64_t m = nw[k].lo;
            while (m) { const int c = __builtin_ctzll(m); m &= m - 1; dist[r * W + c] = (int16_t)d; }
            m = nw[k].hi;
            while (m) { const int c = __builtin_ctzll(m); m &= m - 1; dist[r * W + 64 + c] = (int16_t)d; }
        }
    }
}

__device__ inline void fill_init(const DevEnv &e, const uint32_t *bits, int16_t *dist, bool bfs_style) {
    // bfs_style: makeBfsMap's initial copy (obstacle -1, free -2); else -1 everywhere (A* distances)
    const int cells = e.H * e.W;
    for (int k = lane_id(); k < cells; k += 64) {
        const int r = k / e.W, c = k - r * e.W;
        dist[k] = bfs_style ? (obstacle_at(e, bits, r, c) ? (int16_t)-1 : (int16_t)-2) : (int16_t)-1;
    }
}

}  // namespace

// One wave per agent BFS event (makeBfsMap on reset / goal change).
__global__ __launch_bounds__(256) void bfs_kernel(DevEnv e, int parity, int all) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6;
    const int cells = e.H * e.W;
    int16_t *dist = reinterpret_cast<int16_t *>(smem) + (size_t)wave * ((cells + 7) & ~7);
    const uint32_t count = all ? (uint32_t)(e.B * e.N) : e.counters[C_BFS_COUNT + parity];
    const uint32_t *list = e.bfs_list + (size_t)parity * e.B * e.N;
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t item = blockIdx.x * (blockDim.x >> 6) + wave; item < count; item += nwaves) {
        const uint32_t ai = all ? item : list[item];
        const int b = (int)(ai / (uint32_t)e.N);
        const uint32_t *bits = env_map(e, b);
        const uint32_t gl = e.goal[ai];
        fill_init(e, bits, dist, true);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        wave_bfs(e, bits, prow(gl), pcol(gl), dist);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        int16_t *outp = e.bfs + (size_t)ai * cells;
        for (int k = lane_id(); k < cells; k += 64) outp[k] = dist[k];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}

// One wave per human (re)plan: BFS from the current position, then lane 0
// walks back from the goal (astar_4 parent rule, see the file header) and
// writes start->goal (FixedPathHuman) or start->goal->start (Human / LoopingHuman).
__global__ __launch_bounds__(256) void replan_kernel(DevEnv e, int parity, int all) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6;
    const int cells = e.H * e.W;
    int16_t *dist = reinterpret_cast<int16_t *>(smem) + (size_t)wave * ((cells + 7) & ~7);
    const uint32_t count = all ? (uint32_t)e.B : e.counters[C_REPLAN_COUNT + parity];
    const uint32_t *list = e.replan_list + (size_t)parity * e.B;
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    const int W = e.W;
    for (uint32_t item = blockIdx.x * (blockDim.x >> 6) + wave; item < count; item += nwaves) {
        const int b = all ? (int)item : (int)list[item];
        const uint32_t *bits = env_map(e, b);
        const uint32_t st = e.hpos[b], gl = e.hgoal[b];
        fill_init(e, bits, dist, false);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        wave_bfs(e, bits, prow(st), pcol(st), dist);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane_id() == 0) {
            uint32_t *path = e.hpath + (size_t)b * e.Lmax;
            const int gr = prow(gl), gc = pcol(gl);
            const int d = (st == gl) ? -1 : dist[gr * W + gc];
            if (d <= 0) {
                // start == goal (astar_4 returns []) or unreachable (returns ValueError): the
                // reference crashes right after; keep the human in place and count it.
                atomicAdd(&e.counters[C_UNREACHABLE], 1u);
                path[0] = st;
                e.hlen[b] = 1;
            } else {
                const bool round_trip = e.human_mode != 2;
                const int len = round_trip ? 2 * d + 1 : d + 1;
                if (len > e.Lmax) {
                    atomicAdd(&e.counters[C_PATH_OVERFLOW], 1u);
                    path[0] = st;
                    e.hlen[b] = 1;
                } else {
                    int r = gr, c = gc;
                    for (int k = d; k >= 0; --k) {
                        const uint32_t cell = pack(r, c);
                        path[k] = cell;
                        if (round_trip) path[2 * d - k] = cell;
                        if (k == 0) break;
                        // parent: neighbour with dist k-1 and the largest (h, row, col)
                        int br = -1, bc = -1, bh = -1;
                        const int nr[4] = {r, r - 1, r, r + 1}, nc[4] = {c - 1, c, c + 1, c};
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            if (nr[q] < 0 || nr[q] >= e.H || nc[q] < 0 || nc[q] >= W) continue;
                            if (dist[nr[q] * W + nc[q]] != k - 1) continue;
                            const int h = abs(nr[q] - gr) + abs(nc[q] - gc);
                            if (h > bh || (h == bh && (nr[q] > br || (nr[q] == br && nc[q] > bc)))) {
                                bh = h; br = nr[q]; bc = nc[q];
                            }
                        }
                        if (br < 0) {   // cannot happen for a consistent BFS image; never index with -1
                            atomicAdd(&e.counters[C_BAD_STATUS], 1u);
                            break;
                        }
                        r = br; c = bc;
                    }
                    e.hlen[b] = len;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}

static size_t search_lds(const DevEnv &e) { return (size_t)4 * ((e.H * e.W + 7) & ~7) * sizeof(int16_t); }

void launch_bfs(const DevEnv &e, int parity, bool all, hipStream_t s) {
    const long items = all ? (long)e.B * e.N : (long)e.B * e.N;
    int grid = (int)((items + 3) / 4);
    if (!all && grid > 256) grid = 256;   // grid-stride over the (device-counted) list
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(bfs_kernel, dim3(grid), dim3(256), search_lds(e), s, e, parity, all ? 1 : 0);
}

void launch_replan(const DevEnv &e, int parity, bool all, hipStream_t s) {
    int grid = (int)((e.B + 3) / 4);
    if (!all && grid > 256) grid = 256;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(replan_kernel, dim3(grid), dim3(256), search_lds(e), s, e, parity, all ? 1 : 0);
}

}  // namespace mapf
