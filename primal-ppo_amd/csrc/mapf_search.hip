// primal-ppo_amd/csrc/mapf_search.hip -- BFS distance maps and human A* paths.
//
// ONE kernel serves both searches a step can trigger (work lists filled by
// step_kernel; at reset: every env and every agent):
//  * makeBfsMap (mapf_gym.py:211-244) for every agent whose goal changed:
//    bfs[b][i] = obstacleMap copy with free cells -2, then the level-order
//    distance from the goal (goal = 0).
//  * Human.getAstarPath (mapf_gym.py:33-37; astar_4.py:21-109) for every
//    human that reached the end of its path and drew a new goal.  astar_4's
//    heap pops in the total order of the keys (f, g, row, col) -- duplicate
//    entries of one cell share their key, so the parent field of the heap
//    tuple never matters -- and pops are monotone under the consistent
//    Manhattan heuristic; `parents[c]` is overwritten whenever
//    new_g <= g_scores[c] (astar_4.py:58).  Hence parent(c) is the LAST
//    expanded neighbour p with d(p) = d(c) - 1, i.e. the one with the largest
//    key (h(p), row, col): every such p has a smaller key than c and is
//    expanded before c.  astar_4's path is therefore: BFS distances from the
//    start (stopped at the goal's level), then a walk back from the goal
//    taking at each step the neighbour with distance d-1 and the largest
//    (manhattan-to-goal, row, col).  Pinned by tests/golden/g3_search.npz
//    (the reference's own astar_4 outputs) and the oracle's literal heap A*.
//
// Layout: one wave per work item; grid rows on the lanes (row r = lane + 64k,
// k < RW), each row a W-bit mask in registers (u32 / u64 / 2 x u64).  One BFS
// level = one frontier dilation: horizontal neighbours by shifting the row,
// vertical neighbours by DPP wave_shr:1 / wave_shl:1 (no LDS round trip).
// Distances land in a per-wave LDS image initialised from a precomputed
// init image (obstacle -1 / free -2) by 16-byte copies, and leave (BFS maps)
// as one 16-byte-per-lane sweep.
#include "mapf_common.h"
#include "mapf_kernels.h"

namespace mapf {

namespace {

struct Row2 { uint64_t lo, hi; };

// ---- row operations for the three row widths ------------------------------
__device__ inline uint32_t r_or(uint32_t a, uint32_t b) { return a | b; }
__device__ inline uint64_t r_or(uint64_t a, uint64_t b) { return a | b; }
__device__ inline Row2 r_or(Row2 a, Row2 b) { return {a.lo | b.lo, a.hi | b.hi}; }
__device__ inline uint32_t r_and(uint32_t a, uint32_t b) { return a & b; }
__device__ inline uint64_t r_and(uint64_t a, uint64_t b) { return a & b; }
__device__ inline Row2 r_and(Row2 a, Row2 b) { return {a.lo & b.lo, a.hi & b.hi}; }
__device__ inline uint32_t r_andn(uint32_t a, uint32_t b) { return a & ~b; }
__device__ inline uint64_t r_andn(uint64_t a, uint64_t b) { return a & ~b; }
__device__ inline Row2 r_andn(Row2 a, Row2 b) { return {a.lo & ~b.lo, a.hi & ~b.hi}; }
__device__ inline uint32_t r_nb(uint32_t a) { return (a << 1) | (a >> 1); }
__device__ inline uint64_t r_nb(uint64_t a) { return (a << 1) | (a >> 1); }
__device__ inline Row2 r_nb(Row2 a) {
    return {(a.lo << 1) | (a.lo >> 1) | (a.hi << 63), (a.hi << 1) | (a.hi >> 1) | (a.lo >> 63)};
}
__device__ inline bool r_any(uint32_t a) { return a != 0; }
__device__ inline bool r_any(uint64_t a) { return a != 0; }
__device__ inline bool r_any(Row2 a) { return (a.lo | a.hi) != 0; }
__device__ inline bool r_test(uint32_t a, int c) { return (a >> c) & 1u; }
__device__ inline bool r_test(uint64_t a, int c) { return (a >> c) & 1ull; }
__device__ inline bool r_test(Row2 a, int c) { return c < 64 ? ((a.lo >> c) & 1ull) : ((a.hi >> (c - 64)) & 1ull); }
template <class T> __device__ inline T r_bit(int c);
template <> __device__ inline uint32_t r_bit<uint32_t>(int c) { return 1u << c; }
template <> __device__ inline uint64_t r_bit<uint64_t>(int c) { return 1ull << c; }
template <> __device__ inline Row2 r_bit<Row2>(int c) { return c < 64 ? Row2{1ull << c, 0} : Row2{0, 1ull << (c - 64)}; }
template <class T> __device__ inline T r_zero() { return T{}; }

// DPP cross-lane moves: lane i receives lane i-1 (wave_shr:1) / lane i+1 (wave_shl:1); edge lanes get 0.
__device__ inline uint32_t dpp_from_below(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, false);
}
__device__ inline uint32_t dpp_from_above(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false);
}
__device__ inline uint64_t dpp_from_below(uint64_t x) {
    return ((uint64_t)dpp_from_below((uint32_t)(x >> 32)) << 32) | dpp_from_below((uint32_t)x);
}
__device__ inline uint64_t dpp_from_above(uint64_t x) {
    return ((uint64_t)dpp_from_above((uint32_t)(x >> 32)) << 32) | dpp_from_above((uint32_t)x);
}
__device__ inline Row2 dpp_from_below(Row2 x) { return {dpp_from_below(x.lo), dpp_from_below(x.hi)}; }
__device__ inline Row2 dpp_from_above(Row2 x) { return {dpp_from_above(x.lo), dpp_from_above(x.hi)}; }
__device__ inline uint32_t rdlane(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
__device__ inline uint64_t rdlane(uint64_t x, int l) {
    return ((uint64_t)rdlane((uint32_t)(x >> 32), l) << 32) | rdlane((uint32_t)x, l);
}
__device__ inline Row2 rdlane(Row2 x, int l) { return {rdlane(x.lo, l), rdlane(x.hi, l)}; }

__device__ inline uint64_t bits64_at(const uint32_t *row, int WW, int off) {
    // 64 bits from bit `off` of a padded row of WW u32 words (past the end: 1s = obstacle)
    const int w = off >> 5, s = off & 31;
    auto word = [&](int k) -> uint64_t { return (k < WW) ? (uint64_t)row[k] : 0xFFFFFFFFull; };
    const uint64_t a = word(w) | (word(w + 1) << 32);
    const uint64_t b = word(w + 2);
    return s == 0 ? a : ((a >> s) | (b << (64 - s)));
}

template <class T> __device__ inline T free_row(const DevEnv &e, const uint32_t *bits, int r);
template <> __device__ inline uint64_t free_row<uint64_t>(const DevEnv &e, const uint32_t *bits, int r) {
    if (r >= e.H) return 0;
    const uint64_t f = ~bits64_at(bits + (size_t)(r + e.P) * e.WW, e.WW, e.P);
    return e.W >= 64 ? f : (f & ((1ull << e.W) - 1));
}
template <> __device__ inline uint32_t free_row<uint32_t>(const DevEnv &e, const uint32_t *bits, int r) {
    return (uint32_t)free_row<uint64_t>(e, bits, r);
}
template <> __device__ inline Row2 free_row<Row2>(const DevEnv &e, const uint32_t *bits, int r) {
    if (r >= e.H) return {0, 0};
    const uint32_t *row = bits + (size_t)(r + e.P) * e.WW;
    Row2 f = {~bits64_at(row, e.WW, e.P), ~bits64_at(row, e.WW, e.P + 64)};
    if (e.W < 128) f.hi &= (1ull << (e.W - 64)) - 1;
    return f;
}

template <class T>
__device__ inline void write_level(int16_t *dist, int W, int r, T m, int d);
template <>
__device__ inline void write_level<uint32_t>(int16_t *dist, int W, int r, uint32_t m, int d) {
    while (m) { const int c = __builtin_ctz(m); m &= m - 1; dist[r * W + c] = (int16_t)d; }
}
template <>
__device__ inline void write_level<uint64_t>(int16_t *dist, int W, int r, uint64_t m, int d) {
    while (m) { const int c = __builtin_ctzll(m); m &= m - 1; dist[r * W + c] = (int16_t)d; }
}
template <>
__device__ inline void write_level<Row2>(int16_t *dist, int W, int r, Row2 m, int d) {
    write_level<uint64_t>(dist, W, r, m.lo, d);
    write_level<uint64_t>(dist + 64, W, r, m.hi, d);
}

// Level-synchronous BFS over free cells from (sr, sc); writes levels >= 1 into
// dist (dist[start] is set by the caller).  Stops after the level that reaches
// (stop_r, stop_c) when stop_r >= 0.
template <class T, int RW>
__device__ void wave_bfs(const T (&fre)[RW], int sr, int sc, int16_t *dist, int W, int stop_r, int stop_c) {
    const int lane = lane_id();
    T fr[RW], vis[RW];
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        fr[k] = (lane + 64 * k == sr) ? r_bit<T>(sc) : r_zero<T>();
        vis[k] = fr[k];
    }
    for (int d = 1;; ++d) {
        T up[RW], dn[RW], nw[RW];
#pragma unroll
        for (int k = 0; k < RW; ++k) { up[k] = dpp_from_below(fr[k]); dn[k] = dpp_from_above(fr[k]); }
        if (RW == 2) {
            const T a = rdlane(fr[0], 63), b = rdlane(fr[RW - 1], 0);
            if (lane == 0) up[RW - 1] = a;       // row 64 <- row 63
            if (lane == 63) dn[0] = b;           // row 63 <- row 64
        }
        bool any = false, hit = false;
#pragma unroll
        for (int k = 0; k < RW; ++k) {
            nw[k] = r_andn(r_and(r_or(r_or(r_nb(fr[k]), up[k]), dn[k]), fre[k]), vis[k]);
            any |= r_any(nw[k]);
        }
        if (__ballot(any) == 0ull) break;
#pragma unroll
        for (int k = 0; k < RW; ++k) {
            vis[k] = r_or(vis[k], nw[k]);
            fr[k] = nw[k];
            write_level<T>(dist, W, lane + 64 * k, nw[k], d);
            if (lane + 64 * k == stop_r && r_test(nw[k], stop_c)) hit = true;
        }
        if (stop_r >= 0 && __ballot(hit) != 0ull) break;
    }
}

__device__ inline void copy_init(int16_t *dist, const int16_t *init, int cells_pad) {
    const uint4 *src = reinterpret_cast<const uint4 *>(init);
    uint4 *dst = reinterpret_cast<uint4 *>(dist);
    for (int k = lane_id(); k < cells_pad / 8; k += 64) dst[k] = src[k];
}

}  // namespace

template <class T, int RW>
__global__ __launch_bounds__(256) void search_kernel(DevEnv e, int parity, int all) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = lane_id();
    const int W = e.W, cells = e.H * e.W;
    const int cells_pad = (cells + 7) & ~7;
    int16_t *dist = reinterpret_cast<int16_t *>(smem) + (size_t)wave * cells_pad;
    const uint32_t n_replan = all ? (uint32_t)e.B : e.counters[C_REPLAN_COUNT + parity];
    const uint32_t n_bfs = !e.keep_bfs ? 0u : (all ? (uint32_t)(e.B * e.N) : e.counters[C_BFS_COUNT + parity]);
    const uint32_t total = n_replan + n_bfs;
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t item = blockIdx.x * (blockDim.x >> 6) + wave; item < total; item += nwaves) {
        const bool replan = item < n_replan;
        uint32_t ai = 0;
        int b;
        if (replan) {
            b = all ? (int)item : (int)e.replan_list[(size_t)parity * e.B + item];
        } else {
            const uint32_t k = item - n_replan;
            ai = all ? k : e.bfs_list[(size_t)parity * e.B * e.N + k];
            b = (int)(ai / (uint32_t)e.N);
        }
        const uint32_t *bits = env_map(e, b);
        const int16_t *init = e.bfs_init + (e.shared_map ? 0 : (size_t)b * cells_pad);
        T fre[RW];
#pragma unroll
        for (int k = 0; k < RW; ++k) fre[k] = free_row<T>(e, bits, lane + 64 * k);
        copy_init(dist, init, cells_pad);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (!replan) {
            // makeBfsMap from the agent's goal (the goal cell gets 0 even on an obstacle)
            const uint32_t gl = e.goal[ai];
            if (lane == 0) dist[prow(gl) * W + pcol(gl)] = 0;
            wave_bfs<T, RW>(fre, prow(gl), pcol(gl), dist, W, -1, -1);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            int16_t *outp = e.bfs + (size_t)ai * cells;
            if ((cells & 7) == 0) {
                const uint4 *src = reinterpret_cast<const uint4 *>(dist);
                uint4 *dst = reinterpret_cast<uint4 *>(outp);
                for (int k = lane; k < cells / 8; k += 64) dst[k] = src[k];
            } else {
                for (int k = lane; k < cells; k += 64) outp[k] = dist[k];
            }
        } else {
            const uint32_t st = e.hpos[b], gl = e.hgoal[b];
            const int gr = prow(gl), gc = pcol(gl);
            if (lane == 0) dist[prow(st) * W + pcol(st)] = 0;
            if (st != gl) wave_bfs<T, RW>(fre, prow(st), pcol(st), dist, W, gr, gc);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                uint32_t *path = e.hpath + (size_t)b * e.Lmax;
                const int d = (st == gl) ? -1 : dist[gr * W + gc];
                if (d <= 0) {
                    // start == goal (astar_4 returns []) or unreachable (it returns a
                    // ValueError): the reference crashes right after; keep the human put.
                    atomicAdd(&e.counters[C_UNREACHABLE], 1u);
                    path[0] = st;
                    e.hlen[b] = 1;
                } else {
                    const bool round_trip = e.human_mode != 2;
                    const int len = round_trip ? 2 * d + 1 : d + 1;
                    int r = gr, c = gc;
                    for (int k = d; k >= 0; --k) {
                        const uint32_t cell = pack(r, c);
                        path[k] = cell;
                        if (round_trip) path[2 * d - k] = cell;
                        if (k == 0) break;
                        // parent: neighbour at distance k-1 with the largest (h, row, col)
                        const int16_t vl = c > 0 ? dist[r * W + c - 1] : (int16_t)-9;
                        const int16_t vu = r > 0 ? dist[(r - 1) * W + c] : (int16_t)-9;
                        const int16_t vr = c + 1 < W ? dist[r * W + c + 1] : (int16_t)-9;
                        const int16_t vd = r + 1 < e.H ? dist[(r + 1) * W + c] : (int16_t)-9;
                        int br = -1, bc = -1, bh = -1;
                        auto cand = [&](int16_t v, int nr, int nc) {
                            if (v != k - 1) return;
                            const int h = abs(nr - gr) + abs(nc - gc);
                            if (h > bh || (h == bh && (nr > br || (nr == br && nc > bc)))) { bh = h; br = nr; bc = nc; }
                        };
                        cand(vl, r, c - 1); cand(vu, r - 1, c); cand(vr, r, c + 1); cand(vd, r + 1, c);
                        if (br < 0) { atomicAdd(&e.counters[C_BAD_STATUS], 1u); break; }
                        r = br; c = bc;
                    }
                    e.hlen[b] = len;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

template <class T, int RW>
static void launch_search_t(const DevEnv &e, int parity, bool all, hipStream_t s) {
    const size_t lds = (size_t)4 * ((e.H * e.W + 7) & ~7) * sizeof(int16_t);
    long items = all ? (long)e.B + (e.keep_bfs ? (long)e.B * e.N : 0) : (long)e.B + (e.keep_bfs ? (long)e.B * e.N : 0);
    long grid = (items + 3) / 4;
    const long cap = all ? 8192 : 128;   // step lists are short: a small grid-strided grid
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((search_kernel<T, RW>), dim3((unsigned)grid), dim3(256), lds, s, e, parity, all ? 1 : 0);
}

void launch_search(const DevEnv &e, int parity, bool all, hipStream_t s) {
    const bool two_rows = e.H > 64;
    if (e.W <= 32) {
        if (two_rows) launch_search_t<uint32_t, 2>(e, parity, all, s); else launch_search_t<uint32_t, 1>(e, parity, all, s);
    } else if (e.W <= 64) {
        if (two_rows) launch_search_t<uint64_t, 2>(e, parity, all, s); else launch_search_t<uint64_t, 1>(e, parity, all, s);
    } else {
        if (two_rows) launch_search_t<Row2, 2>(e, parity, all, s); else launch_search_t<Row2, 1>(e, parity, all, s);
    }
}

}  // namespace mapf
