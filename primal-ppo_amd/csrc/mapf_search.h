// primal-ppo_amd/csrc/mapf_search.h -- wave-level grid searches (device code).
//
// Two kinds of work item, both one wave each:
//  * makeBfsMap (mapf_gym.py:211-244) for an agent whose goal changed:
//    bfs[b][i] = obstacleMap copy with free cells -2, then the level-order
//    distance from the goal (goal = 0, even on an obstacle).
//  * the human's next path (Human.getAstarPath, mapf_gym.py:33-37, astar_4.py:
//    21-109) between hnext_start[b] and hnext_goal[b], into the path buffer
//    the human is NOT using (hcur[b] ^ 1).
//
// astar_4 as BFS + walk-back.  astar_4's heap pops in the total order of the
// keys (f, g, row, col) -- duplicate entries of one cell share their key, so
// the parent field of the heap tuple never matters -- and the pops are
// monotone under the consistent Manhattan heuristic; `parents[c]` is
// overwritten whenever new_g <= g_scores[c] (astar_4.py:58).  So parent(c) is
// the LAST expanded neighbour p with d(p) = d(c) - 1, i.e. the one with the
// largest key (h(p), row, col) -- every such p has a smaller key than c and is
// expanded before c is popped.  The path is therefore: BFS distances from the
// start (stopped at the goal's level), then a walk back from the goal taking,
// at each step, the neighbour at distance d-1 with the largest
// (manhattan-to-goal, row, col).  Pinned by tests/golden/g3_search.npz (the
// reference's own astar_4 outputs) and by the oracle's literal heap A*.
//
// Register-only BFS.  Grid rows live on the lanes (row r = lane + 64k, k < RW),
// each row a W-bit mask (u32 / u64 / 2 x u64).  One BFS level = one frontier
// dilation: horizontal neighbours by shifting the row, vertical neighbours by
// DPP wave_shr:1 / wave_shl:1.  A BFS map is written level by level into a
// per-wave LDS image (each lane stores the few cells its row gains at that
// level), then swept out coalesced.  The A* walk-back needs only d mod 4, kept
// as 2 bit planes in registers: the grid graph is bipartite, so two adjacent
// reachable cells differ by exactly one level and "d(p) == d(c) - 1" <=> p
// visited and d(p) = d(c) - 1 (mod 4).
#pragma once
#include "mapf_common.h"

namespace mapf {
namespace srch {

struct Row2 { uint64_t lo, hi; };

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
__device__ inline uint32_t r_shl1(uint32_t a) { return a << 1; }
__device__ inline uint64_t r_shl1(uint64_t a) { return a << 1; }
__device__ inline Row2 r_shl1(Row2 a) { return {a.lo << 1, (a.hi << 1) | (a.lo >> 63)}; }
__device__ inline uint32_t r_shr1(uint32_t a) { return a >> 1; }
__device__ inline uint64_t r_shr1(uint64_t a) { return a >> 1; }
__device__ inline Row2 r_shr1(Row2 a) { return {(a.lo >> 1) | (a.hi << 63), a.hi >> 1}; }
__device__ inline bool r_any(uint32_t a) { return a != 0; }
__device__ inline bool r_any(uint64_t a) { return a != 0; }
__device__ inline bool r_any(Row2 a) { return (a.lo | a.hi) != 0; }
__device__ inline uint32_t r_get(uint32_t a, int c) { return (a >> c) & 1u; }
__device__ inline uint32_t r_get(uint64_t a, int c) { return (uint32_t)((a >> c) & 1ull); }
__device__ inline uint32_t r_get(Row2 a, int c) {
    return c < 64 ? (uint32_t)((a.lo >> c) & 1ull) : (uint32_t)((a.hi >> (c - 64)) & 1ull);
}
template <class T> __device__ inline T r_bit(int c);
template <> __device__ inline uint32_t r_bit<uint32_t>(int c) { return 1u << c; }
template <> __device__ inline uint64_t r_bit<uint64_t>(int c) { return 1ull << c; }
template <> __device__ inline Row2 r_bit<Row2>(int c) { return c < 64 ? Row2{1ull << c, 0} : Row2{0, 1ull << (c - 64)}; }
template <class T> __device__ inline T r_zero() { return T{}; }
// lowest set column / clear it
__device__ inline int r_ctz(uint32_t a) { return __builtin_ctz(a); }
__device__ inline int r_ctz(uint64_t a) { return __builtin_ctzll(a); }
__device__ inline int r_ctz(Row2 a) { return a.lo ? __builtin_ctzll(a.lo) : 64 + __builtin_ctzll(a.hi); }
__device__ inline uint32_t r_pop(uint32_t a) { return a & (a - 1u); }
__device__ inline uint64_t r_pop(uint64_t a) { return a & (a - 1ull); }
__device__ inline Row2 r_pop(Row2 a) { return a.lo ? Row2{a.lo & (a.lo - 1ull), a.hi} : Row2{0ull, a.hi & (a.hi - 1ull)}; }

// lane i <- lane i-1 (DPP wave_shr:1) / lane i <- lane i+1 (wave_shl:1); edge lanes read 0
// (bound_ctrl: the edge lane writes 0 itself, so no zeroed destination is needed -- one
// v_mov fewer per word and BFS level)
__device__ inline uint32_t from_below(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, true);
}
__device__ inline uint32_t from_above(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, true);
}
__device__ inline uint64_t from_below(uint64_t x) {
    return ((uint64_t)from_below((uint32_t)(x >> 32)) << 32) | from_below((uint32_t)x);
}
__device__ inline uint64_t from_above(uint64_t x) {
    return ((uint64_t)from_above((uint32_t)(x >> 32)) << 32) | from_above((uint32_t)x);
}
__device__ inline Row2 from_below(Row2 x) { return {from_below(x.lo), from_below(x.hi)}; }
__device__ inline Row2 from_above(Row2 x) { return {from_above(x.lo), from_above(x.hi)}; }
__device__ inline uint32_t rdlane(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
__device__ inline uint64_t rdlane(uint64_t x, int l) {
    return ((uint64_t)rdlane((uint32_t)(x >> 32), l) << 32) | rdlane((uint32_t)x, l);
}
__device__ inline Row2 rdlane(Row2 x, int l) { return {rdlane(x.lo, l), rdlane(x.hi, l)}; }

template <class P>
__device__ inline uint64_t bits64_at(P row, int WW, int off) {
    const int w = off >> 5, s = off & 31;
    auto word = [&](int k) -> uint64_t { return (k < WW) ? (uint64_t)row[k] : 0xFFFFFFFFull; };
    const uint64_t a = word(w) | (word(w + 1) << 32);
    const uint64_t b = word(w + 2);
    return s == 0 ? a : ((a >> s) | (b << (64 - s)));
}
// free cells of map row r as a row mask; `bits` a global or LDS pointer to the padded rows
template <class P> __device__ inline uint64_t free_row64(const DevEnv &e, P bits, int r) {
    if (r >= e.H) return 0;
    const uint64_t f = ~bits64_at(bits + (size_t)(r + e.P) * e.WW, e.WW, e.P);
    return e.W >= 64 ? f : (f & ((1ull << e.W) - 1));
}
template <class T> struct FreeRow;
template <> struct FreeRow<uint64_t> {
    template <class P> __device__ static uint64_t get(const DevEnv &e, P bits, int r) { return free_row64(e, bits, r); }
};
template <> struct FreeRow<uint32_t> {
    template <class P> __device__ static uint32_t get(const DevEnv &e, P bits, int r) {
        return (uint32_t)free_row64(e, bits, r);
    }
};
template <> struct FreeRow<Row2> {
    template <class P> __device__ static Row2 get(const DevEnv &e, P bits, int r) {
        if (r >= e.H) return {0, 0};
        const P row = bits + (size_t)(r + e.P) * e.WW;
        Row2 f = {~bits64_at(row, e.WW, e.P), ~bits64_at(row, e.WW, e.P + 64)};
        if (e.W < 128) f.hi &= (1ull << (e.W - 64)) - 1;
        return f;
    }
};

// Level-synchronous BFS over free cells from (sr, sc).  V = visited rows,
// D[k] = bit k of each visited cell's distance.  Stops after the level that
// reaches (stop_r, stop_c) when stop_r >= 0 and returns that level; returns the
// last level otherwise (-1 if the stop cell was never reached).
template <class T, int RW, int K>
__device__ int bfs_planes(const T (&fre)[RW], int sr, int sc, int stop_r, int stop_c, T (&V)[RW], T (&D)[K][RW]) {
    const int lane = lane_id();
    T fr[RW];
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        fr[k] = (lane + 64 * k == sr) ? r_bit<T>(sc) : r_zero<T>();
        V[k] = fr[k];
#pragma unroll
        for (int q = 0; q < K; ++q) D[q][k] = r_zero<T>();
    }
    if (stop_r == sr && stop_c == sc) return 0;
    int d = 1;
    for (;; ++d) {
        T up[RW], dn[RW], nw[RW];
#pragma unroll
        for (int k = 0; k < RW; ++k) { up[k] = from_below(fr[k]); dn[k] = from_above(fr[k]); }
        if (RW == 2) {
            const T a = rdlane(fr[0], 63), b = rdlane(fr[RW - 1], 0);
            if (lane == 0) up[RW - 1] = a;      // row 64 <- row 63
            if (lane == 63) dn[0] = b;          // row 63 <- row 64
        }
        bool any = false, hit = false;
#pragma unroll
        for (int k = 0; k < RW; ++k) {
            nw[k] = r_andn(r_and(r_or(r_or(r_nb(fr[k]), up[k]), dn[k]), fre[k]), V[k]);
            any |= r_any(nw[k]);
            if (lane + 64 * k == stop_r && r_get(nw[k], stop_c)) hit = true;
        }
        if (__ballot(any) == 0ull) return stop_r >= 0 ? -1 : d - 1;
#pragma unroll
        for (int k = 0; k < RW; ++k) {
            V[k] = r_or(V[k], nw[k]);
            fr[k] = nw[k];
#pragma unroll
            for (int q = 0; q < K; ++q)
                if ((d >> q) & 1) D[q][k] = r_or(D[q][k], nw[k]);
        }
        if (stop_r >= 0 && __ballot(hit) != 0ull) return d;
    }
}

// makeBfsMap straight into an LDS image: `img` holds the map's -1 / -2 cells
// (obstacle / free); the start cell gets 0 and every cell reached at level d gets
// d, written by the lane holding its row as the level is found (a frontier row
// has few cells) -- no distance bit planes to maintain or decode.
template <class T, int RW>
__device__ void bfs_to_img(const T (&fre)[RW], int sr, int sc, int16_t *img, int W) {
    const int lane = lane_id();
    T fr[RW], V[RW];
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        fr[k] = (lane + 64 * k == sr) ? r_bit<T>(sc) : r_zero<T>();
        V[k] = fr[k];
    }
    if ((sr & 63) == lane) img[sr * W + sc] = 0;
    for (int d = 1;; ++d) {
        T up[RW], dn[RW], nw[RW];
#pragma unroll
        for (int k = 0; k < RW; ++k) { up[k] = from_below(fr[k]); dn[k] = from_above(fr[k]); }
        if (RW == 2) {
            const T a = rdlane(fr[0], 63), b = rdlane(fr[RW - 1], 0);
            if (lane == 0) up[RW - 1] = a;      // row 64 <- row 63
            if (lane == 63) dn[0] = b;          // row 63 <- row 64
        }
        bool any = false;
#pragma unroll
        for (int k = 0; k < RW; ++k) {
            nw[k] = r_andn(r_and(r_or(r_or(r_nb(fr[k]), up[k]), dn[k]), fre[k]), V[k]);
            any |= r_any(nw[k]);
        }
        if (__ballot(any) == 0ull) return;
#pragma unroll
        for (int k = 0; k < RW; ++k) {
            V[k] = r_or(V[k], nw[k]);
            fr[k] = nw[k];
            const int r = lane + 64 * k;
            for (T m = nw[k]; r_any(m); m = r_pop(m)) img[r * W + r_ctz(m)] = (int16_t)d;
        }
    }
}

// distance bit planes of the narrow-row BFS map (W <= 32: 12 planes cover any
// distance < 64 * 32 cells)
constexpr int KNARROW = 12;

// bit c of the row held by lane `ln` in slot `sl` (ln, sl, c wave-uniform): a v_readlane
__device__ inline uint32_t word_of(uint32_t x, int) { return x; }
__device__ inline uint32_t word_of(uint64_t x, int w) { return w ? (uint32_t)(x >> 32) : (uint32_t)x; }
__device__ inline uint32_t word_of(Row2 x, int w) {
    const uint64_t q = (w >> 1) ? x.hi : x.lo;
    return (w & 1) ? (uint32_t)(q >> 32) : (uint32_t)q;
}
template <class T, int RW>
__device__ inline uint32_t row_bit(const T (&m)[RW], int sl, int ln, int c) {
    const uint32_t w = word_of(sl ? m[RW - 1] : m[0], c >> 5);
    return ((uint32_t)__builtin_amdgcn_readlane((int)w, ln) >> (c & 31)) & 1u;
}

// byte t (cells 8t .. 8t+7) of a row mask
__device__ inline uint32_t row_byte(uint32_t x, int t) { return (x >> (8 * t)) & 0xFFu; }
__device__ inline uint32_t row_byte(uint64_t x, int t) { return (uint32_t)(x >> (8 * t)) & 0xFFu; }
__device__ inline uint32_t row_byte(Row2 x, int t) { return row_byte(t < 8 ? x.lo : x.hi, t & 7); }

// 8 x 8 bit-matrix transpose: bit j of byte i <-> bit i of byte j
__device__ inline uint64_t transpose8(uint64_t x) {
    uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
    x ^= t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
    x ^= t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
    return x ^ t ^ (t << 28);
}

// makeBfsMap out of registers: the distance bit planes D (bfs_planes), visited V and free
// rows `fre` of the rows this lane holds, decoded straight into the 8x8 tiles (bfs_at) --
// one 16-B store per tile row, issued by the lane holding that row.  Per tile row: the
// byte of each plane over its 8 cells, one 8 x 8 transpose per 8 planes (cell j's
// distance bits), then -2 / -1 for the unreached free / obstacle cells.  Replaces the
// level-by-level LDS image, whose per-level cell stores (a divergent loop per level) set
// the BFS's pace.
template <class T, int RW, int K>
__device__ inline void planes_to_tiles(const T (&V)[RW], const T (&fre)[RW], const T (&D)[K][RW], int kq, int H,
                                       int W, uint4 *__restrict__ dst) {
    const int lane = lane_id();
    const int TW = bfs_tw(W), rows = ((H + 7) >> 3) << 3;
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        const int r = lane + 64 * k;
        if (r >= rows) continue;                     // rows H .. rows-1 decode to -1 (no free / visited bits)
        uint4 *row = dst + (size_t)(r >> 3) * TW * 8 + (r & 7);
        for (int tc = 0; tc < TW; ++tc) {
            const uint32_t un = ~row_byte(V[k], tc) & 0xFFu, fb = row_byte(fre[k], tc);
            uint64_t lo = 0, hi = 0;
#pragma unroll
            for (int q = 0; q < (K < 8 ? K : 8); ++q) lo |= (uint64_t)row_byte(D[q][k], tc) << (8 * q);
            lo = transpose8(lo);
            if (K > 8 && kq > 8) {
#pragma unroll
                for (int q = 8; q < K; ++q) hi |= (uint64_t)row_byte(D[q][k], tc) << (8 * (q - 8));
                hi = transpose8(hi);
            }
            uint32_t o[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint32_t lw = (uint32_t)(lo >> (32 * (m >> 1))), hw = (uint32_t)(hi >> (32 * (m >> 1)));
                const int a = (2 * m) & 3, j = 2 * m;
                const uint32_t x = ((lw >> (8 * a)) & 0xFFu) | (((hw >> (8 * a)) & 0xFFu) << 8) |
                                   (((lw >> (8 * a + 8)) & 0xFFu) << 16) | (((hw >> (8 * a + 8)) & 0xFFu) << 24);
                const uint32_t um = (((un >> j) & 1u) ? 0xFFFFu : 0u) | (((un >> (j + 1)) & 1u) ? 0xFFFF0000u : 0u);
                const uint32_t fm = ((fb >> j) & 1u) | (((fb >> (j + 1)) & 1u) << 16);
                o[m] = x | (um & ~fm);                 // unreached: free -2, obstacle -1
            }
            row[tc * 8] = make_uint4(o[0], o[1], o[2], o[3]);
        }
    }
}

// distance planes of the register BFS map of u64 / two-u64 rows: distances < 512 (mazes
// deeper than that take the LDS image)
constexpr int KWIDE = 9;

// LDS bytes one wave needs
template <class T, int RW>
__host__ __device__ inline size_t wave_lds(int H, int W) {
    const size_t planes = 3 * (size_t)64 * RW * sizeof(T);
    const size_t img = (size_t)((H * W + 7) & ~7) * 2;
    return ((planes > img ? planes : img) + 15) & ~(size_t)15;
}

// One search item on one wave (wave-uniform arguments):
//   replan = false: makeBfsMap of agent ai (env b) from its goal sr_cell into bfs[ai];
//   replan = true:  env b's human path sr_cell -> stop_cell into path buffer `buf`,
//                   its length into hlen[b][buf]; returns that length (0 for a BFS map).
// `lds` = wave_lds<T, RW>(H, W) bytes of this wave's LDS; `map` = the env's padded
// obstacle rows if the caller holds a copy (e.g. in LDS), else read from HBM.
template <class T, int RW>
__device__ __attribute__((always_inline)) inline int search_one(const DevEnv &e, bool replan, int b, uint32_t ai, uint32_t sr_cell, uint32_t stop_cell,
                          int buf, char *lds, const uint32_t *map = nullptr) {
    const int lane = lane_id();
    const int W = e.W, H = e.H;
    int len = 0;
    {
        // the map rows from the caller's LDS copy (typed, so the reads are ds_* and never
        // wait behind the wave's global stores), else from HBM
        T fre[RW];
        if (map) {
            const auto bits = as_lds(const_cast<uint32_t *>(map));
#pragma unroll
            for (int k = 0; k < RW; ++k) fre[k] = FreeRow<T>::get(e, bits, lane + 64 * k);
        } else {
            const uint32_t *bits = env_map(e, b);
#pragma unroll
            for (int k = 0; k < RW; ++k) fre[k] = FreeRow<T>::get(e, bits, lane + 64 * k);
        }
        const int sr = prow(sr_cell), sc = pcol(sr_cell);
        if (!replan) {
            uint4 *dst = reinterpret_cast<uint4 *>(e.bfs + (size_t)ai * bfs_cells(H, W));
            // distances as bit planes in registers, decoded straight into the tiles
            constexpr int K = sizeof(T) == 4 ? KNARROW : KWIDE;
            bool done = false;
            {
                T V[RW], D[K][RW];
                const int maxd = bfs_planes<T, RW, K>(fre, sr, sc, -1, -1, V, D);
                if (sizeof(T) == 4 || maxd < (1 << K)) {
                    planes_to_tiles<T, RW, K>(V, fre, D, 32 - __builtin_clz((unsigned)maxd | 1u), H, W, dst);
                    done = true;
                }
            }
            if (!done) {
                // deeper than the planes hold: the map copy (-1 obstacle / -2 free) in an LDS
                // image, the BFS levels on top, then one coalesced sweep out
                int16_t *img = reinterpret_cast<int16_t *>(lds);
#pragma unroll
                for (int k = 0; k < RW; ++k) {
                    const int r = lane + 64 * k;
                    if (r < H)
                        for (int c = 0; c < W; ++c) img[r * W + c] = r_get(fre[k], c) ? (int16_t)-2 : (int16_t)-1;
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
                bfs_to_img<T, RW>(fre, sr, sc, img, W);
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
                // out in 8x8 tiles (bfs_at): one 16-B store per tile row, -1 past the map's edge
                const int TW = bfs_tw(W), nrows = (int)(bfs_cells(H, W) >> 3);
                for (int k = lane; k < nrows; k += 64) {
                    const int t = k >> 3, r = ((t / TW) << 3) | (k & 7), c0 = (t % TW) << 3;
                    uint4 v;
                    if ((W & 7) == 0 && r < H) {
                        v = *reinterpret_cast<const uint4 *>(img + r * W + c0);
                    } else {
                        uint32_t q[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int ca = c0 + 2 * j, cb = ca + 1;
                            const uint32_t lo = (r < H && ca < W) ? (uint16_t)img[r * W + ca] : 0xFFFFu;
                            const uint32_t hi = (r < H && cb < W) ? (uint16_t)img[r * W + cb] : 0xFFFFu;
                            q[j] = lo | (hi << 16);
                        }
                        v = make_uint4(q[0], q[1], q[2], q[3]);
                    }
                    dst[k] = v;
                }
            }
        } else {
            const int gr = prow(stop_cell), gc = pcol(stop_cell);
            T V2[RW], D2[2][RW];
            const int d = bfs_planes<T, RW, 2>(fre, sr, sc, gr, gc, V2, D2);
            // Predecessor masks per row: bit c of pX[k] = the X neighbour of cell (r, c) lies one
            // BFS level closer to the start (levels compared mod 4: bipartite grid, see header).
            T pL[RW], pR[RW], pU[RW], pD[RW];
            {
                T Lm[4][RW];
#pragma unroll
                for (int k = 0; k < RW; ++k) {
                    const T n0 = r_andn(V2[k], D2[0][k]), n1 = r_and(V2[k], D2[0][k]);
                    Lm[0][k] = r_andn(n0, D2[1][k]);
                    Lm[1][k] = r_andn(n1, D2[1][k]);
                    Lm[2][k] = r_and(n0, D2[1][k]);
                    Lm[3][k] = r_and(n1, D2[1][k]);
                    pL[k] = pR[k] = pU[k] = pD[k] = r_zero<T>();
                }
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int pm = (m + 3) & 3;
                    T up[RW], dn[RW];
#pragma unroll
                    for (int k = 0; k < RW; ++k) { up[k] = from_below(Lm[pm][k]); dn[k] = from_above(Lm[pm][k]); }
                    if (RW == 2) {
                        const T a = rdlane(Lm[pm][0], 63), bb = rdlane(Lm[pm][RW - 1], 0);
                        if (lane == 0) up[RW - 1] = a;
                        if (lane == 63) dn[0] = bb;
                    }
#pragma unroll
                    for (int k = 0; k < RW; ++k) {
                        pL[k] = r_or(pL[k], r_and(Lm[m][k], r_shl1(Lm[pm][k])));
                        pR[k] = r_or(pR[k], r_and(Lm[m][k], r_shr1(Lm[pm][k])));
                        pU[k] = r_or(pU[k], r_and(Lm[m][k], up[k]));
                        pD[k] = r_or(pD[k], r_and(Lm[m][k], dn[k]));
                    }
                }
            }
            uint32_t *path = human_path(e, b, buf);
            if (d <= 0) {
                // start == goal (astar_4 returns []) or unreachable (it returns a ValueError):
                // the reference crashes right after; the human stays put for three steps (the
                // shortest round trip).  Never one: a 1-cell path is left the step after it is
                // switched to, i.e. before the search of the path after it -- deferred beside
                // the next step (mapf_api.cpp: join_deferred) -- is guaranteed done.
                if (lane == 0) {
                    atomicAdd(&e.counters[C_UNREACHABLE], 1u);
                    path[0] = sr_cell; path[1] = sr_cell; path[2] = sr_cell;
                }
                len = 3;
            } else {
                // walk back from the goal on the scalar unit: parent = predecessor neighbour with
                // the largest (manhattan-to-goal, row, col) -- astar_4's last overwrite (:58)
                const bool round_trip = e.human_mode != 2;
                len = round_trip ? 2 * d + 1 : d + 1;
                int r = gr, c = gc;
                for (int k = d; k >= 0; --k) {
                    const uint32_t cell = pack(r, c);
                    if (lane == 0) {
                        path[k] = cell;
                        if (round_trip) path[2 * d - k] = cell;
                    }
                    if (k == 0) break;
                    const int ln = r & 63, sl = r >> 6;
                    const uint32_t bl = row_bit(pL, sl, ln, c), br_ = row_bit(pR, sl, ln, c);
                    const uint32_t bu = row_bit(pU, sl, ln, c), bd = row_bit(pD, sl, ln, c);
                    int nr = -1, nc = -1, bh = -1;
                    auto cand = [&](uint32_t ok, int qr, int qc) {
                        if (!ok) return;
                        const int h = abs(qr - gr) + abs(qc - gc);
                        if (h > bh || (h == bh && (qr > nr || (qr == nr && qc > nc)))) { bh = h; nr = qr; nc = qc; }
                    };
                    cand(bl, r, c - 1); cand(bu, r - 1, c); cand(br_, r, c + 1); cand(bd, r + 1, c);
                    if (nr < 0) { if (lane == 0) atomicAdd(&e.counters[C_BAD_STATUS], 1u); break; }
                    r = nr; c = nc;
                }
            }
            if (lane == 0) e.hlen[b * 2 + buf] = len;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    return len;
}

// All search items of one step (or of a reset), grid-strided over waves.
//   all = 0: the step's work lists (parity); 1: every env's next path + every
//   agent's BFS map; 2: every env's next path only; 3: the step's human paths
//   only; 4: the step's BFS maps only.
template <class T, int RW>
__device__ void search_items(const DevEnv &e, int parity, int all, char *lds, uint32_t wave_id, uint32_t nwaves) {
    const bool every = all == 1 || all == 2;
    const uint32_t n_replan = every ? (uint32_t)e.B : (all == 4 ? 0u : e.counters[C_REPLAN_COUNT + parity]);
    const uint32_t n_bfs = (!e.keep_bfs || all == 2 || all == 3)
                               ? 0u : (every ? (uint32_t)(e.B * e.N) : e.counters[C_BFS_COUNT + parity]);
    const uint32_t total = n_replan + n_bfs;
    for (uint32_t item = wave_id; item < total; item += nwaves) {
        const bool replan = item < n_replan;
        uint32_t ai = 0, sr_cell, stop_cell = NO_CELL;
        int b, buf = 0;
        if (replan) {
            b = every ? (int)item : (int)e.replan_list[(size_t)parity * e.B + item];   // parity = list slot
            stop_cell = e.hnext_goal[b];
            if (stop_cell == NO_CELL) continue;
            sr_cell = e.hnext_start[b];
            buf = e.hcur[b] ^ 1;
        } else {
            const uint32_t k = item - n_replan;
            ai = every ? k : e.bfs_list[(size_t)parity * e.B * e.N + k];
            b = (int)(ai / (uint32_t)e.N);
            sr_cell = e.goal[ai];
        }
        search_one<T, RW>(e, replan, b, ai, sr_cell, stop_cell, buf, lds);
    }
}

}  // namespace srch
}  // namespace mapf
