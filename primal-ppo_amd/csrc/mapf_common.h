// primal-ppo_amd/csrc/mapf_common.h -- device-side layout and helpers shared by
// the MAPF kernels (gfx950, wave64).
//
// HBM layout (Structure of Arrays, one handle = B lockstep envs):
//   map_bits  [nmaps][Hp][WW] u32   obstacle bitmap padded by P=max(F/2,1) cells
//                                   of 1s on every side (off-map == obstacle)
//   pos, goal [B*N] u32             packed cell (row | col << 16)
//   last_act  [B*N] i8              -1 = none (Agent.invalidActions[2] empty)
//   seq       [B*N*S] u32, seq_len/seq_cur [B*N]   agentsSequence
//   hpath     [B][2][Lmax] u32      human path, double buffered: hcur[b] is the
//                                   current path, the other buffer holds the path
//                                   the human will switch to at the end of it
//                                   (precomputed off the critical path)
//   hlen [B][2], hcur/hstep [B], hpos/hnext/hgoal/hentr [B], hnext_start/hnext_goal [B]
//   bfs       [B*N][TH][TW][8][8] i16  agent.bfsMap (keep_bfs) in 8x8-cell tiles, one
//                                   128-B L2 line each (bfs_at); cells past the map's
//                                   edge inside a tile hold -1
//   counters  [32] u32              error counters + work-list counts
//   replan_list [3][B], bfs_list [3][B*N]  per-step work lists, slot = step count mod 3
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mapf_diag.h"   // in-kernel phase stamps: no-ops unless built with -DMAPF_STAMPS

namespace mapf {

constexpr int NA = 5;           // EnvParameters.N_ACTIONS
constexpr int FREECELL_TRIES = 64;

// Agent.dirDict / oppositeAction (mapf_gym.py:97-100); x = row, y = col.
__host__ __device__ constexpr int dr(int a) { return a == 2 ? 1 : (a == 4 ? -1 : 0); }
__host__ __device__ constexpr int dc(int a) { return a == 1 ? 1 : (a == 3 ? -1 : 0); }
__host__ __device__ constexpr int opp(int a) { return a == 0 ? 0 : (a == 1 ? 3 : (a == 2 ? 4 : (a == 3 ? 1 : 2))); }

// Philox purposes (shared spec with oracle/mapf_oracle.c).
enum : uint32_t { P_ENTRANCE = 1, P_HGOAL0 = 2, P_START = 3, P_GOAL0 = 4, P_GOAL = 5,
                  P_HGOAL = 6, P_FIX = 7, P_ACT = 8, P_SAMPLE = 9, P_MAPGEN = 10 };

// counters[] slots
enum : int { C_BAD_ACTION = 0, C_FIX_BOUND = 1, C_EMPTY_VIABLE = 2, C_FREECELL = 3,
             C_UNREACHABLE = 4, C_BAD_STATUS = 5, C_PATH_OVERFLOW = 6,
             C_REPLAN_COUNT = 8,   // [8..10]  by work-list slot (step count mod 3)
             C_BFS_COUNT = 12,     // [12..14]
             C_NUM = 32 };

struct DevEnv {
    int B, N, H, W, F, C, P, Hp, WW, G, S, HS, Lmax;
    int use_da, use_hp, lifelong, human_mode, goal_mode, fix_choice, shared_map, keep_bfs, k_predict, R;
    float action_cost, collision_cost, human_collision_cost, repeat_cost, goal_reward;
    uint32_t env_offset;
    uint64_t seed;
    int constr_d2;            // largest d2 with (R - sqrt(d2)) / R >= 0.01 in fp64 (mapf_gym.py:633)
    int obs_envs;             // envs per observe workgroup
    int step_block;           // threads per step workgroup (64..256)
    int force_agent_lanes;    // use the agent-per-lane step kernel even for N <= 8 (testing)
    const uint32_t *map_bits;
    uint32_t *pos, *goal;
    int8_t *last_act;
    uint32_t *seq;
    int32_t *seq_len, *seq_cur;
    uint32_t *hpath;          // [B][2][Lmax]
    int32_t *hlen;            // [B][2]
    int32_t *hcur, *hstep;
    uint32_t *hpos, *hnext, *hgoal, *hentr;
    uint32_t *hnext_start, *hnext_goal;   // the next path's endpoints (NO_CELL = none)
    uint32_t *hseq;
    int32_t *hseq_len, *hseq_idx;
    uint32_t *hreplans, *clock;
    int16_t *bfs;
    uint32_t *counters, *replan_list, *bfs_list;
    unsigned long long *prof;  // [65536][8] per-wave phase cycles of the MAPF_STAMPS diagnostic build
    const float *cost_lut;    // [R*R+1]: float32(max(R - sqrt(d2), 0) / R) (fp64 like the reference)
    const uint8_t *smask;     // [nmaps][H*W]: static-invalid action mask of each cell (getInvalidActions[0])
    int search_blocks;        // workgroups of the observe launch that run search work
    int band_blocks;          // workgroups of the fused launch that write the zero band (0 = none)
};

constexpr uint32_t NO_CELL = 0xFFFFFFFFu;
// diagnostic buffer prof[]: [PROF_WAVES][8] per-wave phase cycles, then the
// fused kernel's block timeline [PROF_TL_BLOCKS][8] (MAPF_STAMPS builds only)
constexpr size_t PROF_WAVES = 65536, PROF_TL = PROF_WAVES * 8, PROF_TL_BLOCKS = 8192,
                 PROF_WORDS = PROF_TL + PROF_TL_BLOCKS * 8;

__host__ __device__ inline uint32_t pack(int r, int c) { return (uint32_t)(r & 0xFFFF) | ((uint32_t)c << 16); }
__host__ __device__ inline int prow(uint32_t p) { return (int)(p & 0xFFFF); }
__host__ __device__ inline int pcol(uint32_t p) { return (int)(p >> 16); }

// Philox4x32-10 (same constants/rounds as oracle/mapf_oracle.c: philox()).
struct u32x4 { uint32_t x, y, z, w; };
__device__ inline u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        // one v_mad_u64_u32 per product (hi and lo together), not mul_hi + mul_lo
        const uint64_t m0 = (uint64_t)0xD2511F53u * c0, m1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(m0 >> 32), lo0 = (uint32_t)m0;
        uint32_t hi1 = (uint32_t)(m1 >> 32), lo1 = (uint32_t)m1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}

// Uniform random policy (the env-only benchmark's actions): one Philox draw
// (env, P_ACT | (agent >> 3) << 8, clock, 0) serves 8 agents, agent i taking
// 16-bit half-word i & 7 of it, scaled to 0..4.  Shared spec with
// oracle/mapf_oracle.c: oc_random_actions().
__host__ __device__ inline int random_action(const u32x4 &o, int i) {
    const int k = i & 7;
    const uint32_t w = (k >> 1) == 0 ? o.x : (k >> 1) == 1 ? o.y : (k >> 1) == 2 ? o.z : o.w;
    return (int)((((w >> ((k & 1) * 16)) & 0xFFFFu) * (uint32_t)NA) >> 16);
}

// LDS-typed pointers.  A pointer the compiler cannot prove to be LDS is generic and its
// accesses compile to flat_* instructions, which also count in vmcnt: a flat read of LDS
// then waits behind the wave's outstanding global stores.
template <class T> using lds_ptr = __attribute__((address_space(3))) T *;
template <class T> __device__ inline lds_ptr<T> as_lds(T *p) { return (lds_ptr<T>)p; }

// Obstacle test on the padded bitmap (off-map cells read as 1 within P cells); `bits` a
// global, generic or LDS pointer.
template <class P>
__device__ inline bool obstacle_at(const DevEnv &e, P bits, int r, int c) {
    if (r < -e.P || r >= e.H + e.P || c < -e.P || c >= e.W + e.P) return true;
    int rr = r + e.P, cc = c + e.P;
    return (bits[rr * e.WW + (cc >> 5)] >> (cc & 31)) & 1u;
}
__device__ inline bool in_map(const DevEnv &e, int r, int c) { return r >= 0 && r < e.H && c >= 0 && c < e.W; }

__device__ inline const uint32_t *env_map(const DevEnv &e, int b) {
    return e.map_bits + (e.shared_map ? 0 : (size_t)b * e.Hp * e.WW);
}

// agent.bfsMap tiles: an F x F observation window (the BFS channel, ch 6) touches
// ~5 lines of 128 B on average (F = 11) where row-major int16 rows touched ~13.
__host__ __device__ inline int bfs_tw(int W) { return (W + 7) >> 3; }
__host__ __device__ inline size_t bfs_cells(int H, int W) { return (size_t)((H + 7) >> 3) * bfs_tw(W) * 64; }
__host__ __device__ inline int bfs_at(int W, int r, int c) {
    return ((((r >> 3) * bfs_tw(W)) + (c >> 3)) << 6) | ((r & 7) << 3) | (c & 7);
}

__device__ inline uint32_t *human_path(const DevEnv &e, int b, int buf) {
    return e.hpath + ((size_t)b * 2 + buf) * e.Lmax;
}
// Human.getNextPos (mapf_gym.py:46-50), maintained in hnext[b] by the step kernel.
__device__ inline uint32_t human_next(const DevEnv &e, int b) { return e.hnext[b]; }


// Wave-level helpers ---------------------------------------------------------
__device__ inline int lane_id() {   // volatile: never hoisted out of a loop (keeps per-lane invariants from pinning VGPRs)
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
__device__ inline uint64_t ballot(bool p) { return __ballot(p); }
__device__ inline uint32_t shfl32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }
__device__ inline uint64_t shfl64(uint64_t v, int src) {
    uint32_t lo = shfl32((uint32_t)v, src), hi = shfl32((uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

// The padded obstacle bitmap of a shared map held in registers: lane k of the
// wave holds word k (needs Hp*WW <= 64).  Tests are ds_bpermute reads of
// another lane, not HBM loads -- a step running while the chip streams
// observation stores would wait microseconds per loaded word.  Call only with
// every lane of the wave active (the source lanes must execute the permute).
struct RegMap {
    uint32_t w;
    bool on;
    __device__ bool obstacle(const DevEnv &e, const uint32_t *bits, int r, int c) const {
        if (!on) return obstacle_at(e, bits, r, c);
        const bool off = r < -e.P || r >= e.H + e.P || c < -e.P || c >= e.W + e.P;
        const int rr = off ? 0 : r + e.P, cc = off ? 0 : c + e.P;
        const uint32_t word = shfl32(w, rr * e.WW + (cc >> 5));     // every lane permutes
        return off || ((word >> (cc & 31)) & 1u);
    }
};
__host__ __device__ inline bool regmap_fits(const DevEnv &e) { return e.shared_map && e.Hp * e.WW <= 64; }

// torch's NaN semantics for the network's epilogues (fmaxf would turn a NaN into 0, so a
// NaN from an fp16 overflow would never reach the loss and GradScaler's found-inf):
// relu(x) = x <= 0 ? 0 : x  (NaN kept; -0 -> +0), the gradient mask likewise !(y <= 0);
// max_pool2d's running max: a NaN wins (val > max || isnan(val)).
__device__ inline float relu_nan(float v) { return (v > 0.f || v != v) ? v : 0.f; }
__device__ inline float max_nan(float m, float v) { return (v > m || v != v) ? v : m; }

}  // namespace mapf
