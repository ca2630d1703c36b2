// primal-ppo_amd/csrc/mapf_group.h -- lane-group primitives.
//
// One environment = one group of G lanes (G = next pow2 >= N, G <= 64), lane
// i of the group = agent i, so a wave holds 64/G environments.  Every piece of
// the reference that is sequential over agents (getActionStatus's scan,
// fixActions' worklist, jointStep's goal draws) runs as a GROUP-UNIFORM loop:
// every lane of the group executes the same iterations, exchanging per-agent
// values with ds_bpermute (shfl) and 64-bit ballots restricted to the group.
#pragma once
#include "mapf_common.h"

namespace mapf {

struct Group {
    int G, base, i;          // group width, first lane of the group, agent slot
    uint64_t wmask;          // group's lanes within the wave ballot
    __device__ Group(int G_) : G(G_) {
        int lane = lane_id();
        base = lane & ~(G_ - 1);
        i = lane & (G_ - 1);
        wmask = (G_ == 64) ? ~0ull : (((1ull << G_) - 1ull) << base);
    }
    // bit j = predicate of agent j of this group
    __device__ uint64_t ballot(bool p) const { return (__ballot(p) & wmask) >> base; }
    __device__ uint32_t shfl(uint32_t v, int j) const { return shfl32(v, base + j); }
    __device__ int shfl_i(int v, int j) const { return (int)shfl32((uint32_t)v, base + j); }
    __device__ uint64_t shfl64(uint64_t v, int j) const { return mapf::shfl64(v, base + j); }
};

__device__ inline int ctz64(uint64_t x) { return __builtin_ctzll(x); }
__device__ inline int popc64(uint64_t x) { return __popcll(x); }
__device__ inline uint64_t below(int i) { return i >= 64 ? ~0ull : ((1ull << i) - 1ull); }
__device__ inline int nth_bit(unsigned m, int n) {  // position of the n-th set bit (n >= 0)
    for (int t = 0; t < 32; ++t)
        if ((m >> t) & 1u) { if (n == 0) return t; --n; }
    return -1;
}

// util.getFreeCell (util.py:67-76) as a specified Philox stream -- identical
// to oracle/mapf_oracle.c free_cell(): draw k uses counter
// (env, purpose | agent << 8, epoch, k); row = mulhi(w0, H), col = mulhi(w1, W);
// after FREECELL_TRIES rejections the last draw's w2 picks uniformly among
// the admissible cells in row-major order.  `ok(r, c)` must be group-uniform
// (it may ballot).  Returns false when no cell is admissible.
template <class Ok>
__device__ bool group_free_cell(const DevEnv &e, uint32_t env_id, uint32_t purpose, int agent, uint32_t epoch,
                                Ok ok, int &r, int &c) {
    u32x4 o = {0, 0, 0, 0};
    const uint32_t c1 = purpose | ((uint32_t)agent << 8);
    for (int k = 0; k < FREECELL_TRIES; ++k) {
        o = philox(env_id, c1, epoch, (uint32_t)k, e.seed);
        r = (int)__umulhi(o.x, (uint32_t)e.H);
        c = (int)__umulhi(o.y, (uint32_t)e.W);
        if (ok(r, c)) return true;
    }
    int cnt = 0;
    for (int rr = 0; rr < e.H; ++rr)
        for (int cc = 0; cc < e.W; ++cc)
            if (ok(rr, cc)) ++cnt;
    if (cnt == 0) return false;
    int pick = (int)__umulhi(o.z, (uint32_t)cnt);
    for (int rr = 0; rr < e.H; ++rr)
        for (int cc = 0; cc < e.W; ++cc)
            if (ok(rr, cc)) {
                if (pick == 0) { r = rr; c = cc; return true; }
                --pick;
            }
    return false;
}

// The path the human switches to when its current path ends.  The reference
// replans at that end-step (Human.nextStep -> getNextGoal, mapf_gym.py:25-31,
// :42-44; FixedPathHuman.getNextGoal :87-94); its goal draw depends only on
// the clock of that step, `epoch` = clock + len - 1 - hstep, so the path can be
// planned (and searched) ahead of time.  Mode 1: a fresh getFreeCell goal on the
// human's world (entrance marked) from the entrance; mode 2: the next scripted
// pose from the current one; mode 0 (LoopingHuman) never switches.
// hmode: the human mode if the caller has it as a constant (-1: e.human_mode);
// entr: the entrance cell if the caller holds it (have_entr), else read e.hentr[b].
__device__ inline void plan_next_path(const DevEnv &e, int b, uint32_t env_id, uint32_t epoch, int seq_idx,
                                      uint32_t &nstart, uint32_t &ngoal, bool leader, RegMap rm = RegMap{0u, false},
                                      int hmode = -1, uint32_t entr = 0u, bool have_entr = false) {
    nstart = NO_CELL;
    ngoal = NO_CELL;
    if (hmode < 0) hmode = e.human_mode;
    if (hmode == 1) {
        const uint32_t ent = have_entr ? entr : e.hentr[b];
        const uint32_t *bits = env_map(e, b);
        auto ok = [&](int r, int c) -> bool { return !rm.obstacle(e, bits, r, c) && pack(r, c) != ent; };
        int r, c;
        if (group_free_cell(e, env_id, P_HGOAL, 0, epoch, ok, r, c)) { nstart = ent; ngoal = pack(r, c); }
        else if (leader) atomicAdd(&e.counters[C_FREECELL], 1u);
    } else if (hmode == 2) {
        if (seq_idx + 1 < e.hseq_len[b]) {
            nstart = e.hseq[(size_t)b * e.HS + seq_idx];
            ngoal = e.hseq[(size_t)b * e.HS + seq_idx + 1];
        }
    }
}

// Step counters in LDS between the waves of one workgroup (persistent rollout kernels):
// volatile ds_read / ds_write, wave-uniform results.
__device__ inline uint32_t lds_count(const uint32_t *c) {
    return (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)*reinterpret_cast<volatile __attribute__((address_space(3))) uint32_t *>(as_lds(const_cast<uint32_t *>(c))));
}
// publish: every earlier LDS write of the wave lands before the counter moves
__device__ inline void publish_count(uint32_t *c, uint32_t v) {
    __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0)
    if (lane_id() == 0) *reinterpret_cast<volatile __attribute__((address_space(3))) uint32_t *>(as_lds(c)) = v;
}
// the smallest of the n (<= 64) counters p[0..n), wave-uniform
__device__ inline uint32_t group_min(const uint32_t *p, int n) {
    const int l = lane_id();
    uint32_t x = l < n ? *reinterpret_cast<volatile __attribute__((address_space(3))) uint32_t *>(
                             as_lds(const_cast<uint32_t *>(p + l)))
                       : 0xFFFFFFFFu;
    for (int o = 1; o < n; o <<= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o));
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
// pacing: wait until each of the n (<= 64) counters p[0..n) has reached v
__device__ inline void wait_group_min(const uint32_t *p, int n, uint32_t v) {
    const int l = lane_id();
    for (;;) {
        uint32_t x = l < n ? *reinterpret_cast<volatile __attribute__((address_space(3))) uint32_t *>(
                                 as_lds(const_cast<uint32_t *>(p + l)))
                           : 0xFFFFFFFFu;
        for (int o = 1; o < n; o <<= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o));
        if ((uint32_t)__builtin_amdgcn_readfirstlane((int)x) >= v) return;
        __builtin_amdgcn_s_sleep(1);
    }
}

}  // namespace mapf
