// primal-ppo_amd/csrc/mapf_step_pairs.h -- the step for N <= 8 agents per env.
//
// Same semantics as step_kernel (mapf_step.hip, which documents the reference
// lines), different mapping: one lane per ORDERED PAIR (i, j) of agents, NP*NP
// lanes per env (NP = next pow2 >= N), i.e. one env per wave at N = 8.  The
// pairwise part of getRestrictedActions / getTrainValid (mapf_gym.py:363-402,
// :535-550) is one lane's work instead of a loop over j; per-agent results are
// OR-reduced across the NP lanes of agent i's row.  Serial parts
// (getActionStatus's scan, fixActions' worklist) run on per-env uniform
// values.  8x the waves of the agent-per-lane kernel at N = 8: the latency of
// each wave's short dependent chains hides behind the others.
//
// Lane roles: row i = agent i (its NP lanes hold agent i's values, replicated),
// lane j of the row also holds agent j's values ("column" copies).  Outputs
// and state are written by lane j == 0 of each row.
#pragma once
#include "mapf_group.h"
#include "mapf_kernels.h"
#include "mapf_observe.h"
#include "mapf_pyset.h"

namespace mapf {

namespace pairs {

// bit of the action whose move is (dr, dc), 0 if none (|dr| + |dc| > 1)
__device__ inline unsigned abit(int r, int c) {
    if (r == 0 && c == 0) return 1u;
    if (r == 0 && c == 1) return 1u << 1;
    if (r == 1 && c == 0) return 1u << 2;
    if (r == 0 && c == -1) return 1u << 3;
    if (r == -1 && c == 0) return 1u << 4;
    return 0u;
}
// actions t of agent i with |p_i + d(t) - p_j|_1 <= 1, for p_j - p_i = (r, c)
__device__ inline unsigned keys_of(int r, int c) {
    unsigned m = 0;
#pragma unroll
    for (int t = 0; t < NA; ++t)
        if (abs(dr(t) - r) + abs(dc(t) - c) <= 1) m |= 1u << t;
    return m;
}

template <int NP>
__device__ inline uint32_t row_or(uint32_t v) {
#pragma unroll
    for (int s = 1; s < NP; s <<= 1) v |= (uint32_t)__shfl_xor((int)v, s, 64);
    return v;
}

}  // namespace pairs

// Work-list appends whose slot comes from a returning atomic (one wave-aggregated
// atomicAdd per list).  The step only issues the atomic; step_pairs_finish()
// reads its result and stores the items as late as the caller can (the fused
// kernel: after the observation stores), so no wave waits on the round trip.
struct PairsDeferred {
    uint64_t bmask = 0, rmask = 0;     // lanes appending to bfs_list / replan_list
    uint32_t bret = 0, rret = 0;       // the leader lane's atomicAdd result
    uint32_t bitem = 0, ritem = 0;
    // INLINE steps (the multi-step rollout kernel): no lists, the wave searches itself
    uint32_t bgoal = 0;                // the new goal of a bmask lane's agent
    uint32_t rstart = 0, rgoal = 0;    // the human's next path (wave-uniform)
    int rbuf = 0;                      // ... into this path buffer
};

// The state of one wave's env kept in registers across the steps of the
// multi-step rollout kernel (RES steps): no state loads at the top of a step, so
// a step never waits (vmcnt counts loads AND stores on gfx9) behind the previous
// step's observation stores.  The human's current path is copied into the wave's
// LDS (lp) whenever it switches, so the per-step path reads are LDS reads.
struct EnvRegs {
    uint32_t pi, pj, gi;          // per lane (i, j): cells of agents i and j, agent i's goal
    int la;                       //                  agent i's last action (-1 = none)
    float creg;                   //                  cost_lut[lane] (calculateCostReward's table in lanes)
    uint32_t clock, hp, hn, hng, hgoal, hstart, hentr, replans;   // per env (wave-uniform)
    int hs, hcur, hlen0, hlen1;
    uint32_t *lp;                 // LDS copy of path buffer hcur (Lmax cells)
};

// path buffer `buf` of env b (len cells) into the wave's LDS copy
__device__ inline void env_regs_path_to_lds(const DevEnv &e, int b, int buf, int len, uint32_t *lp) {
    const uint32_t *p = human_path(e, b, buf);
    for (int k = lane_id(); k < len; k += 64) lp[k] = p[k];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <int NP>
__device__ inline void env_regs_load(const DevEnv &e, int b, EnvRegs &r, uint32_t *lp) {
    const int lane = lane_id(), i = lane / NP, j = lane % NP;
    const bool vi = i < e.N, vj = j < e.N;
    const size_t ai = (size_t)b * e.N + i, aj = (size_t)b * e.N + j;
    r.pi = vi ? e.pos[ai] : 0u;
    r.pj = vj ? e.pos[aj] : 0u;
    r.gi = vi ? e.goal[ai] : 0u;
    r.la = vi ? (int)e.last_act[ai] : -1;
    const int RR = e.R * e.R;
    r.creg = RR < 64 ? e.cost_lut[lane <= RR ? lane : 0] : 0.f;
    r.clock = e.clock[b];
    r.hentr = e.hentr[b];
    r.hp = e.hpos[b];
    r.hn = e.hnext[b];
    r.hng = e.hnext_goal[b];
    r.hgoal = e.hgoal[b];
    r.hstart = e.hnext_start[b];
    r.replans = 0u;
    r.hs = e.hstep[b];
    r.hcur = e.hcur[b];
    r.hlen0 = e.hlen[(size_t)b * 2];
    r.hlen1 = e.hlen[(size_t)b * 2 + 1];
    r.lp = lp;
    env_regs_path_to_lds(e, b, r.hcur, r.hcur ? r.hlen1 : r.hlen0, lp);
}

template <int NP>
__device__ inline void env_regs_store(const DevEnv &e, int b, const EnvRegs &r) {
    const int lane = lane_id(), i = lane / NP, j = lane % NP;
    if (i < e.N && j == 0) {
        const size_t ai = (size_t)b * e.N + i;
        e.pos[ai] = r.pi;
        e.goal[ai] = r.gi;
        e.last_act[ai] = (int8_t)r.la;
    }
    if (lane == 0) {
        e.clock[b] = r.clock;
        e.hpos[b] = r.hp;
        e.hnext[b] = r.hn;
        e.hnext_goal[b] = r.hng;
        e.hgoal[b] = r.hgoal;
        e.hnext_start[b] = r.hstart;
        e.hreplans[b] += r.replans;
        e.hstep[b] = r.hs;
        e.hcur[b] = r.hcur;
    }
}

__device__ inline void step_pairs_finish(const DevEnv &e, const PairsDeferred &d, int slot) {
    const int lane = lane_id();
    if (d.bmask) {
        const uint32_t base = __builtin_amdgcn_readlane(d.bret, __builtin_ctzll(d.bmask));
        if ((d.bmask >> lane) & 1ull)
            e.bfs_list[(size_t)slot * e.B * e.N + base + __popcll(d.bmask & ((1ull << lane) - 1ull))] = d.bitem;
    }
    if (d.rmask) {
        const uint32_t base = __builtin_amdgcn_readlane(d.rret, __builtin_ctzll(d.rmask));
        if ((d.rmask >> lane) & 1ull)
            e.replan_list[(size_t)slot * e.B + base + __popcll(d.rmask & ((1ull << lane) - 1ull))] = d.ritem;
    }
}

// One env's step on its NP*NP lanes; `gt` = the lane's index among the step
// lanes of the launch (env = gt / (NP*NP)).  FEED: also hand the post-step
// cells, goals and human state to the workgroup's observation (LDS `ob`,
// whose first env is b0) -- the fused step+observe kernel; needs COMMIT.
//
// rm: the shared map in registers (NP = 8 only: one env per wave, so every
// lane takes part in each map read); dfr: the deferred list appends.
// INLINE (NP = 8, the multi-step rollout kernel): no work lists -- the search
// items are left in dfr for step_pairs_search_inline() on the same wave.
// RES (with INLINE): the env state lives in *rs (EnvRegs) instead of HBM.
template <int NP, bool FEED, bool INLINE = false, bool RES = false>
__device__ __forceinline__ void step_pairs_env(const DevEnv &e, int32_t *__restrict__ actions, const StepOut &out,
                                               uint32_t flags, int slot, int gt, const ObsLds &ob, int b0,
                                               RegMap rm, PairsDeferred &dfr, EnvRegs *rs = nullptr) {
    using namespace pairs;
    constexpr int L = NP * NP;
    constexpr uint32_t ROW = (1u << NP) - 1u;
    const int N = e.N;
    // one env per wave at NP = 8: make the env index (and everything derived from
    // per-env loads) wave-uniform, i.e. scalar registers / SALU, not 64 VALU lanes
    const int b = (L == 64) ? __builtin_amdgcn_readfirstlane(gt / L) : gt / L;
    if (!INLINE && gt == 0 && (flags & 1u)) {
        e.counters[C_REPLAN_COUNT + (slot + 1) % 3] = 0;
        e.counters[C_BFS_COUNT + (slot + 1) % 3] = 0;
    }
    if (b >= e.B) return;
    STAMP_BEGIN();
    const int lane = lane_id();
    const int base = lane & ~(L - 1), li = lane - base;
    const int i = li / NP, j = li % NP;
    const uint64_t emask = (L == 64) ? ~0ull : (((1ull << L) - 1ull) << base);
    auto eballot = [&](bool p) -> uint64_t { return (__ballot(p) & emask) >> base; };   // bit (k*NP + m)
    auto agents_of = [&](uint64_t m) -> uint32_t {   // stride-NP row-0 bits -> compact agent mask
        if constexpr (NP == 8) {     // gather bit 8k -> k in three shift-or folds (not eight extracts)
            m &= 0x0101010101010101ull;
            m |= m >> 7;
            m |= m >> 14;
            m |= m >> 28;
            return (uint32_t)m & 0xFFu;
        }
        uint32_t a = 0;
#pragma unroll
        for (int k = 0; k < NP; ++k) a |= (uint32_t)((m >> (k * NP)) & 1ull) << k;
        return a;
    };
    const bool vi = i < N, vj = j < N;
    const bool head = j == 0;               // lane that writes agent i's outputs
    const size_t ai = (size_t)b * N + i, aj = (size_t)b * N + j;
    const uint32_t env_id = e.env_offset + (uint32_t)b;
    // ---- every per-env / per-agent load is issued here, in two dependent rounds
    const uint32_t clock = RES ? rs->clock : e.clock[b];
    // calculateCostReward's table (cost_lut[d2], d2 <= R*R) in lanes: lane k holds
    // entry k, read with one permute instead of an fp64 sqrt + divide per lane
    const int RR = e.R * e.R;
    const bool lutreg = L == 64 && RR < 64;      // one env per wave: every lane is active
    const float creg = !lutreg ? 0.f : RES ? rs->creg : e.cost_lut[lane_id() <= RR ? lane_id() : 0];
    const uint32_t hp = RES ? rs->hp : e.hpos[b], hn = RES ? rs->hn : e.hnext[b];
    const int hs = RES ? rs->hs : e.hstep[b], hcur = RES ? rs->hcur : e.hcur[b];
    const int2 hlen2 = RES ? make_int2(rs->hlen0, rs->hlen1) : *reinterpret_cast<const int2 *>(e.hlen + (size_t)b * 2);
    // RES: human modes 0 / 1 and random goals only (rollout_fusable), so the scripted
    // human's and the goal sequences' loads are compiled out of the rollout loop
    const int hmode = RES ? (e.human_mode == 1 ? 1 : 0) : e.human_mode;
    const int gmode = RES ? 1 : e.goal_mode;
    const uint32_t hng = hmode == 1 ? (RES ? rs->hng : e.hnext_goal[b]) : NO_CELL;
    const int hsi = hmode == 2 ? e.hseq_idx[b] : 0, hsl = hmode == 2 ? e.hseq_len[b] : 0;

    const uint32_t pi = RES ? rs->pi : (vi ? e.pos[ai] : 0u), pj = RES ? rs->pj : (vj ? e.pos[aj] : 0u);
    const int ri = prow(pi), ci = pcol(pi), rj = prow(pj), cj = pcol(pj);
    const uint32_t gi = RES ? rs->gi : (vi ? e.goal[ai] : 0u);
    const int la = RES ? rs->la : (vi ? (int)e.last_act[ai] : -1);
    int a_i, a_j;
    if (flags & 2u) {                       // random policy: one env-uniform Philox draw for all N <= 8 agents
        const u32x4 o = philox(env_id, P_ACT, clock, 0u, e.seed);
        a_i = random_action(o, i);
        a_j = random_action(o, j);
        if (vi && head) actions[ai] = a_i;
    } else {
        a_i = vi ? actions[ai] : 0;
        a_j = vj ? actions[aj] : 0;
        if (vi && head && (a_i < 0 || a_i >= NA)) atomicAdd(&e.counters[C_BAD_ACTION], 1u);
        if (a_i < 0 || a_i >= NA) a_i = 0;
        if (a_j < 0 || a_j >= NA) a_j = 0;
    }
    // human.nextStep does not depend on the agents: decide it now, issue its path loads in round 2
    const int Lc = hcur ? hlen2.y : hlen2.x;
    int cur2 = hcur, hs2 = hs + 1, seq_idx = 0;
    bool swapped = false, at_end = hs >= Lc - 1;
    if (at_end) {
        hs2 = 0;
        if (hmode == 1) {
            if (hng != NO_CELL) { cur2 = hcur ^ 1; swapped = true; }
        } else if (hmode == 2) {
            seq_idx = hsi + 1;
            if (seq_idx < hsl) { cur2 = hcur ^ 1; swapped = true; }
        }
    }
    const int L2 = cur2 ? hlen2.y : hlen2.x;
    const uint32_t *p2 = human_path(e, b, cur2);
    if (RES && cur2 != hcur) env_regs_path_to_lds(e, b, cur2, L2, rs->lp);   // the path switches
    const uint32_t *p2r = RES ? rs->lp : p2;                                  // ... read from LDS
    const uint32_t hp_new = p2r[hs2];
    const uint32_t hn_new = p2r[hs2 + 1 < L2 ? hs2 + 1 : L2 - 1];
    unsigned st_mask = 0x1Fu;
    if (rm.on) {                            // getInvalidActions' static list from the register map
        unsigned m = 0;
#pragma unroll
        for (int k = 1; k < NA; ++k) m |= (unsigned)rm.obstacle(e, nullptr, ri + dr(k), ci + dc(k)) << k;
        if (vi) st_mask = m;
    } else if (vi) {
        st_mask = (unsigned)e.smask[(e.shared_map ? 0 : (size_t)b * e.H * e.W) + ri * e.W + ci];
    }
    unsigned hu_mask = 0;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        if ((st_mask >> k) & 1u) continue;
        const uint32_t x = pack(ri + dr(k), ci + dc(k));
        if (x == hn || (pi == hn && x == hp)) hu_mask |= 1u << k;
    }
    const unsigned rep_mask = la >= 0 ? 1u << opp(la) : 0u;
    STAMP(0);

    // ---- the pair (i, j): restricted-action keys and conflicts with j's actual action
    unsigned kij = 0, cij = 0;
    if (vi && vj && i != j) {
        const int r = rj - ri, c = cj - ci;
        if (abs(r) + abs(c) <= 2) {
            kij = keys_of(r, c);
            const int er = r + dr(a_j), ec = c + dc(a_j);        // Y_j - p_i
            cij = abit(er, ec);                                   // vertex: p_i + d(t) == Y_j
            if (er == 0 && ec == 0) cij |= abit(r, c);            // swap: p_i + d(t) == p_j, Y_j == p_i
        }
    }
    const uint64_t Mb = eballot((cij >> a_i) & 1u);                 // M_i = bits [i*NP, i*NP+NP)
    const uint32_t kc = row_or<NP>(kij | (cij << 8));
    const unsigned keys = kc & 0x1Fu, conf = (kc >> 8) & 0x1Fu;
    const unsigned good = ~(st_mask | hu_mask | rep_mask | keys) & 0x1Fu;
    const uint32_t Mi = (uint32_t)(Mb >> (i * NP)) & ROW;
    STAMP(1);

    // ---- getActionStatus
    int s0;
    bool cb = false;
    if ((st_mask >> a_i) & 1u) s0 = -1;
    else if ((hu_mask >> a_i) & 1u) s0 = -2;
    else if ((good >> a_i) & 1u) s0 = 1;
    else if (Mi) { s0 = -3; cb = true; }
    else s0 = ((rep_mask >> a_i) & 1u) ? -4 : 1;
    const uint32_t cbm = agents_of(eballot(head && vi && cb));
    uint32_t T = 0;
    for (uint32_t rem = cbm; rem; rem &= rem - 1) {
        const int k = __builtin_ctz(rem);
        if (!((T >> k) & 1u)) T |= ((uint32_t)(Mb >> (k * NP)) & ROW) | (1u << k);
    }
    const int st = ((T >> i) & 1u) ? -3 : s0;

    // selects, not a switch (each case's branch reloaded spilled scalars: step_group)
    float c_act = e.action_cost, c_rep = e.repeat_cost, c_col = e.collision_cost, c_hum = e.human_collision_cost;
    asm volatile("" : "+s"(c_act), "+s"(c_rep), "+s"(c_col), "+s"(c_hum));
    float rw = c_act;
    rw = st == -4 ? c_rep : rw;
    rw = (st == -1 || st == -3) ? c_col : rw;
    rw = st == -2 ? c_hum : rw;
    const int Xr = ri + dr(a_i), Xc = ci + dc(a_i);
    const uint32_t shadow = agents_of(eballot(head && vi && st == 1 && Xr == prow(gi) && Xc == pcol(gi)));
    float cost = 0.f;
    {   // max(R - ||h - x||, 0) / R in float64, then float32 (mapf_gym.py:513-526)
        const int d0 = prow(hn) - Xr, d1 = pcol(hn) - Xc;
        const int d2 = d0 * d0 + d1 * d1;
        if (lutreg) {
            const float c = __shfl(creg, d2 < RR ? d2 : 0, 64);    // every lane permutes
            cost = d2 < RR ? c : 0.f;
        } else if (d2 < RR) {
            cost = (float)(((double)e.R - sqrt((double)d2)) / (double)e.R);
        }
    }
    if (vi) {
        if (head) {
            if (out.status) out.status[ai] = (int8_t)st;
            if (out.reward) out.reward[ai] = rw;
            if (out.cost) out.cost[ai] = cost;
        }
        if (out.train_valid) {
            float *tv = out.train_valid + ai * NA;
            for (int t = j; t < NA; t += NP)
                tv[t] = (((good >> t) & 1u) || (((keys >> t) & 1u) && !((conf >> t) & 1u))) ? 1.f : 0.f;
        }
    }
    if (li == 0 && out.shadow_goals) out.shadow_goals[b] = __popc(shadow);
    STAMP(2);
    if (!(flags & 1u)) return;

    // ---- fixActions (worklist; agent values row-replicated, j's copies in column).
    // Same semantics as step_kernel (mapf_step.hip): reference set order for a
    // two-agent eviction (mapf_pyset.h), empty viable set -> stay, deadlock after
    // fix_draws(N) draws -> unplaced agents stay, blocked movers revert.
    int fixed = a_i;
    const uint32_t need = agents_of(eballot(head && vi && (st == -1 || st == -2 || st == -3)));
    if (need) {
        const int st_j = (int)shfl32((uint32_t)st, base + j * NP);
        const unsigned good_j = shfl32(good, base + j * NP);
        int asg_i = (vi && st == 1) ? a_i : -1;
        int asg_j = (vj && st_j == 1) ? a_j : -1;
        // worklist agents with a good action take its min at once (it collides with nothing:
        // it never enters U and is never evicted, so its turn decides nothing -- step_group)
        if (vi && st < 0 && good) asg_i = __builtin_ctz(good);
        if (vj && st_j < 0 && good_j) asg_j = __builtin_ctz(good_j);
        const uint32_t qm = agents_of(eballot(head && vi && st < 0 && !good));
        int q = (vi && st < 0 && !good) ? __popc(qm & ((1u << i) - 1u)) : -1;
        int next_q = __popc(qm), hd = 0, draws = 0;
        const unsigned viable_i = ~(st_mask | hu_mask) & 0x1Fu;
        while (hd < next_q) {
            const int idx = __builtin_ctz(agents_of(eballot(head && vi && q == hd)));
            const unsigned good_idx = shfl32(good, base + idx * NP);
            int newa = -1;
            uint32_t ev = 0;
            bool swap_ev = false;
            if (good_idx) {
                newa = __builtin_ctz(good_idx);
            } else {
                const unsigned viable = shfl32(viable_i, base + idx * NP);
                unsigned cjm = 0;          // in row idx: idx's actions colliding with agent j's assignment
                if (i == idx && vj && j != idx && asg_j >= 0) {
                    const int r = rj - ri, c = cj - ci;
                    if (abs(r) + abs(c) <= 2) {
                        const int er = r + dr(asg_j), ec = c + dc(asg_j);
                        cjm = abit(er, ec);
                        if (er == 0 && ec == 0) cjm |= abit(r, c);
                    }
                }
                unsigned U = 0;
#pragma unroll
                for (int t = 0; t < NA; ++t)
                    if (eballot((cjm >> t) & 1u)) U |= 1u << t;
                const unsigned fr = viable & ~U;
                if (fr) {
                    newa = __builtin_ctz(fr);
                } else {
                    if (draws >= fix_draws(N)) {      // deadlock: idx stays queued
                        if (li == 0) atomicAdd(&e.counters[C_FIX_BOUND], 1u);
                        break;
                    }
                    const int nv = __popc(viable);
                    newa = 0;
                    if (nv == 0) {
                        if (li == 0) atomicAdd(&e.counters[C_EMPTY_VIABLE], 1u);
                    } else {
                        int pick;
                        if (e.fix_choice == 0) pick = draws % nv;
                        else pick = (int)__umulhi(philox(env_id, P_FIX | ((uint32_t)idx << 8), clock, (uint32_t)draws,
                                                         e.seed).x, (uint32_t)nv);
                        newa = nth_bit(viable, pick);
                    }
                    ++draws;
                    ev = (uint32_t)(eballot((cjm >> newa) & 1u) >> (idx * NP)) & ROW;   // evicted agents
                    if (__builtin_expect(__popc(ev) == 2, 0)) {
                        // restrictedAction[idx][newa] of agent j, computed in row idx, moved to group lane j
                        unsigned rb = 0;
                        if (i == idx && vj && j != idx) {
                            const int Xr = ri + dr(newa), Xc = ci + dc(newa);
#pragma unroll
                            for (int t = 0; t < NA; ++t) {
                                const int yr = rj + dr(t), yc = cj + dc(t);
                                if ((yr == Xr && yc == Xc) || (Xr == rj && Xc == cj && yr == ri && yc == ci)) rb |= 1u << t;
                            }
                        }
                        const unsigned rbk = shfl32(rb, base + idx * NP + (li < NP ? li : 0));
                        const int ja = __builtin_ctz(ev), jb = 31 - __builtin_clz(ev);
                        const int asg_k = li < NP ? asg_j : -1;          // row 0: lane k holds agent k's
                        if constexpr (L == 64) {   // one env per wave: scalar operands
                            const int ba = __builtin_amdgcn_readlane(asg_j, ja), bb = __builtin_amdgcn_readlane(asg_j, jb);
                            swap_ev = evict_pair_swapped(WaveGroup(), N, li < NP ? rbk : 0u, asg_k, ja, ba, jb, bb);
                        } else {
                            const int ba = (int)shfl32((uint32_t)asg_j, base + ja), bb = (int)shfl32((uint32_t)asg_j, base + jb);
                            swap_ev = evict_pair_swapped(Group(L), N, li < NP ? rbk : 0u, asg_k, ja, ba, jb, bb);
                        }
                    }
                }
            }
            ++hd;
            if ((ev >> i) & 1u) {
                const int rank = __popc(ev & ((1u << i) - 1u));
                asg_i = -1;
                q = next_q + (swap_ev ? 1 - rank : rank);
            }
            if ((ev >> j) & 1u) asg_j = -1;
            next_q += __popc(ev);
            if (i == idx) { asg_i = newa; q = -1; }
            if (j == idx) asg_j = newa;
        }
        if (hd < next_q) {     // deadlock fallback (fix_revert_blocked in the pair layout)
            if (vi && asg_i < 0) asg_i = 0;
            if (vj && asg_j < 0) asg_j = 0;
            uint32_t frontier = agents_of(eballot(head && vi && asg_i == 0));
            while (frontier) {
                const bool blk = vi && vj && asg_i > 0 && ((frontier >> j) & 1u) &&
                                 pack(ri + dr(asg_i), ci + dc(asg_i)) == pj;
                const uint64_t bm = eballot(blk);
                uint32_t nb = 0;
#pragma unroll
                for (int k = 0; k < NP; ++k) nb |= (uint32_t)(((bm >> (k * NP)) & ROW) != 0ull) << k;
                if ((nb >> i) & 1u) asg_i = 0;
                if ((nb >> j) & 1u) asg_j = 0;
                frontier = nb;
            }
        }
        fixed = asg_i >= 0 ? asg_i : 0;
    }
    STAMP(3);

    // ---- takeStep + lifelong goals
    const int nr = ri + dr(fixed), nc = ci + dc(fixed);
    const uint32_t np = vi ? pack(nr, nc) : 0xFFFFFFFFu;
    const bool reached = vi && e.lifelong && np == gi;
    uint32_t ng = gi;
    if (gmode == 0) {
        if (reached && head) {
            int cur = e.seq_cur[ai];
            const int len = e.seq_len[ai];
            const uint32_t *s = e.seq + ai * e.S;
            if (cur >= len) ng = s[len - 1];
            else ng = s[cur++];
            e.seq_cur[ai] = cur;
        }
    } else {
        // getNextGoal(worldWithAgentsAndGoals()) in agent order (mapf_gym.py:620-627)
        for (uint32_t rem = agents_of(eballot(head && reached)); rem; rem &= rem - 1) {
            const int k = __builtin_ctz(rem);
            const uint32_t mypos = (i <= k) ? np : pi;
            const uint32_t mygoal = ng;
            const uint32_t *bits = env_map(e, b);
            auto ok = [&](int r, int c) -> bool {
                if (rm.obstacle(e, bits, r, c)) return false;
                const uint32_t cell = pack(r, c);
                return eballot(head && vi && (mypos == cell || mygoal == cell)) == 0ull;
            };
            int r, c;
            if (!group_free_cell(e, env_id, P_GOAL, k, clock, ok, r, c)) {
                if (li == 0) atomicAdd(&e.counters[C_FREECELL], 1u);
                const uint32_t npk = shfl32(np, base + k * NP);
                r = prow(npk); c = pcol(npk);
            }
            if (i == k) ng = pack(r, c);
        }
    }
    if constexpr (RES) {
        if (vi) { rs->pi = np; rs->gi = ng; rs->la = fixed; }
        const uint32_t npj = shfl32(np, base + j * NP);          // agent j's new cell (row j)
        if (vj) rs->pj = npj;
    } else if (vi && head) {
        e.pos[ai] = np;
        e.goal[ai] = ng;
        e.last_act[ai] = (int8_t)fixed;
    }
    if (e.keep_bfs) {                       // agent.bfsMap recompute (makeBfsMap on goal change, :627)
        const uint64_t bm = __ballot(vi && head && reached);
        if (bm) {
            if (!INLINE && lane == __builtin_ctzll(bm))
                dfr.bret = atomicAdd(&e.counters[C_BFS_COUNT + slot], (uint32_t)__popcll(bm));
            dfr.bmask = bm;
            dfr.bitem = (uint32_t)ai;
            dfr.bgoal = ng;
        }
    }
    STAMP(4);

    // ---- human.nextStep (see step_kernel): side effects of the advance decided above
    if (at_end) {
        if (hmode == 1) {
            if (RES) {
                if (swapped) { rs->hgoal = hng; rs->replans += 1u; }
            } else if (swapped && li == 0) {
                e.hgoal[b] = hng; e.hreplans[b] += 1u;
            }
        } else if (hmode == 2) {
            if (li == 0) {
                e.hgoal[b] = e.hseq[(size_t)b * e.HS + (seq_idx < hsl ? seq_idx : hsl - 1)];
                e.hseq_idx[b] = seq_idx;
            }
        }
    }
    if (swapped) {
        uint32_t ns, ngl;
        plan_next_path(e, b, env_id, clock + (uint32_t)L2, seq_idx, ns, ngl, li == 0, rm, hmode,
                       RES ? rs->hentr : 0u, RES);
        if (RES) {
            rs->hstart = ns;
            rs->hng = ngl;
        } else if (li == 0) {
            e.hnext_start[b] = ns;
            e.hnext_goal[b] = ngl;
        }
        const uint64_t rmk = __ballot(li == 0 && ngl != NO_CELL);
        if (rmk) {
            if (!INLINE && lane == __builtin_ctzll(rmk))
                dfr.rret = atomicAdd(&e.counters[C_REPLAN_COUNT + slot], (uint32_t)__popcll(rmk));
            dfr.rmask = rmk;
            dfr.ritem = (uint32_t)b;
            dfr.rstart = ns;
            dfr.rgoal = ngl;
            dfr.rbuf = cur2 ^ 1;
        }
    }
    if (RES) {
        rs->hcur = cur2;
        rs->hs = hs2;
        rs->hp = hp_new;
        rs->hn = hn_new;
        rs->clock = clock + 1u;
    } else if (li == 0) {
        e.hcur[b] = cur2;
        e.hstep[b] = hs2;
        e.hpos[b] = hp_new;
        e.hnext[b] = hn_new;
        e.clock[b] = clock + 1u;
    }
    STAMP(5);

    if (vi && head) {
        const int d0 = prow(hp_new) - nr, d1 = pcol(hp_new) - nc;
        const float cv = (d0 * d0 + d1 * d1 <= e.constr_d2) ? 1.f : 0.f;
        if (out.actions_fixed) out.actions_fixed[ai] = fixed;
        if (out.goals_reached) out.goals_reached[ai] = reached ? 1.f : 0.f;
        if (out.constraints) out.constraints[ai] = cv;
        if (out.reward_total) out.reward_total[ai] = reached ? rw + e.goal_reward : rw;
    }
    STAMP(6);
    if constexpr (FEED) {
        const int le = b - b0;
        if (vi && head) {
            ob.spos[le * N + i] = np;
            ob.sgoal[le * N + i] = ng;
        }
        if (li == 0) ob.shn[le] = hn_new;
        if (e.use_hp && e.C >= 6) {       // human.path[1..K] of the path it walks after the step
            const int kp = e.k_predict;
            for (int q = 1 + li; q <= kp && q < L2; q += L) ob.shp[le * kp + q - 1] = p2r[q];
            if (li == 0) ob.shpn[le] = min(kp, L2 - 1);
        } else if (li == 0) {
            ob.shpn[le] = 0;
        }
    }
    STAMP_END();
}

}  // namespace mapf
