// primal-ppo_amd/csrc/mapf_step.h -- one env's lockstep step on a lane group (device code),
// shared by step_kernel (mapf_step.hip) and the wide rollout kernel (mapf_rollout_wide.hip).
//
// Reference semantics (Nielsencu/primal-ppo mapf_gym.py), in runner.py:64-100
// order: getActionStatus (:434-480) -> calculateActionReward (:483-511) ->
// calculateCostReward (:528-533) -> getTrainValid (:535-550) -> jointStep
// (:614-637: fixActions :552-612, takeStep :158-161, lifelong goals :623-627,
// human.nextStep :25-31, constraintsViolated :631-633).  The masks that the
// reference recomputes at the END of jointStep (getUnconditionallyGoodActions
// :404-430) are a pure function of the state, so this kernel recomputes them
// at the START of the next step instead of storing them.
//
// Mapping: lane = agent, G lanes per env (mapf_group.h).  Conflicts are never
// materialised as the reference's restrictedAction dict: for distinct agent
// positions (guaranteed: starts are validated distinct and resolved moves
// never collide), the dict's content is exactly
//   (j, b) in R_i[a]  <=>  p_i+d(a) == p_j+d(b)  or  (p_i+d(a) == p_j and p_j+d(b) == p_i)
// and its key set is  a in keys(i) <=> exists j != i: |p_i+d(a) - p_j|_1 <= 1.
// (The reference's pruning test, mapf_gym.py:387, never removes a true
// conflict when positions differ.)
//
// HBM traffic per agent-step: ~16 B state read, ~50 B outputs (+ rare BFS /
// replan work lists) -- latency bound, not bandwidth bound.
#pragma once
#include "mapf_group.h"
#include "mapf_kernels.h"
#include "mapf_pyset.h"

namespace mapf {

// The search work of one inline step (instead of the work lists): lanes of the agents
// whose goal changed and, group-uniform, the human's next path to search.
struct StepInline {
    uint64_t bmask;        // agents whose bfsMap must be rebuilt (keep_bfs)
    uint32_t goal;         // per lane: the agent's goal after the step
    bool replan;           // the human's next path: rstart -> rgoal into path buffer rbuf
    uint32_t rstart, rgoal;
    int rbuf;
};

// Where a step reads its static tables: the env's padded obstacle rows and the cost
// table in LDS (the persistent rollout's copies; the static action mask is then derived
// from the rows), or from HBM (nullptr).
// An env's state held in registers by a persistent caller (the wide rollout's stepping
// wave): read instead of HBM at the start of a step and updated at its end (the HBM
// copy is still written, for everything else that reads it).
struct StepRegs {
    uint32_t pp, gg;     // per lane: the agent's cell and goal
    int la;              // per lane: its last action (-1 none)
    uint32_t clock, hp, hn;
    int hs, hcur, hl0, hl1;
    uint32_t hq;         // per lane q in 1..k_predict: human.path[q] after the step (NO_CELL past its end)
};

__device__ inline void step_regs_load(const DevEnv &e, int b, int i, StepRegs &r) {
    const bool act = i < e.N;
    const size_t ai = (size_t)b * e.N + i;
    r.pp = act ? e.pos[ai] : 0xFFFFFFFFu;
    r.gg = act ? e.goal[ai] : 0u;
    r.la = act ? (int)e.last_act[ai] : -1;
    r.clock = e.clock[b];
    r.hp = e.hpos[b];
    r.hn = e.hnext[b];
    r.hs = e.hstep[b];
    r.hcur = e.hcur[b];
    r.hl0 = e.hlen[b * 2];
    r.hl1 = e.hlen[b * 2 + 1];
    r.hq = NO_CELL;
}

// The cells within distance 2 of an agent (the neighbour grid's 12 slots) and, per slot, the
// folded pair tests of step_group (keys / conflicts of an agent there, see pair()).
constexpr int NBR_DR[12] = {-2, -1, -1, -1, 0, 0, 0, 0, 1, 1, 1, 2};
constexpr int NBR_DC[12] = {0, -1, 0, 1, -2, -1, 1, 2, -1, 0, 1, 0};
constexpr int cabs(int x) { return x < 0 ? -x : x; }
constexpr unsigned nbr_keys(int R, int C) {
    unsigned m = 0;
    for (int t = 0; t < NA; ++t)
        if (cabs(dr(t) - R) + cabs(dc(t) - C) <= 1) m |= 1u << t;
    return m;
}
constexpr uint32_t nbr_conf(int R, int C) {
    uint32_t tab = 0;
    for (int aj = 0; aj < NA; ++aj) {
        const int YR = R + dr(aj), YC = C + dc(aj);
        for (int t = 0; t < NA; ++t)
            if ((dr(t) == YR && dc(t) == YC) || (dr(t) == R && dc(t) == C && YR == 0 && YC == 0))
                tab |= 1u << (5 * aj + t);
    }
    return tab;
}
#define MAPF_NBR12(F) {F(NBR_DR[0], NBR_DC[0]), F(NBR_DR[1], NBR_DC[1]), F(NBR_DR[2], NBR_DC[2]), \
    F(NBR_DR[3], NBR_DC[3]), F(NBR_DR[4], NBR_DC[4]), F(NBR_DR[5], NBR_DC[5]), F(NBR_DR[6], NBR_DC[6]), \
    F(NBR_DR[7], NBR_DC[7]), F(NBR_DR[8], NBR_DC[8]), F(NBR_DR[9], NBR_DC[9]), F(NBR_DR[10], NBR_DC[10]), \
    F(NBR_DR[11], NBR_DC[11])}
constexpr unsigned NKEYS[12] = MAPF_NBR12(nbr_keys);
constexpr uint32_t NCONF[12] = MAPF_NBR12(nbr_conf);
#undef MAPF_NBR12

// the registers back to HBM (the REGS caller, once after its last step)
__device__ inline void step_regs_store(const DevEnv &e, int b, int i, const StepRegs &r) {
    if (i < e.N) {
        const size_t ai = (size_t)b * e.N + i;
        e.pos[ai] = r.pp;
        e.goal[ai] = r.gg;
        e.last_act[ai] = (int8_t)r.la;
    }
    if (i == 0) {
        e.hcur[b] = r.hcur;
        e.hstep[b] = r.hs;
        e.hpos[b] = r.hp;
        e.hnext[b] = r.hn;
        e.clock[b] = r.clock;
    }
}

struct StepSrc {
    const uint32_t *map = nullptr;
    const float *cost = nullptr;
    uint8_t *grid = nullptr;      // (H + 4) x (W + 4) u16 of LDS scratch, whole-wave envs only
};

// One env's step on the group g (lane i of the group = agent i; G >= N).  The
// search work a committed step creates (BFS maps of the agents whose goal
// changed, the human's next path) goes to the work lists of slot `parity`, or,
// with `inl`, to the caller, which searches it inline (mapf_rollout_wide.hip).
// Grp: Group (G lanes per env, exchanges through ds_bpermute) or, when the env is the
// whole wave, WaveGroup (exchanges by v_readlane: the agent loops' indices are
// wave-uniform, and a readlane costs a few cycles where a bpermute costs an LDS round trip).
// REGS: the env's state comes from and goes back to `rg` (register-resident, persistent
// callers) instead of being loaded from HBM (it is still stored to HBM).
// LANEPTR (the wide rollout): `actions` and every per-agent pointer of `out` are already this
// lane's element (shadow_goals this env's), held in VGPRs by the caller, and `have` says which
// outputs exist (bit k = the k-th StepOut field) -- the output bases then take no SGPRs in the
// step loop, where they were spilled to VGPR lanes and read back at every store.
template <class Grp, bool REGS = false, bool LANEPTR = false>
__device__ __attribute__((always_inline)) inline void step_group(const DevEnv &e, int32_t *__restrict__ actions,
                                                                const StepOut &out, uint32_t flags, int parity, int b,
                                                                const Grp &g, StepInline *inl, StepSrc src,
                                                                StepRegs &rg, uint32_t have = 0) {
    const int N = e.N;
    STAMP_BEGIN();
    const int i = g.i;
    const bool act = i < N;
    const size_t ai = (size_t)b * N + i;
    const size_t oi = LANEPTR ? 0 : ai, ob = LANEPTR ? 0 : (size_t)b;   // output element indices
    auto has = [&](int k, const void *p) { return LANEPTR ? ((have >> k) & 1u) != 0 : p != nullptr; };
    const uint32_t env_id = e.env_offset + (uint32_t)b;
    const uint32_t clock = REGS ? rg.clock : e.clock[b];

    // ---- human.nextStep (:25-31, :42-44, :65-70, :87-94): where the human goes --
    // It depends on nothing the agents do, so its state and path cells are read here,
    // in the same round of loads as the agents' state (the writes stay at the end).
    // The path switched to at an end-step was searched one path ahead (buffer hcur ^ 1).
    const int hs = REGS ? rg.hs : e.hstep[b], hcur = REGS ? rg.hcur : e.hcur[b];
    const int hl0 = REGS ? rg.hl0 : e.hlen[b * 2], hl1 = REGS ? rg.hl1 : e.hlen[b * 2 + 1];
    const int hL = hcur ? hl1 : hl0;
    int cur2 = hcur, hs2 = hs + 1, seq_idx = 0;
    bool swapped = false;
    uint32_t hgoal_new = NO_CELL;
    if (hs >= hL - 1) {
        hs2 = 0;
        if (e.human_mode == 1) {
            const uint32_t hng = e.hnext_goal[b];
            if (hng != NO_CELL) {
                cur2 = hcur ^ 1;
                swapped = true;
                hgoal_new = hng;
            }
        } else if (e.human_mode == 2) {
            const int idx = e.hseq_idx[b] + 1;
            const int len = e.hseq_len[b];
            seq_idx = idx;
            if (idx >= len) {
                hgoal_new = e.hseq[(size_t)b * e.HS + len - 1];   // path kept, restarts at [0]
            } else {
                hgoal_new = e.hseq[(size_t)b * e.HS + idx];
                cur2 = hcur ^ 1;
                swapped = true;
            }
        }
    }
    const int hL2 = cur2 ? hl1 : hl0;
    const uint32_t *hpath2 = human_path(e, b, cur2);
    // REGS (the persistent caller keeps everything else in registers / LDS): read the two path
    // cells as vector loads.  Uniform addresses would make them scalar loads, counted in
    // lgkmcnt with the LDS operations -- and the first LDS wait of the step would then wait
    // for these HBM reads.
    int vz = 0;
    if constexpr (REGS) asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    const uint32_t hp_new = hpath2[hs2 + vz];
    const uint32_t hn_new = hpath2[(hs2 + 1 < hL2 ? hs2 + 1 : hL2 - 1) + vz];
    // and the observation's predicted cells human.path[1..K] (getObservations :293-297), in
    // the same round: read after the step's output stores they would wait for those stores
    // (only with the HP channel: an unused load still holds its register, and the next step's
    // reload of it would wait vmcnt behind every store issued meanwhile)
    if constexpr (REGS) rg.hq = (e.use_hp && e.C >= 6 && i >= 1 && i <= e.k_predict && i < hL2) ? hpath2[i] : NO_CELL;

    // ---- state -----------------------------------------------------------
    const uint32_t pp = REGS ? rg.pp : (act ? e.pos[ai] : 0xFFFFFFFFu);
    const int pr = act ? prow(pp) : -100, pc = act ? pcol(pp) : -100;
    const uint32_t gg = REGS ? rg.gg : (act ? e.goal[ai] : 0u);
    const int la = REGS ? rg.la : (act ? (int)e.last_act[ai] : -1);
    int a = 0;
    if (flags & 2u) {          // random policy fused in: same stream as random_actions_kernel
        if (act) {
            a = random_action(philox(env_id, P_ACT | ((uint32_t)(i >> 3) << 8), clock, 0u, e.seed), i);
            actions[oi] = a;
        }
    } else if (act) {
        a = actions[oi];
        if (a < 0 || a >= NA) { atomicAdd(&e.counters[C_BAD_ACTION], 1u); a = 0; }
    }
    // REGS callers hold the map rows, cost table and neighbour grid in LDS: typed as such
    const uint32_t *bits = env_map(e, b);
    const auto lmap = as_lds(src.map);
    auto obstacle = [&](int r, int c) -> bool {
        if constexpr (REGS) return obstacle_at(e, lmap, r, c);
        else return obstacle_at(e, bits, r, c);
    };
    const uint32_t hp = REGS ? rg.hp : e.hpos[b], hn = REGS ? rg.hn : human_next(e, b);

    // ---- getInvalidActions (mapf_gym.py:339-360) ---------------------------
    // static part: a per-cell 5-bit mask precomputed from the map (off-map / obstacle),
    // or the same five obstacle tests on the LDS rows
    unsigned st_mask = 0x1Fu;
    if (act) {
        if (REGS) {
            // an agent's four neighbours lie inside the padded rows (P >= 1, mapf_api.cpp), so
            // the five words load with no bounds test: five reads in flight, one wait
            st_mask = 0;
            uint32_t w[NA];
#pragma unroll
            for (int k = 0; k < NA; ++k) w[k] = lmap[(pr + dr(k) + e.P) * e.WW + ((pc + dc(k) + e.P) >> 5)];
#pragma unroll
            for (int k = 0; k < NA; ++k) st_mask |= ((w[k] >> ((pc + dc(k) + e.P) & 31)) & 1u) << k;
        } else {
            st_mask = e.smask[(e.shared_map ? 0 : (size_t)b * e.H * e.W) + pr * e.W + pc];
        }
    }
    unsigned hu_mask = 0;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        const int r = pr + dr(k), c = pc + dc(k);
        if ((st_mask >> k) & 1u) continue;
        if (pack(r, c) == hn) hu_mask |= 1u << k;
        else if (pp == hn && pack(r, c) == hp) hu_mask |= 1u << k;
    }
    const unsigned rep_mask = la >= 0 ? 1u << opp(la) : 0u;

    STAMP(0);
    // ---- getRestrictedActions (:363-402), evaluated against actual actions --
    const int Xr = pr + dr(a), Xc = pc + dc(a);
    unsigned keys = 0, conf = 0;   // conf: my actions t that collide with some j's actual action
    uint64_t M = 0;                // agents j colliding with my actual action
    unsigned hitM = 0;             // grid path: M != 0 (M is then built lazily, per scanned agent)
    // the pair test of agent j at (qr, qc) taking action aj (only pairs within distance 2 matter)
    auto pair = [&](int j, int qr, int qc, int aj) {
        const int Yr = qr + dr(aj), Yc = qc + dc(aj);
        unsigned cj = 0;
#pragma unroll
        for (int t = 0; t < NA; ++t) {
            const int tr = pr + dr(t), tc = pc + dc(t);
            if (abs(tr - qr) + abs(tc - qc) <= 1) keys |= 1u << t;
            if ((tr == Yr && tc == Yc) || (tr == qr && tc == qc && Yr == pr && Yc == pc)) cj |= 1u << t;
        }
        conf |= cj;
        if ((cj >> a) & 1u) M |= 1ull << j;
    };
    if (REGS && src.grid) {
        // The agents within distance 2 straight from an LDS grid (the env is the whole wave,
        // its lanes the agents): 12 neighbour cells per lane instead of a loop over all N
        // agents.  Grid = (H + 4) x (W + 4) u16, 2-cell border; a cell holds its agent's
        // index | action << 8 (0xFFFF empty) -- positions are distinct, so at most one --
        // so one read gives a neighbour and its action, no cross-lane exchange.
        const int GW = e.W + 4, gwords = ((e.H + 4) * GW * 2 + 3) >> 2;
        const int lane = lane_id();
        const auto grid = as_lds(reinterpret_cast<uint16_t *>(src.grid));
        // cleared 16 B per lane (the grid's LDS area is 16-B aligned and padded to 16 B)
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const auto grid128 = as_lds(reinterpret_cast<u32x4 *>(src.grid));
        for (int k = lane; k < ((gwords + 3) >> 2); k += 64) grid128[k] = u32x4(0xFFFFFFFFu);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // lanes past N read around the grid's cell (0, 0) (result dropped): no branch per read
        const int me = act ? (pr + 2) * GW + pc + 2 : 2 * GW + 2;
        if (act) grid[me] = (uint16_t)(i | (a << 8));
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // A neighbour's offset is fixed by its slot, so pair()'s tests fold into constants:
        // NKEYS[o] = the keys it contributes, NCONF[o] bits 5aj..5aj+4 = my actions colliding
        // with its action aj (same target, or a swap).  All twelve reads issue back to back,
        // then one wait and a branch-free fold.
        int nb[12];
#pragma unroll
        for (int o = 0; o < 12; ++o) {
            const int v = (int)grid[me + NBR_DR[o] * GW + NBR_DC[o]];
            nb[o] = act ? v : 0xFFFF;
        }
#pragma unroll
        for (int o = 0; o < 12; ++o) {
            const bool h = nb[o] != 0xFFFF;
            const unsigned cj = h ? (NCONF[o] >> (5 * (nb[o] >> 8))) & 0x1Fu : 0u;
            keys |= h ? NKEYS[o] : 0u;
            conf |= cj;
            hitM |= (cj >> a) & 1u;     // M itself is built only for the scan's agents (below)
        }
    } else {
        for (int j = 0; j < N; ++j) {
            const uint32_t pj = g.shfl(pp, j);
            const int aj = g.shfl_i(a, j);
            if (!act || j == i) continue;
            const int qr = prow(pj), qc = pcol(pj);
            if (abs(qr - pr) + abs(qc - pc) > 2) continue;
            pair(j, qr, qc, aj);
        }
    }
    const unsigned good = ~(st_mask | hu_mask | rep_mask | keys) & 0x1Fu;   // setdiff1d (:423)

    STAMP(1);
    // ---- getActionStatus (:434-480) ----------------------------------------
    int s0;
    bool cb = false;
    if ((st_mask >> a) & 1u) s0 = -1;
    else if ((hu_mask >> a) & 1u) s0 = -2;
    else if ((good >> a) & 1u) s0 = 1;
    else if (M || hitM) { s0 = -3; cb = true; }
    else s0 = ((rep_mask >> a) & 1u) ? -4 : 1;
    // sequential scan: agent k is skipped if an earlier agent already set it to
    // -3; an agent taking the conflict branch sets itself and all of M_k to -3
    // (overwriting earlier statuses, :471-472).
    uint64_t T = 0;
    for (uint64_t rem = g.ballot(act && cb); rem; rem &= rem - 1) {
        const int k = ctz64(rem);
        uint64_t Mk;
        if (REGS && src.grid) {
            // M_k = the agents whose actual action collides with k's: same target, or a swap
            // (a symmetric relation, so every lane tests itself against k) -- built here for
            // the few agents in the conflict branch instead of per lane over 12 grid slots
            const int kr = __builtin_amdgcn_readlane(pr, k), kc = __builtin_amdgcn_readlane(pc, k);
            const int kxr = __builtin_amdgcn_readlane(Xr, k), kxc = __builtin_amdgcn_readlane(Xc, k);
            Mk = g.ballot(act && i != k && ((Xr == kxr && Xc == kxc) || (Xr == kr && Xc == kc && kxr == pr && kxc == pc)));
        } else {
            Mk = g.shfl64(M, k);
        }
        if (!((T >> k) & 1ull)) T |= Mk | (1ull << k);
    }
    const int st = ((T >> i) & 1ull) ? -3 : s0;

    // ---- calculateActionReward (:483-511) ----------------------------------
    // selects, not a switch: each case's branch reloaded the env's spilled scalars.  The
    // four costs are pinned in SGPRs first: otherwise the selects become a select of field
    // ADDRESSES and one vector load from the kernel arguments, which the reward's stores
    // then wait for with vmcnt(0).
    float c_act = e.action_cost, c_rep = e.repeat_cost, c_col = e.collision_cost, c_hum = e.human_collision_cost;
    asm volatile("" : "+s"(c_act), "+s"(c_rep), "+s"(c_col), "+s"(c_hum));
    float rw = c_act;
    rw = st == -4 ? c_rep : rw;
    rw = (st == -1 || st == -3) ? c_col : rw;
    rw = st == -2 ? c_hum : rw;
    const bool shadow_hit = act && st == 1 && Xr == prow(gg) && Xc == pcol(gg);
    const uint64_t shadow_mask = g.ballot(shadow_hit);

    // ---- calculateCostReward (:528-533): pre-step human next position -------
    // REGS callers with the table in LDS never touch the HBM copy: a value that MAY come
    // from a global load makes every later use (and every reuse of its register) wait
    // vmcnt(0), i.e. for the whole step's stores, even on the LDS path.
    const int cd0 = prow(hn) - Xr, cd1 = pcol(hn) - Xc;
    const int cd2 = cd0 * cd0 + cd1 * cd1;
    const bool cin = cd2 <= e.R * e.R;
    if (act && has(3, out.cost)) {
        if (REGS && src.cost) {
            out.cost[oi] = cin ? as_lds(src.cost)[cd2] : 0.f;
        } else {
            const float c = cin ? e.cost_lut[cd2] : 0.f;
            // REGS: the load's wait here, on this path only, so nothing is pending at the join
            if constexpr (REGS) __builtin_amdgcn_s_waitcnt(0x0F70);
            out.cost[oi] = c;
        }
    }

    if (act) {
        if (has(0, out.status)) out.status[oi] = (int8_t)st;
        if (has(1, out.reward)) out.reward[oi] = rw;
        if (has(4, out.train_valid)) {   // getTrainValid (:535-550)
            float *tv = out.train_valid + oi * NA;
#pragma unroll
            for (int t = 0; t < NA; ++t)
                tv[t] = (((good >> t) & 1u) || (((keys >> t) & 1u) && !((conf >> t) & 1u))) ? 1.f : 0.f;
        }
    }
    if (i == 0 && has(2, out.shadow_goals)) out.shadow_goals[ob] = popc64(shadow_mask);
    if (inl) inl->replan = false;
    if (!(flags & 1u)) return;

    STAMP(2);
    // ---- jointStep: fixActions (:552-612) ----------------------------------
    // Worklist semantics of the reference; evictions appended in its set order
    // (mapf_pyset.h).  States the reference does not survive: an
    // empty viable set (random.choice([]) raises, :588) stays and evicts as if 0
    // had been drawn; a deadlock (the while loop never ends, :563) is declared
    // after fix_draws(N) draws: the unplaced agents stay and blocked movers are
    // reverted to stay until none is left (fix_revert_blocked).
    int fixed = a;
    const uint64_t need = g.ballot(act && (st == -1 || st == -2 || st == -3));
    if (need) {
        int assigned = (act && st == 1) ? a : -1;
        // Worklist agents with a good action take its min at once: a good action collides
        // with no action of any agent (no agent within reach of its target), so it never
        // enters another agent's conflict set U and is never evicted -- its turn in the
        // sequential order decides nothing.  The loop walks only the others, in order (an
        // evicted agent re-queued later may still have one: the loop keeps that case).
        const bool wl = act && st < 0;
        if (wl && good) assigned = __builtin_ctz(good);
        const uint64_t qm = g.ballot(wl && !good);
        int q = (wl && !good) ? popc64(qm & below(i)) : -1;
        int next_q = popc64(qm), head = 0, draws = 0;
        const unsigned viable_me = ~(st_mask | hu_mask) & 0x1Fu;
        while (head < next_q) {
            const uint64_t hm = g.ballot(act && q == head);
            const int idx = ctz64(hm);
            const unsigned good_idx = g.shfl(good, idx);
            if (good_idx) {
                ++head;
                if (i == idx) { assigned = __builtin_ctz(good_idx); q = -1; }
                continue;
            }
            const unsigned viable = g.shfl(viable_me, idx);
            const uint32_t pidx = g.shfl(pp, idx);
            const int ir = prow(pidx), ic = pcol(pidx);
            unsigned cj = 0;   // idx's actions that collide with MY assigned action
            if (act && i != idx && assigned >= 0 && abs(pr - ir) + abs(pc - ic) <= 2) {
                const int Yr = pr + dr(assigned), Yc = pc + dc(assigned);
#pragma unroll
                for (int t = 0; t < NA; ++t) {
                    const int tr = ir + dr(t), tc = ic + dc(t);
                    if ((tr == Yr && tc == Yc) || (tr == pr && tc == pc && Yr == ir && Yc == ic)) cj |= 1u << t;
                }
            }
            unsigned U = 0;
#pragma unroll
            for (int t = 0; t < NA; ++t)
                if (g.ballot((cj >> t) & 1u)) U |= 1u << t;
            const unsigned fr = viable & ~U;
            if (fr) {
                ++head;
                if (i == idx) { assigned = __builtin_ctz(fr); q = -1; }
                continue;
            }
            if (draws >= fix_draws(N)) {        // deadlock: idx stays queued
                if (i == 0) atomicAdd(&e.counters[C_FIX_BOUND], 1u);
                break;
            }
            const int nv = __popc(viable);
            int rsel = 0;
            if (nv == 0) {      // reference: random.choice([]) raises IndexError
                if (i == idx) atomicAdd(&e.counters[C_EMPTY_VIABLE], 1u);
            } else {
                int pick;
                if (e.fix_choice == 0) pick = draws % nv;
                else pick = (int)__umulhi(philox(env_id, P_FIX | ((uint32_t)idx << 8), clock, (uint32_t)draws, e.seed).x,
                                          (uint32_t)nv);
                rsel = nth_bit(viable, pick);
            }
            ++draws;
            ++head;
            const uint64_t ev = g.ballot((cj >> rsel) & 1u);   // evicted agents (at most two)
            int rank = popc64(ev & below(i));
            if (__builtin_expect(popc64(ev) == 2, 0)) {
                const int ja = ctz64(ev), jb = 63 - __builtin_clzll(ev);
                // restrictedAction[idx][rsel] as (j, b) masks on lane j
                const int Xr = ir + dr(rsel), Xc = ic + dc(rsel);
                unsigned rb = 0;
                if (act && i != idx) {
#pragma unroll
                    for (int t = 0; t < NA; ++t) {
                        const int yr = pr + dr(t), yc = pc + dc(t);
                        if ((yr == Xr && yc == Xc) || (Xr == pr && Xc == pc && yr == ir && yc == ic)) rb |= 1u << t;
                    }
                }
                if (evict_pair_swapped(g, N, rb, assigned, ja, g.shfl_i(assigned, ja), jb, g.shfl_i(assigned, jb)))
                    rank = 1 - rank;
            }
            if ((ev >> i) & 1ull) { assigned = -1; q = next_q + rank; }
            next_q += popc64(ev);
            if (i == idx) { assigned = rsel; q = -1; }
        }
        if (head < next_q) {
            if (act && assigned < 0) assigned = 0;
            fix_revert_blocked(g, act, pp, assigned);
        }
        fixed = assigned >= 0 ? assigned : 0;
    }

    STAMP(3);
    // ---- takeStep (:158-161) + lifelong goals (:623-627) --------------------
    const int nr = pr + dr(fixed), nc = pc + dc(fixed);
    const uint32_t np = act ? pack(nr, nc) : 0xFFFFFFFFu;
    const bool reached = act && e.lifelong && np == gg;
    uint32_t ng = gg;
    int cur = 0;
    if (e.goal_mode == 0) {
        if (reached) {   // Sequence.getNext (util.py:33-39)
            cur = e.seq_cur[ai];
            const int len = e.seq_len[ai];
            const uint32_t *s = e.seq + ai * e.S;
            if (cur >= len) ng = s[len - 1];
            else ng = s[cur++];
            e.seq_cur[ai] = cur;
        }
    } else {
        // getNextGoal(worldWithAgentsAndGoals()) for the reached agents in
        // index order: agents <= k at new positions, > k at old; goals of
        // agents < k already replaced (mapf_gym.py:200-209, :620-627).
        for (uint64_t rem = g.ballot(reached); rem; rem &= rem - 1) {
            const int k = ctz64(rem);
            const uint32_t mypos = (i <= k) ? np : pp;
            const uint32_t mygoal = ng;
            auto ok = [&](int r, int c) -> bool {
                if (obstacle(r, c)) return false;
                const uint32_t cell = pack(r, c);
                return g.ballot(act && (mypos == cell || mygoal == cell)) == 0ull;
            };
            int r, c;
            if (!group_free_cell(e, env_id, P_GOAL, k, clock, ok, r, c)) {
                if (i == k) atomicAdd(&e.counters[C_FREECELL], 1u);
                r = prow(g.shfl(np, k)); c = pcol(g.shfl(np, k));
            }
            if (i == k) ng = pack(r, c);
        }
    }
    const uint64_t bmask = g.ballot(reached && e.keep_bfs);
    if (inl) {
        inl->bmask = bmask;
        inl->goal = ng;
    }
    if constexpr (REGS) {
        if (act) {
            rg.pp = np;
            rg.gg = ng;
            rg.la = fixed;
        }
    }
    if (act) {
        if constexpr (!REGS) {      // REGS: the caller stores the registers once, at its end
            e.pos[ai] = np;
            e.goal[ai] = ng;
            e.last_act[ai] = (int8_t)fixed;
        }
        if (reached && e.keep_bfs && !inl) {
            const uint32_t slot = atomicAdd(&e.counters[C_BFS_COUNT + parity], 1u);
            e.bfs_list[(size_t)parity * e.B * N + slot] = (uint32_t)ai;
        }
    }

    STAMP(4);
    // ---- human.nextStep, state writes (the move itself was read at the top) ------
    {
        if (swapped || hs >= hL - 1) {
            if (e.human_mode == 1 && swapped && i == 0) { e.hgoal[b] = hgoal_new; e.hreplans[b] += 1u; }
            if (e.human_mode == 2 && i == 0) { e.hgoal[b] = hgoal_new; e.hseq_idx[b] = seq_idx; }
        }
        const int L2 = hL2;
        if (swapped) {
            uint32_t ns, hg;
            plan_next_path(e, b, env_id, clock + (uint32_t)L2, seq_idx, ns, hg, i == 0);
            if (inl) {     // group-uniform: the search into the buffer the human is not using
                inl->replan = hg != NO_CELL;
                inl->rstart = ns;
                inl->rgoal = hg;
                inl->rbuf = cur2 ^ 1;
            }
            if (i == 0) {
                e.hnext_start[b] = ns;
                e.hnext_goal[b] = hg;
                if (hg != NO_CELL && !inl) {
                    const uint32_t slot = atomicAdd(&e.counters[C_REPLAN_COUNT + parity], 1u);
                    e.replan_list[(size_t)parity * e.B + slot] = (uint32_t)b;
                }
            }
        }
        if (!REGS && i == 0) {
            e.hcur[b] = cur2;
            e.hstep[b] = hs2;
            e.hpos[b] = hp_new;
            e.hnext[b] = hn_new;
            e.clock[b] = clock + 1u;
        }
        if constexpr (REGS) {
            rg.hcur = cur2;
            rg.hs = hs2;
            rg.hp = hp_new;
            rg.hn = hn_new;
            rg.clock = clock + 1u;
        }
    }

    STAMP(5);
    // ---- outputs ------------------------------------------------------------
    if (act) {
        const int d0 = prow(hp_new) - nr, d1 = pcol(hp_new) - nc;
        const float cv = (d0 * d0 + d1 * d1 <= e.constr_d2) ? 1.f : 0.f;   // (:632-633)
        if (has(5, out.actions_fixed)) out.actions_fixed[oi] = fixed;
        if (has(6, out.goals_reached)) out.goals_reached[oi] = reached ? 1.f : 0.f;
        if (has(7, out.constraints)) out.constraints[oi] = cv;
        if (has(8, out.reward_total)) out.reward_total[oi] = reached ? rw + e.goal_reward : rw;   // runner.py:89-91
    }
    STAMP(6);
    STAMP_END();
}

}  // namespace mapf
