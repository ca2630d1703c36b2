// primal-ppo_amd/csrc/mapf_pyset.h -- fixActions' eviction order (mapf_gym.py:588-596).
//
// When fixActions' random branch picks action r for agent idx, the reference
// evicts the assigned agents that conflict with it in the iteration order of
//     set(tuple(x) for x in agentActionPairs) & set(tuple(x) for x in np.array(restrictedAction[r]))
// (CPython 3.10: Objects/setobject.c set_add_entry / set_table_resize /
// set_insert_clean / set_intersection, Objects/tupleobject.c tuplehash).  The
// tuples hold small ints, whose hashes are not randomised, so the order is a
// pure function of the operands -- restated here exactly as
// oracle/mapf_oracle.c oc_evict_order does (tests pin both to the reference's
// g2_evict fixture).
//
// The assigned pairs are pairwise conflict-free (status-1 actions, good
// actions, first-fit picks and evictions keep it so), so at most one assigned
// agent ends on idx's target and at most one swaps with idx: a pick evicts at
// most two agents, and only the two-agent case has an order to decide.
// Everything here is group-uniform (every lane of the env's lane group runs the
// same iterations); it runs only on that rare branch.
#pragma once
#include "mapf_group.h"

namespace mapf {

// The lane group of one env when it is the whole wave (one env per wave): the
// same interface as Group, but exchanges are v_readlane into scalar registers,
// so the set emulation runs on the SALU and costs the kernel no VGPRs.
struct WaveGroup {
    int i;
    __device__ WaveGroup() : i(lane_id()) {}
    __device__ uint64_t ballot(bool p) const { return __ballot(p); }
    __device__ uint32_t shfl(uint32_t v, int j) const { return (uint32_t)__builtin_amdgcn_readlane((int)v, j); }
    __device__ int shfl_i(int v, int j) const { return __builtin_amdgcn_readlane(v, j); }
    __device__ uint64_t shfl64(uint64_t v, int j) const {
        return (uint64_t)shfl((uint32_t)v, j) | ((uint64_t)shfl((uint32_t)(v >> 32), j) << 32);
    }
};

// tuplehash((a, b)) for small ints (hash(-1) == -2), 64-bit xxHash lanes
__device__ inline uint64_t py_hash_pair(int a, int b) {
    const uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL, P5 = 2870177450012600261ULL;
    uint64_t acc = P5;
    const uint64_t la = (uint64_t)(int64_t)(a == -1 ? -2 : a), lb = (uint64_t)(int64_t)(b == -1 ? -2 : b);
    acc += la * P2; acc = (acc << 31) | (acc >> 33); acc *= P1;
    acc += lb * P2; acc = (acc << 31) | (acc >> 33); acc *= P1;
    acc += 2ULL ^ (P5 ^ 3527539ULL);
    return acc == ~0ULL ? 1546275796ULL : acc;
}

// first empty slot on the probe path of `h` (LINEAR_PROBES 9, PERTURB_SHIFT 5)
__device__ inline int pyset_probe(uint64_t occ, uint64_t mask, uint64_t h) {
    uint64_t perturb = h, i = h & mask;
    for (;;) {
        if (!((occ >> i) & 1ull)) return (int)i;
        if (i + 9 <= mask)
            for (uint64_t j = 1; j <= 9; ++j)
                if (!((occ >> (i + j)) & 1ull)) return (int)(i + j);
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
    }
}

// position of the n-th set bit of m (n >= 0), 64 if none
__device__ inline int nth_bit64(uint64_t m, int n) {
    for (; m; m &= m - 1)
        if (n-- == 0) return ctz64(m);
    return 64;
}

// The two-agent eviction: agents ja != jb (assigned actions ba, bb) conflict
// with idx's pick.  Group lane j (j < N) holds rb = the actions b with (j, b) in
// restrictedAction[idx][r] and asg = agent j's assigned action (-1 = none).
// Returns true when the reference appends jb before ja.
//
// No per-lane storage: the iterated operand's elements are re-enumerated from
// the masks when needed and their slots are packed 5 bits each into one word
// (operands hold at most 6 elements, tables at most 32 slots), so with
// GR = WaveGroup everything stays in scalar registers.
template <class GR>
__device__ inline bool evict_pair_swapped(const GR &g, int N, unsigned rb, int asg, int ja, int ba, int jb, int bb) {
    const int li = g.i;
    const bool agent = li < N;
    const uint64_t am = g.ballot(agent && asg >= 0);
    const uint64_t rm = g.ballot(agent && rb != 0u);
    const int nP = popc64(am) + 1;                  // + (-1, -1): idx itself is unassigned
    int nR = 0;
    for (uint64_t rem = rm; rem; rem &= rem - 1) nR += __popc(g.shfl(rb, ctz64(rem)));
    // set_intersection iterates the smaller operand (ties: the right one, set(restrictedAction[r]))
    const bool fromR = nR <= nP;
    const int n = fromR ? nR : nP;
    const int u = ctz64(~am & below(N));            // set(agentActionPairs): (-1, -1) enters at agent u
    const int before = popc64(am & below(u));
    auto elem = [&](int k, int &j, int &b) {        // element k of the iterated operand, in insertion order
        if (fromR) {                                // restrictedAction list order = ascending (j, b)
            for (uint64_t rem = rm; rem; rem &= rem - 1) {
                const int jj = ctz64(rem);
                const unsigned bm = g.shfl(rb, jj);
                const int c = __popc(bm);
                if (k < c) { j = jj; b = nth_bit(bm, k); return; }
                k -= c;
            }
            j = b = -1;
        } else if (k == before) {
            j = b = -1;
        } else {                                    // agent order
            j = nth_bit64(am, k < before ? k : k - 1);
            b = g.shfl_i(asg, j);
        }
    };
    uint64_t occ = 0, mask = 7;
    uint32_t slots = 0;                             // element k's slot in bits [5k, 5k+5)
    int ka = -1, kb = -1;
    for (int k = 0; k < n && k < 6; ++k) {
        int j, b;
        elem(k, j, b);
        if (j == ja && b == ba) ka = k;
        if (j == jb && b == bb) kb = k;
        const int sl = pyset_probe(occ, mask, py_hash_pair(j, b));
        slots |= (uint32_t)sl << (5 * k);
        occ |= 1ull << sl;
        if ((uint64_t)(k + 1) * 5 >= mask * 3) {     // set_table_resize(used * 4): re-insert in slot order
            uint64_t ns = 8;
            while (ns <= (uint64_t)(k + 1) * 4) ns <<= 1;
            const uint64_t old = occ;
            occ = 0;
            mask = ns - 1;
            uint32_t nslots = 0;
            for (uint64_t rem = old; rem; rem &= rem - 1) {
                const int os = ctz64(rem);
                int m = 0;
                while (m < k && (int)((slots >> (5 * m)) & 31u) != os) ++m;
                int jm, bm;
                elem(m, jm, bm);
                const int s2 = pyset_probe(occ, mask, py_hash_pair(jm, bm));
                occ |= 1ull << s2;
                nslots |= (uint32_t)s2 << (5 * m);
            }
            slots = nslots;
        }
    }
    if (ka < 0 || kb < 0) return false;             // not reachable: both are members
    const int slot1 = (int)((slots >> (5 * ka)) & 31u), slot2 = (int)((slots >> (5 * kb)) & 31u);
    // the intersection inserts its members in that operand's slot order into a fresh set
    const uint64_t ha = py_hash_pair(ja, ba), hb = py_hash_pair(jb, bb);
    const bool first_is_b = slot1 > slot2;
    const int f = pyset_probe(0ull, 7, first_is_b ? hb : ha);
    const int s = pyset_probe(1ull << f, 7, first_is_b ? ha : hb);
    // iteration of the result set: ascending slot
    return (f < s) ? first_is_b : !first_is_b;
}

// fixActions' draw budget per call.  The reference loops until its work list
// drains; in a deadlock it never does.  Its own fixtures need at most 65 draws
// (N = 15, rotating picks); a terminating Philox walk needing more than this is
// not expected, a deadlock reaches it at once.  Shared with the oracle
// (OC_FIX_DRAWS).
__host__ __device__ constexpr int fix_draws(int N) { return 16 * N + 64; }

// Deadlock fallback (lane = agent): the agents left unplaced already hold
// assigned == 0; a mover whose target cell holds a staying agent reverts to
// stay, repeated until no mover is blocked.  The placed movers were pairwise
// conflict-free and staying agents occupy distinct cells, so the result has no
// shared cell and no swap; the fixpoint is unique (the oracle computes it in
// another order).  Only the newest stayers can block anyone: O(N) shuffles.
template <class GR>
__device__ inline void fix_revert_blocked(const GR &g, bool act, uint32_t pp, int &assigned) {
    uint64_t frontier = g.ballot(act && assigned == 0);
    while (frontier) {
        const uint32_t tgt = (act && assigned > 0) ? pack(prow(pp) + dr(assigned), pcol(pp) + dc(assigned)) : NO_CELL;
        bool blocked = false;
        for (uint64_t rem = frontier; rem; rem &= rem - 1)
            if (tgt == g.shfl(pp, ctz64(rem))) blocked = true;
        frontier = g.ballot(blocked);
        if (blocked) assigned = 0;
    }
}

}  // namespace mapf
