// primal-ppo_amd/csrc/mapf_reset.hip -- environment resets.
//
// Fixed (FixedMapfGym, mapf_gym.py:648-669 + populateMap :175-184): agent i
// starts at agentsSequence[i].getNext() and takes its first goal from the
// same Sequence (util.py:33-39); the human is a LoopingHuman (:52-63) or a
// FixedPathHuman (:72-81).  Human paths and BFS maps are computed by the
// search kernels right after (launch_replan / launch_bfs with all = true).
//
// Seeded (MapfGym, mapf_gym.py:164-184): Human.getEntrance (:19-23) = a
// free cell on row 0 or column 0, the human goal = getFreeCell of the world
// with the entrance marked, then for every agent in index order a start and
// a goal by getFreeCell on tempMap (obstacles, entrance, earlier starts and
// goals excluded; the agent's own start excluded for its goal).  Draws follow
// the Philox getFreeCell spec (mapf_group.h: group_free_cell).
#include "mapf_group.h"
#include "mapf_kernels.h"

namespace mapf {

__global__ __launch_bounds__(256) void reset_fixed_kernel(DevEnv e) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < e.B * e.N) {
        const uint32_t *s = e.seq + (size_t)t * e.S;
        const int len = e.seq_len[t];
        int cur = 0;
        const uint32_t start = s[cur < len ? cur++ : len - 1];
        const uint32_t goal = cur >= len ? s[len - 1] : s[cur++];
        e.pos[t] = start;
        e.goal[t] = goal;
        e.seq_cur[t] = cur;
        e.last_act[t] = -1;
    }
    if (t < e.B) {
        // the first path is searched into buffer hcur ^ 1 = 0, then promoted (launch_plan)
        e.hstep[t] = 0;
        e.hseq_idx[t] = 1;
        e.clock[t] = 0;
        e.hreplans[t] = 0;
        e.hcur[t] = 1;
        if (e.human_mode == 2) {
            e.hpos[t] = e.hseq[(size_t)t * e.HS + 0];
            e.hgoal[t] = e.hseq[(size_t)t * e.HS + 1];
        }
        e.hentr[t] = e.hpos[t];
        e.hnext_start[t] = e.hpos[t];
        e.hnext_goal[t] = e.hgoal[t];
    }
}

__global__ __launch_bounds__(256) void reset_seeded_kernel(DevEnv e) {
    const int G = e.G, N = e.N;
    const int gt = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = gt / G;
    if (b >= e.B) return;
    Group g(G);
    const int i = g.i;
    const bool act = i < N;
    const size_t ai = (size_t)b * N + i;
    const uint32_t env_id = e.env_offset + (uint32_t)b;
    const uint32_t *bits = env_map(e, b);
    int r, c;
    // Human.getEntrance: free and (row 0 or col 0)
    auto ok_ent = [&](int rr, int cc) { return !obstacle_at(e, bits, rr, cc) && (rr == 0 || cc == 0); };
    if (!group_free_cell(e, env_id, P_ENTRANCE, 0, 0u, ok_ent, r, c)) {
        if (i == 0) atomicAdd(&e.counters[C_FREECELL], 1u);
        r = 0; c = 0;
    }
    const uint32_t ent = pack(r, c);
    auto ok_hg = [&](int rr, int cc) { return !obstacle_at(e, bits, rr, cc) && pack(rr, cc) != ent; };
    if (!group_free_cell(e, env_id, P_HGOAL0, 0, 0u, ok_hg, r, c)) {
        if (i == 0) atomicAdd(&e.counters[C_FREECELL], 1u);
    }
    const uint32_t hgoal = pack(r, c);
    // populateMap: sequential over agents, tempMap excludes entrance, earlier starts and goals
    uint32_t my_start = 0xFFFFFFFFu, my_goal = 0xFFFFFFFFu;
    for (int k = 0; k < N; ++k) {
        auto ok_s = [&](int rr, int cc) -> bool {
            if (obstacle_at(e, bits, rr, cc)) return false;
            const uint32_t cell = pack(rr, cc);
            if (cell == ent) return false;
            return g.ballot(act && i < k && (my_start == cell || my_goal == cell)) == 0ull;
        };
        if (!group_free_cell(e, env_id, P_START, k, 0u, ok_s, r, c)) {
            if (i == k) atomicAdd(&e.counters[C_FREECELL], 1u);
        }
        if (i == k) my_start = pack(r, c);
        auto ok_g = [&](int rr, int cc) -> bool {
            if (obstacle_at(e, bits, rr, cc)) return false;
            const uint32_t cell = pack(rr, cc);
            if (cell == ent) return false;
            return g.ballot(act && ((i < k && (my_start == cell || my_goal == cell)) || (i == k && my_start == cell))) == 0ull;
        };
        if (!group_free_cell(e, env_id, P_GOAL0, k, 0u, ok_g, r, c)) {
            if (i == k) atomicAdd(&e.counters[C_FREECELL], 1u);
        }
        if (i == k) my_goal = pack(r, c);
    }
    if (act) {
        e.pos[ai] = my_start;
        e.goal[ai] = my_goal;
        e.last_act[ai] = -1;
        e.seq_cur[ai] = 0;
    }
    if (i == 0) {
        e.hentr[b] = ent;
        e.hpos[b] = ent;
        e.hgoal[b] = hgoal;
        e.hstep[b] = 0;
        e.hseq_idx[b] = 1;
        e.clock[b] = 0;
        e.hreplans[b] = 0;
        e.hcur[b] = 1;
        e.hnext_start[b] = ent;
        e.hnext_goal[b] = hgoal;
    }
}

void launch_reset_fixed(const DevEnv &e, hipStream_t s) {
    const int n = e.B * e.N > e.B ? e.B * e.N : e.B;
    hipLaunchKernelGGL(reset_fixed_kernel, dim3((n + 255) / 256), dim3(256), 0, s, e);
}

void launch_reset_seeded(const DevEnv &e, hipStream_t s) {
    const long threads = (long)e.B * e.G;
    hipLaunchKernelGGL(reset_seeded_kernel, dim3((int)((threads + 255) / 256)), dim3(256), 0, s, e);
}

}  // namespace mapf
