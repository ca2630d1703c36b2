// primal-ppo_amd/csrc/mapf_rollout_wide.hip -- T committed random-policy steps +
// observations in ONE launch for the configurations the pair-lane rollout kernel
// (mapf_fused.hip, N in 5..8 on a shared map up to 30 wide) does not cover: up to
// 64 agents, per-env maps up to 128 x 128, the BFS channel (C = 7) -- BASELINE
// configs c4 (1024 x 16 per GPU, 40 x 40) and c5 (2048 x 64 per GPU, 80 x 80).
//
// runner.py:64-100 with the uniform policy, T times, per env:
//     step (mapf_step.h: one lane per agent, the whole wave one group)
//     -> agent.bfsMap of every agent whose goal changed (mapf_gym.py:623-627; the
//        BFS channel of this step's observation reads them)
//     -> getAllObservations of the env (mapf_observe.h: LDS bit-stream -> float4)
//     -> the human's next path, if the step queued one (read two steps later at
//        the earliest: mapf_fused.hip)
// One workgroup = one wave = one env for the whole launch.  The split path runs
// the same work as three launches per step in lockstep over all envs, so every
// step waits for the slowest env's BFS chain and pays the launch gaps; here a
// wave searching an 80 x 80 map for ~100 us holds back only its own env while
// the other waves' observation stores keep HBM busy.
//
// The stepping wave keeps the env's state in registers (StepRegs) and stores it to HBM
// once, after its last step; the human's path buffers and lengths, the work the step
// reads back, stay in HBM (a wave's own stores are visible to its later loads).  LDS per wave:
// the nibble table, the env's padded map rows, and one scratch area shared by the
// observation (bit-stream, occupancy, agent grid) and the search (BFS image).
#include <cstdio>
#include <type_traits>

#define MAPF_WIDE_TU   // mapf_diag.h: no block-timeline stamps here (the WSTAMP rows use that region)

#include "mapf_observe.h"
#include "mapf_search.h"
#include "mapf_step.h"

namespace mapf {

struct WideOut {
    int32_t *actions;
    StepOut out;
    float *obs, *vec;
    int slots;
    int xcd_remap;
    int grid;           // the step's neighbour grid: 0 none (agent loop), 1 own LDS, 2 over the scratch
    int overlap;        // pipelined, no BFS channel: one barrier per step (wide_overlap_bytes)
    int exp;            // diagnostic (stamps) builds only (mapf_tuning.diag_exp), 1: no observation
    int prio;           // pipelined: the stepping wave's issue priority (s_setprio; mapf_tuning.wide_prio, default 1: c4 -1.6 %)
    int wpe;            // waves per env: 2 pipelined (stepper + observer), 1 one wave takes both roles
    int epw;            // envs per workgroup (all the envs of one CU, wide_envs_per_group)
    int pair;           // epw > 1: wave w is env w % epw's role w / epw (1), else env w / wpe's role w % wpe (0)
    int slack;          // epw > 1: a pacing wave runs at most `slack` steps ahead of its group's slowest env (< 0: off)
    int env_lds;        // epw > 1: LDS bytes per env (a multiple of 16); the pacing counters follow the envs
    int bfsobs;         // three-wave form: the observers search the BFS maps (mapf_tuning.wide_bfsobs, default 1)
    int fair;           // one-wave form, epw > 1, > 0: a wave more than `fair` steps ahead of its group's slowest
                        // env issues at priority 0, the others at 2, instead of waiting (mapf_tuning.wide_fair)
};

// the kernel's arguments, read from device memory (ArgRing, mapf_kernels.h)
struct WideArgs {
    DevEnv e;
    WideOut ro;
};

__host__ __device__ inline size_t wide_a16(size_t x) { return (x + 15) & ~(size_t)15; }

// observation part of the scratch area: stream | occ | spos | sgoal | shn | shp | shpn | idg
__host__ __device__ inline size_t wide_obs_bytes(const DevEnv &e) {
    const size_t words = (size_t)obs_env_stream_words(e) + (size_t)e.Hp * e.WW + 2 * (size_t)e.N + 1 + e.k_predict + 1;
    return words * 4 + (((size_t)e.H * e.W + 3) & ~(size_t)3);
}

template <class T, int RW>
__host__ __device__ inline size_t wide_scratch_bytes(const DevEnv &e) {
    const size_t o = wide_obs_bytes(e), s = srch::wave_lds<T, RW>(e.H, e.W);
    return wide_a16(o > s ? o : s);
}

// the cost table (calculateCostReward's, R*R + 1 floats) gets an LDS copy up to 1 KiB
__host__ __device__ inline size_t wide_cost_bytes(const DevEnv &e) {
    const size_t n = ((size_t)e.R * e.R + 1) * 4;
    return n <= 1024 ? wide_a16(n) : 0;
}

__host__ __device__ inline size_t wide_grid_bytes(const DevEnv &e) { return wide_a16((size_t)(e.H + 4) * (e.W + 4) * 2); }

// the overlapped pipeline's own areas: a second observation snapshot (spos | sgoal | shn |
// shp | shpn) and the stepper's BFS image
// (+ 2 words after shpn: the agents whose BFS maps the step rebuilds, when the observers search them)
__host__ __device__ inline size_t wide_snap_bytes(const DevEnv &e) { return wide_a16((size_t)(2 * e.N + 4 + e.k_predict) * 4); }
// overlapped form: a ring of WIDE_SNAPS snapshots behind two LDS counters (16 B), so the
// stepper may run up to WIDE_SNAPS - 1 steps ahead of the observer
constexpr int WIDE_SNAPS = 4;
template <class T, int RW>
__host__ __device__ inline size_t wide_overlap_bytes(const DevEnv &e) {
    return 16 + WIDE_SNAPS * wide_snap_bytes(e) + srch::wave_lds<T, RW>(e.H, e.W);
}

// nibble table (256 B) | map rows | cost table | [neighbour grid] | scratch | [snapshot 1 | BFS image]
template <class T, int RW>
__host__ __device__ inline size_t wide_lds_bytes(const DevEnv &e, int grid = 0, bool overlap = false) {
    return 256 + wide_a16((size_t)e.Hp * e.WW * 4) + wide_cost_bytes(e) + (grid == 1 ? wide_grid_bytes(e) : 0) +
           wide_scratch_bytes<T, RW>(e) + (overlap ? wide_overlap_bytes<T, RW>(e) : 0);
}

__device__ inline ObsLds wide_layout(const DevEnv &e, char *smem, int gmode, char *&scratch, float *&cost,
                                    uint8_t *&grid) {
    ObsLds L;
    const int rowsz = e.Hp * e.WW;
    L.lut = reinterpret_cast<const float4 *>(smem);
    L.mapc = reinterpret_cast<uint32_t *>(smem + 256);
    char *cp = smem + 256 + wide_a16((size_t)rowsz * 4);
    cost = wide_cost_bytes(e) ? reinterpret_cast<float *>(cp) : nullptr;
    scratch = cp + wide_cost_bytes(e) + (gmode == 1 ? wide_grid_bytes(e) : 0);
    grid = gmode == 1 ? reinterpret_cast<uint8_t *>(cp + wide_cost_bytes(e))
                      : (gmode == 2 ? reinterpret_cast<uint8_t *>(scratch) : nullptr);
    L.swe = obs_env_stream_words(e);           // a multiple of 4 words
    L.stream_words = L.swe;
    L.rowsz = rowsz;
    L.stream = reinterpret_cast<uint32_t *>(scratch);
    L.occ = L.stream + L.swe;
    L.spos = L.occ + rowsz;
    L.sgoal = L.spos + e.N;
    L.shn = L.sgoal + e.N;
    L.shp = L.shn + 1;
    L.shpn = reinterpret_cast<int32_t *>(L.shp + e.k_predict);
    L.bfsw = nullptr;
    L.bfsown = nullptr;
    L.idg = reinterpret_cast<uint8_t *>(L.shpn + 1);
    L.bfs_win = false;                         // BFS channel straight from the tiled maps
    return L;
}

// the overlapped form's LDS counters (mapf_group.h: lds_count, publish_count)
__device__ inline void wide_wait_ge(const uint32_t *c, uint32_t v) {
    while (lds_count(c) < v) __builtin_amdgcn_s_sleep(1);
}

__device__ inline void wide_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Two-wave pipelined form (128-thread workgroups, where every env's two waves fit on the
// chip at once): wave 0 steps, wave 1 observes the step before from the LDS snapshot,
//     stepper  | step t | A | BFS maps t, snapshot t | B | human path t | step t+1 | A ...
//     observer |  observe t-1  | A |  (waits)        | B |      observe t         | A ...
// so a step's latency-bound chains run while the previous observation's stores issue.
// BFS maps of step t are written between A (observation t-1, which reads the old maps,
// is done) and B; both waves share one scratch area (the BFS image overlays the
// observation's bit-stream, unused between A and B).  Only a step that rebuilt BFS maps
// releases its global stores before B; otherwise neither wave waits on memory at a
// barrier, so the observer's stores and the stepper's outputs keep draining across them.
// Overlapped (no BFS channel, so the observation reads no BFS map): the stepper searches in
// its own BFS image and publishes snapshot t into ring slot t % WIDE_SNAPS through an LDS
// counter; the observer waits for that counter, observes, and counts its observations, which
// the stepper checks only before reusing a slot -- no barrier:
//     stepper  | step t | BFS maps t | snapshot t, published | human path t | step t+1 ...
//     observer | (t published?) | observe t, counted | (t+1 published?) | observe t+1 ...
// so per step the slower wave's MEAN sets the pace, not the mean of the per-step maximum of
// two noisy chains (a barrier per step made each wait for the other's slow steps).
__device__ inline void wide_release_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ inline void wide_plain_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0): the LDS reads of the store loop are done
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// waves_per_eu(2): at most 256 VGPRs, so two waves of every SIMD stay resident (c5: 2,048
// envs = 8 waves per CU; above 256 the launch would run in two rounds)
// MAPF_ARGS_PTR=1 (experiment build, `make argptr`): the arguments are read through a
// device pointer (ArgRing) instead of the kernarg segment -- 123 instead of 454 SGPR spills,
// but every field is then re-loaded through the scalar cache where it is used, and the
// stepper measured slower
#if MAPF_ARGS_PTR
#define WIDE_PARAMS const WideArgs *__restrict__ args, int T_steps
#define WIDE_BIND const DevEnv &e = args->e; const WideOut &ro = args->ro;
#else
#define WIDE_PARAMS DevEnv e, int T_steps, WideOut ro
#define WIDE_BIND
#endif

template <class T, int RW, bool NT>
__device__ __attribute__((always_inline)) inline void rollout_wide_body(const DevEnv &e, int T_steps, const WideOut &ro) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // XCD-aware env order (as the pair-lane rollout): workgroups are dealt round-robin
    // over the 8 XCDs, so each XCD owns one contiguous range of envs
    const int nb = (int)gridDim.x;
    const int wg = (ro.xcd_remap && (nb & 7) == 0) ? ((int)blockIdx.x & 7) * (nb >> 3) + ((int)blockIdx.x >> 3)
                                                   : (int)blockIdx.x;
    // envs per workgroup: all the envs of one CU in one group (the host checks B % epw == 0),
    // so a pacing wave sees how far the group's other envs are
    const int EPW = ro.epw, wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // wave-uniform
    const int k = ro.pair ? wv % EPW : wv / ro.wpe;    // this wave's env in the group
    const int role = ro.pair ? wv / EPW : wv % ro.wpe; // pipelined: 0 steps, 1.. observe
    const int b = wg * EPW + k;
    if (wg * EPW >= e.B) return;
    const int lane = lane_id();
    const bool pipe = ro.wpe >= 2;
    // observing waves per env (pipelined): observer o (role 1 + o) observes the steps t with
    // t % nobs == o
    const int nobs = pipe ? ro.wpe - 1 : 1, obs_o = pipe ? max(role - 1, 0) : 0;
    const int lt = role * 64 + lane, nthr = ro.wpe * 64;   // thread index within the env's waves
    char *esm = smem + (size_t)k * ro.env_lds;
    uint32_t *prog = reinterpret_cast<uint32_t *>(smem + (size_t)EPW * ro.env_lds);   // [EPW] steps observed
    const bool pacing = EPW > 1 && ro.slack >= 0;
    const bool fairw = EPW > 1 && ro.fair > 0 && !(ro.wpe >= 2);
    char *scratch;
    float *lcost;
    uint8_t *grid;
    ObsLds L = wide_layout(e, esm, ro.grid, scratch, lcost, grid);
    const bool ovl = pipe && ro.overlap;
    char *bimg = scratch;                              // where the stepper's BFS maps search
    // overlapped: ctr [0] snapshots published, [1 + o] steps observer o has observed
    uint32_t *ctr = nullptr;
    uint32_t *snap0 = nullptr;                         // overlapped: the snapshot ring
    if (ovl) {
        char *x = scratch + wide_scratch_bytes<T, RW>(e);
        ctr = reinterpret_cast<uint32_t *>(x);
        snap0 = reinterpret_cast<uint32_t *>(x + 16);
        bimg = x + 16 + WIDE_SNAPS * wide_snap_bytes(e);
        if (lt < 4) ctr[lt] = 0u;
        if (obs_o > 0) {                               // observers past the first: their own scratch
            const ptrdiff_t d = (bimg + srch::wave_lds<T, RW>(e.H, e.W) +
                                 (size_t)(obs_o - 1) * wide_scratch_bytes<T, RW>(e)) - scratch;
            L.stream = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(L.stream) + d);
            L.occ = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(L.occ) + d);
            L.idg = L.idg + d;
        }
    }
    auto snap_of = [&](int t) {                        // this step's snapshot
        ObsLds S = L;
        if (ovl) {
            S.spos = snap0 + (size_t)(t & (WIDE_SNAPS - 1)) * (wide_snap_bytes(e) >> 2);
            S.sgoal = S.spos + e.N;
            S.shn = S.sgoal + e.N;
            S.shp = S.shn + 1;
            S.shpn = reinterpret_cast<int32_t *>(S.shp + e.k_predict);
        }
        return S;
    };
    if (lt < 16)
        const_cast<float4 *>(L.lut)[lt] = make_float4((float)(lt & 1), (float)((lt >> 1) & 1), (float)((lt >> 2) & 1), (float)(lt >> 3));
    if (EPW > 1 && (int)threadIdx.x < EPW) prog[threadIdx.x] = 0u;
    const uint32_t *mb = env_map(e, b);
    for (int q = lt; q < L.rowsz; q += nthr) L.mapc[q] = mb[q];
    if (lcost)
        for (int q = lt; q <= e.R * e.R; q += nthr) lcost[q] = e.cost_lut[q];
    __syncthreads();
    StepRegs rs;                           // the stepping wave keeps the env's state in registers
    step_regs_load(e, b, lane, rs);
    // the registers' loads done before the loop: with one still counted at the loop header,
    // the top of every step waited vmcnt(0), i.e. for the previous step's output stores too
    __builtin_amdgcn_s_waitcnt(0x0F70);     // vmcnt(0), expcnt/lgkmcnt untouched
    const StepSrc src{L.mapc, lcost, grid};   // obstacle tests, cost table, neighbour grid in LDS
    const WaveGroup g;                     // the env is the whole wave: exchanges by v_readlane
    const size_t BN = (size_t)e.B * e.N, CFF = (size_t)e.C * e.F * e.F;
    // this lane's output elements as VGPR pointers (step_group<.., LANEPTR>): the nine output
    // bases and the actions base would otherwise hold 20 SGPRs through the loop -- spilled to
    // VGPR lanes and read back (v_readlane pairs) at every store.  Slot buffers advance them
    // by one [B, N] slice per step.
    const size_t lai = (size_t)b * e.N + (size_t)min(lane, e.N - 1);
    auto vptr = [](auto *p, size_t off) {
        uint64_t v = p ? (uint64_t)(p + off) : 0ull;
        asm volatile("" : "+v"(v));          // opaque and lane-held: never re-derived from the base
        return reinterpret_cast<decltype(p)>(v);
    };
    const StepOut &O = ro.out;
    const uint32_t have = (O.status ? 1u : 0u) | (O.reward ? 2u : 0u) | (O.shadow_goals ? 4u : 0u) |
                          (O.cost ? 8u : 0u) | (O.train_valid ? 16u : 0u) | (O.actions_fixed ? 32u : 0u) |
                          (O.goals_reached ? 64u : 0u) | (O.constraints ? 128u : 0u) | (O.reward_total ? 256u : 0u);
    const StepOut lo{vptr(O.status, lai), vptr(O.reward, lai), vptr(O.shadow_goals, (size_t)b), vptr(O.cost, lai),
                     vptr(O.train_valid, lai * NA), vptr(O.actions_fixed, lai), vptr(O.goals_reached, lai),
                     vptr(O.constraints, lai), vptr(O.reward_total, lai)};
    int32_t *const lact = vptr(ro.actions, lai);
    auto step_out = [&](size_t s) {      // slot s of every output (s = 0: the [B]-leading buffers)
        StepOut o = lo;
        if (s) {
            o.status += s * BN;
            o.reward += s * BN;
            o.shadow_goals += s * e.B;
            o.cost += s * BN;
            o.train_valid += s * BN * NA;
            o.actions_fixed += s * BN;
            o.goals_reached += s * BN;
            o.constraints += s * BN;
            o.reward_total += s * BN;
        }
        return o;
    };
    auto bfs_maps = [&](const StepInline &inl) {
        for (uint64_t m = inl.bmask; m; m &= m - 1ull) {
            const int l = ctz64(m);
            const uint32_t gl = (uint32_t)__builtin_amdgcn_readlane((int)inl.goal, l);
            srch::search_one<T, RW>(e, false, b, (uint32_t)b * (uint32_t)e.N + (uint32_t)l, gl, NO_CELL, 0, bimg,
                                    L.mapc);
        }
    };
    // one loop for both forms (every function inlined once: the kernel's code stays
    // within the instruction cache); unpipelined, the one wave takes both roles in the
    // order step -> BFS maps -> snapshot -> human path -> observe
    bool stepper = !pipe || role == 0, observer = !pipe || role >= 1;
    // the stepping wave bounds the pipeline and shares its SIMD with another env's observing
    // wave, whose work waits on store issue anyway: it goes first when both are ready
    if (pipe && stepper && ro.prio) __builtin_amdgcn_s_setprio(3);
    bool observing = true;                 // overlapped form: some wave consumes the snapshots
#ifdef MAPF_STAMPS
    // phase-cost experiment (no observations written): the stepping role alone
    if (ro.exp == 1) observer = observing = false;
#endif
    // Three-wave form: the BFS maps of the agents whose goal changed (nothing in the loop reads
    // them without the BFS channel) are searched by the observer of that step, after its
    // observation, instead of on the stepper's chain (c4: 0.59 of its 4.63 us per step).  Step
    // t's maps are written after step t - 1's (ctr[3]: steps whose maps are done), so an agent's
    // later map wins; an observer that searched drains its stores before it counts.
    const bool bfs_obs = ovl && nobs >= 2 && observing && ro.bfsobs;
    // several observers writing the same in-place buffers, in alternation
    const bool inplace_multi = ovl && nobs >= 2 && observing && !ro.slots;
    WSTAMP_BEGIN();
    for (int t = 0; t < T_steps; ++t) {
        const size_t s = ro.slots ? (size_t)t : 0;
        if (pacing && !pipe && t > ro.slack) wait_group_min(prog, EPW, (uint32_t)(t - ro.slack));
        if (fairw) {
            if ((uint32_t)t > group_min(prog, EPW) + (uint32_t)ro.fair) __builtin_amdgcn_s_setprio(0);
            else __builtin_amdgcn_s_setprio(2);
        }
        StepInline inl;
        if (stepper) step_group<WaveGroup, true, true>(e, lact + s * BN, step_out(s), 3u, 0, b, g, &inl, src, rs, have);
        WSTAMP(0);
        // A: observation t-1 done.  Nothing the observer reads from HBM was written by the step
        // (its outputs and state are not read back), so the stepper does not wait for them.
        if (pipe && !ovl) wide_plain_barrier();
        const ObsLds Lt = snap_of(t);
        if (stepper) {
            if (!bfs_obs) bfs_maps(inl);                 // agent.bfsMap of the agents whose goal changed
            // the slot's previous snapshot (step t - WIDE_SNAPS) has been observed
            if (ovl && observing && t >= WIDE_SNAPS) {
                const int tt = t - WIDE_SNAPS;             // its observer's (tt / nobs + 1)-th step
                wide_wait_ge(ctr + 1 + tt % nobs, (uint32_t)(tt / nobs + 1));
            }
            // snapshot of step t for the observation, all from the registers: cells, goals,
            // the human's next cell and path cells [1..K] (HP channel)
            if (lane < e.N) { Lt.spos[lane] = rs.pp; Lt.sgoal[lane] = rs.gg; }
            const bool hp_ch = e.use_hp && e.C >= 6;
            if (hp_ch && rs.hq != NO_CELL) Lt.shp[lane - 1] = rs.hq;
            if (lane == 0) {
                Lt.shn[0] = rs.hn;
                const int len = rs.hcur ? rs.hl1 : rs.hl0;
                Lt.shpn[0] = hp_ch ? max(0, min(e.k_predict, len - 1)) : 0;
                if (bfs_obs) {
                    reinterpret_cast<uint32_t *>(Lt.shpn)[1] = (uint32_t)inl.bmask;
                    reinterpret_cast<uint32_t *>(Lt.shpn)[2] = (uint32_t)(inl.bmask >> 32);
                }
            }
            if (ovl) publish_count(ctr, (uint32_t)(t + 1));
        }
        WSTAMP(1);
        // B: snapshot t in LDS; the stepper releases only when it rebuilt BFS maps (the
        // observation's BFS channel reads them from HBM)
        if (pipe && !ovl) { if (stepper && inl.bmask) wide_release_barrier(); else wide_plain_barrier(); }
        // the human's next path, into the other buffer (registers only: the observer may be
        // using the scratch by now)
        if (stepper && inl.replan) {
            const int len = srch::search_one<T, RW>(e, true, b, 0u, inl.rstart, inl.rgoal, inl.rbuf, scratch, L.mapc);
            if (inl.rbuf) rs.hl1 = len;
            else rs.hl0 = len;
        }
        WSTAMP(2);
        if (observer && (nobs == 1 || t % nobs == obs_o)) {
            for (int k = lane; k < L.swe + L.rowsz; k += 64) L.stream[k] = 0u;   // stream then occ
            if (ovl) wide_wait_ge(ctr, (uint32_t)(t + 1));   // snapshot t published
            if (pacing && pipe && t > ro.slack) wait_group_min(prog, EPW, (uint32_t)(t - ro.slack));
            wide_sync();
#ifdef MAPF_STAMPS
            const ObsGroup G{lane, 64, 0, 1, L.stream, L.mapc, true, ro.exp};   // exp 2 / 3: mapf_observe.h
#else
            const ObsGroup G{lane, 64, 0, 1, L.stream, L.mapc, true};
#endif
            obs_emit<true, NT>(e, Lt, ro.obs + s * BN * CFF, ro.vec + s * BN * 4, G, b, false);
            wide_sync();
            uint64_t bm = 0;
            uint32_t mygoal = 0;
            if (bfs_obs) {                               // out of the snapshot before its slot is freed
                const uint32_t *w = reinterpret_cast<const uint32_t *>(Lt.shpn) + 1;
                bm = (uint64_t)lds_count(w) | ((uint64_t)lds_count(w + 1) << 32);
                mygoal = Lt.sgoal[min(lane, e.N - 1)];
            }
            // in place with several observers, the [B] buffer's last writer must be step T - 1's:
            // each observer's last observation drains (vmcnt(0)) before it counts, and the final
            // step's observer re-writes its observation once the others have (after the loop)
            if (inplace_multi && t + nobs >= T_steps) __builtin_amdgcn_s_waitcnt(0x0F70);
            if (ovl) publish_count(ctr + 1 + obs_o, (uint32_t)(t / nobs + 1));   // ... and observed
            if (pacing || fairw) publish_count(prog + k, (uint32_t)(t + 1));
            if (bfs_obs) {
                wide_wait_ge(ctr + 3, (uint32_t)t);      // step t - 1's maps written
                for (uint64_t m = bm; m; m &= m - 1ull) {
                    const int l = ctz64(m);
                    const uint32_t gl = (uint32_t)__builtin_amdgcn_readlane((int)mygoal, l);
                    srch::search_one<T, RW>(e, false, b, (uint32_t)b * (uint32_t)e.N + (uint32_t)l, gl, NO_CELL, 0,
                                            reinterpret_cast<char *>(L.stream), L.mapc);
                }
                if (bm) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the maps land before step t + 1's
                publish_count(ctr + 3, (uint32_t)(t + 1));
            }
        }
        WSTAMP(3);
    }
    // In place, observers take alternate steps into the same [B] buffers, so step T - 2's stores
    // (another wave's) may land after step T - 1's: once every other observer's last observation
    // has drained, step T - 1's observer writes its observation again (its snapshot is still in the
    // ring: the stepper has stopped) -- one extra observation per env per launch
    if (inplace_multi && observer && T_steps >= 2 && (T_steps - 1) % nobs == obs_o) {
        for (int o2 = 0; o2 < nobs; ++o2)
            if (o2 != obs_o) wide_wait_ge(ctr + 1 + o2, (uint32_t)((T_steps - o2 + nobs - 1) / nobs));
        const ObsLds Lt = snap_of(T_steps - 1);
        for (int k = lane; k < L.swe + L.rowsz; k += 64) L.stream[k] = 0u;
        wide_sync();
#ifdef MAPF_STAMPS
        const ObsGroup G{lane, 64, 0, 1, L.stream, L.mapc, true, ro.exp};
#else
        const ObsGroup G{lane, 64, 0, 1, L.stream, L.mapc, true};
#endif
        obs_emit<true, NT>(e, Lt, ro.obs, ro.vec, G, b, false);
    }
    if (stepper) step_regs_store(e, b, lane, rs);
    WSTAMP_END(b, role);
}

template <class T, int RW, bool NT>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void rollout_wide_kernel(WIDE_PARAMS) {
    WIDE_BIND
    rollout_wide_body<T, RW, NT>(e, T_steps, ro);
}

// Three waves per env (c4): the stepper and two observers taking alternate steps.  With one
// observer c4 was bounded by it (5.75 us per step against the stepper's 4.45: one wave per
// SIMD issuing each step's 31 KiB of stores).  Three waves per SIMD need <= 168 VGPRs:
// the arguments come through a device pointer (ArgRing), which also frees the ~450 SGPRs the
// by-value arguments spilled to VGPR lanes (152 VGPRs, 129 SGPR spills, no scratch).
template <class T, int RW, bool NT>
__global__ __launch_bounds__(768) __attribute__((amdgpu_waves_per_eu(3))) void rollout_wide3_kernel(
    const WideArgs *__restrict__ args, int T_steps) {
    rollout_wide_body<T, RW, NT>(args->e, T_steps, args->ro);
}

// The three-wave form is not built for 128-bit rows spread over two lanes (maps wider than 64 cells):
// capped at 168 VGPRs (three waves per SIMD), <Row2,2> spilled 136-188 B per lane to scratch
// and <Row2,1> 12 B (4-5 scratch instructions, tools/scratch_audit.py).  Such maps take
// the one- or two-wave form (no BASELINE config is a wide map without the BFS channel, which the
// three-wave form excludes anyway).
template <class T, int RW>
constexpr bool wide3_form() { return !std::is_same<T, srch::Row2>::value; }

template <class T, int RW>
static bool wide_fits(const DevEnv &e) { return wide_lds_bytes<T, RW>(e) <= 64 * 1024; }

// The launch form for this handle's tuning (mapf.h: mapf_tuning; the measured defaults below)
struct WidePlan {
    bool nt = false;     // nontemporal observation stores
    WideOut r{};         // the form fields (no pointers)
    size_t lds = 0;
    int grid = 0, block = 0;
};

template <class T, int RW>
static WidePlan plan_wide_t(const DevEnv &e, int slots, const mapf_tuning &tu) {
    WidePlan p;
    // persistent waves: every CU holds the same number of workgroups (the LDS request caps
    // them at ceil(B / CUs) per CU, 160 KiB of LDS per CU), or the fuller CUs pace each step
    const int ncu = device_cu_count();
    const int occ = (e.B + ncu - 1) / ncu;
    const size_t cap = ((size_t)160 * 1024 / (size_t)occ) & ~(size_t)255;
    // nontemporal observation stores for slot buffers (fresh lines every step) and for a
    // re-written [B] buffer too large to stay resident in the 256 MiB Infinity Cache (c5:
    // 446 MB, measured 94 vs 124 us per step); smaller ones keep plain stores (c2, c4;
    // c4 in place, nt sc1: 6.27 -> 7.03 us per step)
    p.nt = tu.wide_nt >= 0 ? tu.wide_nt != 0 : (slots || (size_t)e.B * e.N * e.C * e.F * e.F * 4 > ((size_t)128 << 20));
    const void *kern = p.nt ? reinterpret_cast<const void *>(rollout_wide_kernel<T, RW, true>)
                            : reinterpret_cast<const void *>(rollout_wide_kernel<T, RW, false>);
    const void *kern3 = nullptr;
    if constexpr (wide3_form<T, RW>())
        kern3 = p.nt ? reinterpret_cast<const void *>(rollout_wide3_kernel<T, RW, true>)
                     : reinterpret_cast<const void *>(rollout_wide3_kernel<T, RW, false>);
    // two waves per env where every env's pair fits at once: the VGPR budget of a SIMD
    // (512 per lane) over the waves it must hold, 4 SIMDs per CU
    const int fit = 512 / ((kernel_vgprs(kern) + 7) & ~7);
    const bool pipe = (2 * e.B + 4 * ncu - 1) / (4 * ncu) <= fit && tu.wide_pipe != 0;
    // the step's neighbour grid: over the scratch when one wave takes both roles (the step
    // runs while the scratch is free), else its own LDS if every env still fits
    WideOut &r = p.r;
    r.slots = slots;
    r.xcd_remap = tu.xcd_remap != 0;
    r.prio = tu.wide_prio;
    r.bfsobs = tu.wide_bfsobs;
    r.grid = 0;
    if (!pipe && wide_grid_bytes(e) <= wide_scratch_bytes<T, RW>(e)) r.grid = 2;
    else if (wide_lds_bytes<T, RW>(e, 1) <= (occ > 1 ? cap : (size_t)64 * 1024)) r.grid = 1;
    if (tu.wide_grid == 0) r.grid = 0;
    // one barrier per step where the observation reads no BFS map and the extra LDS fits
    r.overlap = pipe && e.C < 7 && wide_lds_bytes<T, RW>(e, r.grid, true) <= (occ > 1 ? cap : (size_t)64 * 1024) &&
                tu.wide_overlap != 0;
#ifdef MAPF_STAMPS
    r.exp = tu.diag_exp;
#endif
    size_t lds = wide_lds_bytes<T, RW>(e, r.grid, r.overlap);
    r.wpe = pipe ? 2 : 1;
    // a second observer (overlapped form) where three waves per env fit on the chip at once,
    // its scratch fits the CU's LDS share, and all the envs of a CU fit one workgroup (<= 12
    // waves): three-wave workgroups dealt to a CU one by one did not always land 3 + 3 + 3 + 3
    // on its SIMDs -- a SIMD asked for a fourth wave (4 x 152 VGPRs > 512) and part of the grid
    // ran in a second round (c4: 6.2 or 8.3 us per step by launch); one workgroup per CU is
    // spread evenly
    const int fit3 = kern3 ? 512 / ((kernel_vgprs(kern3) + 7) & ~7) : 0;
    const size_t lds3 = wide_a16(lds + wide_scratch_bytes<T, RW>(e));
    if (kern3 && r.overlap && (3 * e.B + 4 * ncu - 1) / (4 * ncu) <= fit3 && lds3 <= (occ > 1 ? cap : (size_t)64 * 1024) &&
        e.B % occ == 0 && 3 * occ <= 12 && (size_t)occ * lds3 + 32 <= (size_t)device_max_group_lds() &&
        tu.wide_obs >= 2) {
        r.wpe = 3;
        lds = lds3;
    }
    // one wave per env (c5): all the envs of a CU in one workgroup (<= 8 waves:
    // launch_bounds(512) keeps the 256-VGPR budget), each env's LDS at its own offset, then
    // the pacing counters; every wave runs at most `slack` steps ahead of its group's
    // slowest env.  Unpaced, the younger wave of every SIMD (the CU's last-dispatched four
    // envs) ran 8 % slower than the older one through the whole launch and the launch
    // waited for it (tools/stamps_wide.py, "by dispatch rank in CU"): c5 85.5-85.9 -> 79.8
    // us per step, slack 1 (2: 80.0-80.7, 4: 80.9-81.3, 8: 82.4-83.1, groups unpaced 86.8).
    // The barrier-paced pipeline would couple the envs of a group, so never there.
    r.env_lds = (int)wide_a16(lds);
    r.epw = 1;
    const int epw = tu.wide_epw > 0 ? tu.wide_epw : (pipe ? (r.wpe == 3 ? occ : 1) : occ);
    if (epw > 1 && e.B % epw == 0 && epw * r.wpe <= (r.wpe == 3 ? 12 : 8) && (!pipe || r.overlap) &&
        (size_t)epw * r.env_lds + 32 <= (size_t)device_max_group_lds())
        r.epw = epw;
    r.pair = tu.wide_pair;
    // pacing counters count observations: with two observers per env, not in order (no pacing).
    // The stamps build's stepping-only experiment (diag_exp 1) publishes no progress: no pacing.
    const bool stepping_only = r.exp == 1;
    r.fair = r.wpe == 1 && !stepping_only ? tu.wide_fair : 0;
    r.slack = (r.wpe == 3 || r.fair > 0 || stepping_only) ? -1 : tu.wide_slack;
    if (r.epw > 1) lds = (size_t)device_max_group_lds();   // the whole CU: one group per CU
    else if (cap > lds && cap <= 64 * 1024) lds = cap;
    p.lds = lds;
    p.grid = e.B / r.epw;
    p.block = 64 * r.wpe * r.epw;
    return p;
}

template <class T, int RW>
static int launch_wide_t(const DevEnv &e, int steps, const WideOut &ro, const mapf_tuning &tu, ArgRing &ring,
                         hipStream_t s) {
    const WidePlan p = plan_wide_t<T, RW>(e, ro.slots, tu);
    WideOut r = p.r;
    r.actions = ro.actions;
    r.out = ro.out;
    r.obs = ro.obs;
    r.vec = ro.vec;
    if constexpr (wide3_form<T, RW>()) {
        if (r.wpe == 3) {
            const WideArgs *args = push_args(ring, WideArgs{e, r}, s);
            if (!args) return MAPF_ESTATE;
            auto kern3 = p.nt ? rollout_wide3_kernel<T, RW, true> : rollout_wide3_kernel<T, RW, false>;
            hipLaunchKernelGGL(kern3, dim3(p.grid), dim3(p.block), p.lds, s, args, steps);
            return MAPF_OK;
        }
    }
    auto kern = p.nt ? rollout_wide_kernel<T, RW, true> : rollout_wide_kernel<T, RW, false>;
#if MAPF_ARGS_PTR
    const WideArgs *args = push_args(ring, WideArgs{e, r}, s);
    if (!args) return MAPF_ESTATE;
    hipLaunchKernelGGL(kern, dim3(p.grid), dim3(p.block), p.lds, s, args, steps);
#else
    (void)ring;
    hipLaunchKernelGGL(kern, dim3(p.grid), dim3(p.block), p.lds, s, e, steps, r);
#endif
    return MAPF_OK;
}

template <class T> constexpr const char *row_name() {
    return std::is_same<T, uint32_t>::value ? "u32" : (std::is_same<T, uint64_t>::value ? "u64" : "Row2");
}

// the search row type of a W-wide map; RW = 2 above 64 rows
template <class F>
static auto with_row_type(const DevEnv &e, F f) {
    const bool two = e.H > 64;
    if (e.W <= 32) return two ? f(uint32_t{}, std::integral_constant<int, 2>{}) : f(uint32_t{}, std::integral_constant<int, 1>{});
    if (e.W <= 64) return two ? f(uint64_t{}, std::integral_constant<int, 2>{}) : f(uint64_t{}, std::integral_constant<int, 1>{});
    return two ? f(srch::Row2{}, std::integral_constant<int, 2>{}) : f(srch::Row2{}, std::integral_constant<int, 1>{});
}

bool rollout_wide_fusable(const DevEnv &e) {
    // the HP snapshot holds human.path[1..k_predict] one lane per cell (lanes 1..63)
    if (e.use_hp && e.C >= 6 && e.k_predict > 63) return false;
    return with_row_type(e, [&](auto t, auto rw) { return wide_fits<decltype(t), decltype(rw)::value>(e); });
}

int launch_rollout_wide(const DevEnv &e, int T, int32_t *actions, const StepOut &out, float *obs, float *vec,
                        int slots, const mapf_tuning &tu, ArgRing &ring, hipStream_t s) {
    WideOut ro{};
    ro.actions = actions;
    ro.out = out;
    ro.obs = obs;
    ro.vec = vec;
    ro.slots = slots;
    return with_row_type(e, [&](auto t, auto rw) {
        return launch_wide_t<decltype(t), decltype(rw)::value>(e, T, ro, tu, ring, s);
    });
}

void describe_rollout_wide(const DevEnv &e, int slots, const mapf_tuning &tu, char *buf, size_t n) {
    with_row_type(e, [&](auto t, auto rw) {
        const WidePlan p = plan_wide_t<decltype(t), decltype(rw)::value>(e, slots, tu);
        std::snprintf(buf, n, "%s<%s,%d,%s> grid=%d block=%d lds=%zu wpe=%d epw=%d grid_mode=%d overlap=%d slack=%d "
                              "fair=%d prio=%d bfsobs=%d pair=%d remap=%d",
                      p.r.wpe == 3 ? "rollout_wide3_kernel" : "rollout_wide_kernel", row_name<decltype(t)>(),
                      (int)decltype(rw)::value, p.nt ? "true" : "false", p.grid, p.block, p.lds, p.r.wpe, p.r.epw,
                      p.r.grid, p.r.overlap, p.r.slack, p.r.fair, p.r.prio, p.r.bfsobs, p.r.pair, p.r.xcd_remap);
        return 0;
    });
}

}  // namespace mapf
