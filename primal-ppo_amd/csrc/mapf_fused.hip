// primal-ppo_amd/csrc/mapf_fused.hip -- jointStep + getAllObservations in one
// launch (runner.py:84-97 calls env.jointStep then env.getAllObservations).
//
// A workgroup of 256 lanes steps E = 256 / NP^2 envs (step_pairs_env, one lane
// per agent pair) and then observes exactly those envs: the post-step cells,
// goals and human state go straight to LDS, so the observation needs no state
// reload and no second launch.  HBM traffic is the step's state + the
// observation stores; the step's latency-bound chains of one workgroup overlap
// the float4 store streams of the others.
//
// Workgroup roles, in grid order:
//  [0, nband)           the zero band (channel 5 while use_hp is off, all 0 by
//                       construction) of every agent's observation: HBM writes
//                       that need nothing from the step, issued while the step
//                       workgroups run their latency-bound chains; the step
//                       workgroups' float4 expansion skips exactly those float4s
//  [nband, +nsearch)    search work (below)
//  the rest             step + observe of E envs each
//
// The nsearch search workgroups run the search work of the PREVIOUS committed
// step (work-list slot `sslot`): humans' next paths (needed no earlier than
// two steps after they are queued -- a Human path start->goal->start has >= 3
// cells, mapf_gym.py:33-38) and agents' BFS maps (read only by mapf_bfs and
// the BFS channel, which is not fused).  The step of this launch reads none of
// what they write (the path buffer it walks is the other one).
#include <cstdio>

#include "mapf_step_pairs.h"
#include "mapf_search.h"

namespace mapf {

// one wave per env observes on its own (NP = 8, shared map in registers, every
// env's observation a whole number of float4s)
__host__ __device__ inline bool fused_per_wave(const DevEnv &e) {
    return e.G == 8 && regmap_fits(e) && ((e.N * e.C * e.F * e.F) & 3) == 0;
}

template <int NP, bool HOST>
__global__ __launch_bounds__(256) void step_observe_kernel(DevEnv e, int32_t *__restrict__ actions, StepOut out,
                                                           uint32_t flags, int slot, float *__restrict__ obs,
                                                           float *__restrict__ vec, int nsearch, int sslot, int nband) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    TL_STAMP(0);
    TL_HWID();
    if ((int)blockIdx.x < nband) {          // the zero band of every agent's observation
        const size_t K = (size_t)e.B * e.N;
        const size_t k0 = K * blockIdx.x / nband, k1 = K * (blockIdx.x + 1) / nband;
        obs_zero_band_store(e, obs, k0, k1, threadIdx.x, blockDim.x);
        TL_STAMP(1);
        return;
    }
    const int bx = (int)blockIdx.x - nband;
    if constexpr (HOST) {
        if (bx < nsearch) {
            const int wave = threadIdx.x >> 6;
            char *lds = smem + (size_t)wave * srch::wave_lds<uint32_t, 1>(e.H, e.W);
            srch::search_items<uint32_t, 1>(e, sslot, 0, lds, bx * (blockDim.x >> 6) + wave,
                                            nsearch * (blockDim.x >> 6));
            TL_STAMP(1);
            return;
        }
    } else {
        nsearch = 0;
    }
    constexpr int E = 256 / (NP * NP);
    const int blk = bx - nsearch;
    const int b0 = blk * E;
    const int nenv = min(E, e.B - b0);
    // the map words are loaded before the step's loads; at NP = 8 every wave holds
    // the whole shared map (lane k = word k) and the step reads it from registers,
    // and each wave then observes its own env with no workgroup barrier
    const bool regmap = NP == 8 && regmap_fits(e);
    const bool per_wave = regmap && fused_per_wave(e);
    ObsLds L = obs_layout(e, E, smem, per_wave);
    if (nband == 0) {     // the step workgroups write every float: nibble table for their store loops
        float4 *lut = reinterpret_cast<float4 *>(smem + ((obs_lds_bytes(e, E, per_wave) + 15) & ~(size_t)15));
        obs_lut_init(lut);
        __syncthreads();
        L.lut = lut;
    }
    const uint32_t mreg = obs_map_word(e, b0, nenv, regmap ? (int)(threadIdx.x & 63) : (int)threadIdx.x);
    PairsDeferred dfr;
    step_pairs_env<NP, true>(e, actions, out, flags, slot, blk * 256 + (int)threadIdx.x, L, b0,
                             RegMap{mreg, regmap}, dfr);
    TL_STAMP(1);
    if (per_wave) {
        const int le = (int)(threadIdx.x >> 6);
        if (le < nenv) {
            const ObsGroup g = obs_wave_init(e, L, le, mreg);
            TL_STAMP(2);
            obs_emit<false>(e, L, obs, vec, g, b0, nband > 0);
        }
    } else {
        obs_init(e, L, E, b0, nenv, mreg);
        __syncthreads();
        TL_STAMP(2);
        obs_emit<false>(e, L, obs, vec, obs_workgroup(L, nenv), b0, nband > 0);
    }
    step_pairs_finish(e, dfr, slot);
    TL_STAMP(3);
}

// The search work an INLINE step left in `d`, done by the same wave right away:
// agent.bfsMap of every agent whose goal changed (agent order), then the human's
// next path.  Same items, same results as the work-list searches.
// map: the env's padded obstacle rows in the wave's LDS; rs: the resident state,
// whose path lengths take the searched path's.
__device__ inline void step_pairs_search_inline(const DevEnv &e, const PairsDeferred &d, char *lds,
                                                const uint32_t *map, EnvRegs &rs) {
    for (uint64_t m = d.bmask; m; m &= m - 1ull) {
        const int l = __builtin_ctzll(m);
        const uint32_t ai = (uint32_t)__builtin_amdgcn_readlane((int)d.bitem, l);
        const uint32_t g = (uint32_t)__builtin_amdgcn_readlane((int)d.bgoal, l);
        srch::search_one<uint32_t, 1>(e, false, (int)(ai / (uint32_t)e.N), ai, g, NO_CELL, 0, lds, map);
    }
    if (d.rmask) {
        const int l = __builtin_ctzll(d.rmask);
        const int b = __builtin_amdgcn_readlane((int)d.ritem, l);
        const int buf = __builtin_amdgcn_readlane(d.rbuf, l);
        const int len = srch::search_one<uint32_t, 1>(e, true, b, 0u,
                                                      (uint32_t)__builtin_amdgcn_readlane((int)d.rstart, l),
                                                      (uint32_t)__builtin_amdgcn_readlane((int)d.rgoal, l), buf,
                                                      lds, map);
        if (buf) rs.hlen1 = len;
        else rs.hlen0 = len;
    }
}

// T committed random-policy steps + observations in ONE launch
// (mapf_rollout_random; runner.py:64-100 with the uniform policy, T times).
// Each wave owns one env for the whole launch and loops
//     step (pair lanes) -> observe its env (LDS bit-stream -> float4 stores)
//     -> its own search work (BFS maps, the human's next path)
// so a wave's latency-bound step runs while the other waves' observation stores
// drain: no launch boundary, dispatch ramp or state reload per step.  Step t's
// outputs go to slot t of the buffers when `slots` is set (rollout buffers).
struct RolloutOut {
    int32_t *actions;
    StepOut out;
    float *obs, *vec;
    int slots;
    int xcd_remap;
    int sub_lds;        // SUBS > 1: LDS bytes of one 4-env quarter (the pacing counters follow the quarters)
    int slack;          // SUBS > 1: a wave runs at most `slack` steps ahead of its group's slowest env (< 0: off)
    int fair;           // SUBS > 1, > 0: a wave more than `fair` steps ahead of the group's slowest env issues at
                        // priority 0, the others at 2 (no waiting; mapf_tuning.roll_fair)
};
// the kernel's arguments, read from device memory (ArgRing, mapf_kernels.h)
struct RolloutArgs {
    DevEnv e;
    RolloutOut ro;
};

__host__ __device__ inline bool rollout_fusable(const DevEnv &e) {
    return e.G == 8 && e.human_mode != 2 && e.goal_mode == 1 && e.C < 7 && !e.force_agent_lanes && fused_per_wave(e) &&
           e.W <= 30;
}

// LDS of a rollout workgroup: observation layout | nibble table | 4 search scratch | 4 path copies
__host__ __device__ inline size_t rollout_obs_lds(const DevEnv &e) { return ((obs_lds_bytes(e, 4, true) + 15) & ~(size_t)15) + 256; }
__host__ __device__ inline size_t rollout_lds_bytes(const DevEnv &e) {
    return rollout_obs_lds(e) + 4 * srch::wave_lds<uint32_t, 1>(e.H, e.W) + 4 * (size_t)e.Lmax * 4;
}

// NT: nontemporal observation stores -- for slot buffers (fresh HBM lines every step,
// measured faster); re-written [B]-leading buffers keep plain stores (their lines
// stay cache-resident between steps, measured faster).
// SUBS 4-env quarters per workgroup: SUBS = 4 puts all 16 waves of a CU in one workgroup, so
// each can see how far the others are (pacing, below)
template <bool NT, int SUBS>
__global__ __launch_bounds__(256 * SUBS) __attribute__((amdgpu_waves_per_eu(4))) void rollout_random_kernel(
#if MAPF_ARGS_PTR      // experiment build: arguments through a device pointer (mapf_rollout_wide.hip)
    const RolloutArgs *__restrict__ args, int T) {
    const DevEnv &e = args->e;
    const RolloutOut &ro = args->ro;
#else
    DevEnv e, int T, RolloutOut ro) {
#endif
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int E = 4;                     // envs per workgroup, one per wave
    // XCD-aware env order: workgroups are dealt round-robin over the 8 XCDs, so workgroup w
    // takes env block (w % 8) * (grid / 8) + w / 8 -- each XCD owns one contiguous range of
    // envs, and the output lines that several envs share (status: 16 envs per 128-B line)
    // are completed in one XCD's L2 instead of leaving it as partial lines from several.
    const int nb = (int)gridDim.x;
    const int wg = (ro.xcd_remap && (nb & 7) == 0) ? ((int)blockIdx.x & 7) * (nb >> 3) + ((int)blockIdx.x >> 3)
                                                   : (int)blockIdx.x;
    const int sub = SUBS > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8)) : 0;   // this wave's quarter
    const int qt = (int)(threadIdx.x & 255);           // thread index within the quarter
    const int blk = wg * SUBS + sub;                   // the quarter's 4-env block
    const int b0 = blk * E;
    const int nenv = min(E, e.B - b0);
    const int le = qt >> 6;
    char *qsm = smem + (SUBS > 1 ? (size_t)sub * ro.sub_lds : 0);
    uint32_t *prog = reinterpret_cast<uint32_t *>(smem + (size_t)SUBS * ro.sub_lds);   // [4 * SUBS] steps done
    const int gw = sub * E + le;                       // the wave's index in the workgroup
    ObsLds L = obs_layout(e, E, qsm, true);
    float4 *lut = reinterpret_cast<float4 *>(qsm + rollout_obs_lds(e) - 256);
    if (qt < 16) lut[qt] = make_float4((float)(qt & 1), (float)((qt >> 1) & 1), (float)((qt >> 2) & 1), (float)(qt >> 3));
    // envs past B never count: they start at the top
    if (SUBS > 1 && (int)threadIdx.x < 4 * SUBS) prog[threadIdx.x] = wg * SUBS * E + (int)threadIdx.x < e.B ? 0u : 0xFFFFFFFFu;
    __syncthreads();
    L.lut = lut;
    const size_t swl = srch::wave_lds<uint32_t, 1>(e.H, e.W);
    char *slds = qsm + rollout_obs_lds(e) + (size_t)le * swl;
    uint32_t *lpath = reinterpret_cast<uint32_t *>(qsm + rollout_obs_lds(e) + 4 * swl) + (size_t)le * e.Lmax;
    const uint32_t mreg = obs_map_word(e, b0, nenv, (int)(threadIdx.x & 63));
    EnvRegs rs{};
    if (le < nenv) env_regs_load<8>(e, b0 + le, rs, lpath);
    // every prologue load has landed before the loop: otherwise the compiler keeps a
    // register's load "pending" at the loop header and waits vmcnt(0) -- i.e. behind
    // all of the previous step's stores -- where the loop uses it
    __builtin_amdgcn_s_waitcnt(0x0F70);     // vmcnt(0), expcnt/lgkmcnt untouched
    RSTAMP_BEGIN();
    const bool pacing = SUBS > 1 && ro.slack >= 0 && le < nenv;
    const bool fair = SUBS > 1 && ro.fair > 0 && le < nenv;
    for (int t = 0; t < T; ++t) {
        const DevEnv &E = e;
        const RolloutOut &R = ro;
        if (pacing && t > R.slack) wait_group_min(prog, 4 * SUBS, (uint32_t)(t - R.slack));
        if (fair) {
            if ((uint32_t)t > group_min(prog, 4 * SUBS) + (uint32_t)R.fair) __builtin_amdgcn_s_setprio(0);
            else __builtin_amdgcn_s_setprio(2);
        }
        const size_t BN = (size_t)E.B * E.N;
        const size_t s = R.slots ? (size_t)t : 0;
        StepOut o = R.out;
        if (o.status) o.status += s * BN;
        if (o.reward) o.reward += s * BN;
        if (o.shadow_goals) o.shadow_goals += s * E.B;
        if (o.cost) o.cost += s * BN;
        if (o.train_valid) o.train_valid += s * BN * NA;
        if (o.actions_fixed) o.actions_fixed += s * BN;
        if (o.goals_reached) o.goals_reached += s * BN;
        if (o.constraints) o.constraints += s * BN;
        if (o.reward_total) o.reward_total += s * BN;
        PairsDeferred dfr;
        step_pairs_env<8, true, true, true>(E, R.actions + s * BN, o, 3u, 0, blk * 256 + qt,
                                            L, b0, RegMap{mreg, true}, dfr, &rs);
        if (le < nenv) {
            const ObsGroup g = obs_wave_init(E, L, le, mreg);
            obs_emit<false, NT>(E, L, R.obs + s * BN * E.C * E.F * E.F, R.vec + s * BN * 4, g, b0, false);
            step_pairs_search_inline(E, dfr, slds, L.mapc + (size_t)le * L.rowsz, rs);
            if (pacing || fair) publish_count(prog + gw, (uint32_t)(t + 1));
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (le < nenv) env_regs_store<8>(e, b0 + le, rs);
    if (le < nenv) RSTAMP_END(b0 + le);
}

bool rollout_random_fusable(const DevEnv &e) { return rollout_fusable(e) && rollout_lds_bytes(e) <= 64 * 1024; }

// The pair-lane rollout's launch form for this handle's tuning (mapf.h: mapf_tuning).
struct RolloutPlan {
    int subs = 1;        // 4-env quarters per workgroup (4: the 16 waves of a CU in one workgroup)
    int grid = 0;        // workgroups
    size_t lds = 0;      // dynamic LDS request
    int sub_lds = 0, slack = -1, fair = 0, remap = 1;
};

static bool plan_rollout_random(const DevEnv &e, int slots, const mapf_tuning &tu, RolloutPlan &p) {
    if (!rollout_random_fusable(e)) return false;
    const int grid = (e.B + 3) / 4;
    // Persistent waves: every CU should hold the same number of workgroups, or the
    // CUs holding more set the pace of every step.  The LDS request caps the
    // workgroups per CU at ceil(grid / CUs) (160 KiB of LDS per CU).
    const int ncu = device_cu_count();
    int occ = (grid + ncu - 1) / ncu;
    if (tu.roll_occ >= 1 && tu.roll_occ <= 16) occ = tu.roll_occ;
    size_t lds = rollout_lds_bytes(e);
    const size_t cap = ((size_t)160 * 1024 / (size_t)occ) & ~(size_t)255;
    if (occ >= 3 && cap > lds && cap <= 64 * 1024) lds = cap;
    // Slot buffers at four workgroups per CU (c2): one workgroup of all 16 waves instead,
    // each wave paced within `slack` steps of the slowest (RolloutOut::slack).  Unpaced,
    // each SIMD's four waves ran at 12.3 / 14.4 / 16.3 / 18.3 us per step by wave slot
    // (issue goes to the oldest) and the launch waited for the youngest; paced, all run
    // at 16.9 and the launch takes 17.5-17.7 us per step instead of 20.3
    // (tools/stamps_pairs.py, tools/ab_env.sh).
    // In place (c2): the same one workgroup per CU, but issue priority by progress instead of
    // waits: a wave more than 4 steps ahead of the group's slowest env drops to priority 0, the
    // rest run at 2 -- no wave ever idles, and the youngest wave of a SIMD no longer trails
    // (13.9-14.0 -> 11.9-12.0 us per step; roll_fair 0 with roll_group 0: four workgroups, unpaced).
    const size_t sub = (rollout_lds_bytes(e) + 15) & ~(size_t)15;
    const int fair = tu.roll_fair >= 0 ? tu.roll_fair : (slots ? 0 : 4);
    const bool group = occ == 4 && grid % 4 == 0 && 4 * sub + 64 <= (size_t)device_max_group_lds() &&
                       (tu.roll_group < 0 ? slots != 0 || fair > 0 : tu.roll_group != 0);
    p.subs = group ? 4 : 1;
    p.grid = grid / p.subs;
    p.lds = group ? (size_t)device_max_group_lds() : lds;   // grouped: the whole CU
    p.sub_lds = (int)sub;
    p.fair = fair;
    p.slack = fair > 0 ? -1 : tu.roll_slack;
    p.remap = tu.xcd_remap != 0;
    return true;
}

void describe_rollout_random(const DevEnv &e, int slots, const mapf_tuning &tu, char *buf, size_t n) {
    RolloutPlan p;
    if (!plan_rollout_random(e, slots, tu, p)) {
        std::snprintf(buf, n, "none");
        return;
    }
    std::snprintf(buf, n, "rollout_random_kernel<%s,%d> grid=%d block=%d lds=%zu fair=%d slack=%d remap=%d",
                  slots ? "true" : "false", p.subs, p.grid, 256 * p.subs, p.lds, p.subs > 1 ? p.fair : 0,
                  p.subs > 1 ? p.slack : -1, p.remap);
}

int launch_rollout_random(const DevEnv &e, int T, int32_t *actions, const StepOut &out, float *obs, float *vec,
                          int slots, const mapf_tuning &tu, ArgRing &ring, hipStream_t s) {
    RolloutPlan p;
    if (!plan_rollout_random(e, slots, tu, p)) return ROLLOUT_NOT_COVERED;
    const RolloutOut ro{actions, out, obs, vec, slots, p.remap, p.sub_lds, p.slack, p.fair};
    auto launch = [&](auto kern) -> int {
        const dim3 gd(p.grid), bd(256 * p.subs);
#if MAPF_ARGS_PTR
        const RolloutArgs *args = push_args(ring, RolloutArgs{e, ro}, s);
        if (!args) return MAPF_ESTATE;      // a capture found no free argument slot: nothing launched
        hipLaunchKernelGGL(kern, gd, bd, p.lds, s, args, T);
#else
        hipLaunchKernelGGL(kern, gd, bd, p.lds, s, e, T, ro);
#endif
        return MAPF_OK;
    };
    (void)ring;
    if (p.subs == 4) return slots ? launch(rollout_random_kernel<true, 4>) : launch(rollout_random_kernel<false, 4>);
    return slots ? launch(rollout_random_kernel<true, 1>) : launch(rollout_random_kernel<false, 1>);
}

bool step_observe_fusable(const DevEnv &e) {
    if (e.G > 8 || e.force_agent_lanes || e.human_mode == 2 || e.C >= 7) return false;
    const int E = 256 / (e.G * e.G);
    return obs_lds_bytes(e, E, fused_per_wave(e)) <= 64 * 1024;
}

template <int NP>
static void launch_np(const DevEnv &e, int32_t *actions, const StepOut &out, uint32_t flags, int slot, float *obs,
                      float *vec, int nsearch, int sslot, hipStream_t s) {
    constexpr int E = 256 / (NP * NP);
    const bool per_wave = NP == 8 && fused_per_wave(e);
    // zero-band workgroups: whole float4s only, so the step workgroups' slices
    // and the buffer must be 16-B aligned
    int z0, z1, nband = 0;
    const size_t slice = (size_t)E * e.N * e.C * e.F * e.F;
    if (e.band_blocks > 0 && obs_zero_band(e, z0, z1) && (slice & 3) == 0 && ((uintptr_t)obs & 15) == 0)
        nband = e.band_blocks;
    const int grid = (e.B + E - 1) / E + nsearch + nband;
    size_t lds = obs_lds_bytes(e, E, per_wave);
    if (nband == 0) lds = ((lds + 15) & ~(size_t)15) + 256;   // + the nibble table
    if (nsearch > 0) {
        const size_t sl = 4 * srch::wave_lds<uint32_t, 1>(e.H, e.W);
        if (sl > lds) lds = sl;
        hipLaunchKernelGGL((step_observe_kernel<NP, true>), dim3(grid), dim3(256), lds, s, e, actions, out, flags,
                           slot, obs, vec, nsearch, sslot, nband);
    } else {
        hipLaunchKernelGGL((step_observe_kernel<NP, false>), dim3(grid), dim3(256), lds, s, e, actions, out, flags,
                           slot, obs, vec, 0, 0, nband);
    }
}

void launch_step_observe(const DevEnv &e, int32_t *actions, const StepOut &out, uint32_t flags, int slot,
                         float *obs, float *vec, int nsearch, int sslot, hipStream_t s) {
    if (!observe_hosts_search(e)) nsearch = 0;
    switch (e.G) {
        case 1: launch_np<1>(e, actions, out, flags, slot, obs, vec, nsearch, sslot, s); break;
        case 2: launch_np<2>(e, actions, out, flags, slot, obs, vec, nsearch, sslot, s); break;
        case 4: launch_np<4>(e, actions, out, flags, slot, obs, vec, nsearch, sslot, s); break;
        default: launch_np<8>(e, actions, out, flags, slot, obs, vec, nsearch, sslot, s); break;
    }
}

}  // namespace mapf
