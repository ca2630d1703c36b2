// primal-ppo_amd/csrc/mapf_api.cpp -- the C ABI (include/mapf.h) over the HIP kernels.
//
// Host responsibilities: validate configs and reset inputs (the reference
// raises Python exceptions where this returns MAPF_EINVAL), own the device
// SoA state, build the padded obstacle bitmaps and the fp64-derived lookup
// tables, and order the kernels of one step on the caller's stream:
//   step_kernel -> replan_kernel (human paths, if the human can replan)
//               -> bfs_kernel (agent.bfsMap on goal changes, if keep_bfs)
// No allocation, copy or synchronisation happens inside mapf_step /
// mapf_observe, so both can be captured into a hipGraph by the caller.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mapf.h"
#include "mapf_kernels.h"

using namespace mapf;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t _e = (x);                                                                       \
        if (_e != hipSuccess) return fail(MAPF_EDEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)

int next_pow2(int n) {
    int g = 1;
    while (g < n) g <<= 1;
    return g;
}
}  // namespace

struct mapf_env {
    mapf_config cfg;
    int device = 0;
    DevEnv d{};
    int parity = 1;          // work-list slot of the next step (step count mod 3)
    int pending = -1;        // slot whose search work has not been launched yet
    bool ready = false;
    std::vector<void *> allocs;
    int8_t *maps8 = nullptr;  // [nmaps][H][W] int8 maps on the device (uploaded or generated)
    // second stream for a search that runs beside the observe launch (fork/join inside
    // one API call, so the caller's stream -- and a hipGraph capture of it -- sees one
    // sequence); created on first use
    hipStream_t aux = nullptr, aux2 = nullptr;   // aux: BFS maps the observation reads; aux2: deferred work
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_join2 = nullptr;
    // Deferred joins.  A human's next path is read no earlier than two steps after its
    // step queued it (mapf_fused.hip), and agent BFS maps only by the BFS channel
    // (C = 7, joined at once) and mapf_bfs: so the aux-stream search of committed step t
    // runs beside step t+1 and is joined on the caller's stream before step t+2 -- or
    // before anything else reads or rewrites the state (join_deferred).
    long nsteps = 0;                       // committed steps since the reset
    hipEvent_t ev_def[2] = {nullptr, nullptr};
    long def_due[2] = {-1, -1};            // join before the step that would make nsteps exceed this
    int def_next = 0;
    mapf_tuning tune;                      // launch forms (mapf_set_tuning); never the process environment
    ArgRing args;                          // device-resident argument blocks of the persistent kernels
    template <class T>
    int alloc(T *&p, size_t n) {
        void *q = nullptr;
        if (n == 0) n = 1;
        if (hipMalloc(&q, n * sizeof(T)) != hipSuccess) return fail(MAPF_ENOMEM, "hipMalloc failed");
        allocs.push_back(q);
        p = reinterpret_cast<T *>(q);
        return 0;
    }
};

// the per-step launches' tuning fields live in DevEnv (the kernels read them)
static void apply_tuning(DevEnv &d, const mapf_tuning &t) {
    // envs per observe_kernel workgroup: 64/N fills a wave's lanes for N <= 8; above that one
    // env per workgroup measured fastest (c4, 16 agents: 12.4 us vs 14.2 us at 4 envs, tools/sweep_c45.sh)
    d.obs_envs = t.obs_envs > 0 ? t.obs_envs : (d.N > 8 ? 1 : 64 / d.N);
    if (d.obs_envs > d.B) d.obs_envs = d.B;
    d.step_block = t.step_block;
    d.search_blocks = t.search_blocks;
    d.band_blocks = t.band_blocks;   // zero-band workgroups: slower than the waves' table-driven stores (0)
    d.force_agent_lanes = t.agent_lanes;
}

extern "C" {

void mapf_tuning_default(mapf_tuning *t) {
    if (!t) return;
    *t = mapf_tuning{};
    t->roll_occ = 0;
    t->roll_group = -1;
    t->roll_fair = -1;
    t->roll_slack = 1;
    t->wide_nt = -1;
    t->wide_pipe = 1;
    t->wide_grid = 1;
    t->wide_overlap = 1;
    t->wide_obs = 2;
    t->wide_epw = 0;
    t->wide_pair = 0;
    t->wide_slack = 1;
    t->wide_fair = 0;
    t->wide_prio = 1;
    t->wide_bfsobs = 1;
    t->xcd_remap = 1;
    t->obs_envs = 0;
    t->step_block = 256;
    t->search_blocks = 64;
    t->band_blocks = 0;
    t->agent_lanes = 0;
    t->serial_search = 0;
    t->no_defer = 0;
    t->diag_exp = 0;
}

int mapf_get_tuning(const mapf_env *e, mapf_tuning *t) {
    if (!e || !t) return fail(MAPF_EINVAL, "null argument");
    *t = e->tune;
    return MAPF_OK;
}

int mapf_set_tuning(mapf_env *e, const mapf_tuning *t) {
    if (!e || !t) return fail(MAPF_EINVAL, "null argument");
    auto in = [](int v, int lo, int hi) { return v >= lo && v <= hi; };
    auto flag = [&](int v) { return in(v, 0, 1); };
    if (!in(t->roll_occ, 0, 16)) return fail(MAPF_EINVAL, "roll_occ must be in 0..16");
    if (!in(t->roll_group, -1, 1)) return fail(MAPF_EINVAL, "roll_group must be -1, 0 or 1");
    if (!in(t->roll_fair, -1, 1 << 20)) return fail(MAPF_EINVAL, "roll_fair must be >= -1");
    if (!in(t->roll_slack, -1, 1 << 20)) return fail(MAPF_EINVAL, "roll_slack must be >= -1");
    if (!in(t->wide_nt, -1, 1)) return fail(MAPF_EINVAL, "wide_nt must be -1, 0 or 1");
    if (!flag(t->wide_pipe) || !flag(t->wide_grid) || !flag(t->wide_overlap) || !flag(t->wide_pair) ||
        !flag(t->wide_prio) || !flag(t->wide_bfsobs) || !flag(t->xcd_remap) || !flag(t->agent_lanes) ||
        !flag(t->serial_search) || !flag(t->no_defer))
        return fail(MAPF_EINVAL, "wide_pipe/grid/overlap/pair/prio/bfsobs, xcd_remap, agent_lanes, serial_search, "
                                 "no_defer must be 0 or 1");
    if (!in(t->wide_obs, 1, 2)) return fail(MAPF_EINVAL, "wide_obs must be 1 or 2");
    if (!in(t->wide_epw, 0, 12)) return fail(MAPF_EINVAL, "wide_epw must be in 0..12");
    if (!in(t->wide_slack, -1, 1 << 20)) return fail(MAPF_EINVAL, "wide_slack must be >= -1");
    if (!in(t->wide_fair, 0, 1 << 20)) return fail(MAPF_EINVAL, "wide_fair must be >= 0");
    if (!in(t->obs_envs, 0, 64)) return fail(MAPF_EINVAL, "obs_envs must be in 0..64");
    if (t->step_block != 64 && t->step_block != 128 && t->step_block != 256)
        return fail(MAPF_EINVAL, "step_block must be 64, 128 or 256");
    if (!in(t->search_blocks, 1, 1024)) return fail(MAPF_EINVAL, "search_blocks must be in 1..1024");
    if (!in(t->band_blocks, 0, 4096)) return fail(MAPF_EINVAL, "band_blocks must be in 0..4096");
    if (!in(t->diag_exp, 0, 3)) return fail(MAPF_EINVAL, "diag_exp must be in 0..3");
    e->tune = *t;
    apply_tuning(e->d, e->tune);
    return MAPF_OK;
}

const char *mapf_last_error(void) { return g_err.c_str(); }
int mapf_abi_version(void) { return MAPF_ABI_VERSION; }

int mapf_create(const mapf_config *cfg, int device, mapf_env **out) {
    if (!cfg || !out) return fail(MAPF_EINVAL, "null argument");
    const mapf_config &c = *cfg;
    if (c.num_envs < 1) return fail(MAPF_EINVAL, "num_envs must be >= 1");
    if (c.num_agents < 1 || c.num_agents > 64) return fail(MAPF_EINVAL, "num_agents must be in 1..64");
    if (c.height < 1 || c.height > 128 || c.width < 1 || c.width > 128) return fail(MAPF_EINVAL, "height/width must be in 1..128");
    if (c.fov < 1 || c.fov > 16) return fail(MAPF_EINVAL, "fov must be in 1..16");
    if (c.num_channel < 5 || c.num_channel > 7) return fail(MAPF_EINVAL, "num_channel must be 5, 6 or 7");
    if (c.num_channel == 7 && !c.keep_bfs) return fail(MAPF_EINVAL, "num_channel 7 (BFS channel) needs keep_bfs");
    if (c.human_mode < 0 || c.human_mode > 2) return fail(MAPF_EINVAL, "human_mode must be 0, 1 or 2");
    if (c.goal_mode < 0 || c.goal_mode > 1) return fail(MAPF_EINVAL, "goal_mode must be 0 or 1");
    if (c.fix_choice < 0 || c.fix_choice > 1) return fail(MAPF_EINVAL, "fix_choice must be 0 or 1");
    if (c.max_seq < 1) return fail(MAPF_EINVAL, "max_seq must be >= 1");
    if (c.human_mode == 2 && c.max_human_seq < 2) return fail(MAPF_EINVAL, "max_human_seq must be >= 2");
    if (c.penalty_radius < 1 || c.penalty_radius > 64) return fail(MAPF_EINVAL, "penalty_radius must be in 1..64");
    if (c.k_predict < 0 || c.k_predict > 64) return fail(MAPF_EINVAL, "k_predict must be in 0..64");
    if (hipSetDevice(device) != hipSuccess) return fail(MAPF_EDEVICE, "hipSetDevice failed");

    auto *e = new mapf_env();
    e->cfg = c;
    e->device = device;
    DevEnv &d = e->d;
    d.B = c.num_envs; d.N = c.num_agents; d.H = c.height; d.W = c.width; d.F = c.fov; d.C = c.num_channel;
    d.P = c.fov / 2 > 1 ? c.fov / 2 : 1;
    d.Hp = d.H + 2 * d.P;
    d.WW = (d.W + 2 * d.P + 31) / 32;
    d.G = next_pow2(d.N);
    d.S = c.max_seq;
    d.HS = c.max_human_seq > 2 ? c.max_human_seq : 2;
    d.Lmax = 2 * d.H * d.W + 1;
    d.use_da = c.use_da; d.use_hp = c.use_hp; d.lifelong = c.lifelong; d.human_mode = c.human_mode;
    d.goal_mode = c.goal_mode; d.fix_choice = c.fix_choice; d.shared_map = c.shared_map ? 1 : 0;
    d.keep_bfs = c.keep_bfs ? 1 : 0; d.k_predict = c.k_predict; d.R = c.penalty_radius;
    d.action_cost = c.action_cost; d.collision_cost = c.collision_cost; d.human_collision_cost = c.human_collision_cost;
    d.repeat_cost = c.repeat_cost; d.goal_reward = c.goal_reward;
    d.env_offset = (uint32_t)c.env_offset;
    d.seed = c.seed;
    // envs per observe_kernel workgroup: 64/N fills a wave's lanes for N <= 8; above that one
    // env per workgroup measured fastest (c4, 16 agents: 12.4 us vs 14.2 us at 4 envs, tools/sweep_c45.sh)
    mapf_tuning_default(&e->tune);
    apply_tuning(d, e->tune);

    // fp64 lookup table, computed exactly like the reference (numpy sqrt)
    const double R = (double)c.penalty_radius;
    std::vector<float> cost_lut(d.R * d.R + 1);
    d.constr_d2 = -1;
    for (int k = 0; k <= d.R * d.R; ++k) {
        double v = R - std::sqrt((double)k);      // np.linalg.norm -> sqrt (mapf_gym.py:519)
        if (!(v > 0.0)) v = 0.0;
        cost_lut[k] = (float)(v / R);
        if (v / R >= 0.01) d.constr_d2 = k;       // monotone in k (mapf_gym.py:633)
    }

    const size_t BN = (size_t)d.B * d.N;
    const size_t nmaps = d.shared_map ? 1 : (size_t)d.B;
    int rc = 0;
    uint32_t *map_bits = nullptr;
    float *cl = nullptr;
    rc |= e->alloc(map_bits, nmaps * d.Hp * d.WW);
    rc |= e->alloc(d.pos, BN); rc |= e->alloc(d.goal, BN); rc |= e->alloc(d.last_act, BN);
    rc |= e->alloc(d.seq, BN * d.S); rc |= e->alloc(d.seq_len, BN); rc |= e->alloc(d.seq_cur, BN);
    rc |= e->alloc(d.hpath, (size_t)d.B * 2 * d.Lmax);
    rc |= e->alloc(d.hlen, 2 * (size_t)d.B); rc |= e->alloc(d.hstep, d.B); rc |= e->alloc(d.hcur, d.B);
    rc |= e->alloc(d.hpos, d.B); rc |= e->alloc(d.hnext, d.B); rc |= e->alloc(d.hgoal, d.B); rc |= e->alloc(d.hentr, d.B);
    rc |= e->alloc(d.hnext_start, d.B); rc |= e->alloc(d.hnext_goal, d.B);
    rc |= e->alloc(d.hseq, (size_t)d.B * d.HS); rc |= e->alloc(d.hseq_len, d.B); rc |= e->alloc(d.hseq_idx, d.B);
    rc |= e->alloc(d.hreplans, d.B); rc |= e->alloc(d.clock, d.B);
    if (d.keep_bfs) rc |= e->alloc(d.bfs, BN * bfs_cells(d.H, d.W));
    rc |= e->alloc(d.counters, C_NUM);
    rc |= e->alloc(d.prof, PROF_WORDS);
    rc |= e->alloc(d.replan_list, 3 * (size_t)d.B);
    rc |= e->alloc(d.bfs_list, 3 * BN);
    uint8_t *smask = nullptr;
    rc |= e->alloc(smask, nmaps * (size_t)d.H * d.W);
    rc |= e->alloc(e->maps8, nmaps * (size_t)d.H * d.W);
    rc |= e->alloc(cl, cost_lut.size());
    rc |= e->alloc(e->args.base, (ARG_SLOTS + ARG_CAPTURE_SLOTS) * ARG_SLOT_BYTES);
    if (rc) {
        std::string m = g_err;
        mapf_destroy(e);
        return fail(MAPF_ENOMEM, m);
    }
    d.map_bits = map_bits;
    d.smask = smask;
    d.cost_lut = cl;
    if (hipMemcpy(cl, cost_lut.data(), cost_lut.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(d.counters, 0, C_NUM * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(d.prof, 0, PROF_WORDS * sizeof(unsigned long long)) != hipSuccess) {
        mapf_destroy(e);
        return fail(MAPF_EDEVICE, "initial upload failed");
    }
    *out = e;
    return MAPF_OK;
}

int mapf_destroy(mapf_env *e) {
    if (!e) return MAPF_OK;
    (void)hipSetDevice(e->device);
    if (e->aux) {
        (void)hipStreamSynchronize(e->aux);
        (void)hipStreamDestroy(e->aux);
    }
    if (e->aux2) {
        (void)hipStreamSynchronize(e->aux2);
        (void)hipStreamDestroy(e->aux2);
    }
    if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
    if (e->ev_join) (void)hipEventDestroy(e->ev_join);
    if (e->ev_join2) (void)hipEventDestroy(e->ev_join2);
    for (hipEvent_t ev : e->ev_def)
        if (ev) (void)hipEventDestroy(ev);
    for (void *p : e->allocs) (void)hipFree(p);
    delete e;
    return MAPF_OK;
}

int mapf_path_capacity(const mapf_env *e) { return e ? e->d.Lmax : 0; }
int mapf_step_observe_fused(const mapf_env *e) { return e && step_observe_fusable(e->d) ? 1 : 0; }
static bool rollout_random_fused(const mapf_env *e) {
    return e && (rollout_random_fusable(e->d) || rollout_wide_fusable(e->d));
}
int mapf_rollout_random_fused(const mapf_env *e) {
    if (!e) return 0;
    return rollout_random_fusable(e->d) ? 1 : (rollout_wide_fusable(e->d) ? 2 : 0);
}
int mapf_rollout_plan(const mapf_env *e, int32_t slots, char *buf, int32_t n) {
    if (!e || !buf || n < 1) return fail(MAPF_EINVAL, "null argument");
    if (hipSetDevice(e->device) != hipSuccess) return fail(MAPF_EDEVICE, "hipSetDevice failed");
    const int kind = mapf_rollout_random_fused(e);
    if (kind == 1) describe_rollout_random(e->d, slots ? 1 : 0, e->tune, buf, (size_t)n);
    else if (kind == 2) describe_rollout_wide(e->d, slots ? 1 : 0, e->tune, buf, (size_t)n);
    else std::snprintf(buf, (size_t)n, "step_observe");
    return kind;
}

// s waits for the deferred aux-stream searches: every one (all), or those due before the
// step about to be launched
// Deferral is off while s is captured (observe_with_search), so a pending event was recorded
// outside any capture: a captured stream cannot wait on it (the graph would depend on work
// outside itself) -- the caller must join it first (mapf_flush, or any call on an uncaptured
// stream) before beginning the capture.
static int join_deferred(mapf_env *e, hipStream_t s, bool all) {
    if (e->def_due[0] >= 0 || e->def_due[1] >= 0) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        HIPCHK(hipStreamIsCapturing(s, &cap));
        if (cap != hipStreamCaptureStatusNone)
            return fail(MAPF_ESTATE, "a search deferred before this stream capture began is still pending: "
                                     "call mapf_flush on an uncaptured stream before capturing");
    }
    for (int k = 0; k < 2; ++k) {
        if (e->def_due[k] >= 0 && (all || e->nsteps >= e->def_due[k])) {
            HIPCHK(hipStreamWaitEvent(s, e->ev_def[k], 0));
            e->def_due[k] = -1;
        }
    }
    return MAPF_OK;
}

// the searches that end every reset: first human paths + every agent's BFS map, then each
// human's next path
static int reset_searches(mapf_env *e, hipStream_t s) {
    const DevEnv &d = e->d;
    e->nsteps = 0;
    launch_search(d, 0, 1, s);     // first human paths (buffer 0) + every agent's BFS map
    launch_plan(d, 1, s);          // promote them, plan each human's next path
    launch_search(d, 0, 2, s);     // ... and search it (buffer 1)
    HIPCHK(hipGetLastError());
    e->parity = 1;
    e->pending = -1;
    e->ready = true;
    return MAPF_OK;
}

int mapf_reset(mapf_env *e, const mapf_reset_spec *spec, void *stream) {
    if (!e || !spec || !spec->maps) return fail(MAPF_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    if (int rc = join_deferred(e, s, true)) return rc;
    DevEnv &d = e->d;
    const int B = d.B, N = d.N, H = d.H, W = d.W;
    const size_t nmaps = d.shared_map ? 1 : (size_t)B;
    if (spec->mode != 0 && spec->mode != 1) return fail(MAPF_EINVAL, "reset mode must be 0 or 1");
    if (spec->mode == 1 && d.human_mode == 2) return fail(MAPF_EINVAL, "seeded reset needs human_mode 0 or 1");
    if (spec->mode == 1 && spec->seed) d.seed = spec->seed;

    // map values: 0 free / -1 obstacle (the padded bitmaps and static-action masks are built
    // from them on the device, launch_build_maps)
    for (size_t k = 0; k < nmaps * (size_t)H * W; ++k)
        if (spec->maps[k] != 0 && spec->maps[k] != -1) return fail(MAPF_EINVAL, "map values must be 0 (free) or -1 (obstacle)");
    auto free_at = [&](int b, int r, int c) {
        if (r < 0 || r >= H || c < 0 || c >= W) return false;
        const size_t m = d.shared_map ? 0 : (size_t)b;
        return spec->maps[m * H * W + r * W + c] == 0;
    };

    std::vector<uint32_t> seq, hpos, hgoal, hseq;
    std::vector<int32_t> seq_len, hseq_len;
    if (spec->mode == 0) {
        if (!spec->seq || !spec->seq_len) return fail(MAPF_EINVAL, "mode 0 needs seq and seq_len");
        seq.assign((size_t)B * N * d.S, 0u);
        seq_len.assign((size_t)B * N, 0);
        for (int b = 0; b < B; ++b) {
            std::vector<uint32_t> starts;
            for (int i = 0; i < N; ++i) {
                const size_t ai = (size_t)b * N + i;
                const int len = spec->seq_len[ai];
                if (len < 1 || len > d.S) return fail(MAPF_EINVAL, "seq_len out of range");
                seq_len[ai] = len;
                for (int k = 0; k < len; ++k) {
                    const int r = spec->seq[(ai * d.S + k) * 2], c = spec->seq[(ai * d.S + k) * 2 + 1];
                    if (r < 0 || r >= H || c < 0 || c >= W) return fail(MAPF_EINVAL, "sequence cell out of the map");
                    seq[ai * d.S + k] = pack(r, c);
                }
                const int r0 = spec->seq[(ai * d.S) * 2], c0 = spec->seq[(ai * d.S) * 2 + 1];
                if (!free_at(b, r0, c0)) return fail(MAPF_EINVAL, "agent start on an obstacle");
                for (uint32_t s2 : starts)
                    if (s2 == pack(r0, c0)) return fail(MAPF_EINVAL, "two agents start on the same cell");
                starts.push_back(pack(r0, c0));
            }
        }
        hpos.assign(B, 0u); hgoal.assign(B, 0u);
        if (d.human_mode == 2) {
            if (!spec->human_seq || !spec->human_seq_len) return fail(MAPF_EINVAL, "human_mode 2 needs human_seq");
            hseq.assign((size_t)B * d.HS, 0u);
            hseq_len.assign(B, 0);
            for (int b = 0; b < B; ++b) {
                const int len = spec->human_seq_len[b];
                if (len < 2 || len > d.HS) return fail(MAPF_EINVAL, "human_seq_len out of range");
                hseq_len[b] = len;
                for (int k = 0; k < len; ++k) {
                    const int r = spec->human_seq[((size_t)b * d.HS + k) * 2], c = spec->human_seq[((size_t)b * d.HS + k) * 2 + 1];
                    if (!free_at(b, r, c)) return fail(MAPF_EINVAL, "human pose not on a free cell");
                    hseq[(size_t)b * d.HS + k] = pack(r, c);
                }
            }
        } else {
            if (!spec->human_start || !spec->human_goal) return fail(MAPF_EINVAL, "mode 0 needs human_start/goal");
            for (int b = 0; b < B; ++b) {
                const int sr = spec->human_start[2 * b], sc = spec->human_start[2 * b + 1];
                const int gr = spec->human_goal[2 * b], gc = spec->human_goal[2 * b + 1];
                if (!free_at(b, sr, sc) || !free_at(b, gr, gc)) return fail(MAPF_EINVAL, "human start/goal not free");
                if (sr == gr && sc == gc) return fail(MAPF_EINVAL, "human start == goal (astar_4 returns [])");
                hpos[b] = pack(sr, sc);
                hgoal[b] = pack(gr, gc);
            }
        }
    }

    HIPCHK(hipMemcpyAsync(e->maps8, spec->maps, nmaps * (size_t)H * W, hipMemcpyHostToDevice, s));
    launch_build_maps(d, e->maps8, s);
    HIPCHK(hipMemsetAsync(d.counters, 0, C_NUM * sizeof(uint32_t), s));
    if (spec->mode == 0) {
        HIPCHK(hipMemcpyAsync(d.seq, seq.data(), seq.size() * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(d.seq_len, seq_len.data(), seq_len.size() * 4, hipMemcpyHostToDevice, s));
        if (d.human_mode == 2) {
            HIPCHK(hipMemcpyAsync(d.hseq, hseq.data(), hseq.size() * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d.hseq_len, hseq_len.data(), hseq_len.size() * 4, hipMemcpyHostToDevice, s));
        } else {
            HIPCHK(hipMemcpyAsync(d.hpos, hpos.data(), hpos.size() * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d.hgoal, hgoal.data(), hgoal.size() * 4, hipMemcpyHostToDevice, s));
        }
        launch_reset_fixed(d, s);
    } else {
        launch_reset_seeded(d, s);
    }
    const int rc = reset_searches(e, s);
    if (rc != MAPF_OK) return rc;
    HIPCHK(hipStreamSynchronize(s));   // host staging buffers die at return
    return MAPF_OK;
}

int mapf_reset_generated(mapf_env *e, const mapf_mapgen_spec *spec, int8_t *maps_out, void *stream) {
    if (!e || !spec) return fail(MAPF_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    if (int rc = join_deferred(e, s, true)) return rc;
    DevEnv &d = e->d;
    if (d.human_mode == 2) return fail(MAPF_EINVAL, "generated maps need human_mode 0 or 1 (seeded reset)");
    MapGen g{spec->kind, spec->lo, spec->hi, spec->largest ? 1 : 0, spec->density, spec->epoch,
             spec->seed ? spec->seed : d.seed};
    if (spec->kind == MAPF_MAPS_WAREHOUSE) {
        if (spec->lo < 3 || spec->hi < spec->lo) return fail(MAPF_EINVAL, "warehouse length range [lo, hi] invalid");
        const int breadth = (int)((double)spec->hi / (2.0 / 3.0));
        if (d.H < spec->hi || d.W < breadth) return fail(MAPF_EINVAL, "the H x W stack is smaller than the longest warehouse");
    } else if (spec->kind == MAPF_MAPS_RANDOM) {
        if (!(spec->density >= 0.f && spec->density <= 1.f)) return fail(MAPF_EINVAL, "density must be in [0, 1]");
    } else {
        return fail(MAPF_EINVAL, "unknown map kind");
    }
    if (spec->largest && d.H * d.W > LC_MAX_CELLS) return fail(MAPF_EINVAL, "largest component: at most 8192 cells");
    if (spec->seed) d.seed = spec->seed;
    const size_t nmaps = d.shared_map ? 1 : (size_t)d.B;
    launch_mapgen(d, g, e->maps8, s);
    if (maps_out)
        HIPCHK(hipMemcpyAsync(maps_out, e->maps8, nmaps * (size_t)d.H * d.W, hipMemcpyDeviceToDevice, s));
    launch_build_maps(d, e->maps8, s);
    HIPCHK(hipMemsetAsync(d.counters, 0, C_NUM * sizeof(uint32_t), s));
    launch_reset_seeded(d, s);
    return reset_searches(e, s);       // asynchronous: nothing on the host to keep alive
}

static int step_impl(mapf_env *e, int32_t *actions, const mapf_step_out *out, uint32_t flags, void *stream) {
    if (!e || !actions) return fail(MAPF_EINVAL, "null argument");
    if (!e->ready) return fail(MAPF_ESTATE, "mapf_step before mapf_reset");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    StepOut o{};
    if (out) {
        o.status = out->status; o.reward = out->reward; o.shadow_goals = out->shadow_goals; o.cost = out->cost;
        o.train_valid = out->train_valid; o.actions_fixed = out->actions_fixed; o.goals_reached = out->goals_reached;
        o.constraints = out->constraints; o.reward_total = out->reward_total;
    }
    if (e->pending >= 0) {             // previous step's search work was not observed-through
        if (int rc = join_deferred(e, s, true)) return rc;
        launch_search(e->d, e->pending, 0, s);
        e->pending = -1;
    }
    if (int rc = join_deferred(e, s, !(flags & MAPF_STEP_COMMIT))) return rc;
    const int parity = e->parity;
    launch_step(e->d, actions, o, flags, parity, s);
    if (flags & MAPF_STEP_COMMIT) {
        if (e->d.human_mode != 0 || e->d.keep_bfs) e->pending = parity;
        e->parity = (parity + 1) % 3;
        ++e->nsteps;
    }
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

static int flush_search(mapf_env *e, hipStream_t s) {
    if (int rc = join_deferred(e, s, true)) return rc;
    if (e->pending >= 0) {
        launch_search(e->d, e->pending, 0, s);
        e->pending = -1;
        HIPCHK(hipGetLastError());
    }
    return MAPF_OK;
}

int mapf_step(mapf_env *e, const int32_t *actions, const mapf_step_out *out, uint32_t flags, void *stream) {
    return step_impl(e, const_cast<int32_t *>(actions), out, flags & MAPF_STEP_COMMIT, stream);
}

int mapf_step_random(mapf_env *e, int32_t *actions_out, const mapf_step_out *out, uint32_t flags, void *stream) {
    return step_impl(e, actions_out, out, (flags & MAPF_STEP_COMMIT) | 2u, stream);
}

// The pending search (the last step's BFS maps and human paths) beside the observe launch,
// forked off s onto two streams.  Nothing the observation reads is written by the search
// except the listed agents' BFS maps (C = 7): those are searched on e->aux, joined right
// after the observe launch, and exactly their BFS channel is then rewritten (bfs_fixup).
// The rest -- the humans' next paths, and BFS maps without the BFS channel -- runs on
// e->aux2 and stays there past this call (join_deferred), unless s is being captured into
// a graph (a capture must join every fork before it ends).
static int observe_with_search(mapf_env *e, float *obs, float *vec, hipStream_t s) {
    if (!e->aux) {
        HIPCHK(hipStreamCreateWithFlags(&e->aux, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&e->aux2, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&e->ev_join2, hipEventDisableTiming));
        for (hipEvent_t &ev : e->ev_def) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(s, &cap));
    const bool defer = !e->tune.no_defer && cap == hipStreamCaptureStatusNone;
    const bool bfsch = e->d.C >= 7 && e->d.keep_bfs;
    const int parity = e->pending;
    e->pending = -1;
    HIPCHK(hipEventRecord(e->ev_fork, s));
    if (bfsch) {
        HIPCHK(hipStreamWaitEvent(e->aux, e->ev_fork, 0));
        launch_search(e->d, parity, 4, e->aux);                 // the BFS maps the observation reads
        HIPCHK(hipEventRecord(e->ev_join, e->aux));
    }
    HIPCHK(hipStreamWaitEvent(e->aux2, e->ev_fork, 0));
    launch_search(e->d, parity, bfsch ? 3 : 0, e->aux2);        // human paths (+ BFS maps without the channel)
    if (defer) {
        // slot k's previous search was due before an earlier step: joined by now
        const int k = e->def_next;
        HIPCHK(hipEventRecord(e->ev_def[k], e->aux2));
        e->def_due[k] = e->nsteps + 1;
        e->def_next = k ^ 1;
    } else {
        HIPCHK(hipEventRecord(e->ev_join2, e->aux2));
    }
    launch_observe(e->d, obs, vec, 0, parity, s);
    if (bfsch) {
        HIPCHK(hipStreamWaitEvent(s, e->ev_join, 0));
        launch_bfs_fixup(e->d, parity, obs, s);
    }
    if (!defer) HIPCHK(hipStreamWaitEvent(s, e->ev_join2, 0));
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_observe(mapf_env *e, float *obs, float *vec, void *stream) {
    if (!e || !obs || !vec) return fail(MAPF_EINVAL, "null argument");
    if (!e->ready) return fail(MAPF_ESTATE, "mapf_observe before mapf_reset");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    int nsearch = 0, parity = 0;
    if (e->pending >= 0) {
        if (!observe_hosts_search(e->d) || e->d.C >= 7) {   // wide grids / BFS channel: search beside the launch
            if (!e->tune.serial_search) return observe_with_search(e, obs, vec, s);
            if (int rc = flush_search(e, s)) return rc;
        } else {                       // search work rides in the observe launch
            nsearch = e->d.search_blocks;
            parity = e->pending;
            e->pending = -1;
        }
    }
    launch_observe(e->d, obs, vec, nsearch, parity, s);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

static int step_observe_impl(mapf_env *e, int32_t *actions, const mapf_step_out *out, uint32_t flags, float *obs,
                             float *vec, void *stream) {
    if (!e || !actions || !obs || !vec) return fail(MAPF_EINVAL, "null argument");
    if (!e->ready) return fail(MAPF_ESTATE, "mapf_step_observe before mapf_reset");
    if (!step_observe_fusable(e->d)) {          // two launches, same results
        if (int rc = step_impl(e, actions, out, MAPF_STEP_COMMIT | flags, stream)) return rc;
        return mapf_observe(e, obs, vec, stream);
    }
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    if (int rc = join_deferred(e, s, true)) return rc;
    ++e->nsteps;
    StepOut o{};
    if (out) {
        o.status = out->status; o.reward = out->reward; o.shadow_goals = out->shadow_goals; o.cost = out->cost;
        o.train_valid = out->train_valid; o.actions_fixed = out->actions_fixed; o.goals_reached = out->goals_reached;
        o.constraints = out->constraints; o.reward_total = out->reward_total;
    }
    const bool host = observe_hosts_search(e->d);
    int nsearch = 0, sslot = 0;
    if (e->pending >= 0) {
        if (host) { nsearch = e->d.search_blocks; sslot = e->pending; }
        else launch_search(e->d, e->pending, 0, s);
        e->pending = -1;
    }
    const int parity = e->parity;
    launch_step_observe(e->d, actions, o, MAPF_STEP_COMMIT | flags, parity, obs, vec, nsearch, sslot, s);
    if (e->d.human_mode != 0 || e->d.keep_bfs) {
        if (host) e->pending = parity;             // rides in the next launch
        else launch_search(e->d, parity, 0, s);
    }
    e->parity = (parity + 1) % 3;
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_step_observe(mapf_env *e, const int32_t *actions, const mapf_step_out *out, float *obs, float *vec,
                      void *stream) {
    return step_observe_impl(e, const_cast<int32_t *>(actions), out, 0u, obs, vec, stream);
}

int mapf_step_observe_random(mapf_env *e, int32_t *actions_out, const mapf_step_out *out, float *obs, float *vec,
                             void *stream) {
    return step_observe_impl(e, actions_out, out, 2u, obs, vec, stream);
}

int mapf_rollout_random(mapf_env *e, int32_t T, int32_t slots, int32_t *actions_out, const mapf_step_out *out,
                        float *obs, float *vec, void *stream) {
    if (!e || !actions_out || !obs || !vec) return fail(MAPF_EINVAL, "null argument");
    if (T < 0) return fail(MAPF_EINVAL, "T must be >= 0");
    if (!e->ready) return fail(MAPF_ESTATE, "mapf_rollout_random before mapf_reset");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    StepOut o{};
    if (out) {
        o.status = out->status; o.reward = out->reward; o.shadow_goals = out->shadow_goals; o.cost = out->cost;
        o.train_valid = out->train_valid; o.actions_fixed = out->actions_fixed; o.goals_reached = out->goals_reached;
        o.constraints = out->constraints; o.reward_total = out->reward_total;
    }
    if (T == 0) return MAPF_OK;
    if (rollout_random_fused(e)) {
        if (int rc = flush_search(e, s)) return rc;     // the kernel searches inline from here on
        int rc = launch_rollout_random(e->d, T, actions_out, o, obs, vec, slots ? 1 : 0, e->tune, e->args, s);
        if (rc == ROLLOUT_NOT_COVERED)
            rc = launch_rollout_wide(e->d, T, actions_out, o, obs, vec, slots ? 1 : 0, e->tune, e->args, s);
        if (rc != MAPF_OK)
            return fail(MAPF_ESTATE, "every argument slot for captured persistent launches of this handle is taken "
                                     "(16 per handle, ArgRing; mapf_release_captures frees them)");
        HIPCHK(hipGetLastError());
        return MAPF_OK;
    }
    // not covered by the one-launch kernel: T step_observe launches, same results
    const size_t BN = (size_t)e->d.B * e->d.N, obs_t = BN * e->d.C * e->d.F * e->d.F;
    for (int32_t t = 0; t < T; ++t) {
        const size_t k = slots ? (size_t)t : 0;
        mapf_step_out ot{};
        if (out) {
            auto adv = [&](auto *p, size_t n) { return p ? p + k * n : p; };
            ot.status = adv(out->status, BN); ot.reward = adv(out->reward, BN);
            ot.shadow_goals = adv(out->shadow_goals, (size_t)e->d.B); ot.cost = adv(out->cost, BN);
            ot.train_valid = adv(out->train_valid, BN * 5); ot.actions_fixed = adv(out->actions_fixed, BN);
            ot.goals_reached = adv(out->goals_reached, BN); ot.constraints = adv(out->constraints, BN);
            ot.reward_total = adv(out->reward_total, BN);
        }
        if (int rc = step_observe_impl(e, actions_out + k * BN, out ? &ot : nullptr, 2u, obs + k * obs_t,
                                       vec + k * BN * 4, stream))
            return rc;
    }
    return MAPF_OK;
}

int mapf_release_captures(mapf_env *e) {
    if (!e) return fail(MAPF_EINVAL, "null argument");
    e->args.release_captures();
    return MAPF_OK;
}

int mapf_flush(mapf_env *e, void *stream) {
    if (!e) return fail(MAPF_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    return flush_search(e, (hipStream_t)stream);
}

int mapf_random_actions(mapf_env *e, int32_t *actions, void *stream) {
    if (!e || !actions) return fail(MAPF_EINVAL, "null argument");
    if (!e->ready) return fail(MAPF_ESTATE, "mapf_random_actions before mapf_reset");
    HIPCHK(hipSetDevice(e->device));
    launch_random_actions(e->d, actions, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_bfs(mapf_env *e, int16_t *dist, void *stream) {
    if (!e || !dist) return fail(MAPF_EINVAL, "null argument");
    if (!e->d.keep_bfs) return fail(MAPF_ESTATE, "keep_bfs is off");
    HIPCHK(hipSetDevice(e->device));
    if (int rc = flush_search(e, (hipStream_t)stream)) return rc;
    launch_bfs_export(e->d, dist, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

// hsv_to_rgb(h, 1, 1) (matplotlib.colors, util.init_colors) * 255, truncated like astype('uint8')
static void hue_rgb(double h, uint8_t *rgb) {
    const double h6 = h * 6.0;
    const int i = (int)std::floor(h6) % 6;
    const double f = h6 - std::floor(h6), q = 1.0 - f, t = f;
    double r, g, b;
    switch (i) {
        case 0: r = 1; g = t; b = 0; break;
        case 1: r = q; g = 1; b = 0; break;
        case 2: r = 0; g = 1; b = t; break;
        case 3: r = 0; g = q; b = 1; break;
        case 4: r = t; g = 0; b = 1; break;
        default: r = 1; g = 0; b = q; break;
    }
    rgb[0] = (uint8_t)(r * 255.0); rgb[1] = (uint8_t)(g * 255.0); rgb[2] = (uint8_t)(b * 255.0);
}

int mapf_render(mapf_env *e, const int32_t *envs, int32_t n, int32_t scale, uint8_t *frames, void *stream) {
    if (!e || !envs || !frames) return fail(MAPF_EINVAL, "null argument");
    if (!e->ready) return fail(MAPF_ESTATE, "mapf_render before mapf_reset");
    if (n < 0 || n > 65535) return fail(MAPF_EINVAL, "n must be in 0..65535");
    if (scale < 4 || scale > 64) return fail(MAPF_EINVAL, "scale must be in 4..64");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    if (int rc = flush_search(e, s)) return rc;
    if (n == 0) return MAPF_OK;
    RenderSpec rs{};
    rs.scale = scale;
    const uint8_t fixed[9] = {255, 255, 255, 0, 0, 0, 127, 127, 127};   // colours[0], [-1], [-2] * 255
    std::memcpy(rs.palette, fixed, 9);
    for (int a = 0; a < e->d.N; ++a) hue_rgb((double)a / (double)e->d.N, rs.palette + 3 * (3 + a));
    // drawStar(coord, S, S, 5): outerRad = S // 2, innerRad = int(outerRad * 3 / 8)
    const double PI = 3.141592653589793, between = 2.0 * PI / 5.0;
    const int outer = scale / 2, inner = (int)(outer * 3.0 / 8.0);
    for (int i = 0; i < 5; ++i) {
        const double pa = PI / 2.0 + i * between;
        const double ang[3] = {pa - between / 2.0, pa, pa + between / 2.0};
        const int rad[3] = {inner, outer, inner};
        for (int k = 0; k < 3; ++k) {
            rs.star_x[3 * i + k] = rad[k] * std::cos(ang[k]);
            rs.star_y[3 * i + k] = rad[k] * std::sin(ang[k]);
        }
    }
    launch_render(e->d, envs, n, rs, frames, s);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_get_counters(mapf_env *e, uint32_t *host16, void *stream) {
    if (!e || !host16) return fail(MAPF_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    if (int rc = flush_search(e, s)) return rc;
    HIPCHK(hipMemcpyAsync(host16, e->d.counters, 16 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return MAPF_OK;
}

int mapf_get_profile(mapf_env *e, uint64_t *host16, int reset, void *stream) {
    if (!e || !host16) return fail(MAPF_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    std::vector<uint64_t> all(PROF_TL);
    HIPCHK(hipMemcpyAsync(all.data(), e->d.prof, all.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    if (reset) HIPCHK(hipMemsetAsync(e->d.prof, 0, PROF_WORDS * sizeof(uint64_t), s));
    HIPCHK(hipStreamSynchronize(s));
    for (int k = 0; k < 16; ++k) host16[k] = 0;
    for (size_t w = 0; w < 65536; ++w) {   // sums over waves of the LAST launch; [15] = waves
        if (!all[w * 8 + 7]) continue;
        for (int k = 0; k < 7; ++k) host16[k] += all[w * 8 + k];
        host16[15] += 1;
    }
    return MAPF_OK;
}

int mapf_get_wave_profile(mapf_env *e, uint64_t *host, int32_t nwaves, void *stream) {
    if (!e || !host || nwaves < 0 || nwaves > (int)PROF_WAVES) return fail(MAPF_EINVAL, "bad argument");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(host, e->d.prof, (size_t)nwaves * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return MAPF_OK;
}

int mapf_get_timeline(mapf_env *e, uint64_t *host, int32_t nblocks, void *stream) {
    if (!e || !host || nblocks < 0 || nblocks > (int)PROF_TL_BLOCKS) return fail(MAPF_EINVAL, "bad argument");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(host, e->d.prof + PROF_TL, (size_t)nblocks * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return MAPF_OK;
}

int mapf_get_state(mapf_env *e, const mapf_state *h, void *stream) {
    if (!e || !h) return fail(MAPF_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    const DevEnv &d = e->d;
    const size_t BN = (size_t)d.B * d.N;
    std::vector<uint32_t> pos(BN), goal(BN), hpath((size_t)d.B * 2 * d.Lmax), hp(d.B), hn(d.B), hg(d.B), he(d.B), clk(d.B);
    std::vector<int8_t> la(BN);
    std::vector<int32_t> cur(BN), hl(2 * (size_t)d.B), hs(d.B), hc(d.B);
    if (int rc = flush_search(e, s)) return rc;
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipMemcpy(pos.data(), d.pos, BN * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(goal.data(), d.goal, BN * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(la.data(), d.last_act, BN, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cur.data(), d.seq_cur, BN * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hpath.data(), d.hpath, hpath.size() * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hl.data(), d.hlen, 2 * d.B * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hs.data(), d.hstep, d.B * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hc.data(), d.hcur, d.B * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hn.data(), d.hnext, d.B * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hp.data(), d.hpos, d.B * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hg.data(), d.hgoal, d.B * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(he.data(), d.hentr, d.B * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(clk.data(), d.clock, d.B * 4, hipMemcpyDeviceToHost));
    for (size_t k = 0; k < BN; ++k) {
        if (h->pos) { h->pos[2 * k] = prow(pos[k]); h->pos[2 * k + 1] = pcol(pos[k]); }
        if (h->goal) { h->goal[2 * k] = prow(goal[k]); h->goal[2 * k + 1] = pcol(goal[k]); }
        if (h->last_action) h->last_action[k] = la[k];
        if (h->seq_cursor) h->seq_cursor[k] = cur[k];
    }
    for (int b = 0; b < d.B; ++b) {
        const uint32_t *path = hpath.data() + ((size_t)b * 2 + hc[b]) * d.Lmax;
        const int st = hs[b], len = hl[2 * b + hc[b]];
        const uint32_t nx = hn[b];
        if (h->human) {
            int32_t *o = h->human + 10 * b;
            o[0] = prow(hp[b]); o[1] = pcol(hp[b]); o[2] = prow(nx); o[3] = pcol(nx);
            o[4] = prow(hg[b]); o[5] = pcol(hg[b]); o[6] = st; o[7] = len; o[8] = prow(he[b]); o[9] = pcol(he[b]);
        }
        if (h->human_path)
            for (int k = 0; k < d.Lmax; ++k) {
                h->human_path[((size_t)b * d.Lmax + k) * 2] = k < len ? prow(path[k]) : -1;
                h->human_path[((size_t)b * d.Lmax + k) * 2 + 1] = k < len ? pcol(path[k]) : -1;
            }
        if (h->clock) h->clock[b] = clk[b];
    }
    return MAPF_OK;
}

int mapf_set_state(mapf_env *e, const mapf_state *h, void *stream) {
    if (!e || !h) return fail(MAPF_EINVAL, "null argument");
    if (!e->ready) return fail(MAPF_ESTATE, "mapf_set_state before mapf_reset");
    HIPCHK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    DevEnv &d = e->d;
    const size_t BN = (size_t)d.B * d.N;
    if (int rc = flush_search(e, s)) return rc;
    HIPCHK(hipStreamSynchronize(s));
    if (h->pos) {
        std::vector<uint32_t> v(BN);
        for (size_t k = 0; k < BN; ++k) {
            const int r = h->pos[2 * k], c = h->pos[2 * k + 1];
            if (r < 0 || r >= d.H || c < 0 || c >= d.W) return fail(MAPF_EINVAL, "pos out of the map");
            v[k] = pack(r, c);
        }
        HIPCHK(hipMemcpy(d.pos, v.data(), BN * 4, hipMemcpyHostToDevice));
    }
    if (h->goal) {
        std::vector<uint32_t> v(BN);
        for (size_t k = 0; k < BN; ++k) {
            const int r = h->goal[2 * k], c = h->goal[2 * k + 1];
            if (r < 0 || r >= d.H || c < 0 || c >= d.W) return fail(MAPF_EINVAL, "goal out of the map");
            v[k] = pack(r, c);
        }
        HIPCHK(hipMemcpy(d.goal, v.data(), BN * 4, hipMemcpyHostToDevice));
    }
    if (h->last_action) {
        std::vector<int8_t> v(BN);
        for (size_t k = 0; k < BN; ++k) {
            if (h->last_action[k] < -1 || h->last_action[k] > 4) return fail(MAPF_EINVAL, "last_action out of range");
            v[k] = (int8_t)h->last_action[k];
        }
        HIPCHK(hipMemcpy(d.last_act, v.data(), BN, hipMemcpyHostToDevice));
    }
    if (h->seq_cursor) HIPCHK(hipMemcpy(d.seq_cur, h->seq_cursor, BN * 4, hipMemcpyHostToDevice));
    if (h->human_path && h->human) {
        // the given path becomes buffer 0 (current); buffer 1 is re-planned below
        std::vector<uint32_t> path((size_t)d.B * 2 * d.Lmax, 0u);
        std::vector<int32_t> hl(2 * (size_t)d.B, 1), hc(d.B, 0);
        for (int b = 0; b < d.B; ++b) {
            const int len = h->human[10 * b + 7];
            if (len < 1 || len > d.Lmax) return fail(MAPF_EINVAL, "human path length out of range");
            hl[2 * b] = len;
            for (int k = 0; k < len; ++k)
                path[(size_t)b * 2 * d.Lmax + k] = pack(h->human_path[((size_t)b * d.Lmax + k) * 2],
                                                        h->human_path[((size_t)b * d.Lmax + k) * 2 + 1]);
        }
        HIPCHK(hipMemcpy(d.hpath, path.data(), path.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d.hlen, hl.data(), hl.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d.hcur, hc.data(), d.B * 4, hipMemcpyHostToDevice));
    }
    if (h->human) {
        std::vector<uint32_t> hp(d.B), hg(d.B), he(d.B);
        std::vector<int32_t> hs(d.B);
        for (int b = 0; b < d.B; ++b) {
            const int32_t *o = h->human + 10 * b;
            hp[b] = pack(o[0], o[1]); hg[b] = pack(o[4], o[5]); hs[b] = o[6]; he[b] = pack(o[8], o[9]);
        }
        HIPCHK(hipMemcpy(d.hpos, hp.data(), d.B * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d.hgoal, hg.data(), d.B * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d.hstep, hs.data(), d.B * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d.hentr, he.data(), d.B * 4, hipMemcpyHostToDevice));
    }
    if (h->clock) HIPCHK(hipMemcpy(d.clock, h->clock, d.B * 4, hipMemcpyHostToDevice));
    if (h->human || h->clock) {
        // position / next position follow the path and step (Human.getPos / getNextPos);
        // the next path is re-planned for the new (clock, step) and searched
        launch_plan(d, 0, s);
        launch_search(d, 0, 2, s);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(s));
    }
    return MAPF_OK;
}

int mapf_gae(const float *rewards, const float *values, const float *v_last, float *adv, float *ret, int32_t T,
             int32_t M, double gamma, double lam, void *stream) {
    if (!rewards || !values || !v_last || !adv || !ret) return fail(MAPF_EINVAL, "null argument");
    if (T < 1 || M < 1) return fail(MAPF_EINVAL, "T and M must be >= 1");
    // numpy: GAMMA * next_nonterminal (python floats) then * f32 array -> f32(gamma);
    //        GAMMA * LAM * next_nonterminal -> f32(gamma * lam)   (runner.py:134-140)
    launch_gae(rewards, values, v_last, adv, ret, T, M, (float)(gamma * 1.0), (float)(gamma * lam * 1.0),
               (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_normalize_advantages(const float *ret, const float *v, const float *cret, const float *cv, float *adv_out,
                              float *cadv_out, int32_t M, double lagrange, int32_t mix, void *stream) {
    if (!ret || !v || !cret || !cv || !adv_out || !cadv_out) return fail(MAPF_EINVAL, "null argument");
    if (M < 1) return fail(MAPF_EINVAL, "M must be >= 1");
    launch_normalize(ret, v, cret, cv, adv_out, cadv_out, M, (float)lagrange, (float)(lagrange + 1.0), mix, nullptr,
                     (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_normalize_advantages_dlam(const float *ret, const float *v, const float *cret, const float *cv,
                                   float *adv_out, float *cadv_out, int32_t M, const float *lam_dev, int32_t mix,
                                   void *stream) {
    if (!ret || !v || !cret || !cv || !adv_out || !cadv_out || !lam_dev) return fail(MAPF_EINVAL, "null argument");
    if (M < 1) return fail(MAPF_EINVAL, "M must be >= 1");
    launch_normalize(ret, v, cret, cv, adv_out, cadv_out, M, 0.f, 1.f, mix, lam_dev, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_advantage_moments(const float *ret, const float *v, const float *cret, const float *cv, int32_t M,
                           const double *mean, double *out, void *stream) {
    if (!ret || !v || !cret || !cv || !out) return fail(MAPF_EINVAL, "null argument");
    if (M < 0) return fail(MAPF_EINVAL, "M must be >= 0");
    launch_moments(ret, v, cret, cv, M, mean, out, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_normalize_advantages_stats(const float *ret, const float *v, const float *cret, const float *cv,
                                    const double *stats, float *adv_out, float *cadv_out, int32_t M, double lagrange,
                                    int32_t mix, void *stream) {
    if (!ret || !v || !cret || !cv || !stats || !adv_out || !cadv_out) return fail(MAPF_EINVAL, "null argument");
    if (M < 0) return fail(MAPF_EINVAL, "M must be >= 0");
    if (M == 0) return MAPF_OK;
    launch_normalize_stats(ret, v, cret, cv, stats, adv_out, cadv_out, M, (float)lagrange, (float)(lagrange + 1.0), mix,
                           nullptr, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_normalize_advantages_stats_dlam(const float *ret, const float *v, const float *cret, const float *cv,
                                         const double *stats, float *adv_out, float *cadv_out, int32_t M,
                                         const float *lam_dev, int32_t mix, void *stream) {
    if (!ret || !v || !cret || !cv || !stats || !adv_out || !cadv_out || !lam_dev)
        return fail(MAPF_EINVAL, "null argument");
    if (M < 0) return fail(MAPF_EINVAL, "M must be >= 0");
    if (M == 0) return MAPF_OK;
    launch_normalize_stats(ret, v, cret, cv, stats, adv_out, cadv_out, M, 0.f, 1.f, mix, lam_dev, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_episode_sum(const float *x, int32_t T, int32_t B, int32_t N, float *out, void *stream) {
    if (!x || !out) return fail(MAPF_EINVAL, "null argument");
    if (T < 0 || B < 1 || N < 1 || N > 128) return fail(MAPF_EINVAL, "need T >= 0, B >= 1, N in 1..128");
    launch_episode_sum(x, T, B, N, out, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

int mapf_sample_actions(const float *ps, int32_t ps_stride, int32_t *actions, int64_t *actions64, int32_t M,
                        uint64_t seed, uint32_t step, void *stream) {
    if (!ps || (!actions && !actions64)) return fail(MAPF_EINVAL, "null argument");
    if (M < 1 || ps_stride < 5) return fail(MAPF_EINVAL, "bad M / stride");
    launch_sample(ps, ps_stride, actions, actions64, M, seed, step, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MAPF_OK;
}

}  // extern "C"
