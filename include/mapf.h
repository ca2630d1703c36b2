/*
 * include/mapf.h -- C ABI of libmapf.so, the MI355X-native batched MAPF env.
 *
 * Drop-in boundary for the reference's per-step env API.
 * The reference (Nielsencu/primal-ppo) has no FFI layer: its boundary is the
 * Python method API of mapf_gym.MapfGym, called by runner.py:30-100 and
 * evaluate.py:218-269 in this fixed order:
 *
 *   MapfGym() / FixedMapfGym(...)   mapf_gym.py:164-173 / :648-669  -> mapf_reset
 *   getAllObservations()            mapf_gym.py:327-336             -> mapf_observe
 *   getActionStatus(a)              mapf_gym.py:434-480             -> mapf_step (status)
 *   calculateActionReward(a, st)    mapf_gym.py:483-511             -> mapf_step (reward, shadow_goals)
 *   calculateCostReward(a)          mapf_gym.py:528-533             -> mapf_step (cost)
 *   getTrainValid(a)                mapf_gym.py:535-550             -> mapf_step (train_valid)
 *   jointStep(a, st)                mapf_gym.py:614-637             -> mapf_step (MAPF_STEP_COMMIT)
 *   jointStep + getAllObservations  runner.py:84-97                 -> mapf_step_observe (one launch)
 *   agent.bfsMap / makeBfsMap       mapf_gym.py:211-244             -> mapf_bfs
 *   renderWorld / MapfGym._render   util.py:189-232, mapf_gym.py:639 -> mapf_render
 *   Runner.run GAE                  runner.py:117-149               -> mapf_gae
 *   Model.train normalisation       model.py:106-113                -> mapf_normalize_advantages
 *   Model.step sampling             model.py:38-40                  -> mapf_sample_actions
 *
 * Conventions
 *  - One handle = B lockstep environments resident on one GPU (Structure of
 *    Arrays in HBM).  The handle owns its device state; the caller owns every
 *    output buffer (device pointers, e.g. torch tensors' data_ptr()).
 *  - Calls are asynchronous on the caller's HIP stream (`stream` is a
 *    hipStream_t passed as void*; NULL = the null stream).  A handle is not
 *    thread-safe: one handle per GPU / process.
 *  - Errors: 0 = OK, negative = error code (MAPF_E*); mapf_last_error() gives
 *    a message (thread-local).  Impossible states the reference raises on
 *    (mapf_gym.py:456,508,588,610; astar_4.py:109) are counted on the device
 *    (mapf_get_counters) instead of raised.
 *  - No C++ exceptions cross this boundary.
 */
#ifndef MAPF_H
#define MAPF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAPF_ABI_VERSION 1

#define MAPF_OK 0
#define MAPF_EINVAL (-1)
#define MAPF_EDEVICE (-2)
#define MAPF_ENOMEM (-3)
#define MAPF_ESTATE (-4)

/* Environment configuration.  Field names follow alg_parameters.py
 * (EnvParameters :27-48, TrainingParameters :76-78, NetParameters :103-104). */
typedef struct mapf_config {
    int32_t num_envs;        /* B: environments on this device                     */
    int32_t num_agents;      /* N: EnvParameters.N_AGENTS, 1..64                    */
    int32_t height, width;   /* H, W: grid, 1..128 each                             */
    int32_t fov;             /* F: EnvParameters.FOV_SIZE, 1..16                    */
    int32_t num_channel;     /* C: 5, 6 (NetParameters.NUM_CHANNEL) or 7 (+BFS ch) */
    int32_t use_da, use_hp;  /* FixedMapfGym(useDA, useHP), mapf_gym.py:662-663    */
    int32_t lifelong;        /* EnvParameters.LIFELONG                              */
    int32_t human_mode;      /* 0 LoopingHuman, 1 Human (random goals), 2 FixedPathHuman */
    int32_t goal_mode;       /* 0 agentsSequence (FixedMapfGym), 1 getFreeCell (MapfGym) */
    int32_t fix_choice;      /* fixActions random.choice: 0 rotating rule, 1 Philox */
    int32_t shared_map;      /* 1: one H x W map for all envs, 0: one map per env    */
    int32_t keep_bfs;        /* maintain agent.bfsMap (makeBfsMap) for every agent   */
    int32_t max_seq;         /* S: agentsSequence capacity per agent (goal_mode 0)  */
    int32_t max_human_seq;   /* human pose sequence capacity (human_mode 2)          */
    int32_t k_predict;       /* TrainingParameters.K_TIMESTEP_PREDICT                */
    int32_t penalty_radius;  /* EnvParameters.PENALTY_RADIUS                         */
    float action_cost;       /* EnvParameters.ACTION_COST                            */
    float collision_cost;    /* EnvParameters.COLLISION_COST                         */
    float human_collision_cost; /* EnvParameters.HUMAN_COLLISION_COST                */
    float repeat_cost;       /* EnvParameters.REPEAT_POS                             */
    float goal_reward;       /* EnvParameters.GOAL_REWARD (runner.py:89-91)          */
    int32_t env_offset;      /* global index of env 0 (RNG counters; sharding)       */
    uint32_t reserved;
    uint64_t seed;           /* Philox key (SetupParameters.SEED)                    */
} mapf_config;

typedef struct mapf_env mapf_env;

/* Reset specification.  All pointers are HOST pointers.
 * mode 0 (FixedMapfGym, mapf_gym.py:648-669): maps + agent sequences +
 *   human start/goal (LoopingHuman) or human pose sequence (FixedPathHuman).
 * mode 1 (MapfGym, mapf_gym.py:164-184): maps + Philox draws for the human
 *   entrance/goal and agent starts/goals (getFreeCell semantics). */
typedef struct mapf_reset_spec {
    int32_t mode;
    int32_t reserved;
    const int8_t *maps;          /* [shared_map ? 1 : B][H][W], values 0 (free) / -1 (obstacle) */
    const int32_t *seq;          /* [B][N][S][2] (row, col)                    mode 0 */
    const int32_t *seq_len;      /* [B][N], 1..S                               mode 0 */
    const int32_t *human_start;  /* [B][2]                                     mode 0, human_mode 0 */
    const int32_t *human_goal;   /* [B][2]                                     mode 0, human_mode 0 */
    const int32_t *human_seq;    /* [B][max_human_seq][2]                      human_mode 2 */
    const int32_t *human_seq_len;/* [B], 2..max_human_seq                      human_mode 2 */
    uint64_t seed;               /* mode 1: overrides config.seed when non-zero */
} mapf_reset_spec;

/* Per-step outputs: DEVICE pointers owned by the caller; NULL = not written. */
typedef struct mapf_step_out {
    int8_t *status;          /* [B][N]  getActionStatus: 1, -1, -2, -3, -4          */
    float *reward;           /* [B][N]  calculateActionReward (before GOAL_REWARD)   */
    int32_t *shadow_goals;   /* [B]     calculateActionReward's shadowGoal           */
    float *cost;             /* [B][N]  calculateCostReward                          */
    float *train_valid;      /* [B][N][5] getTrainValid                              */
    int32_t *actions_fixed;  /* [B][N]  actions after fixActions                      */
    float *goals_reached;    /* [B][N]  jointStep's goalsReached                      */
    float *constraints;      /* [B][N]  jointStep's constraintsViolated               */
    float *reward_total;     /* [B][N]  reward + GOAL_REWARD where goal reached (runner.py:89-91) */
} mapf_step_out;

#define MAPF_STEP_COMMIT 1u  /* apply jointStep (move, goals, human, counters).  Without it
                                only the pre-step outputs are produced and no state changes. */

/* Host-side snapshot of the env state (checkpoint / test hook).  Any pointer
 * may be NULL (skipped).  Cells are (row, col). */
typedef struct mapf_state {
    int32_t *pos;            /* [B][N][2]                                  */
    int32_t *goal;           /* [B][N][2]                                  */
    int32_t *last_action;    /* [B][N]   -1 = none (reset)                 */
    int32_t *seq_cursor;     /* [B][N]   util.Sequence.curIdx              */
    int32_t *human;          /* [B][10]  pos r,c; next r,c; goal r,c; step; path len; entrance r,c */
    int32_t *human_path;     /* [B][path_capacity][2]                      */
    uint32_t *clock;         /* [B]      steps since reset                 */
} mapf_state;

const char *mapf_last_error(void);
int mapf_abi_version(void);

int mapf_create(const mapf_config *cfg, int device, mapf_env **out);
int mapf_destroy(mapf_env *env);
int mapf_path_capacity(const mapf_env *env);       /* human path capacity per env */
/* 1 if mapf_step_observe runs as ONE launch for this configuration (N <= 8,
 * no BFS channel, no scripted human), 0 if it runs as step + observe. */
int mapf_step_observe_fused(const mapf_env *env);

int mapf_reset(mapf_env *env, const mapf_reset_spec *spec, void *stream);

/* Obstacle maps generated on the device, then a seeded reset on them (mode 1 of
 * mapf_reset) -- no host maps, no upload, asynchronous on `stream`.
 *   MAPF_MAPS_WAREHOUSE: MapfGym()'s map (mapf_gym.py:166 -> generateWarehouse(num_block=
 *     [lo, hi]), map_generator.py:127-138): per env (one map if shared_map) a length L
 *     uniform in [lo, hi], breadth int(L / (2/3)), shelves as the reference places them
 *     (bit-exact for a given L), at the top-left of the H x W stack, the rest obstacles.
 *     Needs H >= hi, W >= int(hi / (2/3)).
 *   MAPF_MAPS_RANDOM: random_generator's rule -(rand < p) (map_generator.py:23) over H x W,
 *     p = density.
 *   largest = 1: free cells outside the largest 4-connected free component become
 *     obstacles (H * W <= 8192).
 * Draws: Philox (key = seed, or config.seed if 0; counters (env id, 10, epoch, k)).
 * maps_out: optional DEVICE int8 [shared_map ? 1 : B][H][W] copy of the maps. */
#define MAPF_MAPS_WAREHOUSE 0
#define MAPF_MAPS_RANDOM 1
typedef struct mapf_mapgen_spec {
    int32_t kind;            /* MAPF_MAPS_*                                    */
    int32_t lo, hi;          /* warehouse length range (EnvParameters.WORLD_SIZE) */
    int32_t largest;         /* keep the largest 4-connected free component   */
    float density;           /* random maps: obstacle probability             */
    uint32_t epoch;          /* draw epoch (e.g. the rollout index)           */
    uint64_t seed;           /* 0: config.seed                                */
} mapf_mapgen_spec;
int mapf_reset_generated(mapf_env *env, const mapf_mapgen_spec *spec, int8_t *maps_out, void *stream);

/* One lockstep step for all B envs: actions are DEVICE int32 [B][N] in 0..4. */
int mapf_step(mapf_env *env, const int32_t *actions, const mapf_step_out *out, uint32_t flags, void *stream);

/* Env-only benchmark / random-policy rollouts: draw the uniform random policy's
 * actions on the device (same Philox stream as mapf_random_actions), write them
 * to actions_out (DEVICE int32 [B][N]) and step with them, in one launch. */
int mapf_step_random(mapf_env *env, int32_t *actions_out, const mapf_step_out *out, uint32_t flags, void *stream);

/* getAllObservations for all envs: obs DEVICE float [B][N][C][F][F], vec [B][N][4]. */
int mapf_observe(mapf_env *env, float *obs, float *vec, void *stream);

/* jointStep + getAllObservations in ONE launch (runner.py:84-97 calls them back
 * to back): the committed step of mapf_step followed by mapf_observe, identical
 * outputs.  Each workgroup steps its envs and observes them from LDS; the
 * previous step's search work rides in the same launch (its results are next
 * needed two steps later).  Configurations the fused kernel does not cover
 * (N > 8, scripted humans, the BFS channel, very large maps) run the two
 * launches.  mapf_step_observe_random draws the random policy like
 * mapf_step_random. */
int mapf_step_observe(mapf_env *env, const int32_t *actions, const mapf_step_out *out, float *obs, float *vec,
                      void *stream);
int mapf_step_observe_random(mapf_env *env, int32_t *actions_out, const mapf_step_out *out, float *obs,
                             float *vec, void *stream);

/* Random-policy rollout: T x (mapf_step_observe_random), i.e. runner.py:64-100
 * with the uniform random policy T times, in ONE launch where the configuration
 * allows (mapf_rollout_random_fused; otherwise T launches) -- identical results.
 * slots = 1: step t writes slot t of [T]-leading DEVICE buffers (actions_out
 * [T][B][N], every out field [T][...], obs [T][B][N][C][F][F], vec [T][B][N][4]),
 * i.e. rollout buffers; slots = 0: every step overwrites the same [B]-leading
 * buffers.  Each wave of the one-launch kernel owns one env and loops step ->
 * observe -> its own search work, so steps overlap other envs' store drains. */
int mapf_rollout_random(mapf_env *env, int32_t T, int32_t slots, int32_t *actions_out, const mapf_step_out *out,
                        float *obs, float *vec, void *stream);
/* Which kernel mapf_rollout_random runs for this configuration (0: T per-step
 * launches).  1: the pair-lane kernel -- N in 5..8 with a whole number of float4s
 * per env's observation, one shared map whose padded bitmap fits 64 words
 * (W + 2*(F/2) <= 32, H + 2*(F/2) <= 64), no BFS channel, Human or LoopingHuman,
 * random (MapfGym) goals.  2: the one-wave-per-env kernel -- every other
 * configuration whose per-env LDS (map rows, observation bit-stream, BFS image)
 * fits 64 KiB: up to 64 agents, per-env maps, the BFS channel (c4, c5). */
int mapf_rollout_random_fused(const mapf_env *env);

/* Launch tuning of one handle: which form of a kernel the launches take (the measured choices
 * of DESIGN.md §4 / §9).  The reference has no counterpart (its env is Python); these fields
 * only pick between forms that produce identical results.  mapf_create sets the defaults
 * (mapf_tuning_default); nothing is read from the process environment.  A field at its
 * default means "the measured choice for this configuration", which may depend on B, N, the
 * map size, slots and the device (CU count, LDS size, the kernels' VGPR counts). */
typedef struct mapf_tuning {
    /* pair-lane rollout (mapf_rollout_random_fused == 1: N in 5..8, shared map) */
    int32_t roll_occ;        /* workgroups per CU the LDS request admits: 0 = ceil(grid / CUs), 1..16      */
    int32_t roll_group;      /* the 16 waves of a CU in one workgroup: -1 auto (slots, or roll_fair > 0), 0, 1 */
    int32_t roll_fair;       /* grouped, issue priority by progress: -1 auto (4 in place, 0 slots), 0 off, n */
    int32_t roll_slack;      /* grouped, roll_fair 0: waves paced within n steps of the slowest (< 0 off)  */
    /* one-wave-per-env rollout (mapf_rollout_random_fused == 2: up to 64 agents, per-env maps, C = 7) */
    int32_t wide_nt;         /* nontemporal observation stores: -1 auto (slots, or a [B] buffer > 128 MB), 0, 1 */
    int32_t wide_pipe;       /* 1 auto: a stepping and observing waves per env where they fit; 0 one wave   */
    int32_t wide_grid;       /* 1 auto: the step's LDS neighbour grid where it fits; 0 the agent loop       */
    int32_t wide_overlap;    /* 1 auto: pipelined through LDS counters (no BFS channel); 0 per-step barriers */
    int32_t wide_obs;        /* observing waves per env in the overlapped form: 2 (auto, where they fit) or 1 */
    int32_t wide_epw;        /* envs per workgroup: 0 auto (all the envs of a CU where the form allows), n    */
    int32_t wide_pair;       /* epw > 1: 0 wave w is env w / wpe's role w % wpe, 1 env w % epw's role w / epw */
    int32_t wide_slack;      /* one wave per env, epw > 1: paced within n steps of the group's slowest (< 0 off) */
    int32_t wide_fair;       /* one wave per env, epw > 1: issue priority by progress instead of waits (0 off) */
    int32_t wide_prio;       /* pipelined: the stepping wave issues at priority 3 (0 off)                   */
    int32_t wide_bfsobs;     /* three-wave form: the observers search the rebuilt BFS maps (0: the stepper)  */
    int32_t xcd_remap;       /* persistent kernels: XCD-aware env order (0 off)                            */
    /* per-step launches */
    int32_t obs_envs;        /* envs per observe workgroup: 0 auto (64 / N for N <= 8, else 1), 1..64      */
    int32_t step_block;      /* threads per step workgroup: 64, 128 or 256                                 */
    int32_t search_blocks;   /* workgroups of an observe launch that run search work: 1..1024              */
    int32_t band_blocks;     /* zero-band workgroups of the fused step+observe launch: 0..4096             */
    int32_t agent_lanes;     /* 1: the agent-per-lane step kernel even for N <= 8 (no pair-lane kernels)    */
    int32_t serial_search;   /* 1: wide maps search, then observe, on one stream                           */
    int32_t no_defer;        /* 1: a forked search is joined inside its own call                           */
    int32_t diag_exp;        /* -DMAPF_STAMPS builds only: phase experiment (0 = none)                     */
} mapf_tuning;
void mapf_tuning_default(mapf_tuning *t);
int mapf_get_tuning(const mapf_env *env, mapf_tuning *t);
/* Validates every field (MAPF_EINVAL, nothing changed, on a bad one); takes effect at the next launch. */
int mapf_set_tuning(mapf_env *env, const mapf_tuning *t);
/* The kernel mapf_rollout_random would launch now for `slots`, as text into buf (n bytes, NUL-terminated),
 * e.g. "rollout_wide3_kernel<u64,1,false> wpe=3 epw=4 grid=1 overlap=1 slack=-1 fair=0".  Returns
 * mapf_rollout_random_fused's kind (0: per-step launches, text "step_observe") or a negative error. */
int mapf_rollout_plan(const mapf_env *env, int32_t slots, char *buf, int32_t n);

/* Launch the search work a committed step left pending (agent.bfsMap updates, the
 * humans' next paths) on its own; mapf_observe otherwise runs it inside the
 * observation launch.  Any later call that needs it flushes implicitly.
 * Also joins, on `stream`, the searches that wide maps (the split path) defer onto a
 * second stream: call it on an uncaptured stream before beginning a hipGraph capture
 * of a handle that stepped outside the capture -- a call inside the capture that would
 * have to wait for such a search fails with MAPF_ESTATE instead (a graph cannot depend
 * on work recorded before its capture began). */
int mapf_flush(mapf_env *env, void *stream);

/* Return every argument slot that captured persistent launches of this handle took (16 per
 * handle; a capture past them fails with MAPF_ESTATE and launches nothing).  The store of a
 * launch's argument block is captured with the launch, so every replay re-writes its block
 * (stream-ordered) before its kernel reads it: a graph captured before the release still replays
 * right on its own.  What the release allows is a later capture sharing that slot -- replays of the
 * two graphs must then not overlap in time (two streams at once), or one kernel may read the other's
 * block.  Safest: call it once the graphs holding this handle's captured launches are destroyed. */
int mapf_release_captures(mapf_env *env);

/* Uniform random policy (Philox, counter = env clock): DEVICE int32 [B][N]. */
int mapf_random_actions(mapf_env *env, int32_t *actions, void *stream);

/* Copy agent.bfsMap for every agent: DEVICE int16 [B][N][H][W] (requires keep_bfs). */
int mapf_bfs(mapf_env *env, int16_t *dist, void *stream);

/* renderWorld (util.py:189-232; MapfGym._render, mapf_gym.py:639-646) for n envs at once:
 * envs = DEVICE int32 [n] env indices, frames = DEVICE uint8 [n][H*scale][W*scale][3] RGB.
 * Cells white / black, the human's remaining path as grey arrows and a star, agents' cells
 * in hsv(i / N, 1, 1), their goals as discs, the human as a grey triangle, painted in the
 * reference's order.  Polygons cover the pixels inside or on them (the reference uses cv2,
 * absent here: its edge rasterisation may differ by a pixel).  scale in 4..64. */
int mapf_render(mapf_env *env, const int32_t *envs, int32_t n, int32_t scale, uint8_t *frames, void *stream);

/* Counters of impossible states / clamped events (host uint32[16]); synchronises the stream. */
int mapf_get_counters(mapf_env *env, uint32_t *host16, void *stream);

/* Phase-cycle sums over the waves of the last step launch, recorded by the
 * -DMAPF_STAMPS diagnostic build ([15] = waves; all zero in the product
 * build): host uint64[16]; synchronises. */
int mapf_get_profile(mapf_env *env, uint64_t *host16, int reset, void *stream);
/* Diagnostic builds only: the fused kernel's per-workgroup timeline of its last
 * launch, host [nblocks][8] u64 (100 MHz realtime stamps 0-3, HW_ID, XCC_ID). */
int mapf_get_timeline(mapf_env *env, uint64_t *host, int32_t nblocks, void *stream);
/* Diagnostic build: per-wave phase cycles of the last step launch, uint64 [nwaves][8]
 * (slots 0-6 phases, 7 = 1 if the wave recorded). */
int mapf_get_wave_profile(mapf_env *env, uint64_t *host, int32_t nwaves, void *stream);

int mapf_get_state(mapf_env *env, const mapf_state *host, void *stream);   /* synchronises */
int mapf_set_state(mapf_env *env, const mapf_state *host, void *stream);   /* synchronises */

/* GAE over a [T][M] buffer (runner.py:117-149, numpy float32 semantics:
 * f32(gamma) and f32(gamma*lam) constants, separate multiply and add).
 * All pointers DEVICE float; v_last [M]. */
int mapf_gae(const float *rewards, const float *values, const float *v_last, float *adv, float *ret,
             int32_t T, int32_t M, double gamma, double lam, void *stream);

/* model.py:106-113: adv = norm(ret - v); cadv = norm(cret - cv);
 * norm(x) = (x - mean) / (std_unbiased + 1e-6); if mix: adv = (adv - lam*cadv)/(lam+1).
 * DEVICE float [M] each; adv_out / cadv_out [M]. */
int mapf_normalize_advantages(const float *ret, const float *v, const float *cret, const float *cv,
                              float *adv_out, float *cadv_out, int32_t M, double lagrange, int32_t mix,
                              void *stream);

/* mapf_normalize_advantages with the multiplier in DEVICE memory, lam_dev[2] = {f32(lagrange),
 * f32(lagrange + 1)} (computed on the host in double, as mapf_normalize_advantages does): the
 * form a captured hipGraph of the update replays with a new multiplier every update. */
int mapf_normalize_advantages_dlam(const float *ret, const float *v, const float *cret, const float *cv,
                                   float *adv_out, float *cadv_out, int32_t M, const float *lam_dev, int32_t mix,
                                   void *stream);

/* mapf_normalize_advantages over a minibatch split across ranks (model.py:106-113 on the GLOBAL
 * minibatch).  Per rank, x = ret - v and c = cret - cv over its M rows, in fp64:
 *   mapf_advantage_moments(mean = NULL): out[2] = {sum x, sum c}                -> all-reduce (sum)
 *   mapf_advantage_moments(mean = {mean x, mean c}): out[2] = {sum (x - mean x)^2, sum (c - mean c)^2}
 *                                                                            -> all-reduce (sum)
 *   mapf_normalize_advantages_stats(stats = {mean x, mean c, var x, var c}, unbiased over all ranks'
 *                                   rows): the normalisation of mapf_normalize_advantages.
 * mean, out, stats: DEVICE double pointers; the other arrays DEVICE float [M]. */
int mapf_advantage_moments(const float *ret, const float *v, const float *cret, const float *cv, int32_t M,
                           const double *mean, double *out, void *stream);
int mapf_normalize_advantages_stats(const float *ret, const float *v, const float *cret, const float *cv,
                                    const double *stats, float *adv_out, float *cadv_out, int32_t M, double lagrange,
                                    int32_t mix, void *stream);
/* mapf_normalize_advantages_stats with the multiplier in DEVICE memory, lam_dev[2] as in
 * mapf_normalize_advantages_dlam: the distributed form of Model.train's device update (the
 * multiplier stays where the captured single-rank form keeps it). */
int mapf_normalize_advantages_stats_dlam(const float *ret, const float *v, const float *cret, const float *cv,
                                         const double *stats, float *adv_out, float *cadv_out, int32_t M,
                                         const float *lam_dev, int32_t mix, void *stream);

/* OneEpPerformance.episodeReward / episodeCostReward of every env (runner.py:95-96:
 * `perf.episodeReward += np.sum(rewards)` once per step): x DEVICE float [T][B][N] (one
 * rollout's rewards, goal reward included, or cost rewards); out DEVICE float [B] = the float32
 * sum over t, in order, of numpy's float32 np.sum of x[t][b][0..N-1] (pairwise order; N <= 128). */
int mapf_episode_sum(const float *x, int32_t T, int32_t B, int32_t N, float *out, void *stream);

/* Model.step sampling (model.py:38-40): per row, inverse CDF of ps[M][5]
 * with a Philox uniform (key seed, counter (row, step)).  DEVICE. */
int mapf_sample_actions(const float *ps, int32_t ps_stride, int32_t *actions, int64_t *actions64, int32_t M,
                        uint64_t seed, uint32_t step, void *stream);

/* ---- Policy acting forward: fused elementwise epilogues (csrc/mapf_policy.hip) ----
 * SCRIMPNet.forward (net.py:101-155) under autocast with no grad (Model.step /
 * Model.value, model.py:26-69); each call replaces two or three of torch's passes
 * over one activation.  fp16 tensors are passed as uint16_t bit patterns; all
 * pointers DEVICE, contiguous; dropout p in [0, 1) (0 = off), masks from Philox(seed).
 *   nhwc_bias_relu       x[rows][C] = relu(x + bias)                 conv + F.relu (net.py:104-112)
 *   nhwc_bias_relu_pool2 out = maxpool2(relu(x + bias)), x [B][H][W][C] conv + relu + pool1/pool2
 *   layernorm_f16        y(fp16)[rows][512] = LayerNorm(x fp32, row stride)   transformer.py:7-24
 *   dropout_residual     x(fp32) += dropout(y fp16), n % 4 == 0        Residual(... do1/do2)
 *   gelu_dropout_f16     h = dropout(gelu(h)), n % 4 == 0               MLP_Block (transformer.py:27-45)
 *   tokens               x[B][L+1][D] = dropout(cat(cls, A*VV) + pos)  net.py:124-131 */
int mapf_nhwc_bias_relu(uint16_t *x, const uint16_t *bias, int64_t rows, int32_t C, void *stream);
int mapf_nhwc_bias_relu_pool2(const uint16_t *x, const uint16_t *bias, uint16_t *out, int32_t B, int32_t H, int32_t W,
                              int32_t C, void *stream);
int mapf_layernorm_f16(const float *x, int64_t x_row_stride, const float *gamma, const float *beta, uint16_t *y,
                       int64_t rows, int32_t dim, float eps, void *stream);
/* out[c] = fp16 of the fp32 sum over the rows of g fp16 [rows][C] (fixed order): a linear's bias
 * gradient (the training forward's 17-token linears, net._SplitKLinear; its short 2-D ones,
 * net._LinearBG).  C % 4 == 0, C <= 4096; work: 512 * C floats of scratch.  rows <= 8192 with C % 8 == 0
 * and g 16-B aligned: one launch (a block per 32 columns), else per-block partials then their sum.
 * rows == 0 zeroes out (g may then be NULL).  Capturable. */
int mapf_colsum_f16(const uint16_t *g, uint16_t *out, float *work, int64_t rows, int32_t C, void *stream);
/* Backward of p = maxpool2x2(relu(fp16(r + bias))) (mapf_nhwc_bias_relu_pool2's forward from the raw
 * conv output r fp16 NHWC [B][H][W][C]; the training forward's pooled conv layers, net.py:106-111):
 * dr gets dp at each window's first strictly greatest activation in (row, column) order -- torch's
 * max_pool2d argmax -- where that activation is > 0; 0 elsewhere, including rows / columns no window
 * covers.  dbias = fp16 of the fp32 sum of dr over B, H, W.  work: 512 * C floats.  Capturable. */
int mapf_relu_bias_pool_bwd_f16(const uint16_t *r, const uint16_t *bias, const uint16_t *dp, uint16_t *dr,
                                uint16_t *dbias, float *work, int32_t B, int32_t H, int32_t W, int32_t C,
                                void *stream);
/* Backward of y = relu(conv + bias) over NHWC fp16 rows [rows][C] (mapf_nhwc_bias_relu's forward; the
 * training forward's conv layers): dx = dy where y > 0 else 0 (fp16, [rows][C]), dbias = fp16 of the
 * fp32 sum of dx over the rows (fixed order).  C % 4 == 0, C <= 1024; work: 512 * C floats of
 * scratch.  rows == 0 zeroes dbias.  Capturable. */
int mapf_relu_bias_bwd_f16(const uint16_t *y, const uint16_t *dy, uint16_t *dx, uint16_t *dbias, float *work,
                           int64_t rows, int32_t C, void *stream);
/* Multi-tensor casts in ONE launch (the training forward's fp16 copies of the fp32 weights under
 * autocast, and their fp16 gradients back to fp32: one launch each way instead of one per tensor):
 * dst[i][k] = (fp16) src[i][k] (round to nearest even) or the exact reverse, k < n[i], i < count <= 64.
 * src / dst / n are HOST arrays of device pointers and element counts (copied into the launch's
 * arguments; capturable).  MAPF_EINVAL on a bad count or a null pointer with n[i] > 0. */
int mapf_cast_f32_to_f16_multi(const float *const *src, uint16_t *const *dst, const int64_t *n, int32_t count,
                               void *stream);
int mapf_cast_f16_to_f32_multi(const uint16_t *const *src, float *const *dst, const int64_t *n, int32_t count,
                               void *stream);
/* mapf_cast_f32_to_f16_multi where entry i with cout[i] > 0 is a conv weight stored [Cout][ks][ks][Cin]
 * (channels_last [Cout][Cin][ks][ks], Cout = cout[i], ks = ks[i], Cin = n[i] / (Cout ks ks)) written as
 * its flipped, transposed copy [Cin][ks][ks][Cout]: dst[ci][ky][kx][co] = src[co][ks-1-ky][ks-1-kx][ci]
 * -- the weight of the data gradient dx = conv(dy, w flipped, transposed) (_HipConv) -- in the same launch
 * as the plain casts (cout[i] == 0).  cout / ks: HOST int32 arrays.  MAPF_EINVAL as above or when n[i]
 * is not a multiple of Cout ks ks. */
int mapf_cast_f32_to_f16_multi_flip(const float *const *src, uint16_t *const *dst, const int64_t *n,
                                    const int32_t *cout, const int32_t *ks, int32_t count, void *stream);
/* The PPO update's optimizer tail (model._DeviceUpdate._back, model.py:177-185 of the reference: GradScaler
 * unscale_, clip_grad_norm_(10), Adam step, for torch.optim.Adam(fused, capturable) state): for `count`
 * fp32 tensors p[i], their gradients g[i], Adam moments m[i], v[i] (all four of one dense layout, n[i]
 * elements) and step counters steps[i] (fp32 scalars, equal): found_inf = 1 if any gradient is non-finite
 * (the caller zeroes it first); grad_norm = the 2-norm of g / scale over every tensor; unless found_inf:
 * g' = (g / scale) * min(max_norm / (grad_norm + 1e-6), 1), Adam with step = steps + 1 (no weight decay,
 * no amsgrad), steps += 1; g' is written back to g (found_inf or not: torch's unscale_ + clip leave it
 * so).  scale: the loss scale, fp32 in device memory.  work:
 * work_floats >= sum over tensors of ceil(n / 8192) floats of scratch.  Three kernel kinds, no host
 * synchronisation, no memset: capturable.  Pointer arrays are host arrays of device pointers. */
int mapf_optim_unscale_clip_adam(float *const *p, float *const *g, float *const *m, float *const *v,
                                 const int64_t *n, float *const *steps, int32_t count, const float *scale,
                                 float max_norm, float lr, float beta1, float beta2, float eps, float *found_inf,
                                 float *grad_norm, float *work, int64_t work_floats, void *stream);
/* Backward of z = fp16(LayerNorm(x)) (mapf_layernorm_f16; the training forward's PreNorm,
 * transformer.py:7-24 under autocast): given dz fp16 [rows][512], dx fp32 [rows][512] (contiguous),
 * dgamma / dbeta fp32 [512] (sums over the rows, fixed order).  mean / rstd are recomputed from x as
 * mapf_layernorm_f16 computes them.  dres: NULL, or fp32 [rows][512] added to dx -- the gradient the
 * residual path x + fn(LN(x)) brings to x, so the two need no separate add.  work: 2 * 512 * 512
 * floats of scratch.  rows == 0 zeroes dgamma / dbeta.  No host synchronisation, no memset:
 * capturable. */
int mapf_layernorm_bwd_f16(const float *x, int64_t x_row_stride, const float *gamma, const uint16_t *dz,
                           const float *dres, float *dx, float *dgamma, float *dbeta, float *work, int64_t rows,
                           int32_t dim, float eps, void *stream);

/* The TRAINING forward's dropout + residual + next LayerNorm (round 6; net._DropResLN), one pass:
 * x_out = res + dropout(y) (fp32; res rows res_row_stride floats apart, y fp16 contiguous), z =
 * fp16(LayerNorm(x_out)) -- mapf_dropout_residual_layernorm's arithmetic, out of place.  The dropout's
 * seed is read from DEVICE memory (seed_dev[0], a counter the training forward increments, mixed with
 * the site's salt), so a captured update draws new masks on every replay.  dim 512, p in [0, 1). */
int mapf_dropout_residual_layernorm_train(const float *res, int64_t res_row_stride, const uint16_t *y, float *x_out,
                                          const float *gamma, const float *beta, uint16_t *z, int64_t rows, int32_t dim,
                                          float eps, float p, const uint64_t *seed_dev, uint32_t salt, void *stream);
/* Its backward: mapf_layernorm_bwd_f16 over x_out (contiguous) with dres, plus dy (fp16) = the
 * gradient of the dropped branch: fp16(fp16(dx) * 1 / (1 - p)) where the forward kept, 0 elsewhere. */
int mapf_layernorm_dropout_bwd_f16(const float *x, const float *gamma, const uint16_t *dz, const float *dres, float *dx,
                                   uint16_t *dy, float *dgamma, float *dbeta, float *work, int64_t rows, int32_t dim,
                                   float eps, float p, const uint64_t *seed_dev, uint32_t salt, void *stream);
/* The training forward's MLP GELU + dropout (net._GeluDropout): out = dropout(gelu(h)) fp16 (h kept), and
 * its backward dh = fp16(gelu'(h) * fp16(dout / (1 - p)) where kept) -- torch's masked_scale then its exact
 * GeluBackward; the seed in device memory as above.  n % 4 == 0. */
int mapf_gelu_dropout_train_f16(const uint16_t *h, uint16_t *out, int64_t n, float p, const uint64_t *seed_dev,
                                uint32_t salt, void *stream);
int mapf_gelu_dropout_bwd_f16(const uint16_t *h, const uint16_t *dout, uint16_t *dh, int64_t n, float p,
                              const uint64_t *seed_dev, uint32_t salt, void *stream);
int mapf_dropout_residual(float *x, const uint16_t *y, int64_t n, float p, uint64_t seed, void *stream);
/* mapf_dropout_residual on rows x 512 contiguous x, y, then z = LayerNorm(x) as fp16 (like
 * mapf_layernorm_f16) in one pass; bit-identical to the two calls with the same seed. */
int mapf_dropout_residual_layernorm(float *x, const uint16_t *y, const float *gamma, const float *beta, uint16_t *z,
                                    int64_t rows, int32_t dim, float eps, float p, uint64_t seed, void *stream);
int mapf_gelu_dropout_f16(uint16_t *h, int64_t n, float p, uint64_t seed, void *stream);
int mapf_tokens(float *x, const float *A, const uint16_t *VV, const float *cls, const float *pos, int64_t B, int32_t L,
                int32_t D, float p, uint64_t seed, void *stream);
/* mapf_tokens (D = 512) and z = LayerNorm(x) as fp16 (gamma, beta, eps) in one pass; bit-identical
 * to mapf_tokens then mapf_layernorm_f16.  x may be NULL (the tokens not written: see
 * mapf_linear512_tokens_residual_layernorm). */
int mapf_tokens_layernorm(float *x, const float *A, const uint16_t *VV, const float *cls, const float *pos, int64_t B,
                          int32_t L, int32_t D, float p, uint64_t seed, const float *gamma, const float *beta,
                          float eps, uint16_t *z, void *stream);
/* The TRAINING forward's tokens and the first PreNorm (net._TokensLN; SCRIMPNet.forward, net.py:124-130):
 * x = dropout(cat(cls, A * VV) + pos) fp32 [B][L + 1][512] -- torch's ops and roundings (the product and
 * the sum rounded separately), dropout x * 1 / (1 - p) where kept, the mask from the device seed (graph-safe,
 * as mapf_dropout_residual_layernorm_train) -- and z = fp16(LayerNorm(x)) in one pass.  A: fp32 [B][L]
 * (the tokeniser's softmax), VV: fp16 [B][512], cls: fp32 [512], pos: fp32 [L + 1][512].  L == 16. */
int mapf_tokens_layernorm_train(float *x, const float *A, const uint16_t *VV, const float *cls, const float *pos,
                                int64_t B, int32_t L, float p, const uint64_t *seed_dev, uint32_t salt, const float *gamma,
                                const float *beta, float eps, uint16_t *z, void *stream);
/* Its backward after LayerNorm's (mapf_layernorm_bwd_f16 with the residual's gradient as dres): given
 * dx fp32 [B][L + 1][512], the same mask: g = dx / (1 - p) where kept; dA fp32 [B][L] = sum over the
 * columns of g[.][t + 1] VV; dVV fp16 [B][512] = sum over t of g[.][t + 1] A[.][t]; dpos fp32 [L + 1][512]
 * and dcls fp32 [512] the sums of g over B (fixed order).  work: 512 * (L + 1) * 512 floats. */
int mapf_tokens_train_bwd(const float *dx, const float *A, const uint16_t *VV, float *dA, uint16_t *dVV, float *dpos,
                          float *dcls, float *work, int64_t B, int32_t L, float p, const uint64_t *seed_dev,
                          uint32_t salt, void *stream);
/* Row tiles per workgroup of the mapf_linear512_* kernels (process-wide; bit-identical results
 * either way, for A/B timing): 2 (128 rows share each staged 512 x 32 weight chunk), 1 (64 rows),
 * or 0 (default: 1, the faster or within 1 % for every form at the c3 shape, round 5).  MAPF_EINVAL
 * on another value. */
int mapf_linear512_select(int32_t row_tiles);
/* LDS stages of the mapf_linear512_* kernels' K ring (process-wide, bit-identical results): 2, 3, 4
 * (stages - 1 weight/activation chunks in flight) or 0 (default, as measured).  MAPF_EINVAL otherwise. */
int mapf_linear512_stages(int32_t stages);
/* K per staged chunk of the mapf_linear512_* kernels (process-wide, bit-identical results: the same
 * MFMA sequence per element): 32 (64-B half-line LDS rows), 64 (full 128-B lines, two stages; with 2
 * row tiles all 160 KiB of a CU's LDS) or 0 (default: 32).  MAPF_EINVAL otherwise. */
int mapf_linear512_kdepth(int32_t k);

/* 512 x 512 Linear (w: fp16 [512 out][512 in], torch's layout; bias fp16 [512]) on `rows` contiguous fp16
 * rows a[rows][512] with its epilogue, one launch (MFMA GEMM; the linear's fp16 output stays on chip):
 *   mapf_linear512_gelu_dropout        out = dropout(gelu(a w^T + b)) fp16    = lin + mapf_gelu_dropout_f16
 *   mapf_linear512_residual_layernorm  x += dropout(a w^T + b); z = LayerNorm(x) fp16
 *                                                                  = lin + mapf_dropout_residual_layernorm
 * The same dropout masks as those kernels for the same seed (only the GEMM's summation order differs). */
int mapf_linear512_gelu_dropout(const uint16_t *a, const uint16_t *w, const uint16_t *bias, uint16_t *out, int64_t rows,
                                float p, uint64_t seed, void *stream);
int mapf_linear512_residual_layernorm(const uint16_t *a, const uint16_t *w, const uint16_t *bias, float *x,
                                      const float *gamma, const float *beta, uint16_t *z, int64_t rows, float eps,
                                      float p, uint64_t seed, void *stream);

/* mapf_linear512_residual_layernorm that writes the updated residual rows back only for rows
 * g % x_every == 0 (z for every row): before a block that keeps only token 0 of the stream
 * (the encoder's last block), the other tokens' fp32 rows are never needed again. */
int mapf_linear512_residual_layernorm_rows(const uint16_t *a, const uint16_t *w, const uint16_t *bias, float *x,
                                           const float *gamma, const float *beta, uint16_t *z, int64_t rows, float eps,
                                           float p, uint64_t seed, int32_t x_every, void *stream);

/* mapf_linear512_residual_layernorm on the first block's residual stream without it in HBM: the
 * input rows x (B sequences x (L + 1) tokens) are the tokens of mapf_tokens (A, VV, cls, pos,
 * tok_p, tok_seed: same values and mask bits) recomputed in the epilogue; x is written with
 * tokens + dropout(linear(a)), z = LayerNorm of it.  With mapf_tokens_layernorm(x = NULL, ...)
 * before it, the tokens' fp32 copy is never written nor read back. */
int mapf_linear512_tokens_residual_layernorm(const uint16_t *a, const uint16_t *w, const uint16_t *bias, float *x,
                                             const float *gamma, const float *beta, uint16_t *z, int64_t B, int32_t L,
                                             float eps, float p, uint64_t seed, const float *tok_A,
                                             const uint16_t *tok_VV, const float *tok_cls, const float *tok_pos,
                                             float tok_p, uint64_t tok_seed, void *stream);
/* out[B][q_rows][512] = softmax(q k^T * scale) v per head (heads = 16, head_dim = 32, n <= 32 tokens;
 * fp16 in/out, fp32 scores and softmax, P rounded to fp16 for P.V like flash SDPA) --
 * transformer.py:48-85's attention for the first q_rows queries.  Strides in fp16 elements between
 * consecutive tokens / sequences of q and of k, v (multiples of 8; q, k, v 16-B aligned). */
int mapf_attention_f16(const uint16_t *q, const uint16_t *k, const uint16_t *v, uint16_t *out, int64_t B, int32_t n,
                       int32_t q_rows, int64_t q_token_stride, int64_t q_seq_stride, int64_t kv_token_stride,
                       int64_t kv_seq_stride, int32_t heads, int32_t head_dim, float scale, void *stream);

/* The gradient of mapf_attention_f16 (the training forward's attention, transformer.py:48-85):
 * given q, k, v (strides as mapf_attention_f16), its fp16 output `out` and the output gradient
 * `dout` ([B][q_rows][heads * head_dim] at out_token_stride / out_seq_stride), writes dq (q's
 * strides) and dk, dv (k's / v's strides) as fp16: P recomputed in fp32, D = rowsum(dout * out).
 * n <= 32, heads 16, head_dim 32; every pointer 16-B aligned, strides multiples of 8. */
int mapf_attention_bwd_f16(const uint16_t *q, const uint16_t *k, const uint16_t *v, const uint16_t *out,
                           const uint16_t *dout, uint16_t *dq, uint16_t *dk, uint16_t *dv, int64_t B, int32_t n,
                           int32_t q_rows, int64_t q_token_stride, int64_t q_seq_stride, int64_t kv_token_stride,
                           int64_t kv_seq_stride, int64_t out_token_stride, int64_t out_seq_stride, int32_t heads,
                           int32_t head_dim, float scale, void *stream);
/* Which kernel mapf_attention_bwd_f16 launches (process-wide): 1 (default, round 6) the MFMA form, one
 * wave per (sequence, head), P and dS rounded to fp16 as MFMA operands; 0 the VALU form, one wave per
 * three heads, P and dS in fp32.  MAPF_EINVAL otherwise. */
int mapf_attention_bwd_select(int32_t form);

/* ---- PPO loss (model.py:115-175) ------------------------------------------
 * All loss terms of one minibatch update over R = rows x agents elements with A actions each,
 * plus d(all_loss)/d(new_ps, new_v, new_cv, policy_sig), in one launch.  Device pointers: fp32
 * new_ps / old_ps / policy_sig / train_valid [R][A], int64 action [R], fp32 new_v, old_v, returns,
 * new_cv, old_cv, cost_returns, advantage, cost_advantage [R]; sig_fp16 != 0 when policy_sig was
 * fp16 (autocast): its clamp bounds and 1 - sig round to fp16 like torch's.  HOST pointer coef[6]
 * = {CLIP_RANGE, ENTROPY_COEF, VALUE_COEF, VALID_COEF, COST_VALUE_COEF, COST_COEF * lambda}.
 * loss[1] (device) = all_loss; terms[7] (device) = {policy, entropy, critic, valid, cost critic,
 * cost, clip_frac}; the grads have the shapes of their inputs.  Deterministic (fixed-order reduction). */
int mapf_ppo_loss(const float *new_ps, const float *old_ps, const int64_t *action, const float *new_v,
                  const float *old_v, const float *returns, const float *new_cv, const float *old_cv,
                  const float *cost_returns, const float *advantage, const float *cost_advantage,
                  const float *policy_sig, int32_t sig_fp16, const float *train_valid, int64_t R, int32_t A,
                  const float *coef, float *loss, float *terms, float *grad_ps, float *grad_v, float *grad_cv,
                  float *grad_sig, void *stream);

/* SCRIMPNet's 128- and 256-channel convolutions (net.py:104-111: conv1a / conv1b 3x3 128->128,
 * conv2 2x2 128->256, conv2a / conv2b 2x2 256->256; and 2x2 256->128, conv2's data gradient over the
 * flipped weight in the training backward; stride 1, zero padding `pad`) as an MFMA
 * implicit GEMM (csrc/mapf_conv.hip).  x: fp16 NHWC [nimg][H][W][Cin]; w_packed: fp16
 * [Cout][ks][ks][Cin] (torch's weight permuted); y: fp16 NHWC [nimg][Ho][Wo][Cout], Ho = H + 2 pad -
 * ks + 1.  fp32 accumulation, output rounded to fp16; relu = 1: then + bias (fp16, rounded again)
 * and ReLU -- the autocast conv followed by mapf_nhwc_bias_relu.  MAPF_EINVAL for other shapes. */
int mapf_conv_nhwc_f16(const uint16_t *x, const uint16_t *w_packed, const uint16_t *bias, uint16_t *y, int64_t nimg,
                       int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t ks, int32_t pad, int32_t relu,
                       void *stream);

/* mapf_conv_nhwc_f16 + bias + ReLU + 2x2 max-pool (net.py:106-107 / 110-111: relu(conv) then
 * MaxPool2d(2), floor), y fp16 NHWC [nimg][Ho / 2][Wo / 2][Cout]: the conv's output never goes to
 * HBM (tiles of whole images; 128 -> 128 3x3 and 256 -> 256 2x2 with Ho * Wo <= the tile).
 * Same values as mapf_conv_nhwc_f16(relu = 0) then mapf_nhwc_bias_relu_pool2. */
int mapf_conv_nhwc_pool_f16(const uint16_t *x, const uint16_t *w_packed, const uint16_t *bias, uint16_t *y, int64_t nimg,
                            int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t ks, int32_t pad, void *stream);

/* Which implicit-GEMM form mapf_conv_nhwc_f16 / mapf_conv_nhwc_pool_f16 launch (process-wide; values
 * to fp16 rounding of a different summation order, for A/B timing): 2 the image-resident form
 * wherever its geometry applies (whole images per workgroup, each input channel slice DMA'd into
 * LDS once and read by every tap), 0 the per-tap staged form, 1 (default) the faster of the two
 * as measured per layer (image-resident for the 3x3 and the pooled layers).  MAPF_EINVAL on
 * another value. */
int mapf_conv_select(int32_t impl);

/* conv1 (net.py:104, 3x3, padding 1, Cin = num_channel <= 7, Cout = 128) from the fp32 NCHW observation
 * x_nchw [nimg][Cin][H][W] (cast to fp16 as autocast does); w fp16 [Cout][64]: torch's [Cout][Cin][3][3]
 * flattened per output channel (K = Cin * 9 in (c, ky, kx) order) and zero-padded to 64;
 * y fp16 NHWC [nimg][H][W][Cout] = relu(fp16(fp16(conv) + bias)) -- the MIOpen path's NHWC copy, cast,
 * conv and mapf_nhwc_bias_relu in one launch. */
int mapf_conv_first_f32(const float *x_nchw, const uint16_t *w, const uint16_t *bias, uint16_t *y, int64_t nimg,
                        int32_t Cin, int32_t H, int32_t W, int32_t Cout, void *stream);

/* mapf_ppo_loss with coef[6] in DEVICE memory (captured-graph updates: the Lagrangian term changes
 * every update without re-capturing). */
int mapf_ppo_loss_dcoef(const float *new_ps, const float *old_ps, const int64_t *action, const float *new_v,
                        const float *old_v, const float *returns, const float *new_cv, const float *old_cv,
                        const float *cost_returns, const float *advantage, const float *cost_advantage,
                        const float *policy_sig, int32_t sig_fp16, const float *train_valid, int64_t R, int32_t A,
                        const float *coef_dev, float *loss, float *terms, float *grad_ps, float *grad_v,
                        float *grad_cv, float *grad_sig, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* MAPF_H */
