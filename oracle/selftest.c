/*
 * oracle/selftest.c -- TEST INFRASTRUCTURE ONLY: drives the CPU oracle
 * (mapf_oracle.c, compiled into the same executable) through every entry point
 * with AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle asan`;
 * tests/test_oracle_asan.py runs it).  Episodes on random 0.3-density maps
 * (deadlocks, empty viable sets, unreachable goals), warehouses with dense
 * agents, FOV 3..11, 5..7 channels, DA/HP, fixed and seeded resets; A*, BFS, GAE,
 * the eviction-order sets.  Exit status 0 = every invariant held and the
 * sanitizers stayed quiet.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mapf_oracle.c"

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); ++fails; } } while (0)

static oc_config cfg_of(int H, int W, int N, int F, int C, int da, int hp, int hmode, int gmode, int fix, uint64_t seed) {
    oc_config c;
    memset(&c, 0, sizeof c);
    c.num_envs = 1; c.num_agents = N; c.height = H; c.width = W; c.fov = F; c.num_channel = C;
    c.use_da = da; c.use_hp = hp; c.lifelong = 1; c.human_mode = hmode; c.goal_mode = gmode; c.fix_choice = fix;
    c.shared_map = 1; c.keep_bfs = 1; c.max_seq = 4; c.max_human_seq = 4; c.k_predict = 5; c.penalty_radius = 5;
    c.action_cost = -0.3f; c.collision_cost = -2.f; c.human_collision_cost = -2.f; c.repeat_cost = -0.35f;
    c.goal_reward = 1.5f; c.seed = seed;
    return c;
}

static void run_episode(const int8_t *map, oc_config c, uint32_t env_id, int steps) {
    const int N = c.num_agents, F = c.fov, C = c.num_channel;
    oc_env *e = oc_create(&c, env_id);
    oc_reset_random(e, map);
    float *obs = malloc(sizeof(float) * N * C * F * F), vec[64 * 4];
    int act[64], fixed[64], pos[128], goal[128], sh;
    int8_t st[64];
    float rw[64], cost[64], valid[64 * 5], goals[64], constr[64];
    for (int t = 0; t < steps; ++t) {
        oc_random_actions(e, act);
        oc_step(e, act, st, rw, &sh, cost, valid, fixed, goals, constr);
        oc_observe(e, obs, vec);
        oc_get_agents(e, pos, goal);
        for (int i = 0; i < N; ++i) {
            CHECK(fixed[i] >= 0 && fixed[i] < 5, "env %u t %d: fixed action %d", env_id, t, fixed[i]);
            CHECK(map[pos[2 * i] * c.width + pos[2 * i + 1]] == 0, "env %u t %d: agent %d on an obstacle", env_id, t, i);
            for (int j = 0; j < i; ++j)
                CHECK(pos[2 * i] != pos[2 * j] || pos[2 * i + 1] != pos[2 * j + 1], "env %u t %d: agents %d, %d share a cell",
                      env_id, t, i, j);
        }
    }
    free(obs);
    oc_destroy(e);
}

int main(void) {
    /* random 0.3-density maps, no component filtering: unreachable goals and boxed-in agents happen */
    for (uint32_t env = 0; env < 24; ++env) {
        const int H = 8 + (int)(env % 5) * 3, W = 9 + (int)(env % 4) * 4, N = 2 + (int)(env % 7);
        int8_t *m = malloc((size_t)H * W);
        oc_gen_map(1, 0, 0, 0.3f, env, 99, env, H, W, m);
        int free_cells = 0;
        for (int k = 0; k < H * W; ++k) free_cells += m[k] == 0;
        if (free_cells > 2 * N + 4)
            run_episode(m, cfg_of(H, W, N, 3 + 2 * (int)(env % 5), 5 + (int)(env % 3), env & 1, (env >> 1) & 1, 1, 1,
                                  (int)(env & 1), 7 + env), env, 150);
        free(m);
    }
    /* warehouses, dense agents (the per-agent lane path's sizes) */
    for (uint32_t env = 0; env < 4; ++env) {
        int8_t m[40 * 60];
        oc_gen_map(0, 10, 14, 0.f, env, 5, env, 14, 21, m);
        run_episode(m, cfg_of(14, 21, 16, 9, 6, 1, 1, 1, 1, 1, 3), env, 120);
    }
    /* FixedMapfGym reset with LoopingHuman and sequences */
    {
        int8_t m[10 * 15];
        oc_gen_map(0, 10, 10, 0.f, 0, 1, 0, 10, 15, m);
        oc_config c = cfg_of(10, 15, 3, 9, 6, 0, 0, 0, 0, 0, 1);
        oc_env *e = oc_create(&c, 0);
        int seq[3 * 4 * 2] = {0, 0, 9, 14, 5, 0, 9, 0,  0, 2, 9, 12, 0, 5, 0, 7,  9, 5, 0, 14, 4, 0, 2, 0};
        int len[3] = {4, 4, 4};
        oc_reset_fixed(e, m, seq, len, 0, 14, 9, 1, NULL, 0);
        int act[3] = {1, 2, 3}, fixed[3], sh;
        int8_t st[3];
        float rw[3], cost[3], valid[15], goals[3], constr[3], obs[3 * 6 * 81], vec[12];
        for (int t = 0; t < 60; ++t) {
            act[0] = t % 5; act[1] = (t * 3) % 5; act[2] = (t * 7 + 1) % 5;
            oc_step(e, act, st, rw, &sh, cost, valid, fixed, goals, constr);
            oc_observe(e, obs, vec);
        }
        int rc[2 * 300];
        CHECK(oc_get_human_path(e, rc, 300) > 0, "human path empty");
        oc_destroy(e);
    }
    /* searches on a random map */
    {
        int8_t m[30 * 30];
        oc_gen_map(1, 0, 0, 0.25f, 3, 7, 3, 30, 30, m);
        int16_t d[30 * 30];
        int path[2 * 1000];
        for (int k = 0; k < 50; ++k) {
            const int sr = (k * 7) % 30, sc = (k * 11) % 30, gr = (k * 13 + 5) % 30, gc = (k * 17 + 3) % 30;
            if (m[sr * 30 + sc] || m[gr * 30 + gc]) continue;
            oc_bfs_map(m, 30, 30, gr, gc, d);
            const int n = oc_astar(m, 30, 30, sr, sc, gr, gc, path, 1000);
            CHECK(n < 0 ? d[sr * 30 + sc] == -2 : (sr == gr && sc == gc ? n == 0 : n == d[sr * 30 + sc] + 1),
                  "astar length %d vs bfs %d", n, d[sr * 30 + sc]);
        }
    }
    /* GAE */
    {
        enum { T = 64, M = 33 };
        float r[T * M], v[T * M], vl[M], adv[T * M], ret[T * M];
        for (int k = 0; k < T * M; ++k) { r[k] = (float)((k * 37) % 11) - 5.f; v[k] = (float)((k * 13) % 7) * 0.25f; }
        for (int k = 0; k < M; ++k) vl[k] = 0.5f;
        oc_gae(r, v, vl, adv, ret, T, M, 0.95, 0.95);
        for (int k = 0; k < T * M; ++k) CHECK(ret[k] == ret[k], "gae NaN");
    }
    /* eviction-order sets */
    {
        int pairs[64], rj[5], rb[5], out[8];
        uint32_t x = 12345;
        for (int it = 0; it < 20000; ++it) {
            const int N = 2 + (int)((x = x * 1664525u + 1013904223u) >> 27);
            for (int j = 0; j < N; ++j) pairs[j] = ((x = x * 1664525u + 1013904223u) >> 29) < 5 ? (int)(x >> 29) : -1;
            pairs[it % N] = -1;
            const int nr = 1 + (int)((x = x * 1664525u + 1013904223u) >> 30);
            for (int k = 0; k < nr; ++k) { rj[k] = (int)((x = x * 1664525u + 1013904223u) % (uint32_t)N); rb[k] = (int)(x >> 29) % 5; }
            const int n = oc_evict_order(pairs, N, rj, rb, nr, out);
            CHECK(n >= 0 && n <= nr, "evict count %d", n);
        }
    }
    if (fails) fprintf(stderr, "selftest: %d failures\n", fails);
    else printf("selftest: OK\n");
    return fails ? 1 : 0;
}
