/*
 * oracle/mapf_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A literal single-environment CPU restatement of the reference's hot path
 * (Nielsencu/primal-ppo @ /root/reference). Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product path
 * (primal-ppo_amd/csrc, libmapf.so) never links or calls this file.
 *
 * It deliberately follows the reference's *structure* (per-agent invalid-action
 * lists, the restrictedAction dict built pair by pair with its pruning test,
 * the sequential getActionStatus scan, the fixActions worklist, the heap A*,
 * the queue BFS) so that the device kernels, which use a different
 * formulation (bitmasks, wave ballots, BFS + walk-back for A*), are checked
 * against an independent statement of the same semantics.
 *
 * Parity pins: the .npz fixtures under tests/golden/, generated from the reference itself by
 * tests/golden/make_golden.py (see DESIGN.md "Oracle").
 *
 * RNG: the reference draws from numpy's MT19937 / Python random.  Those
 * streams cannot be reproduced on the GPU, so "random" mode draws from a
 * specified Philox4x32-10 stream (same distributions as the reference:
 * getFreeCell = uniform over cells whose world value is 0, by rejection).
 * The device implements the identical stream, so random mode is also
 * checked bit-exactly (device vs this file); fixed mode (FixedMapfGym) is
 * additionally pinned against the reference's own outputs.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -shared -fPIC).
 */
#include <stdint.h>
#ifdef OC_DIAG
#include <stdio.h>
#endif
#include <stdlib.h>
#include <string.h>
#include <math.h>

#define OC_NA 5
#define OC_FREECELL_TRIES 64

/* must match include/mapf.h: mapf_config (field for field) */
typedef struct oc_config {
    int32_t num_envs, num_agents, height, width, fov, num_channel;
    int32_t use_da, use_hp, lifelong, human_mode, goal_mode, fix_choice;
    int32_t shared_map, keep_bfs, max_seq, max_human_seq, k_predict, penalty_radius;
    float action_cost, collision_cost, human_collision_cost, repeat_cost, goal_reward;
    int32_t env_offset;
    uint32_t reserved;
    uint64_t seed;
} oc_config;

typedef struct { int r, c; } oc_cell;

/* Agent.dirDict / oppositeAction: mapf_gym.py:97-100 (x = row, y = col) */
static const int DR[OC_NA] = {0, 0, 1, 0, -1};
static const int DC[OC_NA] = {0, 1, 0, -1, 0};
static const int OPP[OC_NA] = {0, 3, 4, 1, 2};

enum { P_ENTRANCE = 1, P_HGOAL0 = 2, P_START = 3, P_GOAL0 = 4, P_GOAL = 5,
       P_HGOAL = 6, P_FIX = 7, P_ACT = 8 };

typedef struct {
    oc_cell pos, goal;
    unsigned inv_static, inv_human, inv_repeat; /* invalidActions[0..2] (mapf_gym.py:107-110) */
    int n_restr[OC_NA];                         /* restrictedAction (mapf_gym.py:112-113) */
    int *restr_j[OC_NA], *restr_b[OC_NA];
    unsigned good;                              /* unconditionallyGoodActions */
    int seq_cur;                                /* util.Sequence.curIdx (util.py:14-39) */
} oc_agent;

typedef struct oc_env {
    oc_config cfg;
    int H, W, N, F, C;
    int8_t *map;          /* obstacleMap: 0 free, -1 obstacle */
    oc_agent *ag;
    oc_cell *seq; int *seq_len;     /* agentsSequence: N x max_seq */
    /* human (mapf_gym.py:9-94) */
    oc_cell hpos, hgoal, hentr;
    oc_cell *hpath; int hlen, hstep, hcap;
    oc_cell *hseq; int hseq_len, hseq_idx;
    int16_t *bfs;          /* agent.bfsMap per agent, H*W */
    uint32_t env_id, clock, hreplans, errors;
    uint32_t fix_empty, fix_deadlock;   /* states the reference raises on / never leaves (fix_actions) */
    /* scratch */
    int *world; int *tmp;
} oc_env;

/* ------------------------------------------------------------------ */
/* Philox4x32-10 (shared spec with primal-ppo_amd/csrc/mapf_rng.h)      */
static inline uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
static void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed, uint32_t out[4]) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int i = 0; i < 10; ++i) {
        uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
uint32_t oc_philox_word(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed, int w) {
    uint32_t o[4]; philox(c0, c1, c2, c3, seed, o); return o[w & 3];
}

/* util.getFreeCell (util.py:67-76): uniform over cells with world==0 by
 * rejection.  Philox stream: draw k uses counter (env, purpose|agent<<8,
 * epoch, k); row = mulhi(w0,H), col = mulhi(w1,W).  After 64 rejected draws
 * the last draw's w2 picks uniformly among the admissible cells in
 * row-major order (same distribution, bounded time).  pred: 0 = world==0,
 * 1 = world==0 && (r==0 || c==0)   (Human.getEntrance, mapf_gym.py:19-23).
 * Returns 0 on success, -1 if no admissible cell. */
static int free_cell(const oc_env *e, const int *world, int pred, uint32_t purpose,
                     int agent, uint32_t epoch, oc_cell *out) {
    uint32_t o[4] = {0, 0, 0, 0};
    uint32_t c1 = purpose | ((uint32_t)agent << 8);
    for (int k = 0; k < OC_FREECELL_TRIES; ++k) {
        philox(e->env_id, c1, epoch, (uint32_t)k, e->cfg.seed, o);
        int r = (int)mulhi32(o[0], (uint32_t)e->H), c = (int)mulhi32(o[1], (uint32_t)e->W);
        if (world[r * e->W + c] == 0 && (pred == 0 || r == 0 || c == 0)) { out->r = r; out->c = c; return 0; }
    }
    int cnt = 0;
    for (int r = 0; r < e->H; ++r)
        for (int c = 0; c < e->W; ++c)
            if (world[r * e->W + c] == 0 && (pred == 0 || r == 0 || c == 0)) ++cnt;
    if (cnt == 0) return -1;
    int pick = (int)mulhi32(o[2], (uint32_t)cnt);
    for (int r = 0; r < e->H; ++r)
        for (int c = 0; c < e->W; ++c)
            if (world[r * e->W + c] == 0 && (pred == 0 || r == 0 || c == 0)) {
                if (pick == 0) { out->r = r; out->c = c; return 0; }
                --pick;
            }
    return -1;
}

/* ------------------------------------------------------------------ */
/* astar_4 (astar_4.py:21-109), literal: binary heap ordered like the    */
/* Python tuples (f, g, (x, y), parent); parents dict overwritten when    */
/* new_g <= g_scores (the `<` test at :58/:71/:85/:99).                   */
typedef struct { int f, g, x, y; } hent;
static int hless(const hent *a, const hent *b) {
    if (a->f != b->f) return a->f < b->f;
    if (a->g != b->g) return a->g < b->g;
    if (a->x != b->x) return a->x < b->x;
    return a->y < b->y;   /* equal (f,g,cell) entries are interchangeable */
}
static void hpush(hent *h, int *n, hent v) {
    int i = (*n)++;
    h[i] = v;
    while (i > 0) { int p = (i - 1) / 2; if (!hless(&h[i], &h[p])) break; hent t = h[i]; h[i] = h[p]; h[p] = t; i = p; }
}
static hent hpop(hent *h, int *n) {
    hent top = h[0];
    h[0] = h[--(*n)];
    int i = 0;
    for (;;) {
        int l = 2 * i + 1, r = l + 1, m = i;
        if (l < *n && hless(&h[l], &h[m])) m = l;
        if (r < *n && hless(&h[r], &h[m])) m = r;
        if (m == i) break;
        hent t = h[i]; h[i] = h[m]; h[m] = t; i = m;
    }
    return top;
}

/* returns path length (goal ... start order, like construct_path_from_dict),
 * 0 when start == goal (reference returns []), -1 when no path exists
 * (reference *returns* a ValueError). world: passable iff != -1. */
int oc_astar(const int8_t *world, int H, int W, int sr, int sc, int gr, int gc, int *out_rc, int cap) {
    if (sr == gr && sc == gc) return 0;     /* norm < 0.1 (astar_4.py:30) */
    int cells = H * W;
    int *g_scores = (int *)malloc(sizeof(int) * cells);
    int *parent = (int *)malloc(sizeof(int) * cells);
    char *closed = (char *)calloc(cells, 1);
    hent *heap = (hent *)malloc(sizeof(hent) * (4 * cells + 8));
    int n = 0, found = 0;
    for (int i = 0; i < cells; ++i) { g_scores[i] = -1; parent[i] = -1; }
    hent s = {0, 0, sr, sc};
    hpush(heap, &n, s);
    const int size_h = H - 1, size_w = W - 1;
    while (n > 0) {
        hent cur = hpop(heap, &n);
        if (cur.x == gr && cur.y == gc) { found = 1; break; }
        int ci = cur.x * W + cur.y;
        if (closed[ci]) continue;
        closed[ci] = 1;
        int x = cur.x, y = cur.y;
        /* neighbour order: left, up, right, down (astar_4.py:54-107) */
        int nx[4] = {x, x - 1, x, x + 1}, ny[4] = {y - 1, y, y + 1, y};
        int ok[4] = {y > 0, x > 0, y < size_w, x < size_h};
        for (int k = 0; k < 4; ++k) {
            if (!ok[k]) continue;
            int ni = nx[k] * W + ny[k];
            if (world[ni] == -1 || closed[ni]) continue;
            int new_g = cur.g + 1;
            if (g_scores[ni] >= 0 && g_scores[ni] < new_g) {
                /* keep parent */
            } else {
                g_scores[ni] = new_g;
                parent[ni] = ci;
            }
            int h = abs(nx[k] - gr) + abs(ny[k] - gc);
            hent v = {h + g_scores[ni], g_scores[ni], nx[k], ny[k]};
            hpush(heap, &n, v);
        }
    }
    int len = -1;
    if (found) {
        int cur = gr * W + gc, start = sr * W + sc;
        len = 0;
        out_rc[2 * len] = gr; out_rc[2 * len + 1] = gc; ++len;
        while (cur != start) {
            cur = parent[cur];
            if (len < cap) { out_rc[2 * len] = cur / W; out_rc[2 * len + 1] = cur % W; }
            ++len;
        }
    }
    free(g_scores); free(parent); free(closed); free(heap);
    return len;
}

/* makeBfsMap (mapf_gym.py:211-244): copy of obstacleMap, free cells -> -2,
 * level-order BFS from the goal over cells equal to -2. */
void oc_bfs_map(const int8_t *map, int H, int W, int gr, int gc, int16_t *out) {
    int cells = H * W;
    for (int i = 0; i < cells; ++i) out[i] = map[i] == 0 ? -2 : map[i];
    int *q = (int *)malloc(sizeof(int) * (cells + 1));
    char *opened = (char *)calloc(cells, 1);
    int head = 0, tail = 0, value = -1;
    q[tail++] = gr * W + gc; opened[gr * W + gc] = 1;
    int end = 0;
    while (end < tail) {
        end = tail; ++value;
        while (head < end) {
            int node = q[head++];
            int r = node / W, c = node % W;
            out[node] = (int16_t)value;
            int nb[4][2] = {{r - 1, c}, {r + 1, c}, {r, c - 1}, {r, c + 1}};
            int ok[4] = {r > 0, r + 1 < H, c > 0, c + 1 < W};
            for (int k = 0; k < 4; ++k) {
                if (!ok[k]) continue;
                int ni = nb[k][0] * W + nb[k][1];
                if (out[ni] == -2 && !opened[ni]) { opened[ni] = 1; q[tail++] = ni; }
            }
        }
    }
    free(q); free(opened);
}

/* ------------------------------------------------------------------ */
static int in_map(const oc_env *e, int r, int c) { return r >= 0 && r < e->H && c >= 0 && c < e->W; }

/* Human.getAstarPath (mapf_gym.py:33-37) / FixedPathHuman (:83-85) */
static int human_astar(oc_env *e, oc_cell from, oc_cell to, int round_trip) {
    int cap = e->H * e->W + 4;
    int *rc = (int *)malloc(sizeof(int) * 2 * cap);
    int len = oc_astar(e->map, e->H, e->W, from.r, from.c, to.r, to.c, rc, cap);
    if (len <= 0) {           /* [] or ValueError: the reference crashes next; this build's */
        free(rc); e->errors++; /* human stays put three steps (csrc/mapf_search.h: search_one) */
        e->hpath[0] = from; e->hpath[1] = from; e->hpath[2] = from; e->hlen = 3; return -1;
    }
    int n = 0;
    for (int k = len - 1; k >= 0; --k) { e->hpath[n].r = rc[2 * k]; e->hpath[n].c = rc[2 * k + 1]; ++n; }
    if (round_trip)
        for (int k = 1; k < len; ++k) { e->hpath[n].r = rc[2 * k]; e->hpath[n].c = rc[2 * k + 1]; ++n; }
    e->hlen = n;
    free(rc);
    return 0;
}

/* Human.getNextPos (mapf_gym.py:46-50) */
static oc_cell human_next(const oc_env *e) {
    if (e->hstep >= e->hlen - 1) return e->hpath[e->hlen - 1];
    return e->hpath[e->hstep + 1];
}

/* Human.nextStep (mapf_gym.py:25-31) + getNextGoal variants (:42-44, :65-70, :87-94) */
static void human_next_step(oc_env *e) {
    if (e->hstep >= e->hlen - 1) {
        if (e->cfg.human_mode == 1) {                   /* Human: new random goal */
            int cells = e->H * e->W;
            for (int i = 0; i < cells; ++i) e->tmp[i] = e->map[i];
            e->tmp[e->hentr.r * e->W + e->hentr.c] = 1;     /* self.world[entrance] = 1 */
            if (free_cell(e, e->tmp, 0, P_HGOAL, 0, e->clock, &e->hgoal) != 0) e->errors++;
            human_astar(e, e->hpos, e->hgoal, 1);
            e->hreplans++;
        } else if (e->cfg.human_mode == 2) {            /* FixedPathHuman */
            e->hseq_idx++;
            if (e->hseq_idx >= e->hseq_len) {
                e->hgoal = e->hseq[e->hseq_len - 1];
            } else {
                e->hgoal = e->hseq[e->hseq_idx];
                human_astar(e, e->hpos, e->hgoal, 0);
            }
        }                                                /* LoopingHuman: reuse the path */
        e->hstep = 0;
    } else {
        e->hstep++;
    }
    e->hpos = e->hpath[e->hstep];
}

/* Sequence.getNext (util.py:33-39) */
static oc_cell seq_next(oc_env *e, int i) {
    oc_agent *a = &e->ag[i];
    int len = e->seq_len[i];
    oc_cell *s = e->seq + (size_t)i * e->cfg.max_seq;
    if (a->seq_cur >= len) return s[len - 1];
    return s[a->seq_cur++];
}

/* ------------------------------------------------------------------ */
/* getInvalidActions (mapf_gym.py:339-360) */
static void get_invalid_actions(oc_env *e) {
    oc_cell hn = human_next(e), hc = e->hpos;
    for (int i = 0; i < e->N; ++i) {
        oc_agent *a = &e->ag[i];
        unsigned st = 0, hu = 0;
        for (int k = 0; k < OC_NA; ++k) {
            int r = a->pos.r + DR[k], c = a->pos.c + DC[k];
            if (!in_map(e, r, c)) st |= 1u << k;
            else if (e->map[r * e->W + c] != 0) st |= 1u << k;
            else if (r == hn.r && c == hn.c) hu |= 1u << k;
            else if (a->pos.r == hn.r && a->pos.c == hn.c && r == hc.r && c == hc.c) hu |= 1u << k;
        }
        a->inv_static = st; a->inv_human = hu;
    }
}

static void restr_add(oc_env *e, int i, int act, int j, int b) {
    oc_agent *a = &e->ag[i];
    a->restr_j[act][a->n_restr[act]] = j;
    a->restr_b[act][a->n_restr[act]] = b;
    a->n_restr[act]++;
}

/* getRestrictedActions (mapf_gym.py:363-402), including its pruning test */
static void get_restricted_actions(oc_env *e) {
    for (int i = 0; i < e->N; ++i) for (int k = 0; k < OC_NA; ++k) e->ag[i].n_restr[k] = 0;
    for (int one = 0; one < e->N; ++one)
        for (int two = one + 1; two < e->N; ++two) {
            oc_agent *A = &e->ag[one], *B = &e->ag[two];
            int dr = A->pos.r - B->pos.r, dc = A->pos.c - B->pos.c;
            int cur = dr * dr + dc * dc;
            if (cur > 4) continue;
            for (int i = 0; i < OC_NA; ++i) {
                int er = A->pos.r + DR[i], ec = A->pos.c + DC[i];
                int d1 = (er - B->pos.r) * (er - B->pos.r) + (ec - B->pos.c) * (ec - B->pos.c);
                if (d1 <= cur) {
                    for (int j = 0; j < OC_NA; ++j) {
                        int fr = B->pos.r + DR[j], fc = B->pos.c + DC[j];
                        if (er == fr && ec == fc) { restr_add(e, one, i, two, j); restr_add(e, two, j, one, i); }
                    }
                    if (er == B->pos.r && ec == B->pos.c) {
                        restr_add(e, one, i, two, OPP[i]); restr_add(e, two, OPP[i], one, i);
                    }
                }
            }
        }
}

/* getUnconditionallyGoodActions (mapf_gym.py:404-430): setdiff1d(arange(5), bad) */
static void get_good_actions(oc_env *e) {
    get_invalid_actions(e);
    get_restricted_actions(e);
    for (int i = 0; i < e->N; ++i) {
        oc_agent *a = &e->ag[i];
        unsigned bad = a->inv_static | a->inv_human | a->inv_repeat;
        for (int k = 0; k < OC_NA; ++k) if (a->n_restr[k] > 0) bad |= 1u << k;
        a->good = (~bad) & 0x1Fu;
    }
}

/* getActionStatus (mapf_gym.py:434-480) */
static void action_status(const oc_env *e, const int *act, int *st) {
    for (int i = 0; i < e->N; ++i) st[i] = 0;
    for (int i = 0; i < e->N; ++i) {
        if (st[i] != 0) continue;
        const oc_agent *a = &e->ag[i];
        int x = act[i];
        if (a->inv_static >> x & 1) st[i] = -1;
        else if (a->inv_human >> x & 1) st[i] = -2;
        else if (a->good >> x & 1) st[i] = 1;
        else {
            for (int k = 0; k < a->n_restr[x]; ++k)
                if (act[a->restr_j[x][k]] == a->restr_b[x][k]) { st[i] = -3; st[a->restr_j[x][k]] = -3; }
            if (st[i] == 0 && (a->inv_repeat >> x & 1)) st[i] = -4;
            else if (st[i] == 0) st[i] = 1;
        }
    }
}

/* ------------------------------------------------------------------ */
/* Obstacle maps, restating primal-ppo_amd/csrc/mapf_maps.hip:
 * kind 0 = MapfGym()'s warehouse (mapf_gym.py:166 -> generateWarehouse, map_generator.py:127-138)
 * of length L = lo + mulhi(philox(env, 10, epoch, 0).x, hi - lo + 1) at the top-left of H x W,
 * the rest -1; kind 1 = random_generator's -(rand < p) (map_generator.py:23), cell q from word
 * q & 3 of philox(env, 10 | 1 << 8, epoch, q >> 2).  Returns L (kind 0) or 0. */
#define P_MAPGEN 10
int oc_gen_map(int kind, int lo, int hi, float density, uint32_t epoch, uint64_t seed, uint32_t env_id,
               int H, int W, int8_t *out) {
    if (kind == 0) {
        uint32_t o[4];
        philox(env_id, P_MAPGEN, epoch, 0, seed, o);
        int L = lo + (int)mulhi32(o[0], (uint32_t)(hi - lo + 1));
        int breadth = (int)((double)L / (2.0 / 3.0));                      /* int(length/lbRatio) */
        int shelves = (int)(((double)breadth * (1.0 - 1.0 / 3.0)) / 6.0);   /* noShelves */
        int free0 = (int)((double)(breadth - shelves * 6) / 2.0);           /* freeSpace */
        for (int r = 0; r < H; ++r)
            for (int c = 0; c < W; ++c) {
                int ob = r >= L || c >= breadth;
                if (!ob && (r & 1) && r <= L - 2 && c >= free0 && c < free0 + shelves * 6 && (c - free0) % 6 < 5) ob = 1;
                out[r * W + c] = ob ? -1 : 0;
            }
        return L;
    }
    for (int q = 0; q < H * W; ++q) {
        uint32_t o[4];
        philox(env_id, P_MAPGEN | (1u << 8), epoch, (uint32_t)(q >> 2), seed, o);
        out[q] = ((double)o[q & 3] * 0x1p-32 < (double)density) ? -1 : 0;
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* CPython 3.10 set iteration order (Objects/setobject.c set_add_entry,
 * set_table_resize, set_insert_clean, set_intersection; Objects/tupleobject.c
 * tuplehash).  fixActions' eviction branch (mapf_gym.py:590-596) appends the
 * evicted agents in the iteration order of
 *     set(tuple(x) for x in agentActionPairs) & set(tuple(x) for x in np.array(restrictedAction[r]))
 * Elements are (int, int) tuples of small ints (numpy int64 hashes like int:
 * hash(-1) == -2), so the order is deterministic: no hash randomisation.
 * Sets here hold at most OC_PYSET_MAX elements (tables of 8 or 32 slots). */
#define OC_PYSET_MAX 8
typedef struct { int n; uint64_t mask, occ; int64_t key[OC_PYSET_MAX]; uint64_t hash[OC_PYSET_MAX]; int slot[OC_PYSET_MAX]; } oc_pyset;

static uint64_t py_hash_small(int64_t v) { return (uint64_t)(v == -1 ? -2 : v); }
uint64_t oc_py_hash_pair(int64_t a, int64_t b) {           /* tuplehash, 64-bit xxHash lanes */
    const uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL, P5 = 2870177450012600261ULL;
    uint64_t acc = P5, lane[2] = {py_hash_small(a), py_hash_small(b)};
    for (int k = 0; k < 2; ++k) { acc += lane[k] * P2; acc = (acc << 31) | (acc >> 33); acc *= P1; }
    acc += 2ULL ^ (P5 ^ 3527539ULL);
    return acc == ~0ULL ? 1546275796ULL : acc;
}
static int pyset_probe(uint64_t occ, uint64_t mask, uint64_t hash) {   /* first empty slot on the probe path */
    uint64_t perturb = hash, i = hash & mask;
    for (;;) {
        if (!(occ >> i & 1)) return (int)i;
        if (i + 9 <= mask)                                    /* LINEAR_PROBES */
            for (uint64_t j = 1; j <= 9; ++j) if (!(occ >> (i + j) & 1)) return (int)(i + j);
        perturb >>= 5;                                        /* PERTURB_SHIFT */
        i = (i * 5 + 1 + perturb) & mask;
    }
}
static void pyset_init(oc_pyset *s) { s->n = 0; s->mask = 7; s->occ = 0; }
static void pyset_add(oc_pyset *s, int64_t key, uint64_t hash) {
    for (int k = 0; k < s->n; ++k) if (s->key[k] == key) return;   /* already present: no change */
    int sl = pyset_probe(s->occ, s->mask, hash);
    s->key[s->n] = key; s->hash[s->n] = hash; s->slot[s->n] = sl; s->n++;
    s->occ |= 1ULL << sl;
    if ((uint64_t)s->n * 5 < s->mask * 3) return;            /* fill*5 < mask*3 (no dummies: fill == used) */
    uint64_t ns = 8;
    while (ns <= (uint64_t)s->n * 4) ns <<= 1;                /* set_table_resize(used*4) */
    int ord[OC_PYSET_MAX], m = s->n;
    for (int k = 0; k < m; ++k) ord[k] = k;
    for (int a = 1; a < m; ++a)                               /* re-insert in old slot order */
        for (int b = a; b > 0 && s->slot[ord[b]] < s->slot[ord[b - 1]]; --b) { int t = ord[b]; ord[b] = ord[b - 1]; ord[b - 1] = t; }
    s->mask = ns - 1; s->occ = 0;
    for (int k = 0; k < m; ++k) { int e2 = ord[k]; s->slot[e2] = pyset_probe(s->occ, s->mask, s->hash[e2]); s->occ |= 1ULL << s->slot[e2]; }
}
static int pyset_iter(const oc_pyset *s, int *ord) {        /* element indices in slot order */
    int m = 0;
    for (int sl = 0; sl <= (int)s->mask; ++sl)
        for (int k = 0; k < s->n; ++k) if (s->slot[k] == sl) ord[m++] = k;
    return m;
}
static int64_t pair_key(int j, int b) { return (int64_t)(j + 1) * 8 + (b + 1); }

/* The evicted agents, in the reference's order.  pairs[j] = agent j's
 * assigned action or -1 (agentActionPairs[j] == [-1, -1]); (rj, rb)[0..nr) =
 * restrictedAction[r] in list order.  Returns the count, agents in out_j. */
int oc_evict_order(const int *pairs, int N, const int *rj, const int *rb, int nr, int *out_j) {
    oc_pyset P, R, X;
    pyset_init(&P); pyset_init(&R); pyset_init(&X);
    int nP = 0, unassigned = 0;
    for (int j = 0; j < N; ++j) { if (pairs[j] >= 0) ++nP; else unassigned = 1; }
    nP += unassigned;                                         /* len(set(pairs)) */
    int rk[OC_PYSET_MAX * 4][2], nR = 0;
    for (int k = 0; k < nr; ++k) {                            /* len(set(restricted)) */
        int dup = 0;
        for (int m = 0; m < nR; ++m) if (rk[m][0] == rj[k] && rk[m][1] == rb[k]) dup = 1;
        if (!dup && nR < OC_PYSET_MAX * 4) { rk[nR][0] = rj[k]; rk[nR][1] = rb[k]; ++nR; }
    }
    int srcj[OC_PYSET_MAX], srcb[OC_PYSET_MAX], ns = 0, ord[OC_PYSET_MAX];
    if (nR > nP) {      /* set_intersection iterates the smaller operand: set(pairs) */
        for (int j = 0; j < N; ++j) {
            int a = pairs[j] >= 0 ? j : -1, b = pairs[j] >= 0 ? pairs[j] : -1;
            pyset_add(&P, pair_key(a, b), oc_py_hash_pair(a, b));
        }
        int m = pyset_iter(&P, ord);
        for (int k = 0; k < m; ++k) {
            int64_t key = P.key[ord[k]];
            int a = (int)(key / 8) - 1, b = (int)(key % 8) - 1;
            for (int q = 0; q < nR; ++q) if (rk[q][0] == a && rk[q][1] == b) { srcj[ns] = a; srcb[ns] = b; ++ns; break; }
        }
    } else {            /* ... set(restricted) */
        for (int q = 0; q < nR; ++q) pyset_add(&R, pair_key(rk[q][0], rk[q][1]), oc_py_hash_pair(rk[q][0], rk[q][1]));
        int m = pyset_iter(&R, ord);
        for (int k = 0; k < m; ++k) {
            int64_t key = R.key[ord[k]];
            int a = (int)(key / 8) - 1, b = (int)(key % 8) - 1;
            if (a >= 0 && pairs[a] == b) { srcj[ns] = a; srcb[ns] = b; ++ns; }
        }
    }
    for (int k = 0; k < ns; ++k) pyset_add(&X, pair_key(srcj[k], srcb[k]), oc_py_hash_pair(srcj[k], srcb[k]));
    int m = pyset_iter(&X, ord);
    for (int k = 0; k < m; ++k) out_j[k] = (int)(X.key[ord[k]] / 8) - 1;
    return m;
}

/* fixActions (mapf_gym.py:552-612).  random.choice(viable): fix_choice==0
 * takes viable[k % len] for the k-th draw of this call (the rule the golden
 * vectors were generated with, tests/golden/make_golden.py rotating_choice);
 * fix_choice==1 takes viable[mulhi(w0, len)] from Philox (P_FIX, agent,
 * clock, draw).  Evicted agents are appended in the reference's set order
 * (oc_evict_order).
 *
 * States the reference does not survive:
 *  - empty viable set: random.choice([]) raises IndexError (:588).  Here the
 *    agent stays (action 0) and evicts what conflicts with staying, as if 0
 *    had been drawn; counted (fix_empty).
 *  - deadlock: agents whose every viable action conflicts with each other's
 *    (e.g. one pushed by the human into a dead end held by another) evict each
 *    other forever -- the reference's while loop never ends.  After
 *    OC_FIX_DRAWS(N) draws in one call the remaining work-list agents stay and
 *    every mover whose target cell holds a staying agent is reverted to stay,
 *    until no mover is left blocked (a unique fixpoint: no two agents share a
 *    cell or swap); counted (fix_deadlock). */
#ifndef OC_FIX_DRAWS
#define OC_FIX_DRAWS(N) (16 * (N) + 64)
#endif
static void fix_actions(oc_env *e, const int *act, const int *st, int *pairs) {
    int N = e->N;
    int *queue = (int *)malloc(sizeof(int) * (N + 2 * (OC_FIX_DRAWS(N) + 1) + 8));
    int qh = 0, qt = 0;
    for (int i = 0; i < N; ++i) pairs[i] = -1;
    for (int i = 0; i < N; ++i) if (st[i] < 0) queue[qt++] = i;
    for (int i = 0; i < N; ++i) if (st[i] == 1) pairs[i] = act[i];
    int draws = 0;
    while (qh < qt) {
        int idx = queue[qh];
        oc_agent *a = &e->ag[idx];
        if (a->good) {
            pairs[idx] = __builtin_ctz(a->good); qh++;   /* problemAgents.remove(idx): idx is at the head */
            continue;
        }
        unsigned viable = (~(a->inv_static | a->inv_human)) & 0x1Fu;
        int done = 0;
        for (int t = 0; t < OC_NA && !done; ++t) {
            if (!(viable >> t & 1)) continue;
            int hit = 0;
            for (int k = 0; k < a->n_restr[t]; ++k) {
                int j = a->restr_j[t][k];
                if (pairs[j] >= 0 && pairs[j] == a->restr_b[t][k]) { hit = 1; break; }
            }
            if (!hit) { pairs[idx] = t; qh++; done = 1; }
        }
        if (done) continue;
        if (draws >= OC_FIX_DRAWS(N)) {
#ifdef OC_DIAG
            fprintf(stderr, "DEADLOCK env %u clock %u human %d,%d next %d,%d\n", e->env_id, e->clock, e->hpos.r, e->hpos.c, human_next(e).r, human_next(e).c);
#endif
            e->fix_deadlock++; e->errors++;
            break;
        }
        int nv = __builtin_popcount(viable), r = 0;
        if (nv == 0) {
#ifdef OC_DIAG
            fprintf(stderr, "EMPTYVIABLE env %u clock %u agent %d\n", e->env_id, e->clock, idx);
#endif
            e->fix_empty++; e->errors++;
        } else {
            int pick = draws % nv;
            if (e->cfg.fix_choice == 1) {
                uint32_t o[4];
                philox(e->env_id, P_FIX | ((uint32_t)idx << 8), e->clock, (uint32_t)draws, e->cfg.seed, o);
                pick = (int)mulhi32(o[0], (uint32_t)nv);
            }
            for (int t = 0; t < OC_NA; ++t) if (viable >> t & 1) { if (pick == 0) { r = t; break; } --pick; }
        }
        draws++;
        /* conflicts = set(pairs) & set(restrictedAction[r]) -> evict, in set order */
        int ev[OC_PYSET_MAX];
        int nev = oc_evict_order(pairs, N, a->restr_j[r], a->restr_b[r], a->n_restr[r], ev);
        for (int k = 0; k < nev; ++k) { pairs[ev[k]] = -1; queue[qt++] = ev[k]; }
        pairs[idx] = r; qh++;
    }
#ifdef OC_DIAG
    if (draws > 8) fprintf(stderr, "DRAWS %d N %d\n", draws, N);
#endif
    if (qh < qt) {      /* deadlock: stay, then revert blocked movers to a fixpoint */
        for (int q = qh; q < qt; ++q) pairs[queue[q]] = 0;
        for (int changed = 1; changed;) {
            changed = 0;
            for (int i = 0; i < N; ++i) {
                if (pairs[i] <= 0) continue;
                int tr = e->ag[i].pos.r + DR[pairs[i]], tc = e->ag[i].pos.c + DC[pairs[i]];
                for (int k = 0; k < N; ++k)
                    if (k != i && pairs[k] == 0 && e->ag[k].pos.r == tr && e->ag[k].pos.c == tc) { pairs[i] = 0; changed = 1; break; }
            }
        }
    }
    free(queue);
}

/* fp64 radial cost (mapf_gym.py:513-526): max(R - ||h - p||, 0) / R */
static double radial_cost(const oc_env *e, oc_cell h, int pr, int pc) {
    double dr = (double)(h.r - pr), dc = (double)(h.c - pc);
    double R = (double)e->cfg.penalty_radius;
    double v = R - sqrt(dr * dr + dc * dc);
    if (!(v > 0.0)) v = 0.0;
    return v / R;
}

/* ------------------------------------------------------------------ */
oc_env *oc_create(const oc_config *cfg, uint32_t env_id) {
    oc_env *e = (oc_env *)calloc(1, sizeof(oc_env));
    e->cfg = *cfg;
    e->H = cfg->height; e->W = cfg->width; e->N = cfg->num_agents; e->F = cfg->fov; e->C = cfg->num_channel;
    e->env_id = env_id;
    int cells = e->H * e->W;
    e->map = (int8_t *)calloc(cells, 1);
    e->ag = (oc_agent *)calloc(e->N, sizeof(oc_agent));
    for (int i = 0; i < e->N; ++i)
        for (int k = 0; k < OC_NA; ++k) {
            e->ag[i].restr_j[k] = (int *)malloc(sizeof(int) * (6 * e->N + 6));
            e->ag[i].restr_b[k] = (int *)malloc(sizeof(int) * (6 * e->N + 6));
        }
    int S = cfg->max_seq > 0 ? cfg->max_seq : 1;
    e->seq = (oc_cell *)calloc((size_t)e->N * S, sizeof(oc_cell));
    e->seq_len = (int *)calloc(e->N, sizeof(int));
    e->hcap = 2 * cells + 4;
    e->hpath = (oc_cell *)calloc(e->hcap, sizeof(oc_cell));
    int HS = cfg->max_human_seq > 0 ? cfg->max_human_seq : 1;
    e->hseq = (oc_cell *)calloc(HS, sizeof(oc_cell));
    e->bfs = (int16_t *)calloc((size_t)e->N * cells, sizeof(int16_t));
    e->world = (int *)calloc(cells, sizeof(int));
    e->tmp = (int *)calloc(cells, sizeof(int));
    return e;
}

void oc_destroy(oc_env *e) {
    if (!e) return;
    for (int i = 0; i < e->N; ++i) for (int k = 0; k < OC_NA; ++k) { free(e->ag[i].restr_j[k]); free(e->ag[i].restr_b[k]); }
    free(e->map); free(e->ag); free(e->seq); free(e->seq_len); free(e->hpath); free(e->hseq);
    free(e->bfs); free(e->world); free(e->tmp); free(e);
}

static void agent_set_pos(oc_agent *a, oc_cell p) {    /* Agent.setPos (mapf_gym.py:134-139) */
    a->pos = p; a->inv_static = a->inv_human = a->inv_repeat = 0;
    for (int k = 0; k < OC_NA; ++k) a->n_restr[k] = 0;
    a->good = 0;
}

static void make_bfs(oc_env *e, int i) {
    if (!e->cfg.keep_bfs) return;
    oc_bfs_map(e->map, e->H, e->W, e->ag[i].goal.r, e->ag[i].goal.c, e->bfs + (size_t)i * e->H * e->W);
}

/* FixedMapfGym.__init__ (mapf_gym.py:648-669) with LoopingHuman (:52-63) or
 * FixedPathHuman (:72-81).  seq: N x max_seq cells (r,c), seq_len[N]. */
int oc_reset_fixed(oc_env *e, const int8_t *map, const int *seq_rc, const int *seq_len,
                   int hsr, int hsc, int hgr, int hgc, const int *hseq_rc, int hseq_len) {
    int cells = e->H * e->W;
    memcpy(e->map, map, cells);
    e->clock = 0; e->errors = 0; e->hreplans = 0; e->fix_empty = e->fix_deadlock = 0;
    int S = e->cfg.max_seq;
    for (int i = 0; i < e->N; ++i) {
        e->seq_len[i] = seq_len[i];
        for (int k = 0; k < seq_len[i]; ++k) {
            e->seq[(size_t)i * S + k].r = seq_rc[2 * ((size_t)i * S + k)];
            e->seq[(size_t)i * S + k].c = seq_rc[2 * ((size_t)i * S + k) + 1];
        }
        e->ag[i].seq_cur = 0;
    }
    /* human */
    if (e->cfg.human_mode == 2) {
        e->hseq_len = hseq_len; e->hseq_idx = 1;
        for (int k = 0; k < hseq_len; ++k) { e->hseq[k].r = hseq_rc[2 * k]; e->hseq[k].c = hseq_rc[2 * k + 1]; }
        e->hpos = e->hseq[0]; e->hgoal = e->hseq[1]; e->hentr = e->hpos;
        human_astar(e, e->hpos, e->hgoal, 0);
    } else {
        e->hpos.r = hsr; e->hpos.c = hsc; e->hgoal.r = hgr; e->hgoal.c = hgc; e->hentr = e->hpos;
        human_astar(e, e->hpos, e->hgoal, 1);
    }
    e->hstep = 0;
    /* populateMap (mapf_gym.py:175-184) */
    for (int i = 0; i < e->N; ++i) {
        agent_set_pos(&e->ag[i], seq_next(e, i));
        e->ag[i].goal = seq_next(e, i);
        make_bfs(e, i);
    }
    get_good_actions(e);
    return (int)e->errors;
}

/* MapfGym.__init__ (mapf_gym.py:164-173) on a given map, Philox draws. */
int oc_reset_random(oc_env *e, const int8_t *map) {
    int cells = e->H * e->W;
    memcpy(e->map, map, cells);
    e->clock = 0; e->errors = 0; e->hreplans = 0; e->fix_empty = e->fix_deadlock = 0;
    for (int i = 0; i < cells; ++i) e->tmp[i] = map[i];
    /* Human.__init__ (mapf_gym.py:10-16) */
    if (free_cell(e, e->tmp, 1, P_ENTRANCE, 0, 0, &e->hentr) != 0) e->errors++;
    e->hpos = e->hentr;
    e->tmp[e->hentr.r * e->W + e->hentr.c] = 1;
    if (e->cfg.human_mode == 0 || e->cfg.human_mode == 1) {
        if (free_cell(e, e->tmp, 0, P_HGOAL0, 0, 0, &e->hgoal) != 0) e->errors++;
        human_astar(e, e->hpos, e->hgoal, 1);
    }
    e->hstep = 0;
    /* populateMap: tempMap = obstacleMap; tempMap[human] = 1; starts = 2; goals = 3 */
    for (int i = 0; i < e->N; ++i) {
        oc_cell s, g;
        if (free_cell(e, e->tmp, 0, P_START, i, 0, &s) != 0) e->errors++;
        agent_set_pos(&e->ag[i], s);
        e->tmp[s.r * e->W + s.c] = 2;
        if (free_cell(e, e->tmp, 0, P_GOAL0, i, 0, &g) != 0) e->errors++;
        e->ag[i].goal = g;
        make_bfs(e, i);
        e->tmp[g.r * e->W + g.c] = 3;
    }
    get_good_actions(e);
    return (int)e->errors;
}

/* One lockstep step exactly as runner.py:64-100 drives it:
 * getActionStatus -> calculateActionReward -> calculateCostReward ->
 * getTrainValid -> jointStep. */
int oc_step(oc_env *e, const int *act, int8_t *status, float *reward, int *shadow, float *cost,
            float *valid, int *fixed, float *goals, float *constr) {
    int N = e->N;
    int *st = (int *)malloc(sizeof(int) * N);
    action_status(e, act, st);
    /* calculateActionReward (mapf_gym.py:483-511) */
    int sh = 0;
    for (int i = 0; i < N; ++i) {
        float rw = 0.f;
        switch (st[i]) {
            case -1: rw = e->cfg.collision_cost; break;
            case -2: rw = e->cfg.human_collision_cost; break;
            case -3: rw = e->cfg.collision_cost; break;
            case -4: rw = e->cfg.repeat_cost; break;
            case 1: {
                int r = e->ag[i].pos.r + DR[act[i]], c = e->ag[i].pos.c + DC[act[i]];
                if (r == e->ag[i].goal.r && c == e->ag[i].goal.c) sh++;
                rw = e->cfg.action_cost;
            } break;
            default: e->errors++;
        }
        reward[i] = rw; status[i] = (int8_t)st[i];
    }
    *shadow = sh;
    /* calculateCostReward (:528-533): original actions, pre-step human next */
    oc_cell hn = human_next(e);
    for (int i = 0; i < N; ++i)
        cost[i] = (float)radial_cost(e, hn, e->ag[i].pos.r + DR[act[i]], e->ag[i].pos.c + DC[act[i]]);
    /* getTrainValid (:535-550) */
    for (int i = 0; i < N; ++i) {
        oc_agent *a = &e->ag[i];
        for (int k = 0; k < OC_NA; ++k) {
            float v = 0.f;
            if (a->good >> k & 1) v = 1.f;
            else if (a->n_restr[k] > 0) {
                v = 1.f;
                for (int m = 0; m < a->n_restr[k]; ++m)
                    if (act[a->restr_j[k][m]] == a->restr_b[k][m]) { v = 0.f; break; }
            }
            valid[i * OC_NA + k] = v;
        }
    }
    /* jointStep (:614-637) */
    int need_fix = 0;
    for (int i = 0; i < N; ++i) if (!(st[i] > 0 || st[i] <= -4)) need_fix = 1;
    if (need_fix) fix_actions(e, act, st, fixed);
    else for (int i = 0; i < N; ++i) fixed[i] = act[i];
    for (int i = 0; i < N; ++i) goals[i] = 0.f;
    for (int i = 0; i < N; ++i) {
        oc_agent *a = &e->ag[i];
        int x = fixed[i];
        oc_cell np = {a->pos.r + DR[x], a->pos.c + DC[x]};
        agent_set_pos(a, np);               /* Agent.takeStep (:158-161) */
        a->inv_repeat = 1u << OPP[x];
        if (e->cfg.lifelong && a->pos.r == a->goal.r && a->pos.c == a->goal.c) {
            goals[i] += 1.f;
            if (e->cfg.goal_mode == 0) {
                a->goal = seq_next(e, i);
            } else {
                /* worldWithAgentsAndGoals (:200-209) */
                int cells = e->H * e->W;
                for (int m = 0; m < cells; ++m) e->tmp[m] = e->map[m];
                for (int k = 0; k < N; ++k) {
                    oc_agent *b = &e->ag[k];
                    if (b->pos.r >= 0 && b->pos.c >= 0) e->tmp[b->pos.r * e->W + b->pos.c] = k + 1;
                    if (b->goal.r >= 0 && b->goal.c >= 0) e->tmp[b->goal.r * e->W + b->goal.c] = k + 1;
                }
                oc_cell g;
                if (free_cell(e, e->tmp, 0, P_GOAL, i, e->clock, &g) != 0) e->errors++;
                a->goal = g;
            }
            make_bfs(e, i);
        }
    }
    human_next_step(e);
    for (int i = 0; i < N; ++i)
        constr[i] = radial_cost(e, e->hpos, e->ag[i].pos.r, e->ag[i].pos.c) >= 0.01 ? 1.f : 0.f;
    get_good_actions(e);
    e->clock++;
    free(st);
    return (int)e->errors;
}

/* observe (mapf_gym.py:246-325) for every agent (getAllObservations :327-336).
 * obs: N x C x F x F float32, vec: N x 4 float32.
 * Channel 6 (C == 7) is this build's BFS-descent extension: 1 where the
 * agent's bfsMap value is >= 0 and smaller than the value at its position. */
void oc_observe(const oc_env *e, float *obs, float *vec) {
    int N = e->N, F = e->F, C = e->C, H = e->H, W = e->W;
    int half = F / 2;
    /* worldWithAgents (:192-198) */
    int *world = e->world;
    for (int m = 0; m < H * W; ++m) world[m] = e->map[m];
    for (int k = 0; k < N; ++k)
        if (e->ag[k].pos.r >= 0 && e->ag[k].pos.c >= 0) world[e->ag[k].pos.r * W + e->ag[k].pos.c] = k + 1;
    oc_cell hn = human_next(e);
    int *visible = (int *)malloc(sizeof(int) * (F * F + 1));
    for (int i = 0; i < N; ++i) {
        const oc_agent *a = &e->ag[i];
        float *o = obs + (size_t)i * C * F * F;
        memset(o, 0, sizeof(float) * C * F * F);
        int tr = a->pos.r - half, tc = a->pos.c - half, nvis = 0;
        for (int r = tr; r < tr + F; ++r)
            for (int c = tc; c < tc + F; ++c) {
                int cell = (r - tr) * F + (c - tc);
                if (!in_map(e, r, c)) { o[0 * F * F + cell] = 1.f; continue; }
                int wv = world[r * W + c];
                if (wv == -1) o[cell] = 1.f;
                else if (wv > 0 && wv == i + 1) o[cell] = 1.f;
                else if (wv > 0) { visible[nvis++] = wv; o[1 * F * F + cell] = 1.f; }
                if (e->cfg.use_da) {   /* USE_INFLATED_HUMAN is True (alg_parameters.py:77) */
                    int dr = hn.r - r, dc = hn.c - c;
                    if (sqrt((double)(dr * dr + dc * dc)) <= (double)e->cfg.penalty_radius)
                        o[4 * F * F + cell] = 1.f;
                }
                if (e->cfg.use_hp && C >= 6) {   /* human.path[1:K+1] (:293-297) */
                    for (int k = 1; k <= e->cfg.k_predict && k < e->hlen; ++k)
                        if (e->hpath[k].r == r && e->hpath[k].c == c) o[5 * F * F + cell] = 1.f;
                }
                if (C >= 7 && e->cfg.keep_bfs) {
                    const int16_t *b = e->bfs + (size_t)i * H * W;
                    int own = b[a->pos.r * W + a->pos.c];
                    int v = b[r * W + c];
                    if (v >= 0 && own >= 0 && v < own) o[6 * F * F + cell] = 1.f;
                }
            }
        if (tr <= a->goal.r && a->goal.r < tr + F && tc <= a->goal.c && a->goal.c < tc + F)
            o[2 * F * F + (a->goal.r - tr) * F + (a->goal.c - tc)] = 1.f;
        for (int v = 0; v < nvis; ++v) {
            const oc_agent *b = &e->ag[visible[v] - 1];
            int x = b->goal.r, y = b->goal.c;
            int mr = x < tr + F - 1 ? x : tr + F - 1; if (mr < tr) mr = tr;   /* max(tr, min(tr+F-1, x)) */
            int mc = y < tc + F - 1 ? y : tc + F - 1; if (mc < tc) mc = tc;
            o[3 * F * F + (mr - tr) * F + (mc - tc)] = 1.f;
        }
        if (tr <= hn.r && hn.r < tr + F && tc <= hn.c && hn.c < tc + F)
            o[4 * F * F + (hn.r - tr) * F + (hn.c - tc)] = 1.f;
        /* vector (:316-323): float64, (dx^2+dy^2) ** .5 via pow, then float32 */
        double v0 = (double)(a->goal.r - a->pos.r), v1 = (double)(a->goal.c - a->pos.c);
        double v2 = pow(v0 * v0 + v1 * v1, 0.5);
        if (v2 != 0.0) { v0 = v0 / v2; v1 = v1 / v2; }
        vec[i * 4 + 0] = (float)v0; vec[i * 4 + 1] = (float)v1; vec[i * 4 + 2] = (float)v2; vec[i * 4 + 3] = 0.f;
    }
    free(visible);
}

/* ------------------------------------------------------------------ */
/* State accessors for the tests. */
void oc_get_agents(const oc_env *e, int *pos_rc, int *goal_rc) {
    for (int i = 0; i < e->N; ++i) {
        pos_rc[2 * i] = e->ag[i].pos.r; pos_rc[2 * i + 1] = e->ag[i].pos.c;
        goal_rc[2 * i] = e->ag[i].goal.r; goal_rc[2 * i + 1] = e->ag[i].goal.c;
    }
}
void oc_get_masks(const oc_env *e, int *st, int *hu, int *rep, int *good) {
    for (int i = 0; i < e->N; ++i) {
        st[i] = (int)e->ag[i].inv_static; hu[i] = (int)e->ag[i].inv_human;
        rep[i] = (int)e->ag[i].inv_repeat; good[i] = (int)e->ag[i].good;
    }
}
/* human: out[0..1] pos, [2..3] next pos, [4..5] goal, [6] step, [7] path len, [8] replans */
void oc_get_human(const oc_env *e, int *out) {
    oc_cell hn = human_next(e);
    out[0] = e->hpos.r; out[1] = e->hpos.c; out[2] = hn.r; out[3] = hn.c;
    out[4] = e->hgoal.r; out[5] = e->hgoal.c; out[6] = e->hstep; out[7] = e->hlen; out[8] = (int)e->hreplans;
}
int oc_get_human_path(const oc_env *e, int *rc, int cap) {
    for (int k = 0; k < e->hlen && k < cap; ++k) { rc[2 * k] = e->hpath[k].r; rc[2 * k + 1] = e->hpath[k].c; }
    return e->hlen;
}
void oc_get_bfs(const oc_env *e, int16_t *out) { memcpy(out, e->bfs, sizeof(int16_t) * e->N * e->H * e->W); }
uint32_t oc_get_errors(const oc_env *e) { return e->errors; }
void oc_get_fix_counts(const oc_env *e, uint32_t *out2) { out2[0] = e->fix_empty; out2[1] = e->fix_deadlock; }
uint32_t oc_get_clock(const oc_env *e) { return e->clock; }

/* Test hook (g2 fuzz scenarios): put the human at path index hstep and set
 * each agent's repeat mask from a previous action (-1 = none, as at reset),
 * then recompute the masks (getUnconditionallyGoodActions). */
void oc_debug_set(oc_env *e, int hstep, const int *prev) {
    e->hstep = hstep;
    e->hpos = e->hpath[hstep];
    for (int i = 0; i < e->N; ++i) e->ag[i].inv_repeat = prev[i] >= 0 ? 1u << OPP[prev[i]] : 0u;
    get_good_actions(e);
}

/* Random policy used by the env-only benchmark: uniform action in {0..4}.
 * One Philox draw (P_ACT | (agent >> 3) << 8, clock, 0) per 8 agents; agent i
 * takes 16-bit half-word i & 7 of the draw, scaled by 5 >> 16 -- shared spec
 * with the device (mapf_common.h: random_action). */
void oc_random_actions(const oc_env *e, int *act) {
    uint32_t o[4];
    for (int i = 0; i < e->N; ++i) {
        if ((i & 7) == 0) philox(e->env_id, P_ACT | ((uint32_t)(i >> 3) << 8), e->clock, 0, e->cfg.seed, o);
        const int k = i & 7;
        act[i] = (int)((((o[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu) * (uint32_t)OC_NA) >> 16);
    }
}

/* ------------------------------------------------------------------ */
/* GAE (runner.py:117-149), numpy float32 semantics: python-float
 * constants rounded to f32, separate multiply and add (no FMA).
 * r, v, adv, ret: T x M row-major; v_last: M. */
void oc_gae(const float *r, const float *v, const float *v_last, float *adv, float *ret,
            int T, int M, double gamma, double lam) {
    const float g = (float)(gamma * 1.0);
    const float gl = (float)(gamma * lam * 1.0);
    for (int m = 0; m < M; ++m) {
        float last = 0.f;
        for (int t = T - 1; t >= 0; --t) {
            float nv = (t == T - 1) ? v_last[m] : v[(size_t)(t + 1) * M + m];
            volatile float gv = g * nv;
            volatile float s = r[(size_t)t * M + m] + gv;
            volatile float delta = s - v[(size_t)t * M + m];
            volatile float gla = gl * last;
            volatile float a = delta + gla;
            last = a;
            adv[(size_t)t * M + m] = a;
        }
    }
    for (size_t k = 0; k < (size_t)T * M; ++k) { volatile float s = adv[k] + v[k]; ret[k] = s; }
}

/* ------------------------------------------------------------------ */
/* OneEpPerformance.episodeReward / episodeCostReward (runner.py:95-96):
 * `perf.episodeReward += np.sum(rewards)` once per step, rewards a float32
 * [1, N] array.  np.sum = numpy's pairwise_sum over the N contiguous floats
 * (below 8: in order from 0; else 8 strided accumulators combined
 * ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the rest in order; N <= 128 is
 * one block) added to the reduction's identity 0.  The python accumulator
 * starts at int 0 and 0 + np.float32 is np.float32 (NEP 50): float32 over
 * the steps.  x: T x B x N; out: B. */
static float np_sum_f32(const float *a, int n) {
    volatile float res;
    if (n < 8) {
        res = 0.f;
        for (int i = 0; i < n; ++i) res = res + a[i];
    } else {
        volatile float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] = r[j] + a[i + j];
        volatile float s01 = r[0] + r[1], s23 = r[2] + r[3], s45 = r[4] + r[5], s67 = r[6] + r[7];
        volatile float lo = s01 + s23, hi = s45 + s67;
        res = lo + hi;
        for (; i < n; ++i) res = res + a[i];
    }
    volatile float z = 0.f + res;
    return z;
}
void oc_episode_sum(const float *x, int T, int B, int N, float *out) {
    for (int b = 0; b < B; ++b) {
        volatile float acc = 0.f;
        for (int t = 0; t < T; ++t) acc = acc + np_sum_f32(x + ((size_t)t * B + b) * N, N);
        out[b] = acc;
    }
}

/* Batched driver used as the CPU baseline: B independent envs, one lockstep
 * random-policy step + observe each (runner.py:64-100 order). Single thread. */
typedef struct { oc_env **envs; int B; } oc_batch;
oc_batch *oc_batch_create(const oc_config *cfg, const int8_t *map, int B) {
    oc_batch *b = (oc_batch *)calloc(1, sizeof(oc_batch));
    b->B = B; b->envs = (oc_env **)calloc(B, sizeof(oc_env *));
    for (int k = 0; k < B; ++k) {
        b->envs[k] = oc_create(cfg, (uint32_t)(cfg->env_offset + k));
        oc_reset_random(b->envs[k], map);
    }
    return b;
}
void oc_batch_destroy(oc_batch *b) { for (int k = 0; k < b->B; ++k) oc_destroy(b->envs[k]); free(b->envs); free(b); }
int oc_batch_run(oc_batch *b, int steps, float *obs, float *vec) {
    int errs = 0;
    for (int s = 0; s < steps; ++s)
        for (int k = 0; k < b->B; ++k) {
            oc_env *e = b->envs[k];
            int N = e->N;
            int act[64], fixed[64], sh; int8_t st[64];
            float rw[64], cost[64], valid[64 * 5], goals[64], constr[64];
            oc_random_actions(e, act);
            errs += oc_step(e, act, st, rw, &sh, cost, valid, fixed, goals, constr);
            oc_observe(e, obs, vec);
            (void)N;
        }
    return errs;
}
