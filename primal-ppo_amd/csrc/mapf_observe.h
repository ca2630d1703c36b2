// primal-ppo_amd/csrc/mapf_observe.h -- getAllObservations for one workgroup's
// envs, as device functions shared by observe_kernel (mapf_observe.hip) and the
// fused step+observe kernel (mapf_fused.hip).
//
// Reference: observe (mapf_gym.py:246-325), getAllObservations (:327-336),
// worldWithAgents (:192-198).  Per agent: C x F x F float32 channels
//   0 obstacle / off-map / self        3 visible agents' goals (clamped to FOV)
//   1 other agents                     4 human next position (+ danger disc if use_da)
//   2 own goal                         5 human.path[1:K+1] cells (use_hp)
//   6 (C = 7, this build's extension) BFS descent: bfsMap >= 0 and < own value
// and the vector [dx/d, dy/d, d, 0], d = (dx^2 + dy^2) ** .5 in float64.
//
// Every channel value is 0/1, so a workgroup first builds its agents'
// observations as ONE contiguous bit-stream in LDS (bit k of the stream =
// float k of the workgroup's slice of obs[B][N][C][F][F]) and then expands
// it with one float4 store per 4 bits: the kernel's HBM traffic is the
// C*F*F*4 bytes per agent it must write plus ~16 B of state per agent.
//
//  obs_init        zero stream / occupancy, stage the padded obstacle rows in LDS
//  obs_load_agents agents' cells and goals, human next cell and path (from HBM;
//                  the fused kernel's step writes them here instead)
//  obs_emit        1 agent occupancy bitmap of each env (worldWithAgents)
//                  2 (agent, FOV row) tasks: F-bit row segments of ch0/ch1 (+ DA, BFS)
//                  3 per agent: own goal, visible agents' goals, human, HP, vector
//                  4 stream -> float4 stores (coalesced, 1 KiB per wave instruction)
#pragma once
#include "mapf_common.h"

namespace mapf {

// LDS carve-up of an observing workgroup (E envs).  per_env: every env has its
// own word-aligned bit-stream (stride swe words) and its own copy of the map
// rows, so one wave can observe its env with no workgroup barrier.
struct ObsLds {
    int swe;                    // per-env stream stride in words (0: one stream for the workgroup)
    uint32_t *stream, *occ, *mapc, *spos, *sgoal, *shn, *shp;
    int32_t *shpn;
    uint8_t *idg;               // [E][H*W] agent index at each occupied cell (read only where occ is set)
    uint32_t *bfsw;             // BFS channel: [E*N][F][WD] dwords = 2*WD int16 cells of each FOV row's
    int32_t *bfsown;            //   bfsMap window, from column (tc & ~1); [E*N] bfsMap at the agent's cell
    const float4 *lut;          // optional [16] float4: nibble -> its 4 bits as 0.f / 1.f (obs_lut_init)
    int stream_words, rowsz;
    bool bfs_win;               // BFS channel read through the LDS windows (else straight from HBM per task)
};

__host__ __device__ inline int obs_stream_words(const DevEnv &e, int E) { return (E * e.N * e.C * e.F * e.F + 31) / 32 + 1; }

__host__ __device__ inline bool obs_bfs_windows(const DevEnv &e) { return e.C >= 7 && e.keep_bfs && (e.W & 1) == 0; }
__host__ __device__ inline int obs_bfs_wd(const DevEnv &e) { return (e.F + 2) >> 1; }   // dwords per window row

__host__ __device__ inline int obs_env_stream_words(const DevEnv &e) {
    return ((e.N * e.C * e.F * e.F + 31) / 32 + 1 + 3) & ~3;
}

__host__ __device__ inline size_t obs_lds_bytes(const DevEnv &e, int E, bool per_env = false) {
    const int rowsz = e.Hp * e.WW;
    const int nmap = (e.shared_map && !per_env) ? 1 : E;
    const size_t sw = per_env ? (size_t)E * obs_env_stream_words(e) : (size_t)((obs_stream_words(e, E) + 3) & ~3);
    const size_t words = sw + (size_t)E * rowsz + (size_t)nmap * rowsz +
                         2 * (size_t)E * e.N + E + (size_t)E * e.k_predict + E;
    const size_t bfs_words = obs_bfs_windows(e) ? (size_t)E * e.N * (e.F * obs_bfs_wd(e) + 1) : 0;
    return (words + bfs_words) * 4 + (((size_t)E * e.H * e.W + 3) & ~(size_t)3);
}

__device__ inline ObsLds obs_layout(const DevEnv &e, int E, char *smem, bool per_env = false) {
    ObsLds L;
    L.swe = per_env ? obs_env_stream_words(e) : 0;
    L.stream_words = per_env ? E * L.swe : obs_stream_words(e, E);
    L.rowsz = e.Hp * e.WW;
    const int nmap = (e.shared_map && !per_env) ? 1 : E;
    L.stream = reinterpret_cast<uint32_t *>(smem);
    L.occ = L.stream + ((L.stream_words + 3) & ~3);
    L.mapc = L.occ + E * L.rowsz;
    L.spos = L.mapc + nmap * L.rowsz;
    L.sgoal = L.spos + E * e.N;
    L.shn = L.sgoal + E * e.N;                  // [E] human next
    L.shp = L.shn + E;                          // [E][k_predict] human.path[1..K]
    L.shpn = reinterpret_cast<int32_t *>(L.shp + E * e.k_predict);   // [E] count
    L.bfsw = reinterpret_cast<uint32_t *>(L.shpn + E);
    L.bfsown = reinterpret_cast<int32_t *>(L.bfsw + (obs_bfs_windows(e) ? (size_t)E * e.N * e.F * obs_bfs_wd(e) : 0));
    L.idg = reinterpret_cast<uint8_t *>(L.bfsown + (obs_bfs_windows(e) ? E * e.N : 0));
    L.lut = nullptr;
    L.bfs_win = obs_bfs_windows(e);
    return L;
}

// the 16-entry nibble -> float4 table (256 B of LDS, 16-B aligned), filled by the
// first 16 threads; the caller synchronises before use
__device__ inline void obs_lut_init(float4 *lut) {
    const int t = (int)threadIdx.x;
    if (t < 16) lut[t] = make_float4((float)(t & 1), (float)((t >> 1) & 1), (float)((t >> 2) & 1), (float)(t >> 3));
}

namespace obsd {

__device__ inline uint32_t seg_at(const uint32_t *row, int WW, int off, int F) {
    const int w = off >> 5, s = off & 31;
    const uint64_t a = (uint64_t)row[w] | ((w + 1 < WW) ? ((uint64_t)row[w + 1] << 32) : 0ull);
    return (uint32_t)(a >> s) & ((1u << F) - 1u);
}

__device__ inline void or_bits(uint32_t *stream, int off, uint32_t seg, int F) {
    if (!seg) return;
    const int w = off >> 5, s = off & 31;
    atomicOr(&stream[w], seg << s);
    if (s + F > 32) {
        const uint32_t hi = seg >> (32 - s);
        if (hi) atomicOr(&stream[w + 1], hi);
    }
}

__device__ inline void set_bit(uint32_t *stream, int off) { atomicOr(&stream[off >> 5], 1u << (off & 31)); }

__device__ inline int isqrt_floor(int x) {
    int r = (int)sqrtf((float)x);
    while (r * r > x) --r;
    while ((r + 1) * (r + 1) <= x) ++r;
    return r;
}

}  // namespace obsd

// Zero the bit-stream and the occupancy maps.  Staging the obstacle rows is
// split so a caller can issue the loads early and store them later:
// obs_map_word() loads word k of the workgroup's maps, obs_init() stores the
// first blockDim.x words from `mreg` and loads+stores the rest itself.
__device__ inline uint32_t obs_map_word(const DevEnv &e, int b0, int nenv, int k) {
    const int rowsz = e.Hp * e.WW;
    const int nw = e.shared_map ? rowsz : nenv * rowsz;
    if (k >= nw) return 0u;
    return e.shared_map ? e.map_bits[k] : e.map_bits[(size_t)b0 * rowsz + k];
}

__device__ inline void obs_init(const DevEnv &e, const ObsLds &L, int E, int b0, int nenv, uint32_t mreg) {
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int k = tid; k < L.stream_words; k += nt) L.stream[k] = 0u;
    for (int k = tid; k < E * L.rowsz; k += nt) L.occ[k] = 0u;
    const int nw = e.shared_map ? L.rowsz : nenv * L.rowsz;
    if (tid < nw) L.mapc[tid] = mreg;
    for (int k = tid + nt; k < nw; k += nt) L.mapc[k] = obs_map_word(e, b0, nenv, k);
}

__device__ inline void obs_load_agents(const DevEnv &e, const ObsLds &L, int b0, int nenv, int tid, int nt) {
    const int N = e.N, K = nenv * N;
    for (int k = tid; k < K; k += nt) {
        L.spos[k] = e.pos[(size_t)b0 * N + k];
        L.sgoal[k] = e.goal[(size_t)b0 * N + k];
    }
    for (int k = tid; k < nenv; k += nt) {
        const int b = b0 + k;
        L.shn[k] = human_next(e, b);
        int cnt = 0;
        if (e.use_hp && e.C >= 6) {
            const int cur = e.hcur[b];
            const int len = e.hlen[b * 2 + cur];
            const uint32_t *path = human_path(e, b, cur);
            for (int q = 1; q <= e.k_predict && q < len; ++q) L.shp[k * e.k_predict + cnt++] = path[q];
        }
        L.shpn[k] = cnt;
    }
}
__device__ inline void obs_load_agents(const DevEnv &e, const ObsLds &L, int b0, int nenv) {
    obs_load_agents(e, L, b0, nenv, (int)threadIdx.x, (int)blockDim.x);
}

// The config-static zero band of an agent's [C][F][F] block: channel 5
// (human.path[1:K+1], mapf_gym.py:293-297) is written only when use_hp is on,
// so with use_hp off every one of its floats is 0 at every step.  Returns the
// band's float offsets [z0, z1) inside the block, or false if there is none.
__host__ __device__ inline bool obs_zero_band(const DevEnv &e, int &z0, int &z1) {
    if (e.use_hp || e.C < 6 || e.F * e.F > 124) return false;    // <= 31 whole float4s (32 lanes per agent)
    z0 = 5 * e.F * e.F;
    z1 = 6 * e.F * e.F;
    return true;
}

// The band's whole float4s of agents [k0, k1) of `obs` (16-B aligned), written
// as zeros by `nt` threads numbered `t`: float4 q of the buffer belongs to the
// band iff 4q >= k*CFF + z0 and 4q + 4 <= k*CFF + z1 for its agent k.  The fused
// launch runs this in workgroups of their own while the step's latency-bound
// chains run in the others; obs_emit(skip_band) then skips exactly these float4s.
__device__ inline void obs_zero_band_store(const DevEnv &e, float *__restrict__ obs, size_t k0, size_t k1, size_t t,
                                           size_t nt) {
    int z0, z1;
    if (!obs_zero_band(e, z0, z1)) return;
    const size_t CFF = (size_t)e.C * e.F * e.F;
    float4 *o4 = reinterpret_cast<float4 *>(obs);
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    for (size_t idx = k0 * 32 + t; idx < k1 * 32; idx += nt) {      // 32 lanes per agent (a band has <= 31 float4s)
        const size_t k = idx >> 5, j = idx & 31;
        const size_t qa = (k * CFF + z0 + 3) >> 2, qb = (k * CFF + z1) >> 2;
        if (qa + j < qb) o4[qa + j] = zero;
    }
}

// Phases 1-4.  Every thread of the workgroup calls it after a __syncthreads()
// that follows obs_init and the agents' staging.  skip_band: the zero band's
// whole float4s were written by obs_zero_band_store in this launch.
// BFSCH = false compiles the BFS channel (C = 7) out (the fused launch never
// has it: step_observe_fusable).  NT: the table-driven store loop (L.lut) uses
// nontemporal stores.
// The threads that observe a run of the workgroup's envs together: the whole
// workgroup (workgroup barriers) or one wave observing its own env (per_env
// layout; wave-level ordering only).
struct ObsGroup {
    int tid, nt;                 // thread index in the group, group size
    int le0, nenv;               // first env (index within the workgroup) and env count
    uint32_t *stream;            // bit 0 = float 0 of env le0's observation
    const uint32_t *mapc;        // map rows: the shared map, or per-env maps at (le - le0) * rowsz
    bool wave;
#ifdef MAPF_STAMPS
    int diag = 0;                // stamps-build experiments: 2 no float stores, 3 stores only (no bit-stream)
#endif
};

__device__ inline void obs_sync(const ObsGroup &g) {
    if (g.wave) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}

__device__ inline ObsGroup obs_workgroup(const ObsLds &L, int nenv) {
    return ObsGroup{(int)threadIdx.x, (int)blockDim.x, 0, nenv, L.stream, L.mapc, false};
}

// One wave observes env le of the workgroup (per_env layout): zero its stream
// and occupancy, copy the map rows it holds in registers (lane k = word k).
__device__ inline ObsGroup obs_wave_init(const DevEnv &e, const ObsLds &L, int le, uint32_t mreg) {
    const int lane = lane_id();
    uint32_t *st = L.stream + (size_t)le * L.swe;
    for (int k = lane; k < L.swe; k += 64) st[k] = 0u;
    for (int k = lane; k < L.rowsz; k += 64) L.occ[le * L.rowsz + k] = 0u;
    uint32_t *mp = L.mapc + le * L.rowsz;
    if (lane < L.rowsz) mp[lane] = mreg;
    ObsGroup g{lane, 64, le, 1, st, mp, true};
    obs_sync(g);
    return g;
}

template <bool BFSCH = true, bool NT = false>
__device__ inline void obs_emit(const DevEnv &e, const ObsLds &L, float *__restrict__ obs, float *__restrict__ vec,
                                const ObsGroup &G, int b0, bool skip_band = false) {
    using namespace obsd;
    const int N = e.N, F = e.F, C = e.C, FF = F * F, CFF = C * FF;
    const int K = G.nenv * N;                 // agents of the group; k below is group-relative
    const int kw = G.le0 * N;                 // first agent of the group within the workgroup
    const int rowsz = L.rowsz;
    const int tid = G.tid, nt = G.nt;
    uint32_t *stream = G.stream;
    b0 += G.le0;                              // first env of the group
    const int E = G.nenv;

    // ---- phase 1: worldWithAgents as a padded bitmap per env + agent index grid ----
    const int HW = e.H * e.W;
#ifdef MAPF_STAMPS
    const int KB = G.diag == 3 ? 0 : K;       // agents whose bits phases 1-3 build
#else
    const int KB = K;
#endif
    for (int k = tid; k < KB; k += nt) {
        const int le = G.le0 + k / N;
        const int r = prow(L.spos[kw + k]), c = pcol(L.spos[kw + k]);
        const int rr = r + e.P, cc = c + e.P;
        atomicOr(&L.occ[le * rowsz + rr * e.WW + (cc >> 5)], 1u << (cc & 31));
        L.idg[le * HW + r * e.W + c] = (uint8_t)(k % N);
    }
    const int half = F / 2;
    const size_t bcells = bfs_cells(e.H, e.W);
    if (BFSCH && L.bfs_win) {
        // the BFS channel's bfsMap windows: every load of the workgroup issued here
        // at once (one HBM latency, not one per FOV-row task), as aligned dwords
        const int WD = obs_bfs_wd(e);
        for (int idx = tid; idx < KB * F * WD; idx += nt) {
            const int task = idx / WD, w = idx - task * WD;
            const int k = task / F, y = task - k * F;
            const int rr = min(max(prow(L.spos[kw + k]) - half + y, 0), e.H - 1);
            const int col = min(max(((pcol(L.spos[kw + k]) - half) & ~1) + 2 * w, 0), e.W - 2);
            const int16_t *bm = e.bfs + ((size_t)b0 * N + k) * bcells;
            L.bfsw[kw * F * WD + idx] = *reinterpret_cast<const uint32_t *>(bm + bfs_at(e.W, rr, col));   // col even
        }
        for (int k = tid; k < KB; k += nt)
            L.bfsown[kw + k] = e.bfs[((size_t)b0 * N + k) * bcells + bfs_at(e.W, prow(L.spos[kw + k]), pcol(L.spos[kw + k]))];
    }
    obs_sync(G);

    // ---- phase 2: (agent, FOV row) ----
    const int R2 = e.R * e.R;
    for (int task = tid; task < KB * F; task += nt) {
        const int k = task / F, y = task - k * F;
        const int le = G.le0 + k / N;
        const int pr = prow(L.spos[kw + k]), pc = pcol(L.spos[kw + k]);
        const int tr = pr - half, tc = pc - half;
        const int rr = tr + y;                       // map row of this FOV row
        const int prow_idx = rr + e.P;               // padded row (always inside)
        const uint32_t *mrow = G.mapc + (e.shared_map ? 0 : (le - G.le0) * rowsz) + prow_idx * e.WW;
        const uint32_t *orow = L.occ + le * rowsz + prow_idx * e.WW;
        uint32_t seg0 = seg_at(mrow, e.WW, tc + e.P, F);
        uint32_t segA = seg_at(orow, e.WW, tc + e.P, F);
        const uint32_t self = (y == half) ? (1u << half) : 0u;
        const int base = k * CFF + y * F;
        or_bits(stream, base, seg0 | self, F);
        or_bits(stream, base + FF, segA & ~self, F);
        // visibleAgents (the agents of this FOV row) -> their goals clamped to the FOV (ch3, :302-308)
        for (uint32_t others = segA & ~self; others; others &= others - 1u) {
            const int cc = tc + __builtin_ctz(others);
            const int kj = le * N + L.idg[le * HW + rr * e.W + cc];
            const int xr = min(max(prow(L.sgoal[kj]), tr), tr + F - 1);
            const int xc = min(max(pcol(L.sgoal[kj]), tc), tc + F - 1);
            set_bit(stream, k * CFF + 3 * FF + (xr - tr) * F + (xc - tc));
        }
        if (e.use_da && rr >= 0 && rr < e.H) {      // ch4 danger area (mapf_gym.py:289-290)
            const uint32_t hn = L.shn[le];
            const int dy = prow(hn) - rr;
            if (dy * dy <= R2) {
                const int w = isqrt_floor(R2 - dy * dy);
                int c0 = max(max(pcol(hn) - w, 0), tc), c1 = min(min(pcol(hn) + w, e.W - 1), tc + F - 1);
                if (c0 <= c1) {
                    const uint32_t m = ((1u << (c1 - c0 + 1)) - 1u) << (c0 - tc);
                    or_bits(stream, base + 4 * FF, m, F);
                }
            }
        }
        if (BFSCH && L.bfs_win && rr >= 0 && rr < e.H) {   // ch6 BFS descent (extension), from LDS
            const int own = L.bfsown[kw + k];
            const uint32_t *win = L.bfsw + ((size_t)kw * F + task) * obs_bfs_wd(e);
            const int c0 = tc & ~1;
            uint32_t m = 0;
            for (int x = 0; x < F; ++x) {
                const int cc = tc + x, wi = cc - c0;
                const int v = (int16_t)(win[wi >> 1] >> ((wi & 1) * 16));
                if (cc >= 0 && cc < e.W && v >= 0 && v < own) m |= 1u << x;
            }
            if (own < 0) m = 0;
            or_bits(stream, base + 6 * FF, m, F);
        } else if (BFSCH && C >= 7 && e.keep_bfs && rr >= 0 && rr < e.H) {   // ch6 BFS descent (extension)
            // the row's window straight from the tiled map: aligned dwords from column tc & ~1
            // (a dword never straddles a tile; columns past the edge read the tile padding's -1
            // or are masked), all loads issued before any is used
            const size_t ai = (size_t)b0 * N + k;
            const int16_t *bm = e.bfs + ai * bcells;
            const int own = bm[bfs_at(e.W, pr, pc)];
            const int c0 = tc & ~1, cmax = bfs_tw(e.W) * 8 - 2;
            uint32_t wv[9];
#pragma unroll
            for (int w = 0; w < 9; ++w)
                if (2 * w < F + 1)
                    wv[w] = *reinterpret_cast<const uint32_t *>(bm + bfs_at(e.W, rr, min(max(c0 + 2 * w, 0), cmax)));
            uint32_t m = 0;
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int cc = tc + x, wi = cc - c0;
                if (x < F) {
                    const int v = (int16_t)(wv[wi >> 1] >> ((wi & 1) * 16));
                    if (cc >= 0 && cc < e.W && v >= 0 && v < own) m |= 1u << x;
                }
            }
            if (own < 0) m = 0;
            or_bits(stream, base + 6 * FF, m, F);
        }
    }

    // ---- phase 3: per agent: own goal (ch2), human next position (ch4), HP cells (ch5), vector ----
    for (int k = tid; k < KB; k += nt) {
        const int le = G.le0 + k / N;
        const int pr = prow(L.spos[kw + k]), pc = pcol(L.spos[kw + k]);
        const int tr = pr - half, tc = pc - half;
        const int base = k * CFF;
        const int gr = prow(L.sgoal[kw + k]), gc = pcol(L.sgoal[kw + k]);
        if (tr <= gr && gr < tr + F && tc <= gc && gc < tc + F) set_bit(stream, base + 2 * FF + (gr - tr) * F + (gc - tc));
        const uint32_t hn = L.shn[le];
        const int hr = prow(hn), hc = pcol(hn);
        if (tr <= hr && hr < tr + F && tc <= hc && hc < tc + F) set_bit(stream, base + 4 * FF + (hr - tr) * F + (hc - tc));
        for (int q = 0; q < L.shpn[le]; ++q) {         // ch5 (:293-297): in-map cells inside the FOV
            const uint32_t cell = L.shp[le * e.k_predict + q];
            const int r = prow(cell), c = pcol(cell);
            if (tr <= r && r < tr + F && tc <= c && c < tc + F) set_bit(stream, base + 5 * FF + (r - tr) * F + (c - tc));
        }
        // vector (:316-323): d = (dx^2 + dy^2) ** .5 in float64 -- the correctly
        // rounded sqrt equals Python's pow(x, .5) for every x >= 0 (no table load)
        const int dx = gr - pr, dy = gc - pc;
        const int d2 = dx * dx + dy * dy;
        float4 v;
        if (d2 == 0) {
            v = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            const double d = __builtin_sqrt((double)d2);
            v = make_float4((float)((double)dx / d), (float)((double)dy / d), (float)d, 0.f);
        }
        reinterpret_cast<float4 *>(vec)[(size_t)b0 * N + k] = v;
    }
    obs_sync(G);
    TL_STAMP(4);
#ifdef MAPF_STAMPS
    if (G.diag == 2) return;
#endif

    // ---- phase 4: bit-stream -> float stores ----
    const size_t total = (size_t)K * CFF;
    float *dst = obs + (size_t)b0 * N * CFF;
    if (G.wave && L.lut && !skip_band && ((K * CFF) & 3) == 0) {
        // one wave, one env, whole float4s: lane l stores float4 q = l + 64k, whose 4 bits
        // are bits 4(l & 7).. of stream word (l >> 3) + 8k -- a lane-constant field (one
        // v_bfe), an 8-lane LDS broadcast -- and the float4 of that nibble comes from the
        // 16-entry LDS table L.lut: one 1 KiB store per wave instruction, constant step.
        const int sh = (tid & 7) * 4;
        const uint32_t *swp = stream + (tid >> 3);
        float4 *dp = reinterpret_cast<float4 *>(dst) + tid;
#pragma unroll 4
        for (int rem = ((K * CFF) >> 2) - tid; rem > 0; rem -= 64) {
            const float4 f = L.lut[__builtin_amdgcn_ubfe(*swp, sh, 4)];
            if constexpr (NT) {   // streaming stores (rollout slot buffers: not re-read by this launch)
                typedef float v4f __attribute__((ext_vector_type(4)));
#if defined(MAPF_SLOT_STORE) && MAPF_SLOT_STORE == 1     // store-policy experiment: nt only (round 2's)
                __builtin_nontemporal_store(v4f{f.x, f.y, f.z, f.w}, reinterpret_cast<v4f *>(dp));
#elif defined(MAPF_SLOT_STORE) && MAPF_SLOT_STORE == 2   // store-policy experiment: sc1 only
                asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dp), "v"(v4f{f.x, f.y, f.z, f.w}) : "memory");
#elif defined(MAPF_SLOT_STORE) && MAPF_SLOT_STORE == 3   // store-policy experiment: plain
                *dp = f;
#else
                // nt sc1: streamed AND not kept in the XCD's L2 (MI355X_MICROARCH: sc1 stores
                // drop the line), so the lines the step outputs merge in stay resident.  A/B on
                // one box: c2 slots 21.3 -> 20.3 us per step, c5 (446 MB in place) 89.1 -> 86.8
                // vs nt alone; plain 23.7, sc1 alone 21.0 (tools/ab_libs.sh, MAPF_SLOT_STORE)
                asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(dp), "v"(v4f{f.x, f.y, f.z, f.w}) : "memory");
#endif
            } else {
#if defined(MAPF_INPLACE_STORE) && MAPF_INPLACE_STORE == 1      // store-policy experiment: sc1
                typedef float v4f __attribute__((ext_vector_type(4)));
                asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dp), "v"(v4f{f.x, f.y, f.z, f.w}) : "memory");
#elif defined(MAPF_INPLACE_STORE) && MAPF_INPLACE_STORE == 2    // store-policy experiment: nt sc1
                typedef float v4f __attribute__((ext_vector_type(4)));
                asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(dp), "v"(v4f{f.x, f.y, f.z, f.w}) : "memory");
#elif defined(MAPF_INPLACE_STORE) && MAPF_INPLACE_STORE == 3    // store-policy experiment: sc0 sc1
                typedef float v4f __attribute__((ext_vector_type(4)));
                asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(dp), "v"(v4f{f.x, f.y, f.z, f.w}) : "memory");
#else
                *dp = f;
#endif
            }
            swp += 8;
            dp += 64;
        }
    } else if (!G.wave && L.lut && !skip_band && ((E * N * CFF) & 3) == 0 && (nt & 7) == 0) {
        // the same table-driven expansion for a workgroup's stream: thread t's float4s
        // q = t + nt*k keep the bit field 4(t & 7) of words (t >> 3) + (nt / 8) k
        int tid = G.tid;
        asm volatile("" : "+v"(tid));      // opaque here: its pointers are not hoisted into the
                                           // persistent kernels' loop prologue (VGPR spills there)
        const int sh = (tid & 7) * 4;
        const uint32_t *swp = stream + (tid >> 3);
        float4 *dp = reinterpret_cast<float4 *>(dst) + tid;
        for (int rem = (int)(total >> 2) - tid; rem > 0; rem -= nt) {
            *dp = L.lut[__builtin_amdgcn_ubfe(*swp, sh, 4)];
            swp += nt >> 3;
            dp += nt;
        }
        for (size_t q = ((total >> 2) << 2) + tid; q < total; q += nt)
            dst[q] = (float)((stream[q >> 5] >> (q & 31)) & 1u);
    } else if (((E * N * CFF) & 3) == 0) {
        int tid = G.tid;
        asm volatile("" : "+v"(tid));      // (as above)
        const size_t n4 = total >> 2;
        float4 *d4 = reinterpret_cast<float4 *>(dst);
        int z0 = 0, z1 = 0;
        if (!(skip_band && obs_zero_band(e, z0, z1))) z0 = z1 = 0;
        int off = (tid * 4) % CFF;                  // float offset of float4 q inside its agent's block
        const int step = (nt * 4) % CFF;
        for (size_t q = tid; q < n4; q += nt) {
            if (!(off >= z0 && off + 4 <= z1)) {
                const uint32_t bitpos = (uint32_t)(q << 2);
                const uint32_t nib = (stream[bitpos >> 5] >> (bitpos & 31)) & 15u;
                const float4 f = make_float4((float)(nib & 1u), (float)((nib >> 1) & 1u), (float)((nib >> 2) & 1u),
                                             (float)((nib >> 3) & 1u));
                d4[q] = f;
            }
            off += step;
            if (off >= CFF) off -= CFF;
        }
        for (size_t q = (n4 << 2) + tid; q < total; q += nt)
            dst[q] = (float)((stream[q >> 5] >> (q & 31)) & 1u);
    } else {
        int tid = G.tid;
        asm volatile("" : "+v"(tid));      // (as above)
        for (size_t q = tid; q < total; q += nt) dst[q] = (float)((stream[q >> 5] >> (q & 31)) & 1u);
    }
}

}  // namespace mapf
