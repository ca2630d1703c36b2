// primal-ppo_amd/csrc/mapf_kernels.h -- host-side launchers of the MAPF kernels.
#pragma once
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "mapf.h"
#include "mapf_common.h"

namespace mapf {

// Launch-configuration queries, cached per device (a process may drive several GPUs with
// different CU counts) and safe to call from several host threads.
inline int device_cu_count() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
    int v = dev < 64 ? cache[dev].load(std::memory_order_relaxed) : 0;
    if (v > 0) return v;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    if (dev < 64) cache[dev].store(v, std::memory_order_relaxed);
    return v;
}

// LDS bytes one workgroup may request (160 KiB on gfx950)
inline int device_max_group_lds() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 64 * 1024;
    int v = dev < 64 ? cache[dev].load(std::memory_order_relaxed) : 0;
    if (v > 0) return v;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || v <= 0) v = 64 * 1024;
    if (dev < 64) cache[dev].store(v, std::memory_order_relaxed);
    return v;
}

// VGPRs per lane of a kernel (one code object per arch: the same on every device here)
inline int kernel_vgprs(const void *fn) {
    static std::mutex m;
    static std::unordered_map<const void *, int> cache;
    std::lock_guard<std::mutex> lock(m);
    auto it = cache.find(fn);
    if (it != cache.end()) return it->second;
    hipFuncAttributes fa{};
    const int v = hipFuncGetAttributes(&fa, fn) == hipSuccess && fa.numRegs > 0 ? fa.numRegs : 512;
    cache.emplace(fn, v);
    return v;
}

struct StepOut {          // device pointers (mapf_step_out)
    int8_t *status;
    float *reward;
    int32_t *shadow_goals;
    float *cost;
    float *train_valid;
    int32_t *actions_fixed;
    float *goals_reached;
    float *constraints;
    float *reward_total;
};

// flags: bit0 commit (jointStep), bit1 random policy (draw actions in-kernel into `actions`)
void launch_step(const DevEnv &e, int32_t *actions, const StepOut &out, uint32_t flags, int parity, hipStream_t s);
bool launch_step_pairs(const DevEnv &e, int32_t *actions, const StepOut &out, uint32_t flags, int slot,
                       hipStream_t s);   // N <= 8: one lane per agent pair; false if N > 8
void launch_random_actions(const DevEnv &e, int32_t *actions, hipStream_t s);
// humans' next paths (replan_list[parity]) + agent BFS maps (bfs_list[parity]);
// all = 1: every env's next path and every agent's map, 2: every env's next path,
// 3 / 4: the step's human paths / BFS maps only
void launch_search(const DevEnv &e, int parity, int all, hipStream_t s);
// agent.bfsMap of every agent, untiled: dist[B*N][H][W] (mapf_bfs)
void launch_bfs_export(const DevEnv &e, int16_t *dist, hipStream_t s);
// plan every human's next path from the state (promote: buffer hcur^1 becomes current first)
void launch_plan(const DevEnv &e, int promote, hipStream_t s);
// observations; the first nsearch workgroups run the search work of `parity`
void launch_observe(const DevEnv &e, float *obs, float *vec, int nsearch, int parity, hipStream_t s);
bool observe_hosts_search(const DevEnv &e);
// after a concurrent search: rewrite the BFS channel of the agents in bfs_list[parity]
void launch_bfs_fixup(const DevEnv &e, int parity, float *obs, hipStream_t s);
// committed step + observations in one launch (mapf_fused.hip); the first nsearch
// workgroups run the search work of list slot sslot (the previous step's)
bool step_observe_fusable(const DevEnv &e);
void launch_step_observe(const DevEnv &e, int32_t *actions, const StepOut &out, uint32_t flags, int slot,
                         float *obs, float *vec, int nsearch, int sslot, hipStream_t s);
// T committed random-policy steps + observations in one launch (mapf_fused.hip): MAPF_OK;
// ROLLOUT_NOT_COVERED (nothing launched) if the configuration is not covered; MAPF_ESTATE
// (nothing launched) if a captured launch found no free argument slot (ArgRing)
// (the kernel's form from the handle's tuning, mapf.h: mapf_tuning); describe_* write the
// form launch_* would take as text (mapf_rollout_plan)
constexpr int ROLLOUT_NOT_COVERED = 1;
bool rollout_random_fusable(const DevEnv &e);
int launch_rollout_random(const DevEnv &e, int T, int32_t *actions, const StepOut &out, float *obs, float *vec,
                           int slots, const mapf_tuning &tu, struct ArgRing &ring, hipStream_t s);
void describe_rollout_random(const DevEnv &e, int slots, const mapf_tuning &tu, char *buf, size_t n);
// the same for up to 64 agents / per-env maps / the BFS channel: one wave per env
// (mapf_rollout_wide.hip); used where the pair-lane rollout does not apply.  Returns MAPF_OK or
// MAPF_ESTATE (a captured launch found no free argument slot, ArgRing).
bool rollout_wide_fusable(const DevEnv &e);
int launch_rollout_wide(const DevEnv &e, int T, int32_t *actions, const StepOut &out, float *obs, float *vec,
                        int slots, const mapf_tuning &tu, struct ArgRing &ring, hipStream_t s);
void describe_rollout_wide(const DevEnv &e, int slots, const mapf_tuning &tu, char *buf, size_t n);

// Device-resident kernel argument blocks.  A persistent kernel whose arguments (DevEnv + its
// output pointers, ~0.5 KiB) do not fit in the SGPR file kept them live from the kernarg
// load on and spilled ~450 SGPRs to VGPR lanes (v_readlane at every use, plus dead stack
// slots).  Read through a `const __restrict__` pointer instead, every field is an invariant
// scalar load the register allocator re-issues where it is used.  The block is written on
// the launch stream by a one-wave kernel that takes it by value (stream-ordered), into the
// next of ARG_SLOTS ring slots: launches on different streams in flight at once never share a
// slot unless more than ARG_SLOTS are.  A launch recorded into a hipGraph keeps its slot's
// address for every replay, so captured launches never take a ring slot (a later direct
// launch would overwrite it between replays): each gets one of ARG_CAPTURE_SLOTS slots of its
// own for the life of the handle, and a capture past them fails (MAPF_ESTATE).  The block's store
// (store_args_kernel) is captured with the kernel, so each replay re-writes its own slot first;
// after release_captures a slot may be shared by two graphs, whose replays must not overlap.
constexpr size_t ARG_SLOT_BYTES = 2048, ARG_SLOTS = 16, ARG_CAPTURE_SLOTS = 16;
struct ArgRing {
    char *base = nullptr;     // (ARG_SLOTS + ARG_CAPTURE_SLOTS) * ARG_SLOT_BYTES of device memory (the handle's)
    unsigned next = 0;        // ring position
    unsigned captured = 0;    // capture slots handed out
    void release_captures() { captured = 0; }
    template <class A>
    A *slot(bool capturing) {
        static_assert(sizeof(A) <= ARG_SLOT_BYTES, "argument block larger than a slot");
        if (capturing) {
            if (captured >= ARG_CAPTURE_SLOTS) return nullptr;
            return reinterpret_cast<A *>(base + (ARG_SLOTS + captured++) * ARG_SLOT_BYTES);
        }
        return reinterpret_cast<A *>(base + (size_t)(next++ % ARG_SLOTS) * ARG_SLOT_BYTES);
    }
};

template <class A>
__global__ __launch_bounds__(64) void store_args_kernel(A a, A *dst) {
    if (threadIdx.x == 0) *dst = a;
}

// a's copy in the ring's next slot (a capture slot while s is being captured), written on
// stream s before the kernel that reads it; nullptr when no capture slot is left
template <class A>
inline const A *push_args(ArgRing &ring, const A &a, hipStream_t s) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess) cap = hipStreamCaptureStatusNone;
    A *slot = ring.slot<A>(cap != hipStreamCaptureStatusNone);
    if (!slot) return nullptr;
    hipLaunchKernelGGL(store_args_kernel<A>, dim3(1), dim3(64), 0, s, a, slot);
    return slot;
}
// renderWorld (util.py:189-232) on the device (mapf_render.hip): frames [n][H*S][W*S][3] u8
struct RenderSpec {
    int scale;
    uint8_t palette[67 * 3];        // 0 free, 1 obstacle, 2 grey (human, path), 3 + i agent i
    double star_x[15], star_y[15];  // drawStar's r cos(a), r sin(a) per vertex (host libm, as the reference's math)
};
void launch_render(const DevEnv &e, const int32_t *envs, int n, const RenderSpec &rs, uint8_t *frames, hipStream_t s);
// obstacle maps on the device (mapf_maps.hip): kind 0 warehouse (length in [lo, hi]), 1 random
// density p; largest: keep only the largest 4-connected free component (H * W <= LC_MAX_CELLS)
struct MapGen {
    int kind, lo, hi, largest;
    float density;
    uint32_t epoch;
    uint64_t seed;
};
constexpr int LC_MAX_CELLS = 8192;
void launch_mapgen(const DevEnv &e, const MapGen &g, int8_t *maps, hipStream_t s);
// the padded obstacle bitmaps and static-action masks from int8 maps [nmaps][H][W] on the device
void launch_build_maps(const DevEnv &e, const int8_t *maps, hipStream_t s);
void launch_reset_fixed(const DevEnv &e, hipStream_t s);
void launch_reset_seeded(const DevEnv &e, hipStream_t s);
void launch_gae(const float *r, const float *v, const float *vl, float *adv, float *ret, int T, int M, float g,
                float gl, hipStream_t s);
void launch_normalize(const float *ret, const float *v, const float *cret, const float *cv, float *adv,
                      float *cadv, int M, float lam, float lam1, int mix, const float *lamd, hipStream_t s);
void launch_moments(const float *ret, const float *v, const float *cret, const float *cv, int M, const double *mean,
                    double *out, hipStream_t s);
void launch_normalize_stats(const float *ret, const float *v, const float *cret, const float *cv, const double *stats,
                            float *adv, float *cadv, int M, float lam, float lam1, int mix, const float *lamd,
                            hipStream_t s);
void launch_episode_sum(const float *x, int T, int B, int N, float *out, hipStream_t s);
void launch_sample(const float *ps, int stride, int32_t *a32, int64_t *a64, int M, uint64_t seed, uint32_t step,
                   hipStream_t s);

}  // namespace mapf
