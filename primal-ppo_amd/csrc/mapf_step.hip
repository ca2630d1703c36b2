// primal-ppo_amd/csrc/mapf_step.hip -- one lockstep env step for B envs: the
// kernels over step_group (mapf_step.h), one group of G lanes per env.
#include "mapf_step.h"

namespace mapf {

__global__ __launch_bounds__(256) void step_kernel(DevEnv e, int32_t *__restrict__ actions, StepOut out,
                                                   uint32_t flags, int parity) {
    const int G = e.G;
    const int gt = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = gt / G;
    if (gt == 0 && (flags & 1u)) {       // zero the next step's work-list slot (consumed two steps ago)
        e.counters[C_REPLAN_COUNT + (parity + 1) % 3] = 0;
        e.counters[C_BFS_COUNT + (parity + 1) % 3] = 0;
    }
    if (b >= e.B) return;                 // whole group leaves together
    StepRegs none;
    if (G == 64) step_group(e, actions, out, flags, parity, b, WaveGroup(), nullptr, StepSrc{}, none);   // env = wave
    else step_group(e, actions, out, flags, parity, b, Group(G), nullptr, StepSrc{}, none);
}

// Uniform random policy (random_action(): one Philox draw per 8 agents).
__global__ __launch_bounds__(256) void random_actions_kernel(DevEnv e, int32_t *__restrict__ actions) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= e.B * e.N) return;
    const int b = t / e.N, i = t - b * e.N;
    const u32x4 o = philox(e.env_offset + (uint32_t)b, P_ACT | ((uint32_t)(i >> 3) << 8), e.clock[b], 0u, e.seed);
    actions[t] = (int32_t)random_action(o, i);
}

void launch_step(const DevEnv &e, int32_t *actions, const StepOut &out, uint32_t flags, int parity, hipStream_t s) {
    if (!e.force_agent_lanes && launch_step_pairs(e, actions, out, flags, parity, s)) return;
    const long threads = (long)e.B * e.G;
    const int blk = e.step_block;
    const int grid = (int)((threads + blk - 1) / blk);
    hipLaunchKernelGGL(step_kernel, dim3(grid), dim3(blk), 0, s, e, actions, out, flags, parity);
}

void launch_random_actions(const DevEnv &e, int32_t *actions, hipStream_t s) {
    const int n = e.B * e.N;
    hipLaunchKernelGGL(random_actions_kernel, dim3((n + 255) / 256), dim3(256), 0, s, e, actions);
}

}  // namespace mapf
