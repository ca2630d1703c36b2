// tools/store_pattern.hip -- what the c2 slot-buffer rollout's store pattern costs.
//
// The rollout kernel's wave for env b writes env b's 23 KB observation slice as 1 KiB
// store instructions (64 lanes x 16 B), 4096 waves at once, into a fresh [B] slice every
// step.  This measures that pattern against an address-interleaved one (concurrent
// instructions of the waves hit adjacent KiB) with plain and nontemporal stores, at the
// same bytes per step, in persistent launches of S steps:
//     hipcc -O3 --offload-arch=gfx950 tools/store_pattern.hip -o tools/store_pattern
//     ./tools/store_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

// CHUNK: per-wave contiguous KiB (the env's slice); else interleaved (KiB k of wave w at
// (k * waves + w)); NT: nontemporal
template <bool CHUNK, bool NT>
__global__ __launch_bounds__(256) void stores(float *buf, int steps, int kib_per_wave, size_t step_floats) {
    const int lane = threadIdx.x & 63;
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int waves = (gridDim.x * blockDim.x) >> 6;
    for (int s = 0; s < steps; ++s) {
        float *base = buf + (size_t)s * step_floats;
        const v4f v = {(float)s, 1.f, 0.f, 1.f};
        for (int k = 0; k < kib_per_wave; ++k) {
            const size_t kib = CHUNK ? (size_t)w * kib_per_wave + k : (size_t)k * waves + w;
            v4f *p = reinterpret_cast<v4f *>(base + kib * 256) + lane;
            if (NT) __builtin_nontemporal_store(v, p);
            else *p = v;
        }
    }
}

int main() {
    const int waves = 4096, kib = 23, steps = 64;        // c2: 4096 envs x ~23 KiB each per step
    const size_t step_floats = (size_t)waves * kib * 256;
    float *buf = nullptr;
    if (hipMalloc(&buf, step_floats * 4 * steps) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char *name, auto kern) {
        hipLaunchKernelGGL(kern, dim3(waves / 4), dim3(256), 0, 0, buf, steps, kib, step_floats);
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(a);
            hipLaunchKernelGGL(kern, dim3(waves / 4), dim3(256), 0, 0, buf, steps, kib, step_floats);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        const double bytes = (double)step_floats * 4 * steps;
        printf("%-34s %7.2f us/step  %6.0f GB/s\n", name, best * 1e3 / steps, bytes / (best * 1e-3) / 1e9);
    };
    run("env chunks, plain", stores<true, false>);
    run("env chunks, nontemporal", stores<true, true>);
    run("interleaved KiB, plain", stores<false, false>);
    run("interleaved KiB, nontemporal", stores<false, true>);
    hipFree(buf);
    return 0;
}
