// tools/store_pattern.hip -- what the c2 slot-buffer rollout's store pattern costs.
//
// The rollout kernel's wave for env b writes env b's 23 KB observation slice as 1 KiB
// store instructions (64 lanes x 16 B), 4096 waves at once, into a fresh [B] slice every
// step.  This measures that pattern against an address-interleaved one (concurrent
// instructions of the waves hit adjacent KiB) with plain and nontemporal stores, at the
// same bytes per step, in persistent launches of S steps:
//     hipcc -O3 --offload-arch=gfx950 tools/store_pattern.hip -o tools/store_pattern
//     ./tools/store_pattern [waves kib_per_wave steps in_place waves_per_workgroup]
// (default: the c2 slot pattern, 4096 23 64 0 4; c4's observer pattern in place: 1024 32 256 1 1)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

// CHUNK: per-wave contiguous KiB (the env's slice); else interleaved (KiB k of wave w at
// (k * waves + w)); NT: nontemporal
template <bool CHUNK, bool NT>
__global__ __launch_bounds__(1024) void stores(float *buf, int steps, int kib_per_wave, size_t step_floats) {
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

#include <cstdlib>
int main(int argc, char **argv) {
    // c2: 4096 envs x ~23 KiB each per step, fresh slices
    const int waves = argc > 1 ? atoi(argv[1]) : 4096, kib = argc > 2 ? atoi(argv[2]) : 23;
    const int steps = argc > 3 ? atoi(argv[3]) : 64, inplace = argc > 4 ? atoi(argv[4]) : 0;
    const int wpg = argc > 5 ? atoi(argv[5]) : 4;
    const size_t slice = (size_t)waves * kib * 256;
    const size_t step_floats = inplace ? 0 : slice;
    printf("%d waves x %d KiB, %d steps, %s, %d waves per workgroup\n", waves, kib, steps,
           inplace ? "in place" : "fresh slices", wpg);
    float *buf = nullptr;
    if (hipMalloc(&buf, slice * 4 * (inplace ? 1 : steps)) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char *name, auto kern) {
        hipLaunchKernelGGL(kern, dim3(waves / wpg), dim3(64 * wpg), 0, 0, buf, steps, kib, step_floats);
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(a);
            hipLaunchKernelGGL(kern, dim3(waves / wpg), dim3(64 * wpg), 0, 0, buf, steps, kib, step_floats);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        const double bytes = (double)slice * 4 * steps;
        printf("%-34s %7.2f us/step  %6.0f GB/s\n", name, best * 1e3 / steps, bytes / (best * 1e-3) / 1e9);
    };
    run("env chunks, plain", stores<true, false>);
    run("env chunks, nontemporal", stores<true, true>);
    run("interleaved KiB, plain", stores<false, false>);
    run("interleaved KiB, nontemporal", stores<false, true>);
    hipFree(buf);
    return 0;
}
