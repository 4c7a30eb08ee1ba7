// Probe: random 16-byte (and 64-byte-per-quad) load rates by working-set size -- how many far-match
// reads per second the memory system serves when the sources are L2-, Infinity-Cache- or
// HBM-resident (the lane-per-page LZ4 decoders read ~500-600 such sources per 16 KiB page).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// each lane: `iters` rounds of 8 independent random 16-B loads inside [0, span)
template <int QUAD>
__global__ __launch_bounds__(64) void gather(const u32x4 *__restrict__ buf, uint32_t span16, int iters, uint32_t *out) {
    uint32_t x = (blockIdx.x * 64 + threadIdx.x) * 2654435761u + 12345u;
    uint32_t acc = 0;
    for (int it = 0; it < iters; it++) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            x = x * 1664525u + 1013904223u;
            uint32_t idx;
            if (QUAD) {   // the 4 lanes of a quad read one 64-byte line (lane j: its j-th 16 bytes)
                const uint32_t q = __builtin_amdgcn_mov_dpp(x, 0x00, 0xF, 0xF, false);
                idx = ((q >> 4) % (span16 >> 2)) * 4 + (threadIdx.x & 3);
            } else {
                idx = (x >> 4) % span16;
            }
            v[u] = buf[idx];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) acc ^= v[u].x ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t big = (size_t)2 << 30;
    u32x4 *buf;
    uint32_t *out;
    hipMalloc(&buf, big);
    hipMalloc(&out, 64);
    hipMemset(buf, 1, big);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const size_t spans[] = {(size_t)1 << 20, (size_t)16 << 20, (size_t)64 << 20, (size_t)192 << 20, big};
    for (int quad = 0; quad < 2; quad++)
        for (size_t sp : spans)
            for (int waves : {4, 8}) {
                const int iters = 256;
                const dim3 grid(256 * waves);
                if (quad) hipLaunchKernelGGL(gather<1>, grid, dim3(64), 0, 0, buf, (uint32_t)(sp / 16), 8, out);
                else hipLaunchKernelGGL(gather<0>, grid, dim3(64), 0, 0, buf, (uint32_t)(sp / 16), 8, out);
                hipEventRecord(e0);
                if (quad) hipLaunchKernelGGL(gather<1>, grid, dim3(64), 0, 0, buf, (uint32_t)(sp / 16), iters, out);
                else hipLaunchKernelGGL(gather<0>, grid, dim3(64), 0, 0, buf, (uint32_t)(sp / 16), iters, out);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                const double loads = (double)grid.x * 64 * iters * 8;
                printf("{\"quad_lines\": %d, \"span_mib\": %zu, \"waves_per_cu\": %d, \"G_lane_loads_per_s\": %.1f, "
                       "\"GB_per_s\": %.0f}\n", quad, sp >> 20, waves, loads / (ms * 1e-3) / 1e9,
                       loads * 16 / (ms * 1e-3) / 1e9);
            }
    return 0;
}
