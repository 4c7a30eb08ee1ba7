// tools/probes/fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the
// lane-per-page LZ4 decoder's access patterns (MI355X_MICROARCH.md: "other access widths
// are uncalibrated"), on buffers far larger than the 256 MiB Infinity Cache:
//   seq16  : every lane streams its own 16 KiB region with 16-byte loads (the stream windows)
//   rand16 : every lane loads 16 bytes at pseudo-random 16-byte-aligned offsets (far matches)
//   line64 : every lane writes its own region in whole 64-byte lines, four 16-byte stores each
//            (the ring flushes)
//   coal16 / coal8 / coal1 : each wave streams its own region, lane-contiguous loads of 16 / 8 / 1
//            bytes (the page-staging kernels; the zstd block pass's sequence lists; its literal
//            gathers) -- round 6, to read FETCH_SIZE beside TCC_EA0_RDREQ_DRAM_32B_sum (32-byte
//            units, 128-byte requests counted as 4) and TCC_BUBBLE_sum
// Known bytes per kernel are printed; compare with the counters of the same dispatch.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/fetch_calib tools/probes/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

__global__ void seq16(const u32x4 *src, uint32_t *sink, size_t per_lane) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const u32x4 *p = src + t * (per_lane / 16);
    u32x4 acc = {0, 0, 0, 0};
    for (size_t k = 0; k < per_lane / 16; k++) acc ^= *(const g_u32x4 *)(uintptr_t)(p + k);
    sink[t] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

__global__ void rand16(const u32x4 *src, uint32_t *sink, size_t nvec, int loads) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t s = 0x9E3779B97F4A7C15ull * (t + 1);
    u32x4 acc = {0, 0, 0, 0};
    for (int k = 0; k < loads; k++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        acc ^= *(const g_u32x4 *)(uintptr_t)(src + (s % nvec));
    }
    sink[t] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

__global__ void line64(u32x4 *dst, size_t per_lane) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    u32x4 *p = dst + t * (per_lane / 16);
    const u32x4 v = {(uint32_t)t, 1u, 2u, 3u};
    for (size_t k = 0; k < per_lane / 16; k += 4) {
        *(g_u32x4 *)(uintptr_t)(p + k) = v;
        *(g_u32x4 *)(uintptr_t)(p + k + 1) = v;
        *(g_u32x4 *)(uintptr_t)(p + k + 2) = v;
        *(g_u32x4 *)(uintptr_t)(p + k + 3) = v;
    }
}

template <typename T>
__global__ void coal(const T *src, uint32_t *sink, size_t per_wave) {
    const size_t w = blockIdx.x, lane = threadIdx.x;
    const T *p = src + w * (per_wave / sizeof(T));
    uint32_t acc = 0;
    for (size_t k = lane; k < per_wave / sizeof(T); k += 64) {
        const T v = *(const __attribute__((address_space(1))) T *)(uintptr_t)(p + k);
        if constexpr (sizeof(T) == 16) acc ^= v.x ^ v.w;
        else if constexpr (sizeof(T) == 8) acc ^= (uint32_t)v ^ (uint32_t)(v >> 32);
        else acc ^= v;
    }
    sink[w * 64 + lane] = acc;
}

int main() {
    const size_t lanes = 256 * 8 * 64;          // 131,072 lanes, as the lane decoder keeps in flight
    const size_t per_lane = 16384;
    const size_t bytes = lanes * per_lane;      // 2 GiB
    u32x4 *buf;
    uint32_t *sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, lanes * 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    const int loads = 256;
    hipLaunchKernelGGL(seq16, dim3(lanes / 64), dim3(64), 0, 0, buf, sink, per_lane);
    hipLaunchKernelGGL(rand16, dim3(lanes / 64), dim3(64), 0, 0, buf, sink, bytes / 16, loads);
    hipLaunchKernelGGL(line64, dim3(lanes / 64), dim3(64), 0, 0, buf, per_lane);
    // coalesced: 2 GiB in 16 KiB regions, one wave each (131,072 waves)
    const size_t waves = bytes / per_lane;
    if (hipMalloc(&sink, waves * 64 * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(coal<u32x4>, dim3(waves), dim3(64), 0, 0, buf, sink, per_lane);
    hipLaunchKernelGGL(coal<uint64_t>, dim3(waves), dim3(64), 0, 0, (const uint64_t *)buf, sink, per_lane);
    hipLaunchKernelGGL(coal<uint8_t>, dim3(waves), dim3(64), 0, 0, (const uint8_t *)buf, sink, per_lane);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"seq16_read_bytes\": %zu, \"rand16_loads\": %zu, \"rand16_read_bytes\": %zu, \"line64_write_bytes\": %zu, \"coal_read_bytes\": %zu}\n",
           bytes, lanes * (size_t)loads, lanes * (size_t)loads * 16, bytes, bytes);
    return 0;
}
