// Probe: throughput and latency of byte-unaligned wide LDS accesses on gfx950
// (ds_read_b64 / ds_read_b128 / ds_write_b64 / ds_write_b128 at arbitrary byte
// addresses vs aligned), the primitive the lane-group LZ4 decoder is built on.
// Each lane owns a 1 KiB LDS region (16 lanes... one wave per workgroup, waves/CU
// set by the grid), addresses are a per-lane LCG inside the region; alignment is
// forced by masking.  Prints ns per wave-instruction per CU for each mode, plus a
// dependent-chain latency (one wave) and an exactness check.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(64) void tp(uint32_t *out, int iters, uint32_t amask) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s[];
    const uint32_t lane = threadIdx.x;
    const uint32_t base = (uint32_t)(uintptr_t)s + lane * 256u;   // 256 B per lane (16 KiB per wave)
    for (uint32_t i = lane; i < 64u * 256u / 4u; i += 64) ((uint32_t *)s)[i] = i * 2654435761u;
    __builtin_amdgcn_wave_barrier();
    uint32_t x = lane * 7919u + blockIdx.x * 104729u + 1u;
    uint32_t acc = 0;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            x = x * 1664525u + 1013904223u;
            const uint32_t a = base + (((x >> 8) % 224u) & amask);
            if (MODE == 0) { u32x2 v; asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a)); acc ^= v.x ^ v.y; }
            if (MODE == 1) { u32x4 v; asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a)); acc ^= v.x ^ v.w; }
            if (MODE == 2) { u32x2 v = {x, acc}; asm volatile("ds_write_b64 %0, %1" : : "v"(a), "v"(v) : "memory"); }
            if (MODE == 3) { u32x4 v = {x, acc, x, acc}; asm volatile("ds_write_b128 %0, %1" : : "v"(a), "v"(v) : "memory"); }
            if (MODE == 4) { uint32_t v; asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a)); acc ^= v; }
            if (MODE == 5) { uint32_t v; asm volatile("ds_read_u8 %0, %1" : "=v"(v) : "v"(a)); acc ^= v; }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// dependent chain: the next address comes from the loaded value (one wave)
template <int W>
__global__ __launch_bounds__(64) void lat(uint32_t *out, int iters, uint32_t amask, uint32_t *cyc) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s[];
    const uint32_t lane = threadIdx.x;
    const uint32_t base = (uint32_t)(uintptr_t)s + lane * 256u;
    for (uint32_t i = lane; i < 64u * 256u / 4u; i += 64) ((uint32_t *)s)[i] = (i * 37u) & 0x7Fu;
    __builtin_amdgcn_wave_barrier();
    uint32_t a = base + ((lane * 13u) & amask);
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        if (W == 8) { u32x2 v; asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a)); a = base + ((v.x ^ v.y) & 0x7Fu & amask); }
        if (W == 16) { u32x4 v; asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a)); a = base + ((v.x ^ v.w) & 0x7Fu & amask); }
        if (W == 4) { uint32_t v; asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a)); a = base + (v & 0x7Fu & amask); }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = (uint32_t)(t1 - t0);
    if (a == 0xFFFFFFFFu) out[0] = a;
}

__global__ void exact(int *ok) {
    __shared__ __attribute__((aligned(16))) uint8_t s[2048];
    const uint32_t t = threadIdx.x;
    for (int i = t; i < 2048; i += 64) s[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    int good = 1;
    for (uint32_t off = 0; off < 16; off++) {
        const uint32_t a = t * 24 + off;
        u32x4 v;
        asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)(s + a)));
        for (int j = 0; j < 16; j++) good &= ((v[j / 4] >> (8 * (j % 4))) & 0xFF) == s[a + j];
        u32x2 w;
        asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(w) : "v"((uint32_t)(uintptr_t)(s + a)));
        for (int j = 0; j < 8; j++) good &= ((w[j / 4] >> (8 * (j % 4))) & 0xFF) == s[a + j];
    }
    __syncthreads();
    // unaligned 16-byte writes at disjoint places
    {
        const uint32_t a = t * 24 + 5;
        u32x4 v = {0x03020100u + t, 0x07060504u, 0x0B0A0908u, 0x0F0E0D0Cu};
        asm volatile("ds_write_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : : "v"((uint32_t)(uintptr_t)(s + a)), "v"(v) : "memory");
        __syncthreads();
        for (int j = 0; j < 16; j++) good &= s[a + j] == (uint8_t)(((v[j / 4]) >> (8 * (j % 4))) & 0xFF);
    }
    atomicAnd(ok, good);
}

template <int MODE>
float run_tp(int waves, uint32_t amask, int iters) {
    uint32_t *out;
    hipMalloc(&out, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipFuncSetAttribute((const void *)tp<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 16384);
    int ncu = 256;
    hipLaunchKernelGGL(tp<MODE>, dim3(ncu * waves), dim3(64), 16384, 0, out, 16, amask);
    hipEventRecord(e0);
    hipLaunchKernelGGL(tp<MODE>, dim3(ncu * waves), dim3(64), 16384, 0, out, iters, amask);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    hipFree(out);
    // cycles (at 2.4 GHz) per wave-instruction per CU
    double instrs = (double)waves * iters * 8;
    return (float)(ms * 1e-3 * 2.4e9 / instrs);
}

template <int W>
float run_lat(uint32_t amask) {
    uint32_t *out, *cyc;
    hipMalloc(&out, 64); hipMalloc(&cyc, 4 * 16);
    hipLaunchKernelGGL(lat<W>, dim3(1), dim3(64), 16384, 0, out, 4096, amask, cyc);
    hipDeviceSynchronize();
    uint32_t c; hipMemcpy(&c, cyc, 4, hipMemcpyDeviceToHost);
    hipFree(out); hipFree(cyc);
    return c / 4096.0f;
}

int main() {
    int *ok; int h = 1;
    hipMalloc(&ok, 4); hipMemcpy(ok, &h, 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(exact, dim3(1), dim3(64), 0, 0, ok);
    hipDeviceSynchronize();
    hipMemcpy(&h, ok, 4, hipMemcpyDeviceToHost);
    printf("{\"exact_unaligned_b64_b128\": %d}\n", h);
    const char *names[] = {"ds_read_b64", "ds_read_b128", "ds_write_b64", "ds_write_b128", "ds_read_b32", "ds_read_u8"};
    const uint32_t masks[] = {~0u, ~3u, ~7u, ~15u};
    const char *mn[] = {"any", "4B", "8B", "16B"};
    for (int waves : {4, 8}) {
        for (int m = 0; m < 4; m++) {
            float r[6];
            r[0] = run_tp<0>(waves, masks[m], 2048);
            r[1] = run_tp<1>(waves, masks[m], 2048);
            r[2] = run_tp<2>(waves, masks[m], 2048);
            r[3] = run_tp<3>(waves, masks[m], 2048);
            r[4] = run_tp<4>(waves, masks[m], 2048);
            r[5] = run_tp<5>(waves, masks[m], 2048);
            printf("{\"waves_per_cu\": %d, \"align\": \"%s\"", waves, mn[m]);
            for (int i = 0; i < 6; i++) printf(", \"%s\": %.2f", names[i], r[i]);
            printf("}\n");
        }
    }
    for (int m = 0; m < 4; m++)
        printf("{\"latency_cycles_one_wave\": true, \"align\": \"%s\", \"b32\": %.1f, \"b64\": %.1f, \"b128\": %.1f}\n", mn[m],
               run_lat<4>(masks[m]), run_lat<8>(masks[m]), run_lat<16>(masks[m]));
    return 0;
}
