// Diagnostic: the rate at which a kernel writes pinned host memory over PCIe, by store width and
// kind (plain or non-temporal), one 64-lane wave per 16 KiB page as the small-batch decoders
// write their pages (direct_out, engine.hip).  Usage: host_write [MiB=32] [reps=20]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int kBytes, bool kNt>
__global__ __launch_bounds__(256) void write_pages(uint8_t *dst, size_t pages) {
    const size_t page = blockIdx.x;
    if (page >= pages) return;
    uint8_t *p = dst + page * 16384;
    for (uint32_t o = threadIdx.x * kBytes; o < 16384; o += 256 * kBytes) {
        if constexpr (kBytes == 4) {
            const uint32_t v = o ^ (uint32_t)page;
            if (kNt) __builtin_nontemporal_store(v, (uint32_t *)(p + o)); else *(uint32_t *)(p + o) = v;
        } else if constexpr (kBytes == 8) {
            const u32x2 v = {o, (uint32_t)page};
            if (kNt) __builtin_nontemporal_store(v, (u32x2 *)(p + o)); else *(u32x2 *)(p + o) = v;
        } else {
            const u32x4 v = {o, (uint32_t)page, o + 1, o + 2};
            if (kNt) __builtin_nontemporal_store(v, (u32x4 *)(p + o)); else *(u32x4 *)(p + o) = v;
        }
    }
}

template <int kBytes, bool kNt>
static void run(uint8_t *dst, size_t bytes, int reps) {
    const size_t pages = bytes / 16384;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((write_pages<kBytes, kNt>), dim3((unsigned)pages), dim3(256), 0, 0, dst, pages);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < reps; r++) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL((write_pages<kBytes, kNt>), dim3((unsigned)pages), dim3(256), 0, 0, dst, pages);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    printf("{\"store_bytes\": %d, \"nontemporal\": %s, \"mib\": %zu, \"best_ms\": %.3f, \"gib_s\": %.2f}\n", kBytes,
           kNt ? "true" : "false", bytes >> 20, best, (double)bytes / (best * 1e-3) / (double)(1u << 30));
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 32;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const size_t bytes = mib << 20;
    uint8_t *h = nullptr, *d = nullptr;
    if (hipHostMalloc((void **)&h, bytes, hipHostMallocDefault) != hipSuccess) return 1;
    if (hipHostGetDevicePointer((void **)&d, h, 0) != hipSuccess) return 1;
    run<4, false>(d, bytes, reps);
    run<4, true>(d, bytes, reps);
    run<8, false>(d, bytes, reps);
    run<8, true>(d, bytes, reps);
    run<16, false>(d, bytes, reps);
    run<16, true>(d, bytes, reps);
    // the same into device memory, then one D2H copy
    uint8_t *dm = nullptr;
    if (hipMalloc((void **)&dm, bytes) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < reps; r++) {
        (void)hipEventRecord(a, 0);
        (void)hipMemcpyAsync(h, dm, bytes, hipMemcpyDeviceToHost, 0);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    printf("{\"d2h_copy\": true, \"mib\": %zu, \"best_ms\": %.3f, \"gib_s\": %.2f}\n", mib, best,
           (double)bytes / (best * 1e-3) / (double)(1u << 30));
    (void)hipFree(dm);
    (void)hipHostFree(h);
    return 0;
}
