// Diagnostic: is a page written into pinned host memory by a 1,024-thread workgroup visible to the
// host once the host sees the flag the workgroup writes after it?  256 workgroups per launch (one
// 16 KiB page + one flag each), 400 launches per variant; the host spins on every flag, then checks
// every byte.  Variants (store kind): 0 plain, 1 nontemporal, 2 system-scope relaxed atomic stores;
// the flag is written after __threadfence_system + barrier (release), or (variant 3) plain stores
// and a system-scope release atomic store of the flag.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int kPages = 256;

__global__ __launch_bounds__(1024) void writer(uint32_t *pages, uint32_t *flags, uint32_t v, int kind) {
    const uint32_t tid = threadIdx.x;
    uint32_t *page = pages + (size_t)blockIdx.x * 4096;
    for (uint32_t i = tid; i < 4096; i += 1024) {
        const uint32_t x = v * 2654435761u + i + blockIdx.x * 7919u;
        if (kind == 1) __builtin_nontemporal_store(x, page + i);
        else if (kind == 2) __hip_atomic_store(page + i, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else page[i] = x;
    }
    if (kind != 3) __threadfence_system();
    __syncthreads();
    if (tid == 0) {
        if (kind == 3) __hip_atomic_store(flags + blockIdx.x * 16, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        else flags[blockIdx.x * 16] = v;
    }
}

int main() {
    uint32_t *h = nullptr, *hf = nullptr, *dp = nullptr, *df = nullptr;
    (void)hipHostMalloc((void **)&h, (size_t)kPages * 16384, hipHostMallocDefault);
    (void)hipHostMalloc((void **)&hf, kPages * 64, hipHostMallocDefault);
    (void)hipHostGetDevicePointer((void **)&dp, h, 0);
    (void)hipHostGetDevicePointer((void **)&df, hf, 0);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int kind = 0; kind < 4; kind++) {
        int bad_pages = 0;
        long bad_words = 0;
        for (uint32_t it = 1; it <= 400; it++) {
            for (int p = 0; p < kPages; p++) ((volatile uint32_t *)hf)[p * 16] = 0;
            hipLaunchKernelGGL(writer, dim3(kPages), dim3(1024), 0, s, dp, df, it, kind);
            for (int p = 0; p < kPages; p++) {
                while (((volatile uint32_t *)hf)[p * 16] != it) {
                }
                int bad = 0;
                const volatile uint32_t *pg = (const volatile uint32_t *)h + (size_t)p * 4096;
                for (uint32_t i = 0; i < 4096; i++) bad += pg[i] != it * 2654435761u + i + (uint32_t)p * 7919u;
                bad_pages += bad != 0;
                bad_words += bad;
            }
            (void)hipStreamSynchronize(s);
        }
        printf("{\"kind\": %d, \"pages\": %d, \"bad_pages\": %d, \"bad_words\": %ld}\n", kind, 400 * kPages, bad_pages, bad_words);
        fflush(stdout);
    }
    return 0;
}
