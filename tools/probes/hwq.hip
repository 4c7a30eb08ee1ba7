// Probe: which pairs of HIP streams run kernels concurrently (GPU_MAX_HW_QUEUES
// maps streams onto a few hardware queues).  Creates 24 streams, then for each
// k launches a ~1 ms spin kernel on stream 0 and on stream k and reports the
// wall time of the pair (about 1 ms = concurrent, about 2 ms = serialized).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void spin(unsigned long long cycles, unsigned *sink) {
    const unsigned long long t0 = clock64();
    unsigned x = threadIdx.x;
    while (clock64() - t0 < cycles) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) sink[0] = x;
}

int main() {
    const int n = 24;
    hipStream_t s[n];
    for (int i = 0; i < n; i++) hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
    hipStream_t hp;
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipStreamCreateWithPriority(&hp, hipStreamNonBlocking, hi);
    unsigned *sink;
    hipMalloc(&sink, 64);
    const unsigned long long cyc = 2000000ull;   // ~1 ms at 2 GHz
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[0], cyc, sink);
    hipDeviceSynchronize();
    auto run = [&](hipStream_t a, hipStream_t b) {
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, cyc, sink);
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, b, cyc, sink);
        hipDeviceSynchronize();
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    const double one = run(s[0], s[0]) / 2.0;
    printf("{\"single_ms\": %.3f, \"pairs\": {", one);
    for (int k = 1; k < n; k++) printf("%s\"0+%d\": %.2f", k > 1 ? ", " : "", k, run(s[0], s[k]) / one);
    printf("}, \"0+high_priority\": %.2f, \"priority_range\": [%d, %d]}\n", run(s[0], hp) / one, lo, hi);
    return 0;
}
