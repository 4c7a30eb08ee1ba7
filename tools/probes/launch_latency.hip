// Diagnostic: host-observed latency of one small kernel (the restore path's floor), p50 over 2000
// launches.  Modes: sync = hipLaunchKernel + hipStreamSynchronize; poll = the kernel writes a flag
// into pinned host memory after a system-scope fence and the host spins on it; query = spin on
// hipStreamQuery; event = hipEventRecord + spin on hipEventQuery.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void touch(volatile uint32_t *flag, uint32_t v) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) *flag = v;
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    uint32_t *h = nullptr;
    (void)hipHostMalloc((void **)&h, 4096, hipHostMallocMapped);
    uint32_t *dflag = nullptr;
    (void)hipHostGetDevicePointer((void **)&dflag, h, 0);
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    const char *names[] = {"sync", "poll", "query", "event"};
    for (int mode = 0; mode < 4; mode++) {
        std::vector<double> t;
        for (int i = 0; i < 2200; i++) {
            *(volatile uint32_t *)h = 0;
            const uint32_t v = (uint32_t)i + 1u;
            auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, (volatile uint32_t *)dflag, v);
            if (mode == 0) {
                (void)hipStreamSynchronize(s);
            } else if (mode == 1) {
                while (*(volatile uint32_t *)h != v) {
                }
            } else if (mode == 2) {
                while (hipStreamQuery(s) != hipSuccess) {
                }
            } else {
                (void)hipEventRecord(ev, s);
                while (hipEventQuery(ev) != hipSuccess) {
                }
            }
            auto t1 = std::chrono::steady_clock::now();
            if (mode == 1) (void)hipStreamSynchronize(s);
            if (i >= 200) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        std::sort(t.begin(), t.end());
        printf("{\"mode\": \"%s\", \"us_p50\": %.1f, \"us_p90\": %.1f}\n", names[mode], t[t.size() / 2], t[t.size() * 9 / 10]);
    }
    return 0;
}
