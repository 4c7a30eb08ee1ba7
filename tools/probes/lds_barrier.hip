// Diagnostic: cycles per barrier-separated round on one CU (one workgroup), for the
// single-page decoder's cost model.  Modes: 0 barrier only, 1 + one dependent LDS read,
// 2 + 8 independent random u16 LDS reads, 3 + 8 random reads and one 16-byte write,
// 4 barrier + LDS atomicOr flag and re-read (the jump rounds' termination test).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

template <int kT>
__global__ __launch_bounds__(kT) void rounds(int mode, int n, unsigned long long *out, unsigned *sink) {
    __shared__ uint16_t buf[32768];
    __shared__ unsigned flag[4];
    const unsigned tid = threadIdx.x;
    for (unsigned i = tid; i < 32768; i += kT) buf[i] = (uint16_t)((i * 2654435761u) >> 17);
    if (tid < 4) flag[tid] = 0;
    __syncthreads();
    unsigned acc = tid, x = tid;
    unsigned long long t0 = clock64();
    for (int r = 0; r < n; r++) {
        if (mode == 1) {
            x = buf[(x + r) & 32767];
        } else if (mode >= 2 && mode <= 3) {
            unsigned v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = buf[((x + u * 4099u) * 2654435761u >> 15) & 32767];
#pragma unroll
            for (int u = 0; u < 8; u++) acc += v[u];
            x = acc;
            if (mode == 3) *(uint4 *)&buf[(tid * 8) & 32767] = make_uint4(acc, acc, acc, acc);
        } else if (mode == 4) {
            if (tid == 0) flag[(r + 1) % 3] = 0;
            if ((x & 7) == 0) atomicOr(&flag[r % 3], 1u);
            x += 1;
        }
        __syncthreads();
        if (mode == 4 && flag[r % 3] == 0) acc++;
    }
    unsigned long long t1 = clock64();
    if (tid == 0) out[0] = t1 - t0;
    if (acc == 0xFFFFFFFFu && x == 1) sink[0] = acc;
}

int main() {
    unsigned long long *d;
    unsigned *s;
    hipMalloc(&d, 8);
    hipMalloc(&s, 4);
    const int n = 1000;
    for (int mode = 0; mode < 5; mode++) {
        for (int t : {256, 1024}) {
            for (int rep = 0; rep < 2; rep++) {
                if (t == 256) hipLaunchKernelGGL(rounds<256>, dim3(1), dim3(256), 0, 0, mode, n, d, s);
                else hipLaunchKernelGGL(rounds<1024>, dim3(1), dim3(1024), 0, 0, mode, n, d, s);
                hipDeviceSynchronize();
            }
            unsigned long long c = 0;
            hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
            printf("{\"mode\": %d, \"threads\": %d, \"cycles_per_round\": %.1f}\n", mode, t, (double)c / n);
        }
    }
    return 0;
}
