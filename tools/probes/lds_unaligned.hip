// Probe: are byte-unaligned 32-bit LDS reads/writes exact on this device?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void probe(uint32_t *out, int *ok) {
    __shared__ __attribute__((aligned(16))) uint8_t s[1024];
    int t = threadIdx.x;
    for (int i = t; i < 1024; i += 64) s[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    // unaligned dword read at t*5+1
    uint32_t a = t * 5 + 1;
    uint32_t v;
    uint32_t addr = (uint32_t)(uintptr_t)(s + a);
    asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    uint32_t want = s[a] | (s[a + 1] << 8) | (s[a + 2] << 16) | ((uint32_t)s[a + 3] << 24);
    out[t] = v;
    int good = v == want;
    __syncthreads();
    // unaligned dword write at t*16 + 3 (disjoint)
    {
        uint32_t addr2 = (uint32_t)(uintptr_t)(s + t * 16 + 3), val = 0xA1B2C3D4u + t;
        asm volatile("ds_write_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : : "v"(addr2), "v"(val) : "memory");
    }
    __syncthreads();
    uint32_t b = t * 16 + 3, w = 0xA1B2C3D4u + t;
    good &= s[b] == (w & 0xFF) && s[b + 1] == ((w >> 8) & 0xFF) && s[b + 2] == ((w >> 16) & 0xFF) && s[b + 3] == (w >> 24);
    atomicAnd(ok, good);
}

int main() {
    uint32_t *out; int *ok; int h = 1;
    hipMalloc(&out, 256); hipMalloc(&ok, 4); hipMemcpy(ok, &h, 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, ok);
    hipError_t e = hipDeviceSynchronize();
    hipMemcpy(&h, ok, 4, hipMemcpyDeviceToHost);
    printf("sync=%s unaligned_ok=%d\n", hipGetErrorString(e), h);
    return 0;
}
