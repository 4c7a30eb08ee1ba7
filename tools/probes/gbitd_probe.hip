// Diagnostic (round 6): the zstd per-lane bit reader with a 32-byte register window
// (scratch/zstd_decode_window.diff) against the three-dword reader it would replace, on random
// streams and random bit consumption, one stream per lane.  Prints the first mismatches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/gbitd_probe tools/probes/gbitd_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;
enum : uint32_t { kUnfinished = 0, kEndOfBuffer = 1, kCompleted = 2, kOverflow = 3 };
struct BitD {
    uint64_t c;
    uint32_t used;
    int32_t ptr, start;
};
__device__ __forceinline__ uint64_t ld64g(const uint8_t *p) {
    const uint32_t s = (uint32_t)(uintptr_t)p & 3u;
    const uint32_t *A = (const uint32_t *)(p - s);
    const uint32_t d0 = A[0], d1 = A[1];
    const uint32_t d2 = s ? A[2] : 0u;
    return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32);
}
__device__ uint32_t old_reload(BitD &b, const uint8_t *in) {
    if (b.used > 64u) return kOverflow;
    if (b.ptr >= b.start + 8) {
        b.ptr -= (int32_t)(b.used >> 3);
        b.used &= 7u;
        b.c = ld64g(in + b.ptr);
        return kUnfinished;
    }
    if (b.ptr == b.start) return b.used < 64u ? kEndOfBuffer : kCompleted;
    int32_t nbytes = (int32_t)(b.used >> 3);
    uint32_t r = kUnfinished;
    if (b.ptr - nbytes < b.start) {
        nbytes = b.ptr - b.start;
        r = kEndOfBuffer;
    }
    b.ptr -= nbytes;
    b.used -= (uint32_t)nbytes * 8u;
    b.c = ld64g(in + b.ptr);
    return r;
}
struct GBitD : BitD {
    int32_t wb;
    u32x4 lo, hi;
};
#ifndef PROBE_GCHUNK_DWORDS
__device__ __forceinline__ u32x4 gchunk(const uint8_t *p) { return *(g_u32x4 *)(uintptr_t)p; }
#else
__device__ __forceinline__ u32x4 gchunk(const uint8_t *p) {
    const uint32_t *q = (const uint32_t *)p;
    return u32x4{q[0], q[1], q[2], q[3]};
}
#endif
__device__ __forceinline__ uint64_t gbitd_take(const GBitD &b) {
    const uint32_t o = (uint32_t)(b.ptr - b.wb), k = o >> 2, s = o & 3u;
    const uint32_t l0 = b.lo.x, l1 = b.lo.y, l2 = b.lo.z, l3 = b.lo.w, h0 = b.hi.x, h1 = b.hi.y;
    const uint32_t d0 = k == 0 ? l0 : k == 1 ? l1 : k == 2 ? l2 : l3;
    const uint32_t d1 = k == 0 ? l1 : k == 1 ? l2 : k == 2 ? l3 : h0;
    const uint32_t d2 = k == 0 ? l2 : k == 1 ? l3 : k == 2 ? h0 : h1;
    return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32);
}
struct PendLoad {
    u32x4 v;
    bool take, shift;
};
__device__ __forceinline__ uint32_t new_issue(GBitD &b, const uint8_t *in, PendLoad &L) {
    uint32_t r = kUnfinished;
    L.take = false;
    if (b.used > 64u) {
        r = kOverflow;
    } else if (b.ptr >= b.start + 8) {
        b.ptr -= (int32_t)(b.used >> 3);
        b.used &= 7u;
        L.take = true;
    } else if (b.ptr == b.start) {
        r = b.used < 64u ? kEndOfBuffer : kCompleted;
    } else {
        int32_t nbytes = (int32_t)(b.used >> 3);
        if (b.ptr - nbytes < b.start) {
            nbytes = b.ptr - b.start;
            r = kEndOfBuffer;
        }
        b.ptr -= nbytes;
        b.used -= (uint32_t)nbytes * 8u;
        L.take = true;
    }
    L.shift = L.take && b.ptr < b.wb;
    L.v = u32x4{0u, 0u, 0u, 0u};
    if (L.shift) L.v = gchunk(in + b.wb - 16);
    return r;
}
__device__ __forceinline__ void new_finish(GBitD &b, const PendLoad &L) {
    if (L.shift) {
        b.hi = b.lo;
        b.lo = L.v;
        b.wb -= 16;
    }
    if (L.take) b.c = gbitd_take(b);
}
__global__ void probe(const uint8_t *buf, uint32_t *bad, uint64_t *info) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    uint64_t s = 0x9E3779B97F4A7C15ull * (t + 1);
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)(s >> 11); };
    const uint8_t *in = buf + (size_t)t * 4096 + (rnd() & 63);
    const int32_t start = (int32_t)(rnd() % 200), n = 8 + (int32_t)(rnd() % 1500);
    BitD a;
    a.start = start;
    a.ptr = start + n - 8;
    a.c = ld64g(in + a.ptr);
    a.used = rnd() % 8;
    GBitD g;
    g.start = start;
    g.ptr = a.ptr;
    g.used = a.used;
    g.wb = g.ptr - (int32_t)((uintptr_t)(in + g.ptr) & 15u);
    g.lo = gchunk(in + g.wb);
    g.hi = u32x4{0u, 0u, 0u, 0u};
    if (g.ptr + 8 > g.wb + 16) g.hi = gchunk(in + g.wb + 16);
    g.c = gbitd_take(g);
    for (int step = 0; step < 3000; step++) {
        if (a.c != g.c || a.ptr != g.ptr || a.used != g.used) {
            if (atomicAdd(bad, 1u) < 16u) {
                const uint32_t k = atomicAdd(bad + 1, 1u);
                info[k * 6 + 0] = t;
                info[k * 6 + 1] = step;
                info[k * 6 + 2] = ((uint64_t)(uint32_t)a.ptr << 32) | (uint32_t)g.wb;
                info[k * 6 + 3] = a.c;
                info[k * 6 + 4] = g.c;
                info[k * 6 + 5] = ((uint64_t)(uintptr_t)in & 63) | ((uint64_t)start << 8) | ((uint64_t)n << 32);
            }
            return;
        }
        const uint32_t u = rnd() % 30;
        a.used = min(a.used + u, 64u);
        g.used = a.used;
        const uint32_t r1 = old_reload(a, in);
        PendLoad L;
        const uint32_t r2 = new_issue(g, in, L);
        new_finish(g, L);
        if (r1 != r2) {
            atomicAdd(bad + 2, 1u);
            return;
        }
        if (r1 == kEndOfBuffer || r1 == kCompleted) return;
    }
}
int main() {
    const int lanes = 64 * 1024;
    std::vector<uint8_t> h((size_t)lanes * 4096 + 4096);
    for (size_t i = 0; i < h.size(); i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
    uint8_t *d;
    uint32_t *bad;
    uint64_t *info;
    if (hipMalloc(&d, h.size()) || hipMalloc(&bad, 16) || hipMalloc(&info, 16 * 6 * 8)) return 1;
    (void)hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
    (void)hipMemset(bad, 0, 16);
    hipLaunchKernelGGL(probe, dim3(lanes / 64), dim3(64), 0, 0, d, bad, info);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    uint32_t hb[4];
    uint64_t hi[96];
    (void)hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hi, info, sizeof(hi), hipMemcpyDeviceToHost);
    printf("{\"mismatch_lanes\": %u, \"status_mismatch\": %u}\n", hb[0], hb[2]);
    for (uint32_t k = 0; k < (hb[1] < 16 ? hb[1] : 16); k++)
        printf("lane %llu step %llu ptr %lld wb %d c_old %016llx c_new %016llx inmod64 %llu start %llu n %llu\n",
               (unsigned long long)hi[k * 6], (unsigned long long)hi[k * 6 + 1], (long long)(int32_t)(hi[k * 6 + 2] >> 32),
               (int32_t)(uint32_t)hi[k * 6 + 2], (unsigned long long)hi[k * 6 + 3], (unsigned long long)hi[k * 6 + 4],
               (unsigned long long)(hi[k * 6 + 5] & 63), (unsigned long long)((hi[k * 6 + 5] >> 8) & 0xFFFFFF),
               (unsigned long long)(hi[k * 6 + 5] >> 32));
    return 0;
}
