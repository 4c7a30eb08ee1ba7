// lds_io.h -- HBM <-> LDS page staging shared by the codec kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tyche {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) { return __builtin_amdgcn_readlane(v, lane); }

// Copies n bytes of global memory (any alignment) into 16-byte-aligned LDS with
// 16-byte loads (1 KiB per wave instruction).  Byte j of src lands at
// lds[head + j], head = src & 15; returns head.  Reads stay inside the 16-byte
// blocks that hold the range, so they never cross a page boundary.
__device__ __forceinline__ uint32_t stage_in(const uint8_t *src, uint32_t n, uint8_t *lds, uint32_t tid,
                                             uint32_t nthreads) {
    uintptr_t a = (uintptr_t)src;
    uint32_t head = (uint32_t)(a & 15u);
    if (n == 0) return head;
    const u32x4 *g = (const u32x4 *)(a - head);
    uint32_t nvec = (head + n + 15u) >> 4;
    u32x4 *l = (u32x4 *)lds;
    uint32_t v = tid;
    for (; v + 3 * nthreads < nvec; v += 4 * nthreads) {   // 4 loads in flight per lane
        u32x4 x0 = __builtin_nontemporal_load(g + v);
        u32x4 x1 = __builtin_nontemporal_load(g + v + nthreads);
        u32x4 x2 = __builtin_nontemporal_load(g + v + 2 * nthreads);
        u32x4 x3 = __builtin_nontemporal_load(g + v + 3 * nthreads);
        l[v] = x0;
        l[v + nthreads] = x1;
        l[v + 2 * nthreads] = x2;
        l[v + 3 * nthreads] = x3;
    }
    for (; v < nvec; v += nthreads) l[v] = __builtin_nontemporal_load(g + v);
    return head;
}

// Writes n bytes from LDS (lds, 16-byte aligned base, data starting at lds[0])
// to global dst (any alignment).  Aligned destinations use 16-byte stores.
__device__ __forceinline__ void stage_out(uint8_t *dst, const uint8_t *lds, uint32_t n, uint32_t tid,
                                          uint32_t nthreads) {
    uintptr_t a = (uintptr_t)dst;
    if ((a & 15u) == 0) {
        uint32_t nvec = n >> 4;
        const u32x4 *l = (const u32x4 *)lds;
        u32x4 *g = (u32x4 *)dst;
        uint32_t v = tid;
        for (; v + 3 * nthreads < nvec; v += 4 * nthreads) {
            u32x4 x0 = l[v], x1 = l[v + nthreads], x2 = l[v + 2 * nthreads], x3 = l[v + 3 * nthreads];
            __builtin_nontemporal_store(x0, g + v);
            __builtin_nontemporal_store(x1, g + v + nthreads);
            __builtin_nontemporal_store(x2, g + v + 2 * nthreads);
            __builtin_nontemporal_store(x3, g + v + 3 * nthreads);
        }
        for (; v < nvec; v += nthreads) __builtin_nontemporal_store(l[v], g + v);
        for (uint32_t j = (nvec << 4) + tid; j < n; j += nthreads) dst[j] = lds[j];
    } else {
        for (uint32_t j = tid; j < n; j += nthreads) dst[j] = lds[j];
    }
}

}  // namespace tyche
