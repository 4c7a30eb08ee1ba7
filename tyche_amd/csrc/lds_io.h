// lds_io.h -- HBM <-> LDS page staging shared by the codec kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tyche {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// LDS accesses at any byte address: gfx950 runs in unaligned DS mode, so a
// 32-bit access through an align(1) type is a single ds_read_b32 / ds_write_b32
// (checked by tools/probes/lds_unaligned.hip).
typedef uint32_t u32_ua __attribute__((aligned(1)));
typedef uint16_t u16_ua __attribute__((aligned(1)));
__device__ __forceinline__ uint32_t lds_ld32(const uint8_t *p) { return *(const u32_ua *)p; }
__device__ __forceinline__ uint32_t lds_ld16(const uint8_t *p) { return *(const u16_ua *)p; }
__device__ __forceinline__ void lds_st32(uint8_t *p, uint32_t v) { *(u32_ua *)p = v; }

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) { return __builtin_amdgcn_readlane(v, lane); }

// inclusive prefix sum over the 64 lanes with DPP row shifts + row broadcasts
__device__ __forceinline__ int32_t wave_incl_sum(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// inclusive max-scan over the 64 lanes (values >= -1; lanes shifted in from outside a row read -1)
__device__ __forceinline__ int32_t wave_incl_max(int32_t v) {
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xA, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xC, 0xF, false));
    return v;
}

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
