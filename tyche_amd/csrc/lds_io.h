// lds_io.h -- HBM <-> LDS page staging shared by the codec kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tyche {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// LDS accesses at any byte address: gfx950 runs in unaligned DS mode, so a
// 32-bit access through an align(1) type is a single ds_read_b32 / ds_write_b32
// (checked by tools/probes/lds_unaligned.hip).
typedef uint32_t u32_ua __attribute__((aligned(1)));
typedef uint16_t u16_ua __attribute__((aligned(1)));
__device__ __forceinline__ uint32_t lds_ld32(const uint8_t *p) { return *(const u32_ua *)p; }
__device__ __forceinline__ uint32_t lds_ld16(const uint8_t *p) { return *(const u16_ua *)p; }
__device__ __forceinline__ void lds_st32(uint8_t *p, uint32_t v) { *(u32_ua *)p = v; }

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// Streaming loads from HBM through the global address space: a generic pointer
// would compile to flat_load, which counts in both vmcnt and lgkmcnt (so every
// later LDS wait would also wait for it) and is waited out of order.
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;
typedef const __attribute__((address_space(1))) uint32_t g_u32;
__device__ __forceinline__ u32x4 gload_nt(const u32x4 *p) { return __builtin_nontemporal_load((g_u32x4 *)(uintptr_t)p); }
__device__ __forceinline__ uint32_t gload_nt(const uint32_t *p) { return __builtin_nontemporal_load((g_u32 *)(uintptr_t)p); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) { return __builtin_amdgcn_readlane(v, lane); }
// i % m for i < 2^20, m >= 1 without an integer divide: v_rcp_f32 (1 ulp)
// leaves the quotient off by at most one, which the two corrections fix (the
// correctly rounded reciprocal cost a ten-instruction div_scale/div_fmas/
// div_fixup sequence per use: LZ4 decode 109.9 -> 104.6 ms per 1M pages)
__device__ __forceinline__ uint32_t mod_small(uint32_t i, uint32_t m) {
    const uint32_t q = (uint32_t)((float)i * __builtin_amdgcn_rcpf((float)m));
    int32_t r = (int32_t)i - (int32_t)(q * m);
    if (r < 0) r += (int32_t)m;
    if (r >= (int32_t)m) r -= (int32_t)m;
    return (uint32_t)r;
}

// 4-byte store to global memory at any byte address (one global_store_dword in
// unaligned access mode)
typedef __attribute__((address_space(1))) u32_ua g_u32_ua;
__device__ __forceinline__ void store_u32_unaligned(uint8_t *p, uint32_t v) { *(g_u32_ua *)(uintptr_t)p = v; }

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
        u32x4 x0 = gload_nt(g + v);
        u32x4 x1 = gload_nt(g + v + nthreads);
        u32x4 x2 = gload_nt(g + v + 2 * nthreads);
        u32x4 x3 = gload_nt(g + v + 3 * nthreads);
        l[v] = x0;
        l[v + nthreads] = x1;
        l[v + 2 * nthreads] = x2;
        l[v + 3 * nthreads] = x3;
    }
    for (; v < nvec; v += nthreads) l[v] = gload_nt(g + v);
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

// adler32 (adler32.c:65) of out[0..n) in LDS: A = 1 + sum b_i, B = n + sum (n - i) b_i, mod 65521
__device__ __forceinline__ uint32_t lds_adler32(const uint8_t *out, uint32_t n, uint32_t lane) {
    uint32_t A = 0;
    uint64_t B = 0;
    for (uint32_t i = lane * 4u; i < n; i += 4u * 64u) {
        uint32_t w = lds_ld32(out + i);
        const uint32_t rem = n - i;
        if (rem < 4u) w &= (1u << (8u * rem)) - 1u;
        const uint32_t b0 = w & 255u, b1 = (w >> 8) & 255u, b2 = (w >> 16) & 255u, b3 = w >> 24;
        const uint32_t s = b0 + b1 + b2 + b3;
        A += s;
        B += (uint64_t)rem * s - (b1 + 2u * b2 + 3u * b3);
    }
    const int32_t a = wave_incl_sum((int32_t)(A % 65521u));
    const int32_t b = wave_incl_sum((int32_t)(uint32_t)(B % 65521u));
    const uint32_t at = (1u + rdlane((uint32_t)a, 64u - 1)) % 65521u;
    const uint32_t bt = (n % 65521u + rdlane((uint32_t)b, 64u - 1)) % 65521u;
    return (bt << 16) | at;
}

}  // namespace tyche
