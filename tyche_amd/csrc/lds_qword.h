// lds_qword.h -- aligned-qword LDS access for the round-4 LZ4 decoders
// (lz4_decode_lc.hip, lz4_decode_quad.hip).
//
// LDS reads and writes at byte-unaligned addresses replay per lane on gfx950
// (~64 cycles per wave instruction against 11-17 for aligned ones,
// tools/probes/lds_wide.hip, profiles/r04_lds_wide.jsonl), so byte-granular
// data (LZ4 literals and matches) goes through naturally aligned qwords and
// v_alignbyte funnel shifts in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lane_ring.h"

namespace tyche {
namespace {

typedef __attribute__((address_space(3))) uint64_t l_u64;
typedef __attribute__((address_space(3))) uint32_t l_u32;
typedef __attribute__((address_space(3))) uint8_t l_u8;
__device__ __forceinline__ uint64_t lq(const uint8_t *p) { return *(const l_u64 *)(const l_u8 *)p; }
__device__ __forceinline__ void lq(uint8_t *p, uint64_t v) { *(l_u64 *)(l_u8 *)p = v; }
__device__ __forceinline__ uint32_t ld32(const uint8_t *p) { return *(const l_u32 *)(const l_u8 *)p; }
__device__ __forceinline__ void ld32(uint8_t *p, uint32_t v) { *(l_u32 *)(l_u8 *)p = v; }
__device__ __forceinline__ uint32_t lb(const uint8_t *p) { return *(const l_u8 *)p; }

#include "byte_funnel.h"

__device__ __forceinline__ uint32_t sel4(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t q) {
    const uint32_t t0 = (q & 1u) ? w1 : w0, t1 = (q & 1u) ? w3 : w2;
    return (q & 2u) ? t1 : t0;
}

// bytes [a, a + 16) of a stream of L bytes, zero outside [0, L); never reads outside it
__device__ __forceinline__ u128 chunk16z(const uint8_t *__restrict__ in, int32_t a, int32_t L) {
    if (a >= L || a + 16 <= 0) return 0;
    if (a >= 0 && a + 16 <= L) return ld16(in + a);
    if (L >= 16) {
        if (a < 0) return ld16(in) << (8 * (-a));
        return ld16(in + L - 16) >> (8 * (a - (L - 16)));
    }
    u128 v = 0;
    for (int32_t k = 15; k >= 0; k--) {
        const int32_t x = a + k;
        v = (v << 8) | ((x >= 0 && x < L) ? ld1(in + x) : 0u);
    }
    return v;
}
// byte p of a stream of L bytes (zero outside it), straight from HBM
__device__ __forceinline__ uint32_t sbyte(const uint8_t *__restrict__ in, int32_t p, int32_t L) {
    return p >= 0 && p < L ? ld1(in + p) : 0u;
}

}  // namespace
}  // namespace tyche
