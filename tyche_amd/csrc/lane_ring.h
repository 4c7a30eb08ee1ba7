// lane_ring.h -- per-lane output rings for the lane-per-page decoders
// (lz4_decode_lane.hip: LZ4 blocks, zstd_decode.hip: zstd sequence execution).
//
// A lane assembles its page in an LDS ring of the last kRing output bytes and
// writes it to HBM only in aligned whole lines; a match whose source is more
// than kRing - 32 bytes back reads the page's already-flushed bytes from HBM
// (the unflushed tail is < kLine + 16 bytes).  A lane's store followed by its own
// load of the same address returns the stored value (one wave's vector memory
// operations are performed in order), which those far reads rely on.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lds_io.h"

namespace tyche {
namespace {

typedef unsigned __int128 u128;
typedef u32x4 u32x4_ua __attribute__((aligned(1)));
typedef __attribute__((address_space(1))) u32x4_ua g_u32x4_ua;
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) uint64_t g_u64_ua __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) u32x4_ua l_u32x4_ua;

__device__ __forceinline__ u128 ld16(const uint8_t *p) {
    u32x4 v = *(const g_u32x4_ua *)(uintptr_t)p;
    return __builtin_bit_cast(u128, v);
}
// (round-1/2 cache-policy experiments on the lane decoder, r01-r02 logs: non-temporal stream
// loads and line flushes were slower; the default policy stays)
__device__ __forceinline__ u128 ld16s(const uint8_t *p) { return ld16(p); }
__device__ __forceinline__ uint64_t ld8(const uint8_t *p) { return *(const g_u64_ua *)(uintptr_t)p; }
__device__ __forceinline__ void st16(uint8_t *p, u128 v) {
    *(g_u32x4_ua *)(uintptr_t)p = __builtin_bit_cast(u32x4, v);
}
__device__ __forceinline__ void st16f(uint8_t *p, u128 v) { st16(p, v); }
__device__ __forceinline__ uint32_t ld1(const uint8_t *p) { return *(const g_u8 *)(uintptr_t)p; }
__device__ __forceinline__ void st1(uint8_t *p, uint32_t v) { *(g_u8 *)(uintptr_t)p = (uint8_t)v; }

// HBM flush granule (128-byte lines at the 256-byte ring: 34.04-34.08 vs
// 34.14-34.65 ms per 1M pages with 64, within noise): the unflushed tail stays
// below kLine + 16 bytes, so far reads (offset > kRing - 32) need kRing >= kLine + 64
#ifndef TYCHE_LANE_LINE
#define TYCHE_LANE_LINE 64
#endif
template <int32_t kRing>
constexpr int32_t line_for() { return kRing >= TYCHE_LANE_LINE + 64 ? TYCHE_LANE_LINE : 64; }

__device__ __forceinline__ u128 lds16(const uint8_t *p) {
    return __builtin_bit_cast(u128, *(const l_u32x4_ua *)(const __attribute__((address_space(3))) uint8_t *)p);
}
__device__ __forceinline__ void lds16(uint8_t *p, u128 v) {
    *(l_u32x4_ua *)(__attribute__((address_space(3))) uint8_t *)p = __builtin_bit_cast(u32x4, v);
}
// Ring layout per lane: 16 B front slack, kRing bytes, 32 B tail slack.
// 16 bytes of the ring at page position x (valid for any x: the 16 bytes past
// the ring's end mirror its first 16)
template <int32_t kRing>
__device__ __forceinline__ u128 ring_rd(uint8_t *rb, int32_t x) {
    return lds16(rb + ((int32_t)((uint32_t)x % (uint32_t)kRing)));
}
template <int32_t kRing>
__device__ __forceinline__ void ring_wr(uint8_t *rb, int32_t x, u128 v) {
    const int32_t q = (int32_t)((uint32_t)x % (uint32_t)kRing);
    lds16(rb + q, v);
    if (q + 16 > kRing) lds16(rb + q - kRing, v);   // wrapped part, to the ring's start
    if (q < 16) lds16(rb + q + kRing, v);           // mirror of the start, past the end
}
// write out the whole lines of [fl, fin)
template <int32_t kRing>
__device__ __forceinline__ void ring_flush(uint8_t *rb, uint8_t *__restrict__ out, int32_t &fl, int32_t fin) {
    constexpr int32_t kLine = line_for<kRing>();
    static_assert(kRing >= kLine + 64, "ring too small for the flush granule");
    while (fin - fl >= kLine) {
#pragma unroll
        for (int32_t j = 0; j < kLine; j += 16) st16f(out + fl + j, ring_rd<kRing>(rb, fl + j));
        fl += kLine;
    }
}
template <int32_t kRing>
__device__ __forceinline__ void ring_flush_all(uint8_t *rb, uint8_t *__restrict__ out, int32_t &fl, int32_t fin) {
    ring_flush<kRing>(rb, out, fl, fin);
    for (; fl + 16 <= fin; fl += 16) st16(out + fl, ring_rd<kRing>(rb, fl));
    if (fl < fin) {
        const u128 v = ring_rd<kRing>(rb, fl);
        for (int32_t j = 0; fl + j < fin; j++) st1(out + fl + j, (uint32_t)(v >> (8 * j)) & 0xFFu);
        fl = fin;
    }
}
// A 16-byte pattern of period off (1 <= off < 16) from the first off bytes of m,
// and the largest multiple of off <= 16: the store stride that keeps the period.
__device__ __forceinline__ u128 period_pattern(u128 m, int32_t off, int32_t &step) {
    u128 p = m & ((((u128)1) << (8 * off)) - 1);
    for (int32_t len = off; len < 16; len <<= 1) p |= p << (8 * len);
    step = 16 - (int32_t)mod_small(16u, (uint32_t)off);
    return p;
}

}  // namespace
}  // namespace tyche
