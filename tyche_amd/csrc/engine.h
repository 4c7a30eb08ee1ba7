// engine.h -- internal interface between the C-ABI layer (engine.hip) and the
// gfx950 kernels (lz4_decode.hip, lz4_encode.hip, pagegen.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tyche_codec.h"

namespace tyche {

// results[i] value for a page that does not fit the launch's LDS sizing
// (caller passed max_src_length / dst_capacity smaller than a page's sizes)
constexpr int32_t kResultTooLarge = INT32_MIN;

// LZ4 block-format constants (lz4.c:264-281)
constexpr int kMinMatch = 4;
constexpr int kLastLiterals = 5;
constexpr int kMfLimit = 12;
constexpr int kRunMask = 15;

__host__ __device__ inline uint32_t lz4_bound(uint32_t n) {
    return n > 0x7E000000u ? 0u : n + n / 255u + 16u;  // LZ4_COMPRESSBOUND, lz4.h:148
}

// page i of a batch
struct PageRef {
    const uint8_t *src;
    uint32_t src_len;
    uint8_t *dst;
    uint32_t dst_cap;
};

__device__ inline PageRef batch_page(const tyche_batch_t &b, size_t i) {
    PageRef r;
    uint64_t so = b.src_offsets ? b.src_offsets[i] : (uint64_t)i * b.src_stride;
    uint64_t dof = b.dst_offsets ? b.dst_offsets[i] : (uint64_t)i * b.dst_stride;
    r.src = (const uint8_t *)b.src + so;
    r.src_len = b.src_lengths ? b.src_lengths[i] : b.src_length;
    r.dst = (uint8_t *)b.dst + dof;
    r.dst_cap = b.dst_capacities ? b.dst_capacities[i] : b.dst_capacity;
    return r;
}

hipError_t launch_lz4_decode(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s);
hipError_t launch_lz4_encode(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s);
hipError_t launch_zstd_encode(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s);
hipError_t launch_zlib_deflate(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s);
hipError_t launch_zlib_inflate(const tyche_batch_t &b, uint32_t out_cap, hipStream_t s);
hipError_t launch_zstd_decode(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s);
hipError_t launch_pagegen(void *dst, uint64_t stride, uint32_t page_len, uint64_t seed, uint64_t first,
                          size_t count, uint32_t dist, hipStream_t s);

}  // namespace tyche
