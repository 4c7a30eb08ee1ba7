// engine.h -- internal interface between the C-ABI layer (engine.hip) and the
// gfx950 kernels (lz4_decode.hip, lz4_encode.hip, pagegen.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
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

// Per-page metadata is never written by a kernel: read it through the constant
// address space so a wave-uniform index becomes a scalar load (s_load, its own
// lgkmcnt counter) instead of a vector load whose in-order vmcnt wait would also
// drain the previous page's output stores.
template <typename T>
__device__ __forceinline__ T ld_meta(const T *p, size_t i) {
    return ((const __attribute__((address_space(4))) T *)(uintptr_t)p)[i];
}

__device__ inline PageRef batch_page(const tyche_batch_t &b, size_t i) {
    PageRef r;
    uint64_t so = b.src_offsets ? ld_meta(b.src_offsets, i) : (uint64_t)i * b.src_stride;
    uint64_t dof = b.dst_offsets ? ld_meta(b.dst_offsets, i) : (uint64_t)i * b.dst_stride;
    r.src = (const uint8_t *)b.src + so;
    r.src_len = b.src_lengths ? ld_meta(b.src_lengths, i) : b.src_length;
    r.dst = (uint8_t *)b.dst + dof;
    r.dst_cap = b.dst_capacities ? ld_meta(b.dst_capacities, i) : b.dst_capacity;
    return r;
}

// The codec kernels run one 64-lane wave per workgroup: LDS ordering between
// lanes needs no s_barrier, and __syncthreads()'s workgroup fence would wait for
// every outstanding global load (the next page's prefetch) -- a code-motion
// barrier is all that is required.
#define WAVE_SYNC() __builtin_amdgcn_wave_barrier()

// Resident one-wave workgroups per CU for a kernel at `lds` bytes of dynamic
// LDS, as the runtime computes it (LDS granules, VGPRs, the per-CU limits).
// The page loops size their grids to exactly this: one more workgroup per CU
// than fits would run after a resident one finished its whole share of pages.
inline size_t waves_per_cu(const void *kernel, size_t lds) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, 64, lds) == hipSuccess && n > 0) return (size_t)n;
    const size_t granted = (lds + 511u) & ~(size_t)511u;
    return granted ? std::max<size_t>(1, std::min<size_t>(32, (160 * 1024) / granted)) : 32;
}

hipError_t launch_lz4_decode(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s,
                             bool allow_lane = true);
bool lz4_lane_decode_wanted(size_t count, uint32_t in_cap, uint32_t out_cap);
hipError_t launch_lz4_decode_lane(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s);
// large batches, round 4: one page per quad, chunked (lz4_decode_quad.hip)
hipError_t launch_lz4_decode_quad(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s);
// large batches, round 4: one page per lane, chunked, aligned LDS (lz4_decode_lc.hip)
hipError_t launch_lz4_decode_lc(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s);
hipError_t launch_lz4_encode(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s);
hipError_t launch_zstd_encode(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s);
hipError_t launch_zlib_deflate(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s);
hipError_t launch_zlib_inflate(const tyche_batch_t &b, uint32_t out_cap, hipStream_t s);
hipError_t launch_zstd_decode(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s);
// Dynamic page assignment.  The codec kernels run one-wave workgroups that loop
// over pages; when a CU holds a number of waves that is not a multiple of its 4
// SIMDs, the waves sharing a SIMD run slower than the lone ones, and static
// striding (page += gridDim.x) leaves the lone waves idle at the end.  Instead
// each wave starts at blockIdx.x and then claims pages from a per-launch
// counter.  A WorkCounter leases one zeroed device counter for one launch on
// stream s: constructed just before the launch (an async memset on s), it is
// returned to the device's pool when it goes out of scope, right after the
// launch call, as an event recorded on s -- the counter is handed out again
// only once that event has completed, i.e. once the kernel that claims pages
// from it has finished, whatever stream or thread asks next.
//
// claims = false: the launch's grid covers all its pages, so no wave ever claims
// one (every claim returns >= gridDim.x >= count whatever the counter holds):
// the counter is a shared scratch word, with no memset and no event -- two
// fewer stream operations on the small-batch latency path.
class WorkCounter {
  public:
    explicit WorkCounter(hipStream_t s, bool claims = true);
    ~WorkCounter();
    WorkCounter(const WorkCounter &) = delete;
    WorkCounter &operator=(const WorkCounter &) = delete;
    unsigned *get() const { return p_; }   // nullptr if no counter could be allocated

  private:
    hipStream_t s_;
    int dev_ = -1, idx_ = -1;
    unsigned *p_ = nullptr;
};
// A device scratch buffer of at least `bytes` for one launch on stream s,
// returned to the device's pool when it goes out of scope (right after the
// launch) as an event on s, and handed out again only once that event has
// completed -- the WorkCounter scheme for kernels that need workspace.
class ScratchLease {
  public:
    ScratchLease(hipStream_t s, size_t bytes);
    ~ScratchLease();
    ScratchLease(const ScratchLease &) = delete;
    ScratchLease &operator=(const ScratchLease &) = delete;
    void *get() const { return p_; }   // nullptr if no buffer could be allocated

  private:
    hipStream_t s_;
    int dev_ = -1, idx_ = -1;
    void *p_ = nullptr;
};
// Bytes held by the current device's scratch pool in leases no launch uses
// (freed on demand: callers sizing work by hipMemGetInfo may count them as free).
size_t scratch_idle_bytes();
// Per-device, thread-safe launch preparation: raises `kernel`'s dynamic-LDS
// limit to the CU's 160 KiB once per (device, kernel) and returns the current
// device's CU count.
size_t prepare_launch(const void *kernel);
// Tunables and kernel-path switches: TYCHE_<name> from the environment (read
// once per name), overridden in-process by tyche_set_knob -- read on every
// launch, so one process can A/B the paths (the parity tests switch them this
// way rather than with setenv, which would race getenv in other threads).
long knob(const char *name, long dflt);
__device__ __forceinline__ size_t claim_page(unsigned *counter, uint32_t lane) {
    unsigned v = 0;
    if (lane == 0) v = atomicAdd(counter, 1u);
    return (size_t)__builtin_amdgcn_readfirstlane(v) + gridDim.x;
}

hipError_t launch_pagegen(void *dst, uint64_t stride, uint32_t page_len, uint64_t seed, uint64_t first,
                          size_t count, uint32_t dist, hipStream_t s);

}  // namespace tyche
