// pagegen.hip -- fills device memory with synthetic database pages (pagegen.h).
// Not part of the codec path: bench.py and the GPU tests use it to put the
// 1M-page workloads of SURVEY §8d straight into HBM without a 16 GiB upload.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "pagegen.h"

namespace tyche {

namespace {

// one block per page, each thread fills dwords of that page
__global__ __launch_bounds__(256) void pagegen_kernel(uint8_t *dst, uint64_t stride, uint32_t page_len, uint64_t seed,
                                                      uint64_t first, uint32_t dist) {
    __shared__ pg_page_t pg;
    const uint64_t page = blockIdx.x;
    if (threadIdx.x == 0) pg_page_init(&pg, seed, first + page, page_len, dist);
    __syncthreads();
    uint32_t *d = (uint32_t *)(dst + page * stride);
    for (uint32_t w = threadIdx.x; w < page_len / 4; w += blockDim.x) d[w] = pg_page_dword(&pg, w * 4);
}

}  // namespace

hipError_t launch_pagegen(void *dst, uint64_t stride, uint32_t page_len, uint64_t seed, uint64_t first, size_t count,
                          uint32_t dist, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if ((page_len & 3u) || (stride & 3u) || (((uintptr_t)dst) & 3u) || dist >= PG_DIST_COUNT) return hipErrorInvalidValue;
    const size_t chunk = 1u << 20;   // grid.x limit-friendly chunks
    for (size_t c = 0; c < count; c += chunk) {
        size_t n = count - c < chunk ? count - c : chunk;
        hipLaunchKernelGGL(pagegen_kernel, dim3((unsigned)n), dim3(256), 0, s, (uint8_t *)dst + c * stride, stride,
                           page_len, seed, first + c, dist);
    }
    return hipGetLastError();
}

}  // namespace tyche
