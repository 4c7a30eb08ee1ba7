/*
 * oracle/oracle_batch.c -- TEST INFRASTRUCTURE ONLY.
 * Page-range loops over the LZ4 restatement, used by bench.py's cpu_baseline
 * leg (one call per thread; ctypes releases the GIL) and by the tests.  Mirrors
 * the reference's one-codec-call-per-Buffer pattern (src/buffer.c:181-188,
 * 246-253), without the malloc per call.
 */
#include <stdint.h>
#include "oracle.h"
#include "../tyche_amd/csrc/pagegen.h"

long oracle_lz4_compress_pages(const uint8_t *src, uint64_t src_stride, uint32_t page_len, uint8_t *dst,
                               uint64_t dst_stride, int32_t *out_len, long first, long count) {
    long total = 0;
    int cap = oracle_lz4_compress_bound((int)page_len);
    for (long i = first; i < first + count; i++) {
        int r = oracle_lz4_compress_default(src + (uint64_t)i * src_stride, dst + (uint64_t)i * dst_stride,
                                            (int)page_len, cap);
        out_len[i] = r;
        total += r;
    }
    return total;
}

long oracle_lz4_decompress_pages(const uint8_t *src, uint64_t src_stride, const int32_t *in_len, uint8_t *dst,
                                 uint64_t dst_stride, uint32_t page_len, int32_t *rv, long first, long count) {
    long bad = 0;
    for (long i = first; i < first + count; i++) {
        int r = oracle_lz4_decompress_safe(src + (uint64_t)i * src_stride, dst + (uint64_t)i * dst_stride,
                                           in_len[i], (int)page_len);
        rv[i] = r;
        if (r < 0) bad++;
    }
    return bad;
}

void oracle_pagegen(uint8_t *dst, uint64_t dst_stride, uint32_t page_len, uint64_t seed, uint64_t first,
                    long count, uint32_t dist) {
    for (long i = 0; i < count; i++) {
        pg_page_t p;
        pg_page_init(&p, seed, first + (uint64_t)i, page_len, dist);
        uint8_t *d = dst + (uint64_t)i * dst_stride;
        for (uint32_t b = 0; b < page_len; b++) d[b] = (uint8_t)pg_page_byte(&p, b);
    }
}
