/* oracle/oracle.h -- TEST INFRASTRUCTURE ONLY (see lz4_oracle.c header). */
#pragma once
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
int oracle_lz4_compress_bound(int n);
int oracle_lz4_compress(const uint8_t *src, uint8_t *dst, int n, int cap);
int oracle_lz4_compress_default(const uint8_t *src, uint8_t *dst, int n, int cap);
int oracle_lz4_decompress_safe(const uint8_t *src, uint8_t *dst, int in_len, int out_cap);
/* batch helpers for the CPU baseline: pages laid out at fixed strides */
long oracle_lz4_compress_pages(const uint8_t *src, uint64_t src_stride, uint32_t page_len, uint8_t *dst,
                               uint64_t dst_stride, int32_t *out_len, long first, long count);
long oracle_lz4_decompress_pages(const uint8_t *src, uint64_t src_stride, const int32_t *in_len, uint8_t *dst,
                                 uint64_t dst_stride, uint32_t page_len, int32_t *rv, long first, long count);
/* zlib (RFC 1950/1951) restatement: decoded length or negative zlib code */
int oracle_zlib_uncompress(const uint8_t *src, int srclen, uint8_t *dst, int dstcap);
uint32_t oracle_adler32(const uint8_t *p, int n);
/* zstd v1.1.2 frame decoder restatement: decoded size or negative error */
int oracle_zstd_decompress(const uint8_t *src, int srclen, uint8_t *dst, int dstcap);
int oracle_zstd_compress_bound(int n);
uint64_t oracle_xxh64(const uint8_t *p, size_t len, uint64_t seed);
/* host copy of the synthetic page generator (tyche_amd/csrc/pagegen.h) */
void oracle_pagegen(uint8_t *dst, uint64_t dst_stride, uint32_t page_len, uint64_t seed, uint64_t first,
                    long count, uint32_t dist);
#ifdef __cplusplus
}
#endif
