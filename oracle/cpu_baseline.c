/*
 * oracle/cpu_baseline.c -- TEST INFRASTRUCTURE ONLY: the CPU baseline of bench.py.
 *
 * Times the reference's own vendored codecs (LZ4 1.7.5 / zstd 1.1.2 / zlib
 * 1.2.8, compiled from /root/reference/src into oracle/_ref/libtyche_ref.so by
 * oracle/Makefile) the way tyche runs them: one codec call per page
 * (LZ4_compress_default / LZ4_decompress_safe, src/buffer.c:181-183, 248-249;
 * ZSTD_compress(level 1) / ZSTD_decompress, :205, :264; compress2(level 1) /
 * uncompress, :193, :257), pthreads split by page range, one thread per core
 * of the process's affinity mask, best of R repetitions, every page
 * round-tripped and compared.  Pages come from the same generator as the GPU
 * bench (tyche_amd/csrc/pagegen.h, pages first..first+n-1 of the seed).
 *
 *   cpu_baseline <lz4|zstd|zlib> <pages> <page_len> <threads> [reps] [seed]
 *   prints one JSON line: compress / decompress GiB/s of uncompressed bytes
 *
 * Built by oracle/Makefile into oracle/_ref/ (linked against libtyche_ref.so);
 * never linked into the product library.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../tyche_amd/csrc/pagegen.h"

/* the reference's entry points (lz4.h:111-163, zstd.h:63-81, zlib.h:1161-1224) */
int LZ4_compress_default(const char *src, char *dst, int n, int cap);
int LZ4_decompress_safe(const char *src, char *dst, int n, int cap);
size_t ZSTD_compress(void *dst, size_t cap, const void *src, size_t n, int level);
size_t ZSTD_decompress(void *dst, size_t cap, const void *src, size_t n);
size_t ZSTD_compressBound(size_t n);
unsigned ZSTD_isError(size_t code);
int compress2(unsigned char *dst, unsigned long *dlen, const unsigned char *src, unsigned long n, int level);
int uncompress(unsigned char *dst, unsigned long *dlen, const unsigned char *src, unsigned long n);
unsigned long compressBound(unsigned long n);

enum { LZ4 = 1, ZLIB = 2, ZSTD = 3 };
static int g_codec;
static size_t g_n, g_plen, g_cap;
static uint8_t *g_in, *g_comp, *g_out;
static size_t *g_clen;
static uint64_t g_seed;
static int g_threads;
static pthread_barrier_t g_bar;
static double g_t[3];
static volatile long g_bad;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static size_t comp_page(const uint8_t *src, uint8_t *dst) {
    if (g_codec == LZ4) {
        int r = LZ4_compress_default((const char *)src, (char *)dst, (int)g_plen, (int)g_cap);
        return r > 0 ? (size_t)r : 0;
    }
    if (g_codec == ZSTD) {
        size_t r = ZSTD_compress(dst, g_cap, src, g_plen, 1);
        return ZSTD_isError(r) ? 0 : r;
    }
    unsigned long d = g_cap;
    return compress2(dst, &d, src, g_plen, 1) == 0 ? (size_t)d : 0;
}

static long dec_page(const uint8_t *src, size_t n, uint8_t *dst) {
    if (g_codec == LZ4) return LZ4_decompress_safe((const char *)src, (char *)dst, (int)n, (int)g_plen);
    if (g_codec == ZSTD) {
        size_t r = ZSTD_decompress(dst, g_plen, src, n);
        return ZSTD_isError(r) ? -1 : (long)r;
    }
    unsigned long d = g_plen;
    return uncompress(dst, &d, src, n) == 0 ? (long)d : -1;
}

static void *worker(void *arg) {
    const size_t t = (size_t)(uintptr_t)arg;
    const size_t a = t * g_n / (size_t)g_threads, b = (t + 1) * g_n / (size_t)g_threads;
    for (size_t i = a; i < b; i++) {   /* generate this thread's pages (first touch on its own node) */
        pg_page_t p;
        pg_page_init(&p, g_seed, i, (uint32_t)g_plen, 0);
        uint8_t *d = g_in + i * g_plen;
        for (size_t k = 0; k < g_plen; k++) d[k] = (uint8_t)pg_page_byte(&p, (uint32_t)k);
        memset(g_comp + i * g_cap, 0, g_cap);
        memset(g_out + i * g_plen, 0, g_plen);
    }
    pthread_barrier_wait(&g_bar);
    if (t == 0) g_t[0] = now_s();
    pthread_barrier_wait(&g_bar);
    for (size_t i = a; i < b; i++) g_clen[i] = comp_page(g_in + i * g_plen, g_comp + i * g_cap);
    pthread_barrier_wait(&g_bar);
    if (t == 0) g_t[1] = now_s();
    pthread_barrier_wait(&g_bar);
    for (size_t i = a; i < b; i++)
        if (dec_page(g_comp + i * g_cap, g_clen[i], g_out + i * g_plen) != (long)g_plen) __sync_fetch_and_add(&g_bad, 1);
    pthread_barrier_wait(&g_bar);
    if (t == 0) g_t[2] = now_s();
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s <lz4|zstd|zlib> <pages> <page_len> <threads> [reps] [seed]\n", argv[0]);
        return 2;
    }
    g_codec = !strcmp(argv[1], "zstd") ? ZSTD : !strcmp(argv[1], "zlib") ? ZLIB : LZ4;
    g_n = (size_t)atol(argv[2]);
    g_plen = (size_t)atol(argv[3]);
    g_threads = atoi(argv[4]);
    const int reps = argc > 5 ? atoi(argv[5]) : 3;
    g_seed = argc > 6 ? strtoull(argv[6], NULL, 10) : 20170303ull;
    if (g_threads < 1 || (size_t)g_threads > g_n) g_threads = g_n ? (int)g_n : 1;
    g_cap = g_codec == LZ4 ? g_plen + g_plen / 255 + 16 : g_codec == ZSTD ? ZSTD_compressBound(g_plen) : compressBound(g_plen);
    g_cap = (g_cap + 63) & ~(size_t)63;
    g_in = malloc(g_n * g_plen);
    g_comp = malloc(g_n * g_cap);
    g_out = malloc(g_n * g_plen);
    g_clen = calloc(g_n, sizeof(size_t));
    if (!g_in || !g_comp || !g_out || !g_clen) {
        fprintf(stderr, "out of memory\n");
        return 3;
    }
    double best_c = 1e30, best_d = 1e30;
    pthread_t *th = calloc((size_t)g_threads, sizeof(pthread_t));
    for (int r = 0; r < reps; r++) {
        pthread_barrier_init(&g_bar, NULL, (unsigned)g_threads);
        for (int t = 0; t < g_threads; t++) pthread_create(&th[t], NULL, worker, (void *)(uintptr_t)t);
        for (int t = 0; t < g_threads; t++) pthread_join(th[t], NULL);
        pthread_barrier_destroy(&g_bar);
        if (g_t[1] - g_t[0] < best_c) best_c = g_t[1] - g_t[0];
        if (g_t[2] - g_t[1] < best_d) best_d = g_t[2] - g_t[1];
    }
    size_t comp_bytes = 0;
    for (size_t i = 0; i < g_n; i++) comp_bytes += g_clen[i];
    const int same = memcmp(g_in, g_out, g_n * g_plen) == 0;
    const double gib = (double)(g_n * g_plen) / 1073741824.0;
    printf("{\"codec\": \"%s\", \"pages\": %zu, \"page_len\": %zu, \"threads\": %d, \"reps\": %d, "
           "\"compress_gib_s\": %.3f, \"decompress_gib_s\": %.3f, \"combined_gib_s\": %.3f, \"ratio\": %.4f, "
           "\"round_trip_ok\": %s}\n",
           argv[1], g_n, g_plen, g_threads, reps, gib / best_c, gib / best_d, gib / (best_c + best_d),
           comp_bytes ? (double)(g_n * g_plen) / (double)comp_bytes : 0.0, (same && !g_bad) ? "true" : "false");
    return (same && !g_bad) ? 0 : 1;
}
