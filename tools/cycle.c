/*
 * tools/cycle.c -- a tyche-shaped sweep/restore cycle in C over the C ABI
 * (include/tyche_codec.h), the way src/list.c would drive libtyche_codec.so
 * (INTEGRATION.md).  BASELINE configs[4] ("C5") in miniature on one GPU:
 *
 *   - N Buffers of mixed page sizes (8/16/32 KiB uniformly), synthetic
 *     PostgreSQL-like pages (tyche_amd/csrc/pagegen.h); each page carries a
 *     codec tag (a deliberate extension: the reference keeps one codec per
 *     List, src/list.c:169) -- LZ4 for most pages, zlib for every 4th;
 *   - sweep: victims go to the compressor in batches of 250
 *     (COMPRESSOR_BATCH_SIZE, src/list.h:57) through tyche_buffers_compress,
 *     and the compressed block is installed as list__update would
 *     (src/list.c:1058): data swapped, comp_length set, `compressed` flagged;
 *   - restore: T worker threads search with the hot-set bias of `-B 20,80`
 *     (80 % of picks among the first 20 % of ids, as intended by
 *     src/manager.c:320-333); a hit on a compressed page locks the buffer and
 *     restores it through tyche_buffer_restore (the coalescing queue), as
 *     list__search does (src/list.c:563-589);
 *   - afterwards every page (restored during the run, or restored now through
 *     the direct path) is compared with a regenerated copy.
 *
 *   build: see __graft_entry__.build() (gcc, links tyche_amd/libtyche_codec.so)
 *   run:   tools/bin/cycle [buffers] [threads] [restores_per_thread]
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/tyche_codec.h"
#include "../tyche_amd/csrc/pagegen.h"

#define BATCH 250
#define SEED 20170303ull

static size_t g_n;
static Buffer **g_bufs;
static int *g_codec;
static long g_restores;
static volatile long g_bad, g_hits, g_restored, g_restored_bytes;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint64_t splitmix(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint32_t page_len_of(size_t i) {
    uint64_t s = SEED ^ (i * 7919u);
    return 8192u << (splitmix(&s) % 3u);
}

static void fill_page(uint8_t *d, size_t i, uint32_t len) {
    pg_page_t p;
    pg_page_init(&p, SEED, i, len, 0);
    for (uint32_t b = 0; b < len; b++) d[b] = (uint8_t)pg_page_byte(&p, b);
}

static void *restorer(void *arg) {
    uint64_t rng = SEED + (uint64_t)(uintptr_t)arg * 1000003u;
    const size_t hot = g_n / 5 ? g_n / 5 : 1;
    for (long k = 0; k < g_restores; k++) {
        const uint64_t r = splitmix(&rng);
        const size_t id = (r % 100u) < 80u ? (size_t)((r >> 8) % hot) : hot + (size_t)((r >> 8) % (g_n - hot ? g_n - hot : 1));
        if (id >= g_n) continue;
        Buffer *b = g_bufs[id];
        buffer__lock(b);
        if (b->flags & compressed) {
            int st = tyche_buffer_restore(b, g_codec[id]);
            if (st == TYCHE_E_OK) {
                b->flags &= ~compressed;
                __sync_fetch_and_add(&g_restored, 1);
                __sync_fetch_and_add(&g_restored_bytes, (long)b->data_length);
            } else if (st != TYCHE_E_BUFFER_ALREADY_DECOMPRESSED) {
                __sync_fetch_and_add(&g_bad, 1);
            }
        }
        __sync_fetch_and_add(&g_hits, 1);
        buffer__unlock(b);
    }
    return NULL;
}

int main(int argc, char **argv) {
    g_n = argc > 1 ? (size_t)atol(argv[1]) : 65536;
    const int threads = argc > 2 ? atoi(argv[2]) : 16;
    g_restores = argc > 3 ? atol(argv[3]) : 20000;
    if (tyche_device_ready() != 1) {
        fprintf(stderr, "no gfx950 device: %s\n", tyche_last_error());
        return 2;
    }
    g_bufs = calloc(g_n, sizeof(Buffer *));
    g_codec = calloc(g_n, sizeof(int));
    size_t raw_bytes = 0;
    for (size_t i = 0; i < g_n; i++) {
        const uint32_t len = page_len_of(i);
        uint8_t *d = malloc(len);
        fill_page(d, i, len);
        if (buffer__initialize(&g_bufs[i], (bufferid_t)i, len, d, NULL) != TYCHE_E_OK) return 3;
        g_codec[i] = (i % 4u == 3u) ? TYCHE_ZLIB_COMPRESSOR_ID : TYCHE_LZ4_COMPRESSOR_ID;
        raw_bytes += len;
    }
    /* ---- sweep: every page becomes a victim once, 250 per compressor batch */
    const double t0 = now_s();
    size_t comp_bytes = 0, fails = 0;
    Buffer *vict[BATCH];
    void *out[BATCH];
    int st[BATCH];
    for (int codec = TYCHE_LZ4_COMPRESSOR_ID; codec <= TYCHE_ZLIB_COMPRESSOR_ID; codec++) {
        size_t k = 0;
        for (size_t i = 0; i <= g_n; i++) {
            if (i < g_n && g_codec[i] == codec) vict[k++] = g_bufs[i];
            if (k == BATCH || (i == g_n && k)) {
                tyche_buffers_compress(vict, out, st, k, codec, 1);
                for (size_t j = 0; j < k; j++) {
                    if (st[j] != TYCHE_E_OK) { fails++; continue; }
                    free(vict[j]->data);          /* list__update installs the compressed copy */
                    vict[j]->data = out[j];
                    vict[j]->flags |= compressed;
                    comp_bytes += vict[j]->comp_length;
                }
                k = 0;
            }
        }
    }
    const double t1 = now_s();
    /* ---- restore: biased searches from worker threads through the queue */
    tyche_restore_queue_start(1024, 100);
    pthread_t th[256];
    const int nt = threads < 256 ? threads : 256;
    for (int t = 0; t < nt; t++) pthread_create(&th[t], NULL, restorer, (void *)(uintptr_t)t);
    for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
    tyche_restore_queue_stop();
    const double t2 = now_s();
    uint64_t batches = 0, served = 0;
    tyche_restore_queue_stats(&batches, &served);
    size_t still = 0;
    uint8_t *ref = malloc(32768);
    for (size_t i = 0; i < g_n; i++) {
        Buffer *b = g_bufs[i];
        if (b->flags & compressed) {
            still++;
            if (tyche_buffer_restore(b, g_codec[i]) != TYCHE_E_OK) { g_bad++; continue; }
            b->flags &= ~compressed;
        }
        fill_page(ref, i, b->data_length);
        if (memcmp(ref, b->data, b->data_length) != 0) g_bad++;
    }
    free(ref);
    const size_t restored_bytes = (size_t)g_restored_bytes;
    printf("{\"buffers\": %zu, \"raw_gib\": %.3f, \"ratio\": %.3f, \"sweep_fails\": %zu, "
           "\"sweep_s\": %.3f, \"sweep_gib_s\": %.3f, \"restore_threads\": %d, \"searches\": %ld, "
           "\"restored\": %ld, \"restore_s\": %.3f, \"restore_gib_s\": %.3f, \"queue_batches\": %llu, "
           "\"queue_buffers\": %llu, \"mismatches\": %ld, \"still_compressed\": %zu}\n",
           g_n, raw_bytes / 1073741824.0, comp_bytes ? (double)raw_bytes / (double)comp_bytes : 0.0, fails, t1 - t0,
           raw_bytes / 1073741824.0 / (t1 - t0), nt, g_hits, g_restored, t2 - t1,
           restored_bytes / 1073741824.0 / (t2 - t1), (unsigned long long)batches, (unsigned long long)served, g_bad,
           still);
    for (size_t i = 0; i < g_n; i++) buffer__destroy(g_bufs[i], true);
    free(g_bufs);
    free(g_codec);
    return (g_bad || fails) ? 1 : 0;
}
