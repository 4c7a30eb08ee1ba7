/*
 * tools/cycle.c -- a tyche-shaped sweep/restore cycle in C over the C ABI
 * (include/tyche_codec.h), the way src/list.c would drive libtyche_codec.so
 * (INTEGRATION.md).  BASELINE configs[4] ("C5") in miniature on one GPU:
 *
 *   - N Buffers of mixed page sizes (8/16/32 KiB uniformly), synthetic
 *     PostgreSQL-like pages (tyche_amd/csrc/pagegen.h); each page carries a
 *     codec tag (a deliberate extension: the reference keeps one codec per
 *     List, src/list.c:169) -- LZ4 for most pages, zlib for every 4th;
 *   - sweep: victims go to a pool of compressor threads (list.c:142-168's
 *     pool, opts.cpu_count of them there) that take batches of 250
 *     (COMPRESSOR_BATCH_SIZE, src/list.h:57, taken under jobs_lock as in
 *     list.c:1039-1045) through tyche_buffers_compress, and the compressed
 *     block is installed as list__update would (src/list.c:1058): data
 *     swapped, comp_length set, `compressed` flagged;
 *   - restore: T worker threads search with the hot-set bias of `-B 20,80`
 *     (80 % of picks among the first 20 % of ids, as intended by
 *     src/manager.c:320-333); a hit on a compressed page locks the buffer and
 *     restores it through tyche_buffer_restore (the coalescing queue), as
 *     list__search does (src/list.c:563-589);
 *   - afterwards every page (restored during the run, or restored now through
 *     the direct path) is compared with a regenerated copy.
 *
 *   build: see __graft_entry__.build() (gcc, links tyche_amd/libtyche_codec.so)
 *   run:   tools/bin/cycle [buffers] [restore_threads] [restores_per_thread] [compressor_threads]
 *   The engine spreads the work over every visible GPU (or TYCHE_DEVICE_IDS /
 *   TYCHE_DEVICES), so one process drives all of them, as tyche would.
 */
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>
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

static size_t *g_order;                 /* victims, grouped by codec */
static size_t g_next;                   /* next victim to hand out; under g_jobs_lock */
static pthread_mutex_t g_jobs_lock = PTHREAD_MUTEX_INITIALIZER;
static volatile long g_comp_bytes, g_fails;

/* a compressor-pool thread: takes up to BATCH same-codec victims at a time (list.c:1039-1045) */
static void *compressor(void *arg) {
    (void)arg;
    Buffer *vict[BATCH];
    void *out[BATCH];
    int st[BATCH];
    for (;;) {
        size_t a, k = 0;
        pthread_mutex_lock(&g_jobs_lock);
        a = g_next;
        while (a + k < g_n && k < BATCH && g_codec[g_order[a + k]] == g_codec[g_order[a]]) k++;
        g_next = a + k;
        pthread_mutex_unlock(&g_jobs_lock);
        if (k == 0) return NULL;
        const int codec = g_codec[g_order[a]];
        for (size_t j = 0; j < k; j++) vict[j] = g_bufs[g_order[a + j]];
        tyche_buffers_compress(vict, out, st, k, codec, 1);
        for (size_t j = 0; j < k; j++) {
            if (st[j] != TYCHE_E_OK) { __sync_fetch_and_add(&g_fails, 1); continue; }
            free(vict[j]->data);          /* list__update installs the compressed copy */
            vict[j]->data = out[j];
            vict[j]->flags |= compressed;
            __sync_fetch_and_add(&g_comp_bytes, (long)vict[j]->comp_length);
        }
    }
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

/* a crash names its frames (the harness is linked with -rdynamic) */
static void on_fault(int sig) {
    static const char msg[] = "\n*** fatal signal; backtrace:\n";
    void *bt[64];
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(bt, backtrace(bt, 64), 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int main(int argc, char **argv) {
    signal(SIGSEGV, on_fault);
    signal(SIGABRT, on_fault);
    g_n = argc > 1 ? (size_t)atol(argv[1]) : 65536;
    const int threads = argc > 2 ? atoi(argv[2]) : 16;
    g_restores = argc > 3 ? atol(argv[3]) : 20000;
    const int comp_threads = argc > 4 ? atoi(argv[4]) : 16;
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
    /* ---- sweep: every page becomes a victim once; victims grouped by codec, 250 per compressor batch */
    g_order = malloc(g_n * sizeof(size_t));
    size_t m = 0;
    for (int codec = TYCHE_LZ4_COMPRESSOR_ID; codec <= TYCHE_ZLIB_COMPRESSOR_ID; codec++)
        for (size_t i = 0; i < g_n; i++)
            if (g_codec[i] == codec) g_order[m++] = i;
    const double t0 = now_s();
    pthread_t cth[256];
    const int nc = comp_threads < 1 ? 1 : comp_threads < 256 ? comp_threads : 256;
    for (int t = 0; t < nc; t++) pthread_create(&cth[t], NULL, compressor, NULL);
    for (int t = 0; t < nc; t++) pthread_join(cth[t], NULL);
    const double t1 = now_s();
    const size_t comp_bytes = (size_t)g_comp_bytes, fails = (size_t)g_fails;
    /* ---- restore: biased searches from worker threads through the queue */
    tyche_restore_queue_start(1024, getenv("CYCLE_WAIT_US") ? atoi(getenv("CYCLE_WAIT_US")) : 100);
    pthread_t th[1024];
    const int nt = threads < 1024 ? threads : 1024;
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
    printf("{\"buffers\": %zu, \"devices\": %d, \"compressor_threads\": %d, \"raw_gib\": %.3f, \"ratio\": %.3f, "
           "\"sweep_fails\": %zu, \"sweep_s\": %.3f, \"sweep_gib_s\": %.3f, \"restore_threads\": %d, \"searches\": %ld, "
           "\"restored\": %ld, \"restore_s\": %.3f, \"restore_gib_s\": %.3f, \"queue_batches\": %llu, "
           "\"queue_buffers\": %llu, \"mismatches\": %ld, \"still_compressed\": %zu}\n",
           g_n, tyche_active_devices(), nc, raw_bytes / 1073741824.0, comp_bytes ? (double)raw_bytes / (double)comp_bytes : 0.0, fails, t1 - t0,
           raw_bytes / 1073741824.0 / (t1 - t0), nt, g_hits, g_restored, t2 - t1,
           restored_bytes / 1073741824.0 / (t2 - t1), (unsigned long long)batches, (unsigned long long)served, g_bad,
           still);
    for (size_t i = 0; i < g_n; i++) buffer__destroy(g_bufs[i], true);
    free(g_bufs);
    free(g_codec);
    free(g_order);
    return (g_bad || fails) ? 1 : 0;
}
