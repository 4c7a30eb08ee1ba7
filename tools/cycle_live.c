/*
 * tools/cycle_live.c -- BASELINE configs[4] ("C5") as a live cycle over the C ABI:
 * the sweeper and the restorers run AT THE SAME TIME, the way tyche's list code
 * drives its codec (src/list.c).  tools/cycle.c runs the two sides one after the
 * other; this harness interleaves them under a raw-memory budget.
 *
 *   - N Buffers of mixed page sizes (8/16/32 KiB uniformly), synthetic
 *     PostgreSQL-like pages (tyche_amd/csrc/pagegen.h).  The data set starts
 *     compressed with zlib (a page store whose pages arrive deflated); a page
 *     the sweeper compresses again gets LZ4 -- "zlib inflate + lz4 deflate":
 *     restores inflate zlib pages and decode LZ4 pages, sweeps always encode
 *     LZ4.  Each Buffer carries its codec tag (the reference keeps one codec
 *     per List, list.c:169: a deliberate extension).
 *   - restorers (T threads, list__search's restore block, list.c:563-589): pick
 *     ids with the hot-set bias of `-B 20,80` as intended (80 % of picks among
 *     the first 20 % of ids; manager.c:286-333 without the cold-range
 *     underflow of manager.c:329), bump the buffer's popularity, and restore a
 *     compressed hit under the buffer's lock through tyche_buffer_restore (the
 *     coalescing queue); raw bytes grow.
 *   - the sweeper (one thread, list__sweep, list.c:782-891): whenever raw bytes
 *     exceed the budget it sets goal = overflow + 5 % of the budget (:789,
 *     sweep_goal 5), runs the clock (:795-816: skip pending and compressed
 *     buffers, halve the popularity of popular ones, take unpopular raw ones),
 *     and flushes its victims to the compressor pool every 1,000 victims or
 *     when the goal is met (:824-838), waiting for the pool to drain.
 *   - the compressor pool (C threads, list__compressor_start, list.c:996-1066):
 *     takes up to 250 victims per call (list.h:57) and compresses them with ONE
 *     tyche_buffers_compress call (the batch extension of list.c:1051), then
 *     installs each result under the buffer's lock (list__update's swap,
 *     :1058-1060).
 *   - afterwards every page is restored (if still compressed) and compared
 *     with a regenerated copy.
 *
 *   run: tools/bin/cycle_live [buffers] [restorers] [restores_per_thread] [compressors] [raw_budget_pct] [seconds]
 *   seconds > 0: a sustained cycle -- the restorers search until that much wall time has passed
 *   (restores_per_thread then only sets the minimum); the JSON line adds histograms of the
 *   compressor pool's batch sizes, the sweeper's flush sizes and the restore queue's launches.
 *   The engine spreads work over every visible GPU (TYCHE_DEVICE_IDS=0,0 rehearses
 *   the fan-out on one).  Prints one JSON line.
 */
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../include/tyche_codec.h"
#include "../tyche_amd/csrc/pagegen.h"

#define COMP_BATCH 250       /* COMPRESSOR_BATCH_SIZE, list.h:57 */
#define VICTIM_BATCH 1000    /* VICTIM_BATCH_SIZE, list.h:56 */
#define SWEEP_GOAL 5         /* list.c:113 */
#define SEED 20170303ull
#define pending_sweep_flag (1 << 1)

static size_t g_n;
static Buffer **g_bufs;
static volatile int *g_codec;
static long g_restores;
static int64_t g_max_raw;
static volatile int64_t g_raw;             /* raw bytes resident (atomic) */
static volatile long g_bad, g_hits, g_restored, g_restored_bytes, g_restored_zlib, g_restored_lz4;
static volatile long g_swept, g_swept_bytes, g_comp_fails, g_sweeps, g_flushes;
static volatile int g_done;
static double g_deadline;                  /* > 0: restorers search until this time (sustained mode) */
/* power-of-two histograms: compressor-pool call sizes and sweeper flush sizes */
#define HB 11
static volatile long g_comp_hist[HB], g_flush_hist[HB];
static int hbucket(size_t k) {
    int b = 0;
    while ((k >>= 1) && b < HB - 1) b++;
    return b;
}

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

/* ---- the compressor pool: victims[] filled by the sweeper, drained in batches of <= 250 */
static Buffer **g_victims;
static size_t g_vict_n, g_vict_next;
static int g_active;
static pthread_mutex_t g_jobs_lock = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_jobs_cond = PTHREAD_COND_INITIALIZER, g_parent_cond = PTHREAD_COND_INITIALIZER;

static void *compressor(void *arg) {
    (void)arg;
    Buffer *vict[COMP_BATCH];
    void *out[COMP_BATCH];
    int st[COMP_BATCH];
    for (;;) {
        pthread_mutex_lock(&g_jobs_lock);
        while (!g_done && g_vict_next >= g_vict_n) pthread_cond_wait(&g_jobs_cond, &g_jobs_lock);
        if (g_vict_next >= g_vict_n) {   /* done and nothing left */
            pthread_mutex_unlock(&g_jobs_lock);
            return NULL;
        }
        size_t k = 0;
        while (k < COMP_BATCH && g_vict_next < g_vict_n) vict[k++] = g_victims[g_vict_next++];
        g_active++;
        pthread_mutex_unlock(&g_jobs_lock);
        __sync_fetch_and_add(&g_comp_hist[hbucket(k)], 1);
        if (tyche_buffers_compress(vict, out, st, k, TYCHE_LZ4_COMPRESSOR_ID, 1) != TYCHE_E_OK)
            for (size_t j = 0; j < k; j++) st[j] = TYCHE_E_DEVICE;
        for (size_t j = 0; j < k; j++) {
            Buffer *b = vict[j];
            if (st[j] != TYCHE_E_OK) {   /* INTEGRATION.md's caller rule: the page stays raw */
                __sync_fetch_and_add(&g_comp_fails, 1);
                continue;
            }
            buffer__lock(b);             /* list__update's swap (list.c:1058-1060) */
            free(b->data);
            b->data = out[j];
            g_codec[b->id] = TYCHE_LZ4_COMPRESSOR_ID;
            b->flags |= compressed;
            __sync_fetch_and_add(&g_raw, -(int64_t)b->data_length);
            __sync_fetch_and_add(&g_swept, 1);
            __sync_fetch_and_add(&g_swept_bytes, (long)b->data_length);
            buffer__unlock(b);
        }
        pthread_mutex_lock(&g_jobs_lock);
        g_active--;
        pthread_cond_broadcast(&g_parent_cond);
        pthread_mutex_unlock(&g_jobs_lock);
    }
}

/* hand the collected victims to the pool and wait until it has installed them (list.c:824-838) */
static void clear_pending(size_t nv) {
    for (size_t j = 0; j < nv; j++) {
        buffer__lock(g_victims[j]);
        g_victims[j]->flags &= ~pending_sweep_flag;
        buffer__unlock(g_victims[j]);
    }
}
static void flush_victims(size_t nv) {
    __sync_fetch_and_add(&g_flush_hist[hbucket(nv)], 1);
    pthread_mutex_lock(&g_jobs_lock);
    g_vict_n = nv;
    g_vict_next = 0;
    pthread_cond_broadcast(&g_jobs_cond);
    while (g_active > 0 || g_vict_next < g_vict_n) pthread_cond_wait(&g_parent_cond, &g_jobs_lock);
    g_vict_n = g_vict_next = 0;
    pthread_mutex_unlock(&g_jobs_lock);
    __sync_fetch_and_add(&g_flushes, 1);
}

static void *sweeper(void *arg) {
    (void)arg;
    size_t hand = 0;
    while (!g_done) {
        const int64_t raw = g_raw;
        if (raw <= g_max_raw) {
            usleep(100);
            continue;
        }
        const int64_t need = (raw - g_max_raw) + g_max_raw * SWEEP_GOAL / 100;   /* list.c:789 */
        int64_t freed = 0;
        size_t nv = 0, scanned = 0;
        while (freed < need && scanned < 8 * g_n && !g_done) {
            hand = (hand + 1) % g_n;
            scanned++;
            Buffer *b = g_bufs[hand];
            buffer__lock(b);                 /* flags and popularity change under the buffer's lock here */
            if (b->popularity) {             /* list.c:815: halve, move on */
                b->popularity >>= 1;
                buffer__unlock(b);
                continue;
            }
            if (b->flags & (compressed | pending_sweep_flag)) {
                buffer__unlock(b);
                continue;
            }
            b->flags |= pending_sweep_flag;
            buffer__unlock(b);
            g_victims[nv++] = b;
            freed += b->data_length;
            if (nv == VICTIM_BATCH || freed >= need) {
                flush_victims(nv);
                clear_pending(nv);
                nv = 0;
            }
        }
        if (nv) {
            flush_victims(nv);
            clear_pending(nv);
        }
        __sync_fetch_and_add(&g_sweeps, 1);
    }
    return NULL;
}

#define MIN_LZ4_RESTORES 16
static void *restorer(void *arg) {
    uint64_t rng = SEED + (uint64_t)(uintptr_t)arg * 1000003u;
    const size_t hot = g_n / 5 ? g_n / 5 : 1;
    /* each restorer makes g_restores searches, and more (up to 8x) until the run has restored
     * MIN_LZ4_RESTORES pages that the sweeper compressed during it: a short run's searches can
     * otherwise all end before the cold pages the sweeps hit come back */
    for (long k = 0; k < g_restores || (g_deadline > 0 ? now_s() < g_deadline
                                                        : (g_restored_lz4 < MIN_LZ4_RESTORES && k < 8 * g_restores));
         k++) {
        const uint64_t r = splitmix(&rng);
        const size_t id = (r % 100u) < 80u ? (size_t)((r >> 8) % hot) : hot + (size_t)((r >> 8) % (g_n - hot ? g_n - hot : 1));
        if (id >= g_n) continue;
        Buffer *b = g_bufs[id];
        buffer__lock(b);
        if (b->popularity < 255) b->popularity++;   /* the reference never bumps it */
        if (b->flags & compressed) {
            const int codec = g_codec[id];
            const int st = tyche_buffer_restore(b, codec);
            if (st == TYCHE_E_OK) {
                b->flags &= ~compressed;
                __sync_fetch_and_add(&g_raw, (int64_t)b->data_length);
                __sync_fetch_and_add(&g_restored, 1);
                __sync_fetch_and_add(&g_restored_bytes, (long)b->data_length);
                __sync_fetch_and_add(codec == TYCHE_ZLIB_COMPRESSOR_ID ? &g_restored_zlib : &g_restored_lz4, 1);
            } else if (st != TYCHE_E_BUFFER_ALREADY_DECOMPRESSED) {
                __sync_fetch_and_add(&g_bad, 1);
            }
        }
        __sync_fetch_and_add(&g_hits, 1);
        buffer__unlock(b);
    }
    return NULL;
}

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
    const int nr = argc > 2 ? atoi(argv[2]) : 64;
    g_restores = argc > 3 ? atol(argv[3]) : 4000;
    const int ncomp = argc > 4 ? atoi(argv[4]) : 16;
    const int budget_pct = argc > 5 ? atoi(argv[5]) : 25;
    const double seconds = argc > 6 ? atof(argv[6]) : 0.0;
    if (tyche_device_ready() != 1) {
        fprintf(stderr, "no gfx950 device: %s\n", tyche_last_error());
        return 2;
    }
    g_bufs = calloc(g_n, sizeof(Buffer *));
    g_codec = calloc(g_n, sizeof(int));
    g_victims = calloc(VICTIM_BATCH, sizeof(Buffer *));
    size_t total = 0;
    for (size_t i = 0; i < g_n; i++) {
        const uint32_t len = page_len_of(i);
        uint8_t *d = malloc(len);
        fill_page(d, i, len);
        if (buffer__initialize(&g_bufs[i], (bufferid_t)i, len, d, NULL) != TYCHE_E_OK) return 3;
        total += len;
    }
    /* ---- the data set arrives deflated: every page zlib-compressed (untimed setup) */
    const double ts = now_s();
    for (size_t a = 0; a < g_n; a += 4096) {
        const size_t k = g_n - a < 4096 ? g_n - a : 4096;
        void **out = calloc(k, sizeof(void *));
        int *st = calloc(k, sizeof(int));
        if (tyche_buffers_compress(g_bufs + a, out, st, k, TYCHE_ZLIB_COMPRESSOR_ID, 1) != TYCHE_E_OK) {
            fprintf(stderr, "setup compress failed: %s\n", tyche_last_error());
            return 4;
        }
        for (size_t j = 0; j < k; j++) {
            if (st[j] != TYCHE_E_OK) return 5;
            Buffer *b = g_bufs[a + j];
            free(b->data);
            b->data = out[j];
            b->flags |= compressed;
            g_codec[a + j] = TYCHE_ZLIB_COMPRESSOR_ID;
        }
        free(out);
        free(st);
    }
    const double setup_s = now_s() - ts;
    g_raw = 0;
    g_max_raw = (int64_t)(total * (size_t)budget_pct / 100u);

    /* ---- the live cycle */
    tyche_restore_queue_start(1024, getenv("CYCLE_WAIT_US") ? atoi(getenv("CYCLE_WAIT_US")) : 100);
    pthread_t cth[256], sth, rth[1024];
    const int nc = ncomp < 1 ? 1 : ncomp < 256 ? ncomp : 256;
    const int nt = nr < 1 ? 1 : nr < 1024 ? nr : 1024;
    const double t0 = now_s();
    if (seconds > 0) g_deadline = t0 + seconds;
    for (int t = 0; t < nc; t++) pthread_create(&cth[t], NULL, compressor, NULL);
    pthread_create(&sth, NULL, sweeper, NULL);
    for (int t = 0; t < nt; t++) pthread_create(&rth[t], NULL, restorer, (void *)(uintptr_t)t);
    for (int t = 0; t < nt; t++) pthread_join(rth[t], NULL);
    const double t1 = now_s();
    g_done = 1;
    pthread_join(sth, NULL);
    pthread_mutex_lock(&g_jobs_lock);
    pthread_cond_broadcast(&g_jobs_cond);
    pthread_mutex_unlock(&g_jobs_lock);
    for (int t = 0; t < nc; t++) pthread_join(cth[t], NULL);
    tyche_restore_queue_stop();
    uint64_t batches = 0, served = 0, qhist[HB] = {0};
    tyche_restore_queue_stats(&batches, &served);
    tyche_restore_queue_hist(qhist, HB);

    /* ---- verify every page */
    size_t still = 0;
    uint8_t *ref = malloc(32768);
    for (size_t i = 0; i < g_n; i++) {
        Buffer *b = g_bufs[i];
        if (b->flags & compressed) {
            still++;
            if (buffer__decompress(b, g_codec[i]) != TYCHE_E_OK) { g_bad++; continue; }
            b->flags &= ~compressed;
        }
        fill_page(ref, i, b->data_length);
        if (memcmp(ref, b->data, b->data_length) != 0) g_bad++;
    }
    free(ref);
    const double run = t1 - t0;
    printf("{\"buffers\": %zu, \"devices\": %d, \"raw_gib\": %.3f, \"raw_budget_pct\": %d, \"setup_zlib_s\": %.3f, "
           "\"restorers\": %d, \"compressors\": %d, \"searches\": %ld, \"run_s\": %.3f, "
           "\"restored\": %ld, \"restored_zlib\": %ld, \"restored_lz4\": %ld, \"restore_gib_s\": %.3f, "
           "\"swept\": %ld, \"sweep_gib_s\": %.3f, \"sweeps\": %ld, \"flushes\": %ld, \"sweep_fails\": %ld, "
           "\"queue_batches\": %llu, \"queue_buffers\": %llu, \"mismatches\": %ld, \"still_compressed\": %zu}\n",
           g_n, tyche_active_devices(), total / 1073741824.0, budget_pct, setup_s, nt, nc, g_hits, run, g_restored,
           g_restored_zlib, g_restored_lz4, g_restored_bytes / 1073741824.0 / run, g_swept,
           g_swept_bytes / 1073741824.0 / run, g_sweeps, g_flushes, g_comp_fails, (unsigned long long)batches,
           (unsigned long long)served, g_bad, still);
    if (seconds > 0) {   /* the histograms, bucket k = sizes 2^k .. 2^(k+1)-1, as a second JSON line */
        printf("{\"hist_buckets\": \"2^k..2^(k+1)-1\", \"compress_call_sizes\": [");
        for (int i = 0; i < HB; i++) printf("%s%ld", i ? ", " : "", g_comp_hist[i]);
        printf("], \"sweep_flush_sizes\": [");
        for (int i = 0; i < HB; i++) printf("%s%ld", i ? ", " : "", g_flush_hist[i]);
        printf("], \"restore_launch_sizes\": [");
        for (int i = 0; i < HB; i++) printf("%s%llu", i ? ", " : "", (unsigned long long)qhist[i]);
        printf("]}\n");
    }
    for (size_t i = 0; i < g_n; i++) buffer__destroy(g_bufs[i], true);
    return (g_bad || g_comp_fails) ? 1 : 0;
}
