/*
 * tools/stress.c -- many concurrent callers of the drop-in Buffer API
 * (include/tyche_codec.h) with no batching of their own: each thread loops
 * buffer__compress -> install (as list__update would, src/list.c:1058) ->
 * buffer__decompress on pages of 8/16/32 KiB with LZ4, zlib and zstd, and
 * compares every restored page with a regenerated copy.
 *
 * tyche calls the codec exactly like this from opts.cpu_count compressor
 * threads (src/list.c:142-168, 1051; 256 on a 2-socket EPYC host) plus its
 * workers (src/list.c:572).  With more threads than the engine's staging
 * contexts and far more launches in flight than any fixed ring of work
 * counters, this checks that no launch's page claims ever alias another's
 * (engine.h: WorkCounter) and that the shared staging contexts never mix up
 * calls.
 *
 *   run: tools/bin/stress [threads] [iterations_per_thread]
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

#define SEED 20170303ull

static long g_iters;
static volatile long g_bad, g_err, g_ops;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void fill_page(uint8_t *d, uint64_t i, uint32_t len) {
    pg_page_t p;
    pg_page_init(&p, SEED, i, len, 0);
    for (uint32_t b = 0; b < len; b++) d[b] = (uint8_t)pg_page_byte(&p, b);
}

static void *worker(void *arg) {
    const uint64_t tid = (uint64_t)(uintptr_t)arg;
    uint8_t *ref = malloc(32768);
    for (long k = 0; k < g_iters; k++) {
        const uint64_t idx = tid * 1000003ull + (uint64_t)k;
        const uint32_t len = 8192u << (idx % 3u);
        const int codec = 1 + (int)((idx / 3u) % 3u);
        uint8_t *d = malloc(len);
        fill_page(d, idx, len);
        Buffer *b = NULL;
        if (buffer__initialize(&b, (bufferid_t)idx, len, d, NULL) != TYCHE_E_OK) { __sync_fetch_and_add(&g_err, 1); free(d); continue; }
        void *comp = NULL;
        int rc = buffer__compress(b, &comp, codec, 1);
        if (rc != TYCHE_E_OK) {
            fprintf(stderr, "compress rc %d: %s\n", rc, tyche_last_error());
            __sync_fetch_and_add(&g_err, 1);
            buffer__destroy(b, true);
            continue;
        }
        free(b->data);
        b->data = comp;
        rc = buffer__decompress(b, codec);
        if (rc != TYCHE_E_OK) {
            fprintf(stderr, "decompress rc %d: %s\n", rc, tyche_last_error());
            __sync_fetch_and_add(&g_err, 1);
        } else {
            fill_page(ref, idx, len);
            if (b->comp_length != 0 || b->data_length != len || memcmp(ref, b->data, len) != 0) __sync_fetch_and_add(&g_bad, 1);
        }
        __sync_fetch_and_add(&g_ops, 1);
        buffer__destroy(b, true);
    }
    free(ref);
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
    const int threads = argc > 1 ? atoi(argv[1]) : 300;
    g_iters = argc > 2 ? atol(argv[2]) : 8;
    if (tyche_device_ready() != 1) {
        fprintf(stderr, "no gfx950 device: %s\n", tyche_last_error());
        return 2;
    }
    pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
    const double t0 = now_s();
    int started = 0;
    for (int t = 0; t < threads; t++)
        if (pthread_create(&th[t], NULL, worker, (void *)(uintptr_t)t) == 0) started++;
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
    const double t1 = now_s();
    printf("{\"threads\": %d, \"devices\": %d, \"round_trips\": %ld, \"mismatches\": %ld, \"errors\": %ld, "
           "\"seconds\": %.3f}\n", started, tyche_active_devices(), g_ops, g_bad, g_err, t1 - t0);
    free(th);
    return (g_bad || g_err || started != threads) ? 1 : 0;
}
