/*
 * tools/latency.c -- latency of one host batch through the Buffer API
 * (tyche_buffers_decompress / tyche_buffers_compress), the restore and sweep
 * calls of src/list.c:572 and :1051, for a few batch sizes and codecs.
 * Prints one JSON line per (codec, page size, batch): median / p90 microseconds
 * per call over `reps` calls, pages verified.
 *   run: tools/bin/latency [reps]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/tyche_codec.h"
#include "../tyche_amd/csrc/pagegen.h"

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return 1e6 * (double)t.tv_sec + 1e-3 * (double)t.tv_nsec;
}
static int cmpd(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 40;
    if (tyche_device_ready() != 1) {
        fprintf(stderr, "no gfx950 device: %s\n", tyche_last_error());
        return 2;
    }
    const int codecs[3] = {TYCHE_LZ4_COMPRESSOR_ID, TYCHE_ZLIB_COMPRESSOR_ID, TYCHE_ZSTD_COMPRESSOR_ID};
    const char *names[4] = {"none", "lz4", "zlib", "zstd"};
    const uint32_t lens[2] = {16384, 32768};
    const int batches[4] = {1, 8, 64, 512};
    double *t_c = malloc(sizeof(double) * (size_t)reps), *t_d = malloc(sizeof(double) * (size_t)reps);
    int bad = 0;
    for (int ci = 0; ci < 3; ci++)
        for (int li = 0; li < 2; li++)
            for (int bi = 0; bi < 4; bi++) {
                const int n = batches[bi];
                const uint32_t len = lens[li];
                Buffer **bufs = calloc((size_t)n, sizeof(Buffer *));
                void **out = calloc((size_t)n, sizeof(void *));
                int *st = calloc((size_t)n, sizeof(int));
                uint8_t *ref = malloc(len);
                for (int r = 0; r < reps; r++) {
                    for (int i = 0; i < n; i++) {
                        uint8_t *d = malloc(len);
                        pg_page_t p;
                        pg_page_init(&p, 20170303ull, (uint64_t)i, len, 0);
                        for (uint32_t k = 0; k < len; k++) d[k] = (uint8_t)pg_page_byte(&p, k);
                        buffer__initialize(&bufs[i], (bufferid_t)i, len, d, NULL);
                    }
                    double t0 = now_us();
                    tyche_buffers_compress(bufs, out, st, (size_t)n, codecs[ci], 1);
                    double t1 = now_us();
                    for (int i = 0; i < n; i++) {
                        if (st[i] != TYCHE_E_OK) { bad++; continue; }
                        free(bufs[i]->data);
                        bufs[i]->data = out[i];
                    }
                    double t2 = now_us();
                    tyche_buffers_decompress(bufs, st, (size_t)n, codecs[ci]);
                    double t3 = now_us();
                    for (int i = 0; i < n; i++) {
                        pg_page_t p;
                        pg_page_init(&p, 20170303ull, (uint64_t)i, len, 0);
                        for (uint32_t k = 0; k < len; k++) ref[k] = (uint8_t)pg_page_byte(&p, k);
                        if (st[i] != TYCHE_E_OK || memcmp(ref, bufs[i]->data, len) != 0) bad++;
                        buffer__destroy(bufs[i], true);
                    }
                    t_c[r] = t1 - t0;
                    t_d[r] = t3 - t2;
                }
                qsort(t_c, (size_t)reps, sizeof(double), cmpd);
                qsort(t_d, (size_t)reps, sizeof(double), cmpd);
                printf("{\"codec\": \"%s\", \"page_len\": %u, \"batch\": %d, \"compress_us_p50\": %.1f, "
                       "\"compress_us_p90\": %.1f, \"decompress_us_p50\": %.1f, \"decompress_us_p90\": %.1f}\n",
                       names[codecs[ci]], len, n, t_c[reps / 2], t_c[reps * 9 / 10], t_d[reps / 2], t_d[reps * 9 / 10]);
                fflush(stdout);
                free(bufs);
                free(out);
                free(st);
                free(ref);
            }
    free(t_c);
    free(t_d);
    return bad ? 1 : 0;
}
