/* Sequence statistics of zstd frames, through the oracle's decoder
 * (oracle/zstd_oracle.c built with -DZSTD_SEQ_TRACE).  Diagnostics only.
 *
 *   gcc -O2 -DZSTD_SEQ_TRACE -Ioracle tools/zstd_seq_stats.c oracle/zstd_oracle.c -o /tmp/seqstats
 *   /tmp/seqstats frames.bin     (frames.bin: [u32 length][frame] ... -- tools/zstd_seq_stats.py writes it)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include "oracle.h"

static uint64_t nseq, nrep, of_bits, ll_bits, ml_bits, lit, mat, ml_hist[8], ll_hist[8], of_hist[18];

void zstd_seq_trace(uint32_t llc, uint32_t mlc, uint32_t ofc, size_t ll, size_t ml, size_t off) {
    (void)llc; (void)mlc;
    nseq++;
    if (ofc <= 1) nrep++;
    of_bits += ofc;
    ll_bits += ll >= 16 ? 31 - __builtin_clz((uint32_t)ll) : 0;
    ml_bits += ml >= 35 ? 31 - __builtin_clz((uint32_t)(ml - 3)) : 0;
    lit += ll;
    mat += ml;
    ml_hist[ml < 5 ? 0 : ml < 6 ? 1 : ml < 8 ? 2 : ml < 12 ? 3 : ml < 20 ? 4 : ml < 40 ? 5 : ml < 100 ? 6 : 7]++;
    ll_hist[ll == 0 ? 0 : ll < 2 ? 1 : ll < 4 ? 2 : ll < 8 ? 3 : ll < 16 ? 4 : ll < 32 ? 5 : ll < 64 ? 6 : 7]++;
    of_hist[ofc < 18 ? ofc : 17]++;
    (void)off;
}

int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    static uint8_t buf[1 << 20], out[1 << 20];
    uint32_t n, frames = 0;
    while (fread(&n, 4, 1, f) == 1 && n <= sizeof buf && fread(buf, 1, n, f) == n) {
        if (oracle_zstd_decompress(buf, (int)n, out, (int)sizeof out) < 0) { fprintf(stderr, "corrupt frame %u\n", frames); return 1; }
        frames++;
    }
    const double F = frames ? frames : 1;
    printf("frames %u  seq/frame %.1f  rep %.1f%%  offset-extra bits/seq %.2f  ll-extra %.2f  ml-extra %.2f  "
           "lit/frame %.0f  match/seq %.1f\n", frames, nseq / F, 100.0 * nrep / (nseq ? nseq : 1),
           (double)of_bits / nseq, (double)ll_bits / nseq, (double)ml_bits / nseq, lit / F, (double)mat / nseq);
    printf("  ml <5 <6 <8 <12 <20 <40 <100 >=100:");
    for (int i = 0; i < 8; i++) printf(" %.1f", 100.0 * ml_hist[i] / nseq);
    printf("\n  ll 0 1 <4 <8 <16 <32 <64 >=64:");
    for (int i = 0; i < 8; i++) printf(" %.1f", 100.0 * ll_hist[i] / nseq);
    printf("\n  ofcode 0..17:");
    for (int i = 0; i < 18; i++) printf(" %.1f", 100.0 * of_hist[i] / nseq);
    printf("\n");
    return 0;
}
