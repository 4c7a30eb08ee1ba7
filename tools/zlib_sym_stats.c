/* Symbol statistics of zlib streams, through the oracle's inflate
 * (oracle/zlib_oracle.c built with -DZLIB_SYM_TRACE).  Diagnostics only.
 *
 *   gcc -O2 -DZLIB_SYM_TRACE -Ioracle tools/zlib_sym_stats.c oracle/zlib_oracle.c -lm -o /tmp/symstats
 *   /tmp/symstats streams.bin   (tools/zstd_seq_stats.py --codec zlib writes it)
 *
 * "entropy" is the per-stream order-0 entropy of the literal/length and
 * distance symbols plus their extra bits: what an optimal Huffman code of the
 * same tokens would spend, headers excluded.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "oracle.h"

static uint64_t nlit, nmat, mlen, dbits, lhist[8], dhist[8], short_d[17], short_l3[17];
static uint64_t hl[286], hd[30], xbits;
static double ent_bits;
static uint8_t cur_ll[288], cur_d[32];
static uint64_t sym_bits, blocks, fixed_blocks;

void zlib_block_trace(const uint8_t *lens, int nlen, int ndist, int type) {
    blocks++;
    memset(cur_ll, 0, sizeof cur_ll);
    memset(cur_d, 0, sizeof cur_d);
    if (type == 1) {
        fixed_blocks++;
        for (int i = 0; i < 288; i++) cur_ll[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
        for (int i = 0; i < 32; i++) cur_d[i] = 5;
        return;
    }
    memcpy(cur_ll, lens, (size_t)nlen);
    memcpy(cur_d, lens + nlen, (size_t)ndist);
}

static int len_sym(int len, int *xb) {
    const int l = len - 3;
    if (l < 8) { *xb = 0; return 257 + l; }
    if (l == 255) { *xb = 0; return 285; }
    const int h = 31 - __builtin_clz((uint32_t)l);
    *xb = h - 2;
    return 257 + 4 * (h - 1) + ((l >> (h - 2)) & 3);
}
static int dist_sym(int dist, int *xb) {
    const int d = dist - 1;
    if (d < 4) { *xb = 0; return d; }
    const int h = 31 - __builtin_clz((uint32_t)d);
    *xb = h - 1;
    return 2 * h + ((d >> (h - 1)) & 1);
}

void zlib_sym_trace(int len, int dist) {
    if (!len) { nlit++; hl[dist]++; sym_bits += cur_ll[dist]; return; }   /* literal: dist carries the byte */
    int lx, dx;
    const int ls = len_sym(len, &lx), ds = dist_sym(dist, &dx);
    hl[ls]++;
    hd[ds]++;
    sym_bits += (uint64_t)(cur_ll[ls] + cur_d[ds] + lx + dx);
    xbits += (uint64_t)(lx + dx);
    nmat++;
    mlen += (uint64_t)len;
    if (dist <= 16) { short_d[dist]++; if (len == 3) short_l3[dist]++; }
    dbits += (uint64_t)dx;
    lhist[len < 4 ? 0 : len < 5 ? 1 : len < 6 ? 2 : len < 8 ? 3 : len < 12 ? 4 : len < 20 ? 5 : len < 40 ? 6 : 7]++;
    dhist[dist < 4 ? 0 : dist < 16 ? 1 : dist < 64 ? 2 : dist < 256 ? 3 : dist < 1024 ? 4 : dist < 4096 ? 5 : dist < 16384 ? 6 : 7]++;
}

static double entropy(const uint64_t *h, int n) {
    uint64_t t = 0;
    for (int i = 0; i < n; i++) t += h[i];
    double b = 0;
    for (int i = 0; i < n; i++) if (h[i]) b -= (double)h[i] * log2((double)h[i] / (double)t);
    return b;
}

int main(int argc, char **argv) {
    (void)argc;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    static uint8_t buf[1 << 20], out[1 << 20];
    uint32_t n, k = 0;
    uint64_t bytes = 0;
    while (fread(&n, 4, 1, f) == 1 && n <= sizeof buf && fread(buf, 1, n, f) == n) {
        memset(hl, 0, sizeof hl);
        memset(hd, 0, sizeof hd);
        xbits = 0;
        if (oracle_zlib_uncompress(buf, (int)n, out, (int)sizeof out) < 0) { fprintf(stderr, "corrupt stream %u\n", k); return 1; }
        ent_bits += entropy(hl, 286) + entropy(hd, 30) + (double)xbits;
        bytes += n;
        k++;
    }
    const double F = k ? k : 1, M = nmat ? nmat : 1;
    printf("streams %u  bytes/stream %.0f  token entropy bytes/stream %.0f  literals/stream %.0f  matches/stream %.1f  "
           "match len %.2f  dist extra bits %.2f\n", k, bytes / F, ent_bits / 8.0 / F, nlit / F, nmat / F, mlen / M, dbits / M);
    printf("  symbol bytes/stream (code lengths used) %.0f  other (headers, end codes, padding) %.0f  blocks/stream %.2f (fixed %.2f)\n",
           sym_bits / 8.0 / F, bytes / F - sym_bits / 8.0 / F, blocks / F, fixed_blocks / F);
    printf("  len 3 4 5 <8 <12 <20 <40 >=40:");
    for (int i = 0; i < 8; i++) printf(" %.1f", 100.0 * lhist[i] / M);
    printf("\n  dist <4 <16 <64 <256 <1K <4K <16K >=16K:");
    for (int i = 0; i < 8; i++) printf(" %.1f", 100.0 * dhist[i] / M);
    printf("\n  dist 1..16 (%% of matches, of which length 3):");
    for (int i = 1; i <= 16; i++) if (short_d[i]) printf(" %d:%.1f/%.1f", i, 100.0 * short_d[i] / M, 100.0 * short_l3[i] / M);
    printf("\n");
    return 0;
}
