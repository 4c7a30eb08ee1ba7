/*
 * tools/parse_sim.c -- CPU model of the device deflate parse (lz_parse.h, kMin3, 4-way buckets) and
 * variants, to see which parse change closes the ratio gap to zlib level 1 before touching a kernel.
 * Diagnostic only: the cost of a parse is a dynamic-Huffman deflate block's size computed from the
 * symbol histograms (optimal code lengths, extra bits, a fixed header estimate), compared with the
 * system zlib's compress2 level 1 (byte-identical to the reference's zlib 1.2.8 at level 1).
 *
 *   gcc -O2 -o /tmp/parse_sim tools/parse_sim.c -lz -lm && /tmp/parse_sim [pages] [page_len] [zstd]
 * (zstd: the same for zstd level 1's fast parse, ZSTD_compressBlock_fast_generic, and the device's
 * repeat-candidate parse at several table shapes)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "../tyche_amd/csrc/pagegen.h"

#define MAXL 65536
static uint8_t pg[MAXL + 64];
static uint32_t L;

/* ---- tokens and cost */
static uint32_t hist_ll[286], hist_d[30];
static double extra_bits;
static const uint16_t len_base[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t dist_base[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

static void tok_lit(uint8_t c) { hist_ll[c]++; }
static void tok_match(uint32_t len, uint32_t dist) {
    while (len > 0) {   /* chunks of <= 258, never leaving a 1-2 byte tail */
        uint32_t l = len > 258 ? (len - 258 < 3 ? len - 3 : 258) : len;
        int c = 28;
        while (len_base[c] > l) c--;
        hist_ll[257 + c]++;
        extra_bits += len_extra[c];
        int d = 29;
        while (dist_base[d] > dist) d--;
        hist_d[d]++;
        extra_bits += dist_extra[d];
        len -= l;
    }
}
/* optimal (unlimited) Huffman code cost in bits for a histogram */
static double huff_bits(const uint32_t *h, int n) {
    uint64_t w[600];
    int m = 0;
    for (int i = 0; i < n; i++)
        if (h[i]) w[m++] = h[i];
    if (m <= 1) return m ? (double)w[0] : 0.0;
    double total = 0;
    while (m > 1) {   /* repeatedly merge the two smallest (O(n^2), fine for 286 symbols) */
        int a = 0, b = 1;
        if (w[b] < w[a]) { a = 1; b = 0; }
        for (int i = 2; i < m; i++) {
            if (w[i] < w[a]) { b = a; a = i; } else if (w[i] < w[b]) b = i;
        }
        const uint64_t s = w[a] + w[b];
        total += (double)s;
        if (a > b) { int t = a; a = b; b = t; }
        w[a] = s;
        w[b] = w[--m];
    }
    return total;
}
static double block_bytes(void) {
    hist_ll[256]++;
    const double bits = huff_bits(hist_ll, 286) + huff_bits(hist_d, 30) + extra_bits + 8 * 60.0;   /* ~60 B of trees */
    return bits / 8 + 2 + 4;   /* zlib header + adler32 */
}

static uint32_t mlen(uint32_t a, uint32_t b, uint32_t limit) {   /* equal bytes at a, b; a stops before limit */
    uint32_t n = 0;
    while (a + n < limit && pg[a + n] == pg[b + n]) n++;
    return n;
}

/* ---- the device parse (lz_parse.h kMin3, kWays 4): lookups before the block's inserts, greedy walk */
static uint32_t opt_ways = 4, opt_buckets = 1024, opt_seq_insert = 0, opt_rep = 0, opt_d4 = 1, opt_probe = 20;
static double parse_device(void) {
    memset(hist_ll, 0, sizeof hist_ll);
    memset(hist_d, 0, sizeof hist_d);
    extra_bits = 0;
    static uint32_t T[1 << 16][8];
    for (uint32_t i = 0; i < opt_buckets; i++)
        for (int w = 0; w < 8; w++) T[i][w] = 0;
    const uint32_t mflimit = L - 12, matchlimit = L - 5;
    uint32_t cursor = 0, anchor = 0, blk = 0, lastd = 0;
    int lg = 0;
    while ((1u << lg) < opt_buckets) lg++;
    while (blk <= mflimit) {
        uint32_t cand[64], len[64], back[64], ok[64];
        uint32_t h[64];
        for (int l = 0; l < 64; l++) {
            const uint32_t pos = blk + l;
            ok[l] = 0;
            const uint32_t p = pos <= mflimit ? pos : mflimit;
            const uint32_t v = pg[p] | pg[p + 1] << 8 | pg[p + 2] << 16;
            h[l] = (v * 2654435761u) >> (32 - lg);
            if (opt_seq_insert && pos <= mflimit) {   /* the serial parse's view: earlier lanes already inserted */
                for (int w = (int)opt_ways - 1; w > 0; w--) T[h[l]][w] = T[h[l]][w - 1];
                T[h[l]][0] = pos + 1;   /* +1: 0 = empty */
            }
        }
        for (int l = 0; l < 64; l++) {
            const uint32_t pos = blk + l;
            if (pos > mflimit) continue;
            uint32_t best = 0, bc = 0;
            for (uint32_t w = opt_seq_insert ? 1 : 0; w < opt_ways + (opt_seq_insert ? 1 : 0) && w < 8; w++) {
                const uint32_t e = T[h[l]][w];
                if (!e) continue;
                const uint32_t c = e - 1;
                if (c >= pos || pos - c > 32768) continue;
                uint32_t n = mlen(pos, c, matchlimit);
                if (n < 3) continue;
                if (n > best) { best = n; bc = c; }
            }
            if (opt_d4 && pos >= 4) {
                uint32_t n = mlen(pos, pos - 4, matchlimit);
                if (n >= 3 && n >= best) { best = n; bc = pos - 4; }
            }
            if (opt_rep && lastd && pos >= lastd) {
                uint32_t n = mlen(pos, pos - lastd, matchlimit);
                if (n >= 3 && n >= best) { best = n; bc = pos - lastd; }
            }
            if (best >= 3) {
                ok[l] = 1;
                cand[l] = bc;
                len[l] = best;
                uint32_t k = 0;
                while (k < 4 && pos >= k + 1 && bc >= k + 1 && pg[pos - k - 1] == pg[bc - k - 1]) k++;
                back[l] = k;
            }
        }
        if (!opt_seq_insert)
            for (int l = 0; l < 64; l++) {   /* block inserts: the highest lane of a bucket wins */
                const uint32_t pos = blk + l;
                for (int w = (int)opt_ways - 1; w > 0; w--) T[h[l]][w] = T[h[l]][w - 1];
                T[h[l]][0] = (pos <= mflimit ? pos : mflimit) + 1;
            }
        /* greedy walk from the cursor */
        uint32_t l = cursor > blk ? cursor - blk : 0;
        for (; l < 64; l++) {
            if (!ok[l]) continue;
            const uint32_t pos = blk + l;
            if (pos < cursor) continue;
            uint32_t k = back[l];
            if (k > pos - anchor) k = pos - anchor;
            if (k > cand[l]) k = cand[l];
            for (uint32_t i = anchor; i < pos - k; i++) tok_lit(pg[i]);
            tok_match(len[l] + k, pos - cand[l]);
            lastd = pos - cand[l];
            cursor = anchor = pos + len[l];
            if (cursor > mflimit) break;
            l = cursor - blk - 1;   /* next candidate at or after the cursor */
        }
        uint32_t nb = blk + 64;
        if ((cursor & ~63u) > nb) nb = cursor & ~63u;
        blk = nb;
    }
    for (uint32_t i = anchor; i < L; i++) tok_lit(pg[i]);
    return block_bytes();
}

/* ---- deflate_fast as zlib level 1 does it (hash chains, max_chain 4, nice 8, max_insert 4) */
static double parse_zlib_fast(void) {
    memset(hist_ll, 0, sizeof hist_ll);
    memset(hist_d, 0, sizeof hist_d);
    extra_bits = 0;
    static int32_t head[1 << 15], prev[MAXL];
    for (int i = 0; i < (1 << 15); i++) head[i] = -1;
    uint32_t pos = 0;
#define H3(p) ((((uint32_t)pg[p] << 10) ^ ((uint32_t)pg[(p) + 1] << 5) ^ pg[(p) + 2]) & 0x7FFF)
#define INS(p) do { uint32_t hh = H3(p); prev[p] = head[hh]; head[hh] = (int32_t)(p); } while (0)
    while (pos < L) {
        uint32_t best = 0, bd = 0;
        if (pos + 3 <= L) {
            const uint32_t hh = H3(pos);
            int32_t c = head[hh];
            prev[pos] = c;
            head[hh] = (int32_t)pos;
            int chain = 4;
            while (c >= 0 && chain-- > 0 && pos - (uint32_t)c <= 32768 - 262) {
                uint32_t n = mlen(pos, (uint32_t)c, L);
                if (n > 258) n = 258;
                if (n > best) { best = n; bd = pos - (uint32_t)c; if (n >= 8) break; }
                c = prev[c];
            }
        }
        if (best >= 3) {
            tok_match(best, bd);
            if (best <= 4) {
                for (uint32_t i = 1; i < best; i++)
                    if (pos + i + 3 <= L) INS(pos + i);
            }
            pos += best;
        } else {
            tok_lit(pg[pos]);
            pos++;
        }
    }
    return block_bytes();
}


/* ======================================================================= zstd level 1
 * Cost model of one zstd block: Huffman literals + FSE-coded LL/ML/OF codes (entropy) + extra bits +
 * a fixed header estimate.  Sequences carry zstd's repeat-offset coding (history {1, 4, 8}). */
typedef struct { uint32_t ll, ml, off; } zseq;
static zseq zs[MAXL];
static uint32_t nzs, zlit[256], zlits;
static uint32_t zcode_ll(uint32_t ll) {
    static const uint32_t base[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 28, 32, 40, 48, 64,
                                      128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
    int c = 35;
    while (base[c] > ll) c--;
    return (uint32_t)c;
}
static const uint8_t zll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static uint32_t zcode_ml(uint32_t mb) {   /* mb = ml - 3 */
    static const uint32_t base[53] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26,
                                      27, 28, 29, 30, 31, 32, 34, 36, 38, 40, 44, 48, 56, 64, 80, 96, 128, 256, 512, 1024, 2048,
                                      4096, 8192, 16384, 32768, 65536};
    int c = 52;
    while (base[c] > mb) c--;
    return (uint32_t)c;
}
static const uint8_t zml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                     1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static double entropy_bits(const uint32_t *h, int n) {
    double tot = 0, b = 0;
    for (int i = 0; i < n; i++) tot += h[i];
    for (int i = 0; i < n; i++)
        if (h[i]) b -= h[i] * __builtin_log2((double)h[i] / tot);
    return b;
}
/* opt_fse 0: ideal entropy + a fixed 12-byte header per table; otherwise FSE-normalized costs at table
 * logs (opt_fse 1: ours, LL 6 / OF 5 / ML 6; 2: the reference's FSE_optimalTableLog choice) plus an
 * estimate of the NCount header (FSE_writeNCount's variable-width fields, zero runs at 2 bits per 3) */
static int opt_fse;
static int hb32(uint32_t v) { return 31 - __builtin_clz(v); }
static double fse_bits(const uint32_t *h, int n, int maxlog) {
    double tot = 0;
    int mx = 0;
    for (int i = 0; i < n; i++) { tot += h[i]; if (h[i]) mx = i; }
    if (tot == 0) return 0;
    if (opt_fse == 0) return entropy_bits(h, n) + 12 * 8;
    int tl = maxlog;
    if (opt_fse >= 2) {
        const uint32_t src = (uint32_t)tot;
        const int maxsrc = src > 1 ? hb32(src - 1) - 2 : 1;
        const int minb = (hb32(src) + 1) < (hb32((uint32_t)mx ? (uint32_t)mx : 1u) + 2) ? hb32(src) + 1 : hb32((uint32_t)mx ? (uint32_t)mx : 1u) + 2;
        if (maxsrc < tl) tl = maxsrc;
        if (minb > tl) tl = minb;
        if (tl < 5) tl = 5;
        if (opt_fse == 3 && tl > maxlog - 2) tl = maxlog - 2;   /* capped at 7 / 6 / 7 */
        if (opt_fse == 4 && tl > maxlog - 1) tl = maxlog - 1;   /* capped at 8 / 7 / 8 */
    }
    const int cells = 1 << tl;
    int norm[64] = {0}, sum = 0, big = 0;
    for (int i = 0; i < n; i++) {
        if (!h[i]) continue;
        int v = (int)(h[i] * (double)cells / tot + 0.5);
        if (v < 1) v = 1;
        norm[i] = v;
        sum += v;
        if (h[i] > h[big] || !h[big]) big = i;
    }
    norm[big] += cells - sum;
    if (norm[big] < 1) norm[big] = 1;
    double bits = 0;
    for (int i = 0; i < n; i++) if (h[i]) bits += h[i] * (tl - __builtin_log2((double)norm[i]));
    /* header */
    double hdr = 4;
    int remaining = cells + 1, nb = tl + 1, zrun = 0;
    for (int i = 0; i <= mx && remaining > 1; i++) {
        if (!norm[i]) { zrun++; continue; }
        if (zrun) { hdr += 2.0 * ((zrun + 2) / 3); zrun = 0; }
        hdr += nb;
        remaining -= norm[i];
        while (remaining < (1 << (nb - 1)) && nb > 1) nb--;
    }
    return bits + hdr;
}
static uint32_t opt_blk_seq = 0;   /* > 0: zstd_cost cuts the sequences into blocks of at most this many */
static void zlit_add(uint32_t a, uint32_t b) {
    for (uint32_t i = a; i < b; i++) zlit[pg[i]]++;
    zlits += b - a;
}
static double zstd_cost_range(uint32_t i0, uint32_t i1, uint32_t *rep, uint32_t *lp, int last);
static double zstd_cost(void) {
    if (opt_blk_seq) {   /* blocks of <= opt_blk_seq sequences, each with its own literal and sequence tables */
        uint32_t rep[3] = {1, 4, 8}, lp = 0;
        double tot = 6;
        for (uint32_t i = 0; i < nzs || i == 0; i += opt_blk_seq) {
            const uint32_t i1 = i + opt_blk_seq < nzs ? i + opt_blk_seq : nzs;
            tot += zstd_cost_range(i, i1, rep, &lp, i1 == nzs);
            if (i1 == nzs) break;
        }
        return tot;
    }
    uint32_t hl[36] = {0}, hm[53] = {0}, ho[32] = {0};
    double extra = 0;
    uint32_t rep[3] = {1, 4, 8};
    for (uint32_t i = 0; i < nzs; i++) {
        const zseq q = zs[i];
        uint32_t ov;
        if (q.ll) {
            if (q.off == rep[0]) ov = 1;
            else if (q.off == rep[1]) ov = 2;
            else if (q.off == rep[2]) ov = 3;
            else ov = q.off + 3;
        } else {
            if (q.off == rep[1]) ov = 1;
            else if (q.off == rep[2]) ov = 2;
            else if (q.off == rep[0] - 1) ov = 3;
            else ov = q.off + 3;
        }
        /* history update (zstd_decompress.c ZSTD_decodeSequence) */
        if (ov > 3) { rep[2] = rep[1]; rep[1] = rep[0]; rep[0] = q.off; }
        else {
            const uint32_t idx = ov - 1 + (q.ll == 0);
            if (idx) {
                const uint32_t t = idx == 3 ? rep[0] - 1 : rep[idx];
                if (idx != 1) rep[2] = rep[1];
                rep[1] = rep[0];
                rep[0] = t;
            }
        }
        const uint32_t lc = zcode_ll(q.ll), mc = zcode_ml(q.ml - 3);
        uint32_t oc = 31 - (uint32_t)__builtin_clz(ov);
        hl[lc]++; hm[mc]++; ho[oc]++;
        extra += zll_bits[lc] + zml_bits[mc] + oc;
    }
    const double lit_bits = huff_bits(zlit, 256);
    const double bits = lit_bits + fse_bits(hl, 36, opt_fse == 1 ? 6 : 9) + fse_bits(hm, 53, opt_fse == 1 ? 6 : 9) +
                        fse_bits(ho, 32, opt_fse == 1 ? 5 : 8) + extra;
    return bits / 8 + 6 + 3 + 5 + 6 + 45;   /* frame + block + literal headers, jump table, HUF table */
}
/* one block: sequences [i0, i1), literals from *lp (the last block also takes the page's tail) */
static double zstd_cost_range(uint32_t i0, uint32_t i1, uint32_t *rep, uint32_t *lp, int last) {
    uint32_t hl[36] = {0}, hm[53] = {0}, ho[32] = {0}, hlit[256] = {0};
    double extra = 0;
    for (uint32_t i = i0; i < i1; i++) {
        const zseq q = zs[i];
        for (uint32_t b = 0; b < q.ll; b++) hlit[pg[*lp + b]]++;
        *lp += q.ll + q.ml;
        uint32_t ov;
        if (q.ll) {
            if (q.off == rep[0]) ov = 1;
            else if (q.off == rep[1]) ov = 2;
            else if (q.off == rep[2]) ov = 3;
            else ov = q.off + 3;
        } else {
            if (q.off == rep[1]) ov = 1;
            else if (q.off == rep[2]) ov = 2;
            else if (q.off == rep[0] - 1) ov = 3;
            else ov = q.off + 3;
        }
        if (ov > 3) { rep[2] = rep[1]; rep[1] = rep[0]; rep[0] = q.off; }
        else {
            const uint32_t idx = ov - 1 + (q.ll == 0);
            if (idx) {
                const uint32_t t = idx == 3 ? rep[0] - 1 : rep[idx];
                if (idx != 1) rep[2] = rep[1];
                rep[1] = rep[0];
                rep[0] = t;
            }
        }
        const uint32_t lc = zcode_ll(q.ll), mc = zcode_ml(q.ml - 3);
        uint32_t oc = 31 - (uint32_t)__builtin_clz(ov);
        hl[lc]++; hm[mc]++; ho[oc]++;
        extra += zll_bits[lc] + zml_bits[mc] + oc;
    }
    if (last) { for (uint32_t b = *lp; b < L; b++) hlit[pg[b]]++; *lp = L; }
    const double lit_bits = huff_bits(hlit, 256);
    const double bits = lit_bits + fse_bits(hl, 36, opt_fse == 1 ? 6 : 9) + fse_bits(hm, 53, opt_fse == 1 ? 6 : 9) +
                        fse_bits(ho, 32, opt_fse == 1 ? 5 : 8) + extra;
    return bits / 8 + 3 + 5 + 6 + 45;
}
static void zreset(void) { nzs = 0; zlits = 0; memset(zlit, 0, sizeof zlit); }

static uint64_t read64(uint32_t p) { uint64_t v = 0; memcpy(&v, pg + p, 8); return v; }
static uint32_t read32(uint32_t p) { uint32_t v; memcpy(&v, pg + p, 4); return v; }
static uint32_t zhash(uint32_t p, uint32_t bits, uint32_t mls) {
    const uint64_t v = read64(p) << (64 - 8 * mls);
    return (uint32_t)((v * 227718039650203ull) >> (64 - bits));   /* ZSTD_hash6Ptr family (prime6bytes) */
}

/* ZSTD_compressBlock_fast_generic (zstd_compress.c:931-1015) on one page */
static double parse_zstd_fast(uint32_t hbits, uint32_t mls) {
    static uint32_t ht[1 << 17];
    memset(ht, 0, sizeof(uint32_t) << hbits);
    zreset();
    /* the reference compresses from a base with lowestIndex = dictLimit; index 0 = the page start */
    uint32_t ip = 1, anchor = 0, o1 = 1, o2 = 4;
    const uint32_t ilimit = L - 8;
    while (ip < ilimit) {
        const uint32_t h = zhash(ip, hbits, mls), cur = ip, mi = ht[h];
        ht[h] = cur;
        uint32_t ml;
        if (o1 > 0 && ip + 1 >= o1 && read32(ip + 1 - o1) == read32(ip + 1)) {
            ml = mlen(ip + 1 + 4, ip + 1 + 4 - o1, L) + 4;
            ip++;
            zlit_add(anchor, ip);
            zs[nzs++] = (zseq){ip - anchor, ml, o1};
        } else {
            if (mi <= 0 || read32(mi) != read32(ip)) {
                ip += ((ip - anchor) >> 8) + 1;   /* g_searchStrength 8 */
                continue;
            }
            uint32_t m = mi;
            ml = mlen(ip + 4, m + 4, L) + 4;
            while (ip > anchor && m > 0 && pg[ip - 1] == pg[m - 1]) { ip--; m--; ml++; }
            o2 = o1;
            o1 = ip - m;
            zlit_add(anchor, ip);
            zs[nzs++] = (zseq){ip - anchor, ml, o1};
        }
        ip += ml;
        anchor = ip;
        if (ip <= ilimit) {
            ht[zhash(cur + 2, hbits, mls)] = cur + 2;
            ht[zhash(ip - 2, hbits, mls)] = ip - 2;
            while (ip <= ilimit && o2 > 0 && read32(ip) == read32(ip - o2)) {
                const uint32_t rl = mlen(ip + 4, ip + 4 - o2, L) + 4;
                const uint32_t t = o2; o2 = o1; o1 = t;
                ht[zhash(ip, hbits, mls)] = ip;
                zs[nzs++] = (zseq){0, rl, o1};
                ip += rl;
                anchor = ip;
            }
        }
    }
    zlit_add(anchor, L);
    return zstd_cost();
}

/* the device parse with repeat candidates (lz_parse.h kRepCand): nb buckets x ways, hash of hb bytes;
 * a repeat candidate wins when at most opt_rep_slack bytes shorter than the hash candidate (TYCHE_REP_SLACK) */
static uint32_t opt_rep_slack = 3;
static uint32_t opt_parts = 1, opt_seed = 1u << 20, opt_carry_rep = 0, gR = 1, gR2 = 4, opt_warm = 0, opt_all_blocks = 0;
static double parse_zstd_device(uint32_t nb, uint32_t ways, uint32_t hb) {
    static uint32_t T[1 << 16][8];
    zreset();
    uint32_t anchor = 0;
    const uint32_t Lfull = L;
  for (uint32_t part = 0; part < opt_parts; part++) {
    const uint32_t b0 = part == 0 ? 0 : ((Lfull * part) / opt_parts) & ~63u;
    const uint32_t b1 = part + 1 == opt_parts ? Lfull : ((Lfull * (part + 1)) / opt_parts) & ~63u;
    const uint32_t Lp = part + 1 == opt_parts ? Lfull : b1 + 5;
    for (uint32_t i = 0; i < nb; i++) for (int w = 0; w < 8; w++) T[i][w] = 0;
    for (uint32_t blk = b0 > opt_seed ? b0 - opt_seed : 0; blk < b0; blk += 64)
        for (int l = 0; l < 64; l++) {
            const uint32_t pos = blk + l;
            const uint64_t x = read64(pos) & (hb >= 8 ? ~0ull : ((1ull << (8 * hb)) - 1));
            const uint32_t h = (uint32_t)((((x * 0xCF1BBCDCB7A56463ull) >> 32) * (uint64_t)nb) >> 32);
            for (int w = (int)ways - 1; w > 0; w--) T[h][w] = T[h][w - 1];
            T[h][0] = pos + 1;
        }
    const uint32_t mflimit = Lp - 12, matchlimit = Lp - 5;
    uint32_t R = 1, R2 = 4;
    if (opt_carry_rep && part > 0) { R = gR; R2 = gR2; }
    const uint32_t saved_nzs = nzs, saved_zlits = zlits, saved_anchor = anchor;
    uint32_t saved_zlit[256];
    int warm = part > 0 && opt_warm > 0;
  for (int pass = warm ? 0 : 1; pass < 2; pass++) {
    uint32_t cursor = pass == 0 ? (b0 > opt_warm ? b0 - opt_warm : 0) & ~63u : b0;
    uint32_t blk = cursor;
    if (pass == 0) memcpy(saved_zlit, zlit, sizeof zlit);
    const uint32_t plim = pass == 0 ? b0 + 5 : Lp;
    const uint32_t mflimit2 = plim - 12, matchlimit2 = plim - 5;
    (void)mflimit; (void)matchlimit;
#define mflimit mflimit2
#define matchlimit matchlimit2
    while (blk <= mflimit) {
        uint32_t cand[64], len[64], back[64], ok[64], rok[64], h[64];
        for (int l = 0; l < 64; l++) {
            const uint32_t pos = blk + l, p = pos <= mflimit ? pos : mflimit;
            const uint64_t x = read64(p) & (hb >= 8 ? ~0ull : ((1ull << (8 * hb)) - 1));
            const uint64_t hx = x * 0xCF1BBCDCB7A56463ull;
            h[l] = (uint32_t)(((hx >> 32) * (uint64_t)nb) >> 32);
            ok[l] = rok[l] = 0;
            if (pos > mflimit) continue;
            uint32_t best = 0, bc = 0;
            for (uint32_t w = 0; w < ways; w++) {
                const uint32_t e = T[h[l]][w];
                if (!e) continue;
                const uint32_t c = e - 1;
                if (c >= pos || read32(c) != read32(pos)) continue;
                const uint32_t n = mlen(pos, c, matchlimit);
                if (n > best) { best = n; bc = c; }
            }
            uint32_t rn = 0, rn2 = 0;
            if (pos >= R && read32(pos - R) == read32(pos)) rn = mlen(pos, pos - R, matchlimit);
            if (R2 != R && pos >= R2 && read32(pos - R2) == read32(pos)) rn2 = mlen(pos, pos - R2, matchlimit);
            if (rn >= 4 && rn + opt_rep_slack >= best) { best = rn; bc = pos - R; }
            if (rn2 >= 4 && rn2 + opt_rep_slack >= best && !(rn >= 4 && rn >= rn2)) { best = rn2; bc = pos - R2; }
            rok[l] = rn >= 4 || rn2 >= 4;
            if (best >= 4) {
                ok[l] = 1; cand[l] = bc; len[l] = best;
                uint32_t k = 0;
                while (k < 4 && pos >= k + 1 && bc >= k + 1 && pg[pos - k - 1] == pg[bc - k - 1]) k++;
                back[l] = k;
            }
        }
        for (int l = 0; l < 63; l++)   /* a position whose successor has a repeat match starts none (unless itself a repeat) */
            if (rok[l + 1] && !rok[l]) ok[l] = 0;
        for (int l = 0; l < 64; l++) {
            for (int w = (int)ways - 1; w > 0; w--) T[h[l]][w] = T[h[l]][w - 1];
            T[h[l]][0] = ((blk + l) <= mflimit ? blk + l : mflimit) + 1;
        }
        uint32_t l = cursor > blk ? cursor - blk : 0;
        for (; l < 64; l++) {
            if (!ok[l]) continue;
            const uint32_t pos = blk + l;
            uint32_t k = back[l];
            if (k > pos - anchor) k = pos - anchor;
            if (k > cand[l]) k = cand[l];
            const uint32_t off = pos - cand[l];
            zlit_add(anchor, pos - k);
            zs[nzs++] = (zseq){pos - k - anchor, len[l] + k, off};
            if (off != R) { R2 = R; R = off; }
            cursor = anchor = pos + len[l];
            if (cursor > mflimit) break;
            l = cursor - blk - 1;
        }
        uint32_t nbk = blk + 64;
        if ((cursor & ~63u) > nbk) nbk = cursor & ~63u;
        if (opt_all_blocks)   /* a finder wave running ahead of the walk inserts the blocks it skips too */
            for (uint32_t sb = blk + 64; sb < nbk; sb += 64)
                for (int l2 = 0; l2 < 64; l2++) {
                    const uint32_t q = sb + l2 <= mflimit ? sb + l2 : mflimit;
                    const uint64_t x = read64(q) & (hb >= 8 ? ~0ull : ((1ull << (8 * hb)) - 1));
                    const uint32_t h2 = (uint32_t)((((x * 0xCF1BBCDCB7A56463ull) >> 32) * (uint64_t)nb) >> 32);
                    for (int w = (int)ways - 1; w > 0; w--) T[h2][w] = T[h2][w - 1];
                    T[h2][0] = q + 1;
                }
        blk = nbk;
    }
#undef mflimit
#undef matchlimit
    if (pass == 0) {   /* warm-up: keep R, R2 and the table, drop the sequences */
        nzs = saved_nzs; zlits = saved_zlits; anchor = saved_anchor;
        memcpy(zlit, saved_zlit, sizeof zlit);
    }
  }
    gR = R; gR2 = R2;
  }
    zlit_add(anchor, L);
    return zstd_cost();
}

static int main_zstd_split(int n) {
    double raw = 0, d[4] = {0}, dw[4] = {0}, ds[6] = {0};
    const uint32_t sp[6] = {2, 2, 2, 4, 4, 4}, ss[6] = {8192, 16384, 1u << 20, 8192, 16384, 1u << 20};
    const uint32_t warms[4] = {256, 512, 1024, 2048};
    const uint32_t parts[4] = {1, 2, 4, 4}, seeds[4] = {1u << 20, 1u << 20, 1u << 20, 1u << 20};
    for (int i = 0; i < n; i++) {
        pg_page_t p;
        pg_page_init(&p, 20170303ull, (uint64_t)i, L, 0);
        for (uint32_t b = 0; b < L; b++) pg[b] = (uint8_t)pg_page_byte(&p, b);
        memset(pg + L, 0, 64);
        raw += L;
        for (int c = 0; c < 4; c++) {
            opt_parts = parts[c];
            opt_seed = seeds[c];
            opt_carry_rep = c == 3;
            d[c] += parse_zstd_device(1856, 2, 5);
        }
        for (int c = 0; c < 4; c++) {
            opt_parts = 4; opt_seed = 1u << 20; opt_carry_rep = 0; opt_warm = warms[c];
            dw[c] += parse_zstd_device(1856, 2, 5);
        }
        for (int c = 0; c < 6; c++) {
            opt_parts = sp[c]; opt_seed = ss[c]; opt_carry_rep = 0; opt_warm = 256;
            ds[c] += parse_zstd_device(1856, 2, 5);
        }
        opt_warm = 0;
    }
    opt_parts = 1;
    opt_seed = 1u << 20;
    for (int c = 0; c < 4; c++) printf("model: device parse in %u parts, seed %u%s: ratio %.3f\n", parts[c], seeds[c], c == 3 ? ", repeat offsets carried" : "", raw / d[c]);
    for (int c = 0; c < 4; c++) printf("model: device parse in 4 parts, warm-up parse of %u bytes before each: ratio %.3f\n", warms[c], raw / dw[c]);
    for (int c = 0; c < 6; c++) printf("model: device parse in %u parts, hash seed %u bytes, warm-up 256: ratio %.3f\n", sp[c], ss[c], raw / ds[c]);
    return 0;
}

static int main_zstd(int n) {
    double raw = 0, ref = 0, d[8] = {0};
    static const uint32_t cfg[][3] = {{1856, 2, 5}, {4096, 2, 5}, {8192, 2, 5}, {16384, 1, 6}, {4096, 2, 6}, {2048, 4, 5}, {4096, 4, 5}, {928, 4, 5}};
    const int nc = 8;
    opt_fse = 3;   /* sequence tables as the device encodes them (FSE_optimalTableLog capped at 7/6/7) */
    const uint32_t hbits = L <= 16384 ? 14 : 13;
    for (int i = 0; i < n; i++) {
        pg_page_t p;
        pg_page_init(&p, 20170303ull, (uint64_t)i, L, 0);
        for (uint32_t b = 0; b < L; b++) pg[b] = (uint8_t)pg_page_byte(&p, b);
        memset(pg + L, 0, 64);
        raw += L;
        ref += parse_zstd_fast(hbits, 6);
        for (int c = 0; c < nc; c++) d[c] += parse_zstd_device(cfg[c][0], cfg[c][1], cfg[c][2]);
    }
    opt_fse = 0;
    printf("pages %d x %u B (zstd, repeat slack %u)\n", n, L, opt_rep_slack);
    printf("model: level-1 fast parse (hashLog %u, mls 6)   ratio %.3f\n", hbits, raw / ref);
    for (int c = 0; c < nc; c++)
        printf("model: device %5u buckets x %u ways, %u-byte hash  ratio %.3f\n", cfg[c][0], cfg[c][1], cfg[c][2], raw / d[c]);
    return 0;
}

static int main_zstd_allblk(int n) {
    double raw = 0, d0 = 0, d1 = 0;
    for (int i = 0; i < n; i++) {
        pg_page_t p;
        pg_page_init(&p, 20170303ull, (uint64_t)i, L, 0);
        for (uint32_t b = 0; b < L; b++) pg[b] = (uint8_t)pg_page_byte(&p, b);
        memset(pg + L, 0, 64);
        raw += L;
        opt_all_blocks = 0;
        d0 += parse_zstd_device(1856, 2, 5);
        opt_all_blocks = 1;
        d1 += parse_zstd_device(1856, 2, 5);
    }
    opt_all_blocks = 0;
    printf("pages %d x %u B: device parse %.3f, with every block inserted (finder ahead of the walk) %.3f\n", n, L,
           raw / d0, raw / d1);
    return 0;
}

static int main_zstd_fse(int n) {
    double raw = 0, d[5] = {0}, r[5] = {0};
    const uint32_t hbits = L <= 16384 ? 14 : 13;
    for (int i = 0; i < n; i++) {
        pg_page_t p;
        pg_page_init(&p, 20170303ull, (uint64_t)i, L, 0);
        for (uint32_t b = 0; b < L; b++) pg[b] = (uint8_t)pg_page_byte(&p, b);
        memset(pg + L, 0, 64);
        raw += L;
        for (int m = 0; m < 5; m++) {
            opt_fse = m;
            d[m] += parse_zstd_device(1856, 2, 5);
            r[m] += parse_zstd_fast(hbits, 6);
        }
    }
    opt_fse = 0;
    static const char *nm[5] = {"ideal entropy", "FSE logs 6/5/6", "FSE optimal logs (<= 9/8/9)",
                                "FSE optimal logs (<= 7/6/7)", "FSE optimal logs (<= 8/7/8)"};
    printf("pages %d x %u B (zstd sequence tables)\n", n, L);
    for (int m = 0; m < 5; m++) printf("model: %-28s device parse %.3f   level-1 parse %.3f\n", nm[m], raw / d[m], raw / r[m]);
    return 0;
}

/* block cuts: the device encoder starts a new block every 960 sequences (zstd_encode.hip kZBlk);
 * level 1 puts a whole page (<= 128 KiB) in one block */
static int main_zstd_blk(int n) {
    static const uint32_t cuts[5] = {0, 960, 1500, 2000, 4000};
    double raw = 0, d[5] = {0}, r[5] = {0}, ns = 0;
    const uint32_t hbits = L <= 16384 ? 14 : 13;
    opt_fse = 3;
    for (int i = 0; i < n; i++) {
        pg_page_t p;
        pg_page_init(&p, 20170303ull, (uint64_t)i, L, 0);
        for (uint32_t b = 0; b < L; b++) pg[b] = (uint8_t)pg_page_byte(&p, b);
        memset(pg + L, 0, 64);
        raw += L;
        for (int m = 0; m < 5; m++) {
            opt_blk_seq = cuts[m];
            d[m] += parse_zstd_device(1856, 2, 5);
            if (m == 0) ns += nzs;
            r[m] += parse_zstd_fast(hbits, 6);
        }
    }
    opt_blk_seq = 0;
    printf("pages %d x %u B (zstd block cuts, FSE logs <= 7/6/7), %.0f device sequences per page\n", n, L, ns / n);
    for (int m = 0; m < 5; m++) printf("model: blocks of <= %4u sequences  device parse %.3f   level-1 parse %.3f\n", cuts[m], raw / d[m], raw / r[m]);
    return 0;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 200;
    L = argc > 2 ? (uint32_t)atoi(argv[2]) : 16384;
    if (argc > 3 && !strcmp(argv[3], "zstd")) return main_zstd(n);
    if (argc > 3 && !strcmp(argv[3], "zsplit")) return main_zstd_split(n);
    if (argc > 3 && !strcmp(argv[3], "zfse")) return main_zstd_fse(n);
    if (argc > 3 && !strcmp(argv[3], "zallblk")) return main_zstd_allblk(n);
    if (argc > 3 && !strcmp(argv[3], "zblk")) return main_zstd_blk(n);
    static const uint32_t grid[][2] = {{1024, 4}, {2048, 4}, {512, 8}, {1024, 8}, {2048, 8}, {1024, 6}, {4096, 8}};
    const int ng = (int)(sizeof grid / sizeof grid[0]);
    double raw = 0, zl = 0, zf = 0, var[16] = {0}, var_r[16] = {0};
    static uint8_t zbuf[MAXL * 2];
    for (int i = 0; i < n; i++) {
        pg_page_t p;
        pg_page_init(&p, 20170303ull, (uint64_t)i, L, 0);
        for (uint32_t b = 0; b < L; b++) pg[b] = (uint8_t)pg_page_byte(&p, b);
        memset(pg + L, 0, 64);
        uLongf zl_len = sizeof zbuf;
        compress2(zbuf, &zl_len, pg, L, 1);
        raw += L;
        zl += zl_len;
        zf += parse_zlib_fast();
        for (int g = 0; g < ng; g++) {
            opt_buckets = grid[g][0];
            opt_ways = grid[g][1];
            opt_seq_insert = 0;
            var[g] += parse_device();
            opt_seq_insert = 1;
            var_r[g] += parse_device();
        }
    }
    printf("pages %d x %u B\n", n, L);
    printf("zlib level 1 (compress2, real bytes)   ratio %.3f\n", raw / zl);
    printf("model: deflate_fast parse              ratio %.3f\n", raw / zf);
    for (int g = 0; g < ng; g++)
        printf("model: %4u buckets x %u ways: block inserts %.3f, serial inserts %.3f\n", grid[g][0], grid[g][1],
               raw / var[g], raw / var_r[g]);
    return 0;
}
