/*
 * oracle/zlib_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the zlib-wrapped deflate decoder the reference calls in
 * buffer__decompress (src/buffer.c:256-260 -> uncompress, src/zlib/uncompr.c:22-59
 * -> inflate, src/zlib/inflate.c:605, inffast.c, inftrees.c), written from
 * RFC 1950/1951, plus adler32 (src/zlib/adler32.c:65).  It is the parity model
 * for the gfx950 inflate kernel.
 *
 * Result: decoded length (Z_OK), or a negative zlib code: -3 Z_DATA_ERROR for a
 * corrupt or truncated stream, -5 Z_BUF_ERROR when the output capacity is too
 * small while input remains (uncompr.c:47-53).  Where the reference's split
 * between those two codes depends on how far inflate's bit buffer had read
 * ahead, parity is on "failed", not on the code (see tests).
 *
 * Table rules follow inflate_table (inftrees.c:32): over-subscribed code sets
 * are rejected; incomplete ones are rejected except a single one-bit code for
 * literal/length or distance tables; a distance table with no codes is allowed.
 */
#include <stdint.h>
#include <string.h>
#include "oracle.h"
#ifdef ZLIB_SYM_TRACE
void zlib_sym_trace(int len, int dist);   /* tools/zlib_sym_stats.c only */
void zlib_block_trace(const uint8_t *lens, int nlen, int ndist, int type);
#endif

#define Z_OK 0
#define Z_DATA_ERROR (-3)
#define Z_BUF_ERROR (-5)

uint32_t oracle_adler32(const uint8_t *p, int n) {
    uint32_t a = 1, b = 0;
    for (int i = 0; i < n; i++) {
        a = (a + p[i]) % 65521u;
        b = (b + a) % 65521u;
    }
    return (b << 16) | a;
}

typedef struct {
    const uint8_t *in;
    int64_t inlen, pos;      /* pos: next byte to load */
    uint64_t bits;           /* bit buffer, LSB first */
    int nbits;
    int overrun;             /* needed bits past the end of input */
} bitin_t;

static uint32_t need(bitin_t *s, int n) {
    while (s->nbits < n) {
        if (s->pos >= s->inlen) { s->overrun = 1; return 0; }
        s->bits |= (uint64_t)s->in[s->pos++] << s->nbits;
        s->nbits += 8;
    }
    uint32_t v = (uint32_t)(s->bits & ((1ull << n) - 1));
    s->bits >>= n;
    s->nbits -= n;
    return v;
}

typedef struct {
    uint16_t count[16];
    uint16_t symbol[320];
} huff_t;

/* builds a canonical decoder; 0 ok, -1 reject (kind: 0 code-length code, 1 lit/len, 2 dist) */
static int build(huff_t *h, const uint8_t *len, int n, int kind) {
    int offs[16];
    memset(h->count, 0, sizeof(h->count));
    for (int i = 0; i < n; i++) h->count[len[i]]++;
    int max = 0;
    for (int l = 15; l >= 1; l--) if (h->count[l]) { max = l; break; }
    if (max == 0) return kind == 0 ? -1 : 0;       /* no codes at all */
    int left = 1;
    for (int l = 1; l <= 15; l++) {
        left <<= 1;
        left -= h->count[l];
        if (left < 0) return -1;                    /* over-subscribed */
    }
    if (left > 0 && (kind == 0 || max != 1)) return -1;   /* incomplete */
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + h->count[l];
    for (int i = 0; i < n; i++) if (len[i]) h->symbol[offs[len[i]]++] = (uint16_t)i;
    return 0;
}

/* one symbol, or -1 for an invalid code / -2 when input ran out */
static int decode(bitin_t *s, const huff_t *h) {
    int code = 0, first = 0, index = 0;
    for (int l = 1; l <= 15; l++) {
        code |= (int)need(s, 1);
        if (s->overrun) return -2;
        int count = h->count[l];
        if (code - count < first) return h->symbol[index + (code - first)];
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    return -1;
}

static const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

int oracle_zlib_uncompress(const uint8_t *src, int srclen, uint8_t *dst, int dstcap) {
    bitin_t s = {src, srclen, 0, 0, 0, 0};
    int64_t op = 0;
    /* zlib header (RFC 1950; inflate.c HEAD state) */
    uint32_t cmf = need(&s, 8), flg = need(&s, 8);
    if (s.overrun) return Z_DATA_ERROR;
    if (((cmf << 8) | flg) % 31u) return Z_DATA_ERROR;
    if ((cmf & 15) != 8) return Z_DATA_ERROR;
    if ((cmf >> 4) + 8 > 15) return Z_DATA_ERROR;
    if (flg & 0x20) return Z_DATA_ERROR;           /* preset dictionary: Z_NEED_DICT -> Z_DATA_ERROR */
    static __thread huff_t lencode, distcode, clcode;
    int last;
    do {
        last = (int)need(&s, 1);
        int type = (int)need(&s, 2);
        if (s.overrun) return Z_DATA_ERROR;
        if (type == 0) {
            s.bits >>= (s.nbits & 7);
            s.nbits -= (s.nbits & 7);
            uint32_t len = need(&s, 16), nlen = need(&s, 16);
            if (s.overrun) return Z_DATA_ERROR;
            if (len != (~nlen & 0xFFFFu)) return Z_DATA_ERROR;
            /* bytes still in the bit buffer come first */
            for (uint32_t i = 0; i < len; i++) {
                uint32_t b = need(&s, 8);
                if (s.overrun) return Z_DATA_ERROR;
                if (op >= dstcap) return Z_BUF_ERROR;
                dst[op++] = (uint8_t)b;
            }
            continue;
        }
        if (type == 3) return Z_DATA_ERROR;
        if (type == 1) {
            uint8_t lens[320];
            int i = 0;
            for (; i < 144; i++) lens[i] = 8;
            for (; i < 256; i++) lens[i] = 9;
            for (; i < 280; i++) lens[i] = 7;
            for (; i < 288; i++) lens[i] = 8;
            build(&lencode, lens, 288, 1);
            for (i = 0; i < 32; i++) lens[i] = 5;     /* 30, 31 complete the code; they decode as invalid */
            build(&distcode, lens, 32, 2);
#ifdef ZLIB_SYM_TRACE
            zlib_block_trace(lens, 288, 32, 1);
#endif
        } else {
            static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
            int nlen = (int)need(&s, 5) + 257, ndist = (int)need(&s, 5) + 1, ncode = (int)need(&s, 4) + 4;
            if (s.overrun) return Z_DATA_ERROR;
            if (nlen > 286 || ndist > 30) return Z_DATA_ERROR;
            uint8_t lens[320];
            memset(lens, 0, sizeof(lens));
            for (int i = 0; i < ncode; i++) lens[order[i]] = (uint8_t)need(&s, 3);
            if (s.overrun) return Z_DATA_ERROR;
            if (build(&clcode, lens, 19, 0)) return Z_DATA_ERROR;
            int n = 0;
            while (n < nlen + ndist) {
                int sym = decode(&s, &clcode);
                if (sym < 0) return Z_DATA_ERROR;
                if (sym < 16) { lens[n++] = (uint8_t)sym; continue; }
                int rep, val = 0;
                if (sym == 16) {
                    if (n == 0) return Z_DATA_ERROR;
                    val = lens[n - 1];
                    rep = 3 + (int)need(&s, 2);
                } else if (sym == 17) {
                    rep = 3 + (int)need(&s, 3);
                } else {
                    rep = 11 + (int)need(&s, 7);
                }
                if (s.overrun) return Z_DATA_ERROR;
                if (n + rep > nlen + ndist) return Z_DATA_ERROR;
                while (rep--) lens[n++] = (uint8_t)val;
            }
            if (lens[256] == 0) return Z_DATA_ERROR;    /* no end-of-block code */
            if (build(&lencode, lens, nlen, 1)) return Z_DATA_ERROR;
            if (build(&distcode, lens + nlen, ndist, 2)) return Z_DATA_ERROR;
#ifdef ZLIB_SYM_TRACE
            zlib_block_trace(lens, nlen, ndist, 2);
#endif
        }
        for (;;) {
            int sym = decode(&s, &lencode);
            if (sym < 0) return Z_DATA_ERROR;
            if (sym < 256) {
                if (op >= dstcap) return Z_BUF_ERROR;
                dst[op++] = (uint8_t)sym;
#ifdef ZLIB_SYM_TRACE
                zlib_sym_trace(0, sym);
#endif
                continue;
            }
            if (sym == 256) break;
            sym -= 257;
            if (sym >= 29) return Z_DATA_ERROR;
            int len = kLenBase[sym] + (int)need(&s, kLenExtra[sym]);
            int ds = decode(&s, &distcode);
            if (ds < 0 || ds >= 30) return Z_DATA_ERROR;
            int dist = kDistBase[ds] + (int)need(&s, kDistExtra[ds]);
            if (s.overrun) return Z_DATA_ERROR;
            if (dist > op) return Z_DATA_ERROR;         /* invalid distance too far back */
#ifdef ZLIB_SYM_TRACE
            zlib_sym_trace(len, dist);
#endif
            for (int i = 0; i < len; i++) {
                if (op >= dstcap) return Z_BUF_ERROR;
                dst[op] = dst[op - dist];
                op++;
            }
        }
    } while (!last);
    /* adler32 trailer, big endian, after byte alignment */
    s.bits >>= (s.nbits & 7);
    s.nbits -= (s.nbits & 7);
    uint32_t a = need(&s, 8) << 24;
    a |= need(&s, 8) << 16;
    a |= need(&s, 8) << 8;
    a |= need(&s, 8);
    if (s.overrun) return Z_DATA_ERROR;
    if (a != oracle_adler32(dst, (int)op)) return Z_DATA_ERROR;
    return (int)op;
}
