/*
 * oracle/zstd_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the zstd frame decoder the reference calls in
 * buffer__decompress for ZSTD_COMPRESSOR_ID (src/buffer.c:263-266 ->
 * ZSTD_decompress, src/zstd/zstd_decompress.c:1459, vendored zstd v1.1.2).
 * It is the parity model for the gfx950 kernel (tyche_amd/csrc/zstd_decode.hip)
 * and follows the reference function by function:
 *
 *   frame header        ZSTD_frameHeaderSize / ZSTD_getFrameParams   zstd_decompress.c:226-307
 *   block loop          ZSTD_decompressFrame                         zstd_decompress.c:1369-1436
 *   literals section    ZSTD_decodeLiteralsBlock                     zstd_decompress.c:386-509
 *   Huffman tables      HUF_readStats / HUF_readDTableX2             entropy_common.c:168-227, huf_decompress.c:86-131
 *   Huffman streams     HUF_decompress1X2 / 4X2 (+ 4X_hufOnly gate)  huf_decompress.c:178-310, 860-870
 *   FSE headers         FSE_readNCount / FSE_buildDTable             entropy_common.c:65-157, fse_decompress.c:113-168
 *   FSE byte streams    FSE_decompress_usingDTable_generic           fse_decompress.c:218-275
 *   sequences header    ZSTD_decodeSeqHeaders / ZSTD_buildSeqTable   zstd_decompress.c:693-780
 *   sequence decode     ZSTD_decodeSequence                          zstd_decompress.c:851-923
 *   sequence execution  ZSTD_execSequence(+Last7) checks             zstd_decompress.c:803-1003
 *   sequence loop       ZSTD_decompressSequences                     zstd_decompress.c:1006-1061
 *   bit reader          BIT_initDStream / BIT_reloadDStream / BIT_lookBits(Fast)   bitstream.h:260-408
 *
 * The backward bit reader is emulated exactly (64-bit container, the same
 * reload points), so the number of symbols an FSE-compressed Huffman header
 * yields, and what the sequence loop reads from a stream that runs dry, are the
 * reference's.  Huffman literal streams are decoded with the single-symbol
 * (X2) tables in every case; the reference's 4X path may pick the double-symbol
 * X4 decoder (HUF_selectDecoder), which yields the same bytes for every stream
 * that decodes without error.
 *
 * Result: decoded size, or a negative value for any error (buffer.c:264-266
 * only tests ZSTD_isError).  XXH64 content checksums are verified when the
 * frame carries one (zstd_decompress.c:1425-1432).
 */
#include <stdint.h>
#include <string.h>
#include "oracle.h"
#ifdef ZSTD_SEQ_TRACE
void zstd_seq_trace(uint32_t llc, uint32_t mlc, uint32_t ofc, size_t ll, size_t ml, size_t off);
#endif

#define ZE_GENERIC (-1)
#define ZE_PREFIX (-10)
#define ZE_FRAMEPARAM (-14)
#define ZE_WINDOW (-16)
#define ZE_CORRUPT (-20)
#define ZE_CHECKSUM (-22)
#define ZE_DICT (-32)
#define ZE_TABLELOG (-44)
#define ZE_MAXSYM (-48)
#define ZE_DSTSIZE (-70)
#define ZE_SRCSIZE (-72)

#define BLOCKSIZE_MAX (128 * 1024)
#define MAXLL 35
#define MAXML 52
#define MAXOFF 28
#define LONGNBSEQ 0x7F00

/* ------------------------------------------------------------ bit reader */
typedef struct {
    uint64_t c;        /* bitContainer */
    uint32_t used;     /* bitsConsumed */
    const uint8_t *ptr, *start;
} bitd_t;

enum { BD_UNFINISHED = 0, BD_END_OF_BUFFER = 1, BD_COMPLETED = 2, BD_OVERFLOW = 3 };

static uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }   /* little-endian host */
static int highbit32(uint32_t v) { return 31 - __builtin_clz(v); }

/* bitstream.h:260-293.  Returns 0 or a negative error. */
static int bitd_init(bitd_t *b, const uint8_t *src, size_t n) {
    memset(b, 0, sizeof(*b));
    if (n < 1) return ZE_SRCSIZE;
    b->start = src;
    const uint8_t last = src[n - 1];
    if (n >= 8) {
        b->ptr = src + n - 8;
        b->c = rd64(b->ptr);
        b->used = last ? 8 - (uint32_t)highbit32(last) : 0;
        if (!last) return ZE_GENERIC;
    } else {
        b->ptr = src;
        b->c = src[0];
        for (size_t k = 1; k < n; k++) {
            /* switch fall-through of bitstream.h:277-283: bytes 1..3 at 8k, bytes 4..6 at 64-8(8-k)) */
            uint32_t sh = k <= 3 ? 8 * (uint32_t)k : 64 - 8 * (8 - (uint32_t)k);
            b->c += (uint64_t)src[k] << sh;
        }
        b->used = last ? 8 - (uint32_t)highbit32(last) : 0;
        if (!last) return ZE_GENERIC;
        b->used += (uint32_t)(8 - n) * 8;
    }
    return 0;
}

static uint64_t bitd_look(const bitd_t *b, uint32_t nb) {     /* BIT_lookBits */
    return ((b->c << (b->used & 63)) >> 1) >> ((63 - nb) & 63);
}
static uint64_t bitd_look_fast(const bitd_t *b, uint32_t nb) { /* BIT_lookBitsFast, nb >= 1 */
    return (b->c << (b->used & 63)) >> ((64 - nb) & 63);
}
static uint64_t bitd_read(bitd_t *b, uint32_t nb) { uint64_t v = bitd_look(b, nb); b->used += nb; return v; }
static uint64_t bitd_read_fast(bitd_t *b, uint32_t nb) { uint64_t v = bitd_look_fast(b, nb); b->used += nb; return v; }

static int bitd_reload(bitd_t *b) {                           /* BIT_reloadDStream */
    if (b->used > 64) return BD_OVERFLOW;
    if (b->ptr >= b->start + 8) {
        b->ptr -= b->used >> 3;
        b->used &= 7;
        b->c = rd64(b->ptr);
        return BD_UNFINISHED;
    }
    if (b->ptr == b->start) return b->used < 64 ? BD_END_OF_BUFFER : BD_COMPLETED;
    uint32_t nbytes = b->used >> 3;
    int r = BD_UNFINISHED;
    if (b->ptr - nbytes < b->start) { nbytes = (uint32_t)(b->ptr - b->start); r = BD_END_OF_BUFFER; }
    b->ptr -= nbytes;
    b->used -= nbytes * 8;
    b->c = rd64(b->ptr);
    return r;
}
static int bitd_end(const bitd_t *b) { return b->ptr == b->start && b->used == 64; }

/* ------------------------------------------------------------ FSE tables */
typedef struct { uint16_t new_state; uint8_t symbol, nb_bits; } fse_cell_t;
typedef struct { uint32_t log; fse_cell_t cell[512]; } fse_dt_t;

/* entropy_common.c:65-157 (FSE_readNCount).  Returns header bytes or < 0. */
static int read_ncount(int16_t *norm, uint32_t *max_sv, uint32_t *table_log, const uint8_t *hb, size_t hbsize) {
    const uint8_t *const istart = hb, *const iend = hb + hbsize;
    const uint8_t *ip = istart;
    if (hbsize < 4) return ZE_SRCSIZE;
    uint32_t bits;
    memcpy(&bits, ip, 4);
    int nb = (int)(bits & 0xF) + 5;
    if (nb > 15) return ZE_TABLELOG;
    bits >>= 4;
    int bitcount = 4;
    *table_log = (uint32_t)nb;
    int remaining = (1 << nb) + 1, threshold = 1 << nb;
    nb++;
    uint32_t charnum = 0;
    int prev0 = 0;
    while ((remaining > 1) & (charnum <= *max_sv)) {
        if (prev0) {
            uint32_t n0 = charnum;
            while ((bits & 0xFFFF) == 0xFFFF) {
                n0 += 24;
                if (ip < iend - 5) { ip += 2; memcpy(&bits, ip, 4); bits >>= bitcount; }
                else { bits >>= 16; bitcount += 16; }
            }
            while ((bits & 3) == 3) { n0 += 3; bits >>= 2; bitcount += 2; }
            n0 += bits & 3;
            bitcount += 2;
            if (n0 > *max_sv) return ZE_MAXSYM;
            while (charnum < n0) norm[charnum++] = 0;
            if ((ip <= iend - 7) || (ip + (bitcount >> 3) <= iend - 4)) {
                ip += bitcount >> 3;
                bitcount &= 7;
                memcpy(&bits, ip, 4);
                bits >>= bitcount;
            } else {
                bits >>= 2;
            }
        }
        {
            const int16_t max = (int16_t)((2 * threshold - 1) - remaining);
            int16_t count;
            if ((bits & (uint32_t)(threshold - 1)) < (uint32_t)max) {
                count = (int16_t)(bits & (uint32_t)(threshold - 1));
                bitcount += nb - 1;
            } else {
                count = (int16_t)(bits & (uint32_t)(2 * threshold - 1));
                if (count >= threshold) count -= max;
                bitcount += nb;
            }
            count--;
            remaining -= count < 0 ? -count : count;
            norm[charnum++] = count;
            prev0 = !count;
            while (remaining < threshold) { nb--; threshold >>= 1; }
            if ((ip <= iend - 7) || (ip + (bitcount >> 3) <= iend - 4)) {
                ip += bitcount >> 3;
                bitcount &= 7;
            } else {
                bitcount -= (int)(8 * (iend - 4 - ip));
                ip = iend - 4;
            }
            memcpy(&bits, ip, 4);
            bits >>= (bitcount & 31);
        }
    }
    if (remaining != 1) return ZE_CORRUPT;
    if (bitcount > 32) return ZE_CORRUPT;
    *max_sv = charnum - 1;
    ip += (bitcount + 7) >> 3;
    return (int)(ip - istart);
}

/* fse_decompress.c:113-168 (FSE_buildDTable).  Returns 0 or < 0. */
static int build_dtable(fse_dt_t *dt, const int16_t *norm, uint32_t max_sv, uint32_t table_log) {
    uint16_t next[256];
    const uint32_t size = 1u << table_log;
    uint32_t high = size - 1;
    if (max_sv > 255) return ZE_MAXSYM;
    if (table_log > 12) return ZE_TABLELOG;
    dt->log = table_log;
    for (uint32_t s = 0; s <= max_sv; s++) {
        if (norm[s] == -1) { dt->cell[high--].symbol = (uint8_t)s; next[s] = 1; }
        else next[s] = (uint16_t)norm[s];
    }
    const uint32_t mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= max_sv; s++)
        for (int i = 0; i < norm[s]; i++) {
            dt->cell[pos].symbol = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    if (pos != 0) return ZE_GENERIC;
    for (uint32_t u = 0; u < size; u++) {
        const uint8_t s = dt->cell[u].symbol;
        const uint32_t ns = next[s]++;
        dt->cell[u].nb_bits = (uint8_t)(table_log - (uint32_t)highbit32(ns));
        dt->cell[u].new_state = (uint16_t)((ns << dt->cell[u].nb_bits) - size);
    }
    return 0;
}

static void build_dtable_rle(fse_dt_t *dt, uint8_t sym) {   /* FSE_buildDTable_rle, fse_decompress.c:177-193 */
    dt->log = 0;
    dt->cell[0].new_state = 0;
    dt->cell[0].symbol = sym;
    dt->cell[0].nb_bits = 0;
}

/* FSE_decompress_usingDTable_generic (fse_decompress.c:218-275), symbol-by-symbol
 * (the fast/safe variants differ only in BIT_readBitsFast vs BIT_readBits, which
 * agree for nbBits >= 1; fastMode tables never hold 0-bit cells). */
static int fse_sym(fse_dt_t *dt, uint32_t *state, bitd_t *b, int fast) {
    const fse_cell_t c = dt->cell[*state];
    uint64_t low = fast ? bitd_read_fast(b, c.nb_bits) : bitd_read(b, c.nb_bits);
    *state = c.new_state + (uint32_t)low;
    return c.symbol;
}

static int fse_decompress_stream(uint8_t *dst, size_t cap, const uint8_t *src, size_t n, fse_dt_t *dt, int fast) {
    uint8_t *op = dst, *const omax = dst + cap, *const olimit = omax - 3;
    bitd_t b;
    int e = bitd_init(&b, src, n);
    if (e) return e;
    uint32_t s1 = (uint32_t)bitd_read(&b, dt->log); bitd_reload(&b);
    uint32_t s2 = (uint32_t)bitd_read(&b, dt->log); bitd_reload(&b);
    /* 4 symbols per loop; with FSE_MAX_TABLELOG 12 and a 64-bit container both
     * mid-loop reload tests of fse_decompress.c:235-246 are compiled out */
    for (; (bitd_reload(&b) == BD_UNFINISHED) & (op < olimit); op += 4) {
        op[0] = (uint8_t)fse_sym(dt, &s1, &b, fast);
        op[1] = (uint8_t)fse_sym(dt, &s2, &b, fast);
        op[2] = (uint8_t)fse_sym(dt, &s1, &b, fast);
        op[3] = (uint8_t)fse_sym(dt, &s2, &b, fast);
    }
    for (;;) {
        if (op > omax - 2) return ZE_DSTSIZE;
        *op++ = (uint8_t)fse_sym(dt, &s1, &b, fast);
        if (bitd_reload(&b) == BD_OVERFLOW) { *op++ = (uint8_t)fse_sym(dt, &s2, &b, fast); break; }
        if (op > omax - 2) return ZE_DSTSIZE;
        *op++ = (uint8_t)fse_sym(dt, &s2, &b, fast);
        if (bitd_reload(&b) == BD_OVERFLOW) { *op++ = (uint8_t)fse_sym(dt, &s1, &b, fast); break; }
    }
    return (int)(op - dst);
}

/* ------------------------------------------------------------ Huffman */
typedef struct { uint32_t log; uint8_t sym[4096]; uint8_t nb[4096]; } huf_dt_t;

/* entropy_common.c:168-227 (HUF_readStats) + huf_decompress.c:86-131 (HUF_readDTableX2).
 * Returns header bytes or < 0. */
static int huf_read_table(huf_dt_t *dt, const uint8_t *src, size_t n) {
    uint8_t w[256];
    uint32_t rank[17];
    if (!n) return ZE_SRCSIZE;
    size_t isize = src[0], osize;
    if (isize >= 128) {
        osize = isize - 127;
        isize = (osize + 1) / 2;
        if (isize + 1 > n) return ZE_SRCSIZE;
        if (osize >= 256) return ZE_CORRUPT;
        for (size_t k = 0; k < osize; k += 2) {
            w[k] = src[1 + k / 2] >> 4;
            w[k + 1] = src[1 + k / 2] & 15;
        }
    } else {
        if (isize + 1 > n) return ZE_SRCSIZE;
        /* FSE_decompress_wksp(huffWeight, 255, ip+1, iSize, ws, 6), fse_decompress.c:289-305 */
        int16_t norm[256];
        uint32_t max_sv = 255, tlog;
        int hs = read_ncount(norm, &max_sv, &tlog, src + 1, isize);
        if (hs < 0) return hs;
        if ((size_t)hs > isize) return ZE_SRCSIZE;   /* the reference would read outside the header here */
        if (tlog > 6) return ZE_TABLELOG;
        fse_dt_t fdt;
        int e = build_dtable(&fdt, norm, max_sv, tlog);
        if (e) return e;
        int fast = 1;
        const int16_t large = (int16_t)(1 << (tlog - 1));
        for (uint32_t s = 0; s <= max_sv; s++) if (norm[s] >= large) fast = 0;
        int r = fse_decompress_stream(w, 255, src + 1 + hs, isize - (size_t)hs, &fdt, fast);
        if (r < 0) return r;
        osize = (size_t)r;
    }
    memset(rank, 0, sizeof(rank));
    uint32_t total = 0;
    for (size_t k = 0; k < osize; k++) {
        if (w[k] >= 12) return ZE_CORRUPT;
        rank[w[k]]++;
        total += (1u << w[k]) >> 1;
    }
    if (total == 0) return ZE_CORRUPT;
    const uint32_t tlog = (uint32_t)highbit32(total) + 1;
    if (tlog > 12) return ZE_CORRUPT;
    {
        const uint32_t rest = (1u << tlog) - total;
        const uint32_t verif = 1u << highbit32(rest);
        const uint32_t lastw = (uint32_t)highbit32(rest) + 1;
        if (verif != rest) return ZE_CORRUPT;
        w[osize] = (uint8_t)lastw;
        rank[lastw]++;
    }
    if ((rank[1] < 2) || (rank[1] & 1)) return ZE_CORRUPT;
    const uint32_t nsym = (uint32_t)osize + 1;
    /* HUF_readDTableX2: maxTableLog 12 (HufLog), so tableLog <= 13 passes; readStats already bounds it */
    dt->log = tlog;
    uint32_t next = 0;
    for (uint32_t k = 1; k < tlog + 1; k++) {
        const uint32_t cur = next;
        next += rank[k] << (k - 1);
        rank[k] = cur;
    }
    for (uint32_t s = 0; s < nsym; s++) {
        const uint32_t wt = w[s], len = (1u << wt) >> 1;
        for (uint32_t i = rank[wt]; i < rank[wt] + len; i++) {
            dt->sym[i] = (uint8_t)s;
            dt->nb[i] = (uint8_t)(tlog + 1 - wt);
        }
        rank[wt] += len;
    }
    return (int)(isize + 1);
}

/* Decodes exactly `count` symbols from one stream; 0 when the stream ends exactly
 * there (HUF_decodeStreamX2 + BIT_endOfDStream), < 0 otherwise.  Symbols are
 * read through the exact container, reloading where HUF_decodeStreamX2 does. */
static int huf_stream(uint8_t *p, size_t count, const uint8_t *src, size_t n, const huf_dt_t *dt) {
    bitd_t b;
    int e = bitd_init(&b, src, n);
    if (e) return e;
    uint8_t *const pend = p + count;
#define HUF_ONE()                                                          \
    do {                                                                   \
        const uint32_t v = (uint32_t)bitd_look_fast(&b, dt->log);          \
        *p++ = dt->sym[v];                                                 \
        b.used += dt->nb[v];                                               \
    } while (0)
    while ((bitd_reload(&b) == BD_UNFINISHED) && (p + 4 <= pend)) { HUF_ONE(); HUF_ONE(); HUF_ONE(); HUF_ONE(); }
    while ((bitd_reload(&b) == BD_UNFINISHED) && (p < pend)) HUF_ONE();
    while (p < pend) HUF_ONE();
#undef HUF_ONE
    return bitd_end(&b) ? 0 : ZE_CORRUPT;
}

/* HUF_decompress4X2_usingDTable_internal (huf_decompress.c:231-310): the
 * interleaved main loop reloads every stream in lock step; since the decoded
 * bytes and the final end-of-stream test do not depend on where a stream is
 * reloaded (a reload never discards unread bits), each stream is decoded on its
 * own here. */
static int huf_4streams(uint8_t *dst, size_t dsize, const uint8_t *src, size_t n, const huf_dt_t *dt) {
    if (n < 10) return ZE_CORRUPT;
    const size_t l1 = (size_t)src[0] | ((size_t)src[1] << 8);
    const size_t l2 = (size_t)src[2] | ((size_t)src[3] << 8);
    const size_t l3 = (size_t)src[4] | ((size_t)src[5] << 8);
    const size_t l4 = n - (l1 + l2 + l3 + 6);
    if (l4 > n) return ZE_CORRUPT;
    const size_t seg = (dsize + 3) / 4;
    const uint8_t *s = src + 6;
    int e;
    /* BIT_initDStream errors come first, in stream order */
    bitd_t probe;
    if ((e = bitd_init(&probe, s, l1))) return e;
    if ((e = bitd_init(&probe, s + l1, l2))) return e;
    if ((e = bitd_init(&probe, s + l1 + l2, l3))) return e;
    if ((e = bitd_init(&probe, s + l1 + l2 + l3, l4))) return e;
    /* a tiny dsize (only reachable through set_repeat) lets streams 2-3 run past
     * dsize into the literal buffer's slack and leaves stream 4 with no symbols */
    const size_t n4 = dsize > 3 * seg ? dsize - 3 * seg : 0;
    if ((e = huf_stream(dst, seg, s, l1, dt))) return e;
    if ((e = huf_stream(dst + seg, seg, s + l1, l2, dt))) return e;
    if ((e = huf_stream(dst + 2 * seg, seg, s + l1 + l2, l3, dt))) return e;
    if ((e = huf_stream(dst + 3 * seg, n4, s + l1 + l2 + l3, l4, dt))) return e;
    return 0;
}

/* ------------------------------------------------------------ sequences */
static const uint32_t LL_BITS[MAXLL + 1] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                            1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12,
                                            13, 14, 15, 16};
static const uint32_t ML_BITS[MAXML + 1] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                            0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                            1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11,
                                            12, 13, 14, 15, 16};
static const uint32_t LL_BASE[MAXLL + 1] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
                                            16, 18, 20, 22, 24, 28, 32, 40, 48, 64, 0x80, 0x100, 0x200, 0x400, 0x800, 0x1000,
                                            0x2000, 0x4000, 0x8000, 0x10000};
static const uint32_t ML_BASE[MAXML + 1] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18,
                                            19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34,
                                            35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 0x83, 0x103, 0x203, 0x403, 0x803,
                                            0x1003, 0x2003, 0x4003, 0x8003, 0x10003};
static const uint32_t OF_BASE[MAXOFF + 1] = {0, 1, 1, 5, 0xD, 0x1D, 0x3D, 0x7D,
                                             0xFD, 0x1FD, 0x3FD, 0x7FD, 0xFFD, 0x1FFD, 0x3FFD, 0x7FFD,
                                             0xFFFD, 0x1FFFD, 0x3FFFD, 0x7FFFD, 0xFFFFD, 0x1FFFFD, 0x3FFFFD, 0x7FFFFD,
                                             0xFFFFFD, 0x1FFFFFD, 0x3FFFFFD, 0x7FFFFFD, 0xFFFFFFD};
/* default distributions, zstd_internal.h:118-136 */
static const int16_t LL_NORM[MAXLL + 1] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1,
                                           2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1,
                                           -1, -1, -1, -1};
static const int16_t ML_NORM[MAXML + 1] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1,
                                           1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                           1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1,
                                           -1, -1, -1, -1, -1};
static const int16_t OF_NORM[MAXOFF + 1] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1,
                                            1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

typedef struct {
    /* decoder context (ZSTD_DCtx fields used by one frame) */
    fse_dt_t ll, of, ml;           /* current sequence tables (copied, so set_repeat reuses them) */
    fse_dt_t ll_def, of_def, ml_def;
    int fse_entropy, lit_entropy;
    huf_dt_t huf;
    uint32_t rep[3];
    const uint8_t *lit_ptr;
    size_t lit_size;
    uint8_t lit_buf[BLOCKSIZE_MAX + 8];
} dctx_t;

/* ZSTD_buildSeqTable (zstd_decompress.c:693-724).  Returns bytes read or < 0. */
static int build_seq_table(fse_dt_t *dt, int type, uint32_t max, uint32_t max_log, const uint8_t *src, size_t n,
                           const fse_dt_t *def, int flag_repeat) {
    switch (type) {
    case 1:   /* set_rle */
        if (!n) return ZE_SRCSIZE;
        if (src[0] > max) return ZE_CORRUPT;
        build_dtable_rle(dt, src[0]);
        return 1;
    case 0:   /* set_basic */
        *dt = *def;
        return 0;
    case 3:   /* set_repeat */
        if (!flag_repeat) return ZE_CORRUPT;
        return 0;
    default: {
        int16_t norm[MAXML + 1];
        uint32_t tlog;
        int hs = read_ncount(norm, &max, &tlog, src, n);
        if (hs < 0) return ZE_CORRUPT;
        if (tlog > max_log) return ZE_CORRUPT;
        build_dtable(dt, norm, max, tlog);   /* return value ignored by the reference (:720) */
        return hs;
    }
    }
}

/* ZSTD_decodeLiteralsBlock (zstd_decompress.c:386-509).  Returns bytes read or < 0. */
static int decode_literals(dctx_t *d, const uint8_t *src, size_t n) {
    if (n < 3) return ZE_CORRUPT;
    const int type = src[0] & 3;
    const uint32_t lhl = (src[0] >> 2) & 3;
    if (type == 3 || type == 2) {
        if (type == 3 && d->lit_entropy == 0) return ZE_DICT;
        if (n < 5) return ZE_CORRUPT;
        size_t lh, lsize, csize;
        int single = 0;
        uint32_t lhc;
        memcpy(&lhc, src, 4);
        if (lhl <= 1) { single = !lhl; lh = 3; lsize = (lhc >> 4) & 0x3FF; csize = (lhc >> 14) & 0x3FF; }
        else if (lhl == 2) { lh = 4; lsize = (lhc >> 4) & 0x3FFF; csize = lhc >> 18; }
        else { lh = 5; lsize = (lhc >> 4) & 0x3FFFF; csize = (lhc >> 22) + ((size_t)src[4] << 10); }
        if (lsize > BLOCKSIZE_MAX) return ZE_CORRUPT;
        if (csize + lh > n) return ZE_CORRUPT;
        const uint8_t *cs = src + lh;
        int e = 0;
        if (type == 3) {
            /* HUF_decompress{1X,4X}_usingDTable with the previous table */
            e = single ? huf_stream(d->lit_buf, lsize, cs, csize, &d->huf) : huf_4streams(d->lit_buf, lsize, cs, csize, &d->huf);
        } else if (single) {
            /* HUF_decompress1X2_DCtx: table then one stream */
            int hs = huf_read_table(&d->huf, cs, csize);
            if (hs < 0) e = hs;
            else if ((size_t)hs >= csize) e = ZE_SRCSIZE;
            else e = huf_stream(d->lit_buf, lsize, cs + hs, csize - (size_t)hs, &d->huf);
        } else {
            /* HUF_decompress4X_hufOnly */
            if (lsize == 0) e = ZE_DSTSIZE;
            else if ((csize >= lsize) || (csize <= 1)) e = ZE_CORRUPT;
            else {
                int hs = huf_read_table(&d->huf, cs, csize);
                if (hs < 0) e = hs;
                else if ((size_t)hs >= csize) e = ZE_SRCSIZE;
                else e = huf_4streams(d->lit_buf, lsize, cs + hs, csize - (size_t)hs, &d->huf);
            }
        }
        if (e < 0) return ZE_CORRUPT;
        d->lit_ptr = d->lit_buf;
        d->lit_size = lsize;
        d->lit_entropy = 1;
        return (int)(csize + lh);
    }
    size_t lh, lsize;
    if (lhl == 1) { lh = 2; lsize = ((uint32_t)src[0] | ((uint32_t)src[1] << 8)) >> 4; }
    else if (lhl == 3) { lh = 3; lsize = ((uint32_t)src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16)) >> 4; }
    else { lh = 1; lsize = src[0] >> 3; }
    if (type == 0) {   /* set_basic: raw */
        if (lh + lsize > n) return ZE_CORRUPT;
        d->lit_ptr = src + lh;
        d->lit_size = lsize;
        return (int)(lh + lsize);
    }
    /* set_rle */
    if (lhl == 3 && n < 4) return ZE_CORRUPT;
    if (lsize > BLOCKSIZE_MAX) return ZE_CORRUPT;
    memset(d->lit_buf, src[lh], lsize);
    d->lit_ptr = d->lit_buf;
    d->lit_size = lsize;
    return (int)(lh + 1);
}

/* ZSTD_decompressSequences (zstd_decompress.c:1006-1061) + ZSTD_decodeSeqHeaders.
 * ostart: frame start (base == vBase, no dictionary).  Returns bytes written or < 0. */
static int decode_sequences(dctx_t *d, uint8_t *ostart, uint8_t *op0, uint8_t *oend, const uint8_t *src, size_t n) {
    const uint8_t *ip = src, *const iend = src + n;
    uint8_t *op = op0;
    if (n < 1) return ZE_SRCSIZE;
    int nbseq = *ip++;
    if (nbseq) {
        if (nbseq > 0x7F) {
            if (nbseq == 0xFF) {
                if (ip + 2 > iend) return ZE_SRCSIZE;
                nbseq = (int)((uint32_t)ip[0] | ((uint32_t)ip[1] << 8)) + LONGNBSEQ;
                ip += 2;
            } else {
                if (ip >= iend) return ZE_SRCSIZE;
                nbseq = ((nbseq - 0x80) << 8) + *ip++;
            }
        }
        if (ip + 4 > iend) return ZE_SRCSIZE;
        const int llt = *ip >> 6, oft = (*ip >> 4) & 3, mlt = (*ip >> 2) & 3;
        ip++;
        int r = build_seq_table(&d->ll, llt, MAXLL, 9, ip, (size_t)(iend - ip), &d->ll_def, d->fse_entropy);
        if (r < 0) return ZE_CORRUPT;
        ip += r;
        r = build_seq_table(&d->of, oft, MAXOFF, 8, ip, (size_t)(iend - ip), &d->of_def, d->fse_entropy);
        if (r < 0) return ZE_CORRUPT;
        ip += r;
        r = build_seq_table(&d->ml, mlt, MAXML, 9, ip, (size_t)(iend - ip), &d->ml_def, d->fse_entropy);
        if (r < 0) return ZE_CORRUPT;
        ip += r;
    }
    const uint8_t *lit = d->lit_ptr;
    const uint8_t *const lit_end = lit + d->lit_size;
    if (nbseq) {
        d->fse_entropy = 1;
        size_t rep[3] = {d->rep[0], d->rep[1], d->rep[2]};
        bitd_t b;
        if (bitd_init(&b, ip, (size_t)(iend - ip)) < 0) return ZE_CORRUPT;
        uint32_t sll = (uint32_t)bitd_read(&b, d->ll.log); bitd_reload(&b);
        uint32_t sof = (uint32_t)bitd_read(&b, d->of.log); bitd_reload(&b);
        uint32_t sml = (uint32_t)bitd_read(&b, d->ml.log); bitd_reload(&b);
        for (; (bitd_reload(&b) <= BD_COMPLETED) && nbseq;) {
            nbseq--;
            const uint32_t llc = d->ll.cell[sll].symbol, mlc = d->ml.cell[sml].symbol, ofc = d->of.cell[sof].symbol;
            size_t off;
            if (!ofc) off = 0;
            else off = OF_BASE[ofc] + (size_t)bitd_read_fast(&b, ofc);
            if (ofc <= 1) {
                off += (llc == 0);
                if (off) {
                    size_t t = (off == 3) ? rep[0] - 1 : rep[off];
                    t += !t;
                    if (off != 1) rep[2] = rep[1];
                    rep[1] = rep[0];
                    rep[0] = off = t;
                } else {
                    off = rep[0];
                }
            } else {
                rep[2] = rep[1];
                rep[1] = rep[0];
                rep[0] = off;
            }
            const size_t ml = ML_BASE[mlc] + ((mlc > 31) ? (size_t)bitd_read_fast(&b, ML_BITS[mlc]) : 0);
            const size_t ll = LL_BASE[llc] + ((llc > 15) ? (size_t)bitd_read_fast(&b, LL_BITS[llc]) : 0);
#ifdef ZSTD_SEQ_TRACE   /* tools/zstd_seq_stats.c only */
            zstd_seq_trace(llc, mlc, ofc, ll, ml, off);
#endif
            if (LL_BITS[llc] + ML_BITS[mlc] + ofc > 64 - 7 - (9 + 9 + 8)) bitd_reload(&b);
            {   /* FSE_updateState x3 (LL, ML, OF) */
                const fse_cell_t a = d->ll.cell[sll];
                sll = a.new_state + (uint32_t)bitd_read(&b, a.nb_bits);
                const fse_cell_t m = d->ml.cell[sml];
                sml = m.new_state + (uint32_t)bitd_read(&b, m.nb_bits);
                const fse_cell_t o = d->of.cell[sof];
                sof = o.new_state + (uint32_t)bitd_read(&b, o.nb_bits);
            }
            /* ZSTD_execSequence checks (:940-942, 952-954; Last7 :816-818, 829-831) */
            if (ml + ll > (size_t)(oend - op)) return ZE_DSTSIZE;
            if (ll > (size_t)(lit_end - lit)) return ZE_CORRUPT;
            uint8_t *const olit_end = op + ll;
            if (off > (size_t)(olit_end - ostart)) return ZE_CORRUPT;
            memcpy(op, lit, ll);          /* literals never overlap the output */
            lit += ll;
            const uint8_t *m = olit_end - off;
            for (size_t k = 0; k < ml; k++) olit_end[k] = m[k];   /* forward byte copy = overlap semantics */
            op = olit_end + ml;
        }
        if (nbseq) return ZE_CORRUPT;
        d->rep[0] = (uint32_t)rep[0];
        d->rep[1] = (uint32_t)rep[1];
        d->rep[2] = (uint32_t)rep[2];
    }
    const size_t last = (size_t)(lit_end - lit);
    if (last > (size_t)(oend - op)) return ZE_DSTSIZE;
    memcpy(op, lit, last);
    op += last;
    return (int)(op - op0);
}

/* ------------------------------------------------------------ XXH64 (checksum flag) */
#define P1 11400714785074694791ULL
#define P2 14029467366897019727ULL
#define P3 1609587929392839161ULL
#define P4 9650029242287828579ULL
#define P5 2870177450012600261ULL
static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t xround(uint64_t acc, uint64_t in) { acc += in * P2; acc = rotl(acc, 31); return acc * P1; }
static uint64_t xmerge(uint64_t acc, uint64_t v) { v = xround(0, v); acc ^= v; return acc * P1 + P4; }
uint64_t oracle_xxh64(const uint8_t *p, size_t len, uint64_t seed) {
    const uint8_t *const end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const uint8_t *const limit = end - 32;
        do {
            v1 = xround(v1, rd64(p)); v2 = xround(v2, rd64(p + 8));
            v3 = xround(v3, rd64(p + 16)); v4 = xround(v4, rd64(p + 24));
            p += 32;
        } while (p <= limit);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = xmerge(h, v1); h = xmerge(h, v2); h = xmerge(h, v3); h = xmerge(h, v4);
    } else {
        h = seed + P5;
    }
    h += (uint64_t)len;
    while (p + 8 <= end) { h ^= xround(0, rd64(p)); h = rotl(h, 27) * P1 + P4; p += 8; }
    if (p + 4 <= end) { uint32_t v; memcpy(&v, p, 4); h ^= (uint64_t)v * P1; h = rotl(h, 23) * P2 + P3; p += 4; }
    while (p < end) { h ^= (*p) * P5; h = rotl(h, 11) * P1; p++; }
    h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
    return h;
}

/* ------------------------------------------------------------ frame */
static dctx_t g_ctx;   /* test infrastructure: single-threaded use from ctypes */

int oracle_zstd_decompress(const uint8_t *src, int srclen, uint8_t *dst, int dstcap) {
    dctx_t *d = &g_ctx;
    size_t remaining = (size_t)srclen;
    const uint8_t *ip = src;
    uint8_t *const ostart = dst, *const oend = dst + dstcap;
    uint8_t *op = dst;
    build_dtable(&d->ll_def, LL_NORM, MAXLL, 6);
    build_dtable(&d->of_def, OF_NORM, MAXOFF, 5);
    build_dtable(&d->ml_def, ML_NORM, MAXML, 6);
    d->fse_entropy = d->lit_entropy = 0;
    d->rep[0] = 1; d->rep[1] = 4; d->rep[2] = 8;
    /* ZSTD_decompressFrame: srcSize >= frameHeaderSize_min (6) + blockHeaderSize (3) */
    if (remaining < 9) return ZE_SRCSIZE;
    uint32_t magic;
    memcpy(&magic, src, 4);
    const uint8_t fhd = src[4];
    const uint32_t did = fhd & 3, single = (fhd >> 5) & 1, fcs_id = fhd >> 6;
    uint32_t checksum = (fhd >> 2) & 1;
    static const uint32_t did_size[4] = {0, 1, 2, 4}, fcs_size[4] = {0, 2, 4, 8};
    const size_t fh = 5 + !single + did_size[did] + fcs_size[fcs_id] + (single && !fcs_id);
    if (remaining < fh + 3) return ZE_SRCSIZE;
    /* ZSTD_getFrameParams (:244-307).  A skippable magic passes with empty
     * parameters when the header is >= 8 bytes, and the blocks that follow are
     * decoded as usual (ZSTD_decompressFrame does not special-case it). */
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
        if (fh < 8) return ZE_SRCSIZE;
        checksum = 0;
    } else if (magic != 0xFD2FB528u) {
        return ZE_PREFIX;
    } else {
        if (fhd & 0x08) return ZE_FRAMEPARAM;
        size_t pos = 5;
        uint64_t window = 0, fcs = 0;
        uint32_t dict_id = 0;
        if (!single) {
            const uint8_t wl = src[pos++];
            const uint32_t wlog = (wl >> 3) + 10;
            if (wlog > 27) return ZE_WINDOW;   /* ZSTD_WINDOWLOG_MAX (64-bit) */
            window = 1ull << wlog;
            window += (window >> 3) * (wl & 7);
        }
        if (did == 1) { dict_id = src[pos]; pos += 1; }
        else if (did == 2) { dict_id = (uint32_t)src[pos] | ((uint32_t)src[pos + 1] << 8); pos += 2; }
        else if (did == 3) { memcpy(&dict_id, src + pos, 4); pos += 4; }
        if (fcs_id == 0) { if (single) fcs = src[pos]; }
        else if (fcs_id == 1) fcs = ((uint64_t)src[pos] | ((uint64_t)src[pos + 1] << 8)) + 256;
        else if (fcs_id == 2) { uint32_t v; memcpy(&v, src + pos, 4); fcs = v; }
        else memcpy(&fcs, src + pos, 8);
        if (!window) window = (uint32_t)fcs;
        if (window > (1u << 27)) return ZE_WINDOW;
        if (dict_id) return ZE_DICT;   /* no dictionary loaded (dctx->dictID == 0) */
    }
    ip += fh;
    remaining -= fh;
    for (;;) {
        if (remaining < 3) return ZE_SRCSIZE;
        const uint32_t bh = (uint32_t)ip[0] | ((uint32_t)ip[1] << 8) | ((uint32_t)ip[2] << 16);
        const uint32_t last = bh & 1, btype = (bh >> 1) & 3, csize0 = bh >> 3;
        if (btype == 3) return ZE_CORRUPT;
        const size_t csize = btype == 1 ? 1 : csize0;
        ip += 3;
        remaining -= 3;
        if (csize > remaining) return ZE_SRCSIZE;
        int dec;
        if (btype == 2) {
            /* ZSTD_decompressBlock_internal */
            if (csize >= BLOCKSIZE_MAX) return ZE_SRCSIZE;
            int lc = decode_literals(d, ip, csize);
            if (lc < 0) return lc;
            dec = decode_sequences(d, ostart, op, oend, ip + lc, csize - (size_t)lc);
        } else if (btype == 0) {
            if (csize > (size_t)(oend - op)) return ZE_DSTSIZE;
            memcpy(op, ip, csize);
            dec = (int)csize;
        } else {
            if (csize0 > (size_t)(oend - op)) return ZE_DSTSIZE;
            memset(op, ip[0], csize0);
            dec = (int)csize0;
        }
        if (dec < 0) return dec;
        op += dec;
        ip += csize;
        remaining -= csize;
        if (last) break;
    }
    if (checksum) {
        if (remaining < 4) return ZE_CHECKSUM;
        uint32_t rd;
        memcpy(&rd, ip, 4);
        if (rd != (uint32_t)oracle_xxh64(ostart, (size_t)(op - ostart), 0)) return ZE_CHECKSUM;
        remaining -= 4;
    }
    if (remaining) return ZE_SRCSIZE;
    return (int)(op - ostart);
}

/* ZSTD_compressBound (zstd_compress.c:37): FSE_compressBound(n) + 12 */
int oracle_zstd_compress_bound(int n) { return n + (n >> 7) + 512 + 12; }
