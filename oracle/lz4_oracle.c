/*
 * oracle/lz4_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, CPU-only restatement of the LZ4 block codec exactly as the
 * reference vendors it (LZ4 1.7.5, /root/reference/src/lz4/lz4.c).  It is the
 * parity checker for the HIP kernels in tyche_amd/csrc and the "port" CPU
 * baseline in bench.py.  Nothing in the product path links or calls this
 * file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load liboracle.so.
 *
 * Pinning: checked byte-for-byte against tests/golden/ (reference outputs
 * produced by oracle/gen_golden.py from the vendored sources built by
 * oracle/Makefile into oracle/_ref/) and against the reference's own KAT
 * (src/tests.c:342-378 Lorem text -> 2578 B with LZ4 level 1).
 *
 * Written from the algorithm description, not from the reference text:
 *   compress   follows LZ4_compress_generic  lz4.c:459-656 (noDict, notLimited
 *              or limitedOutput, byU16 for n < LZ4_64Klimit else byU32),
 *              entered via LZ4_compress_default lz4.c:697 -> _fast :679 ->
 *              _fast_extState :659 (fresh zeroed table per call, :923).
 *   decompress follows LZ4_decompress_generic lz4.c:1089-1248 instantiated
 *              as LZ4_decompress_safe lz4.c:1251 (endOnInputSize, full,
 *              noDict): same acceptance rules and the same error value
 *              -(bytes of input consumed)-1 at the same consumption point.
 */
#include <stdint.h>
#include <string.h>
#include "oracle.h"

#define O_MINMATCH     4
#define O_LASTLITERALS 5
#define O_MFLIMIT      12                    /* WILDCOPYLENGTH + MINMATCH, lz4.c:266 */
#define O_MINLENGTH    (O_MFLIMIT + 1)       /* lz4.c:267 */
#define O_64K_LIMIT    (65536 + O_MFLIMIT - 1) /* LZ4_64Klimit, lz4.c:373 */
#define O_MAX_DISTANCE 65535
#define O_MAX_INPUT    0x7E000000
#define O_SKIP_TRIGGER 6                     /* lz4.c:374 */

static uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint64_t rd64(const uint8_t *p) {
    return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32);
}

int oracle_lz4_compress_bound(int n) {
    /* LZ4_COMPRESSBOUND, lz4.h:148 */
    if ((unsigned)n > (unsigned)O_MAX_INPUT) return 0;
    return n + n / 255 + 16;
}

/* Position table.  byU16 keeps 8192 16-bit offsets (13-bit hash of 4 bytes,
 * lz4.c:402-408); byU32 keeps 4096 32-bit offsets (12-bit hash of 5 bytes on a
 * 64-bit host, lz4.c:410-419).  Both live in the same 16 KiB state, zeroed per
 * call, so offset 0 is every bucket's initial candidate. */
typedef struct {
    int wide;              /* 0 = byU16, 1 = byU32 */
    union { uint16_t u16[8192]; uint32_t u32[4096]; } t;
} postab_t;

static uint32_t pt_hash(const postab_t *pt, const uint8_t *p) {
    if (!pt->wide) return (rd32(p) * 2654435761u) >> (32 - 13);
    return (uint32_t)(((rd64(p) << 24) * 889523592379ull) >> (64 - 12));
}
static void pt_put_h(postab_t *pt, uint32_t h, uint32_t pos) {
    if (pt->wide) pt->t.u32[h] = pos; else pt->t.u16[h] = (uint16_t)pos;
}
static uint32_t pt_get_h(const postab_t *pt, uint32_t h) {
    return pt->wide ? pt->t.u32[h] : pt->t.u16[h];
}

/* number of equal bytes between in[a..] and in[b..], stopping at limit (LZ4_count) */
static uint32_t common_len(const uint8_t *in, uint32_t a, uint32_t b, uint32_t limit) {
    uint32_t n = 0;
    while (a + n < limit && in[a + n] == in[b + n]) n++;
    return n;
}

/* writes a length continuation: k*255 ... remainder (RUN_MASK/ML_MASK = 15 already in the token) */
static uint8_t *put_len_tail(uint8_t *op, uint32_t rest) {
    while (rest >= 255) { *op++ = 255; rest -= 255; }
    *op++ = (uint8_t)rest;
    return op;
}

int oracle_lz4_compress(const uint8_t *src, uint8_t *dst, int n, int cap) {
    static __thread postab_t pt;   /* 16 KiB state like LZ4_stream_t */
    if ((unsigned)n > (unsigned)O_MAX_INPUT) return 0;
    int limited = cap < oracle_lz4_compress_bound(n);
    memset(&pt, 0, sizeof(pt));
    pt.wide = (n >= O_64K_LIMIT);

    const uint32_t end = (uint32_t)n;
    const uint32_t mflimit = end - O_MFLIMIT;       /* only used when n >= 13 */
    const uint32_t matchlimit = end - O_LASTLITERALS;
    uint32_t ip = 0, anchor = 0;
    uint8_t *op = dst;
    uint8_t *const olimit = dst + cap;

    if (n < O_MINLENGTH) goto last_literals;

    pt_put_h(&pt, pt_hash(&pt, src), 0);
    ip = 1;
    uint32_t fwd_h = pt_hash(&pt, src + ip);

    for (;;) {
        uint32_t cand;
        /* search, with the accelerating skip of lz4.c:519-546 */
        {
            uint32_t fwd = ip, step = 1, attempts = 1u << O_SKIP_TRIGGER;
            for (;;) {
                uint32_t h = fwd_h;
                ip = fwd;
                fwd += step;
                step = attempts++ >> O_SKIP_TRIGGER;
                if (fwd > mflimit) goto last_literals;
                cand = pt_get_h(&pt, h);
                fwd_h = pt_hash(&pt, src + fwd);
                pt_put_h(&pt, h, ip);
                if (pt.wide && cand + O_MAX_DISTANCE < ip) continue;
                if (rd32(src + cand) == rd32(src + ip)) break;
            }
        }
        /* extend backwards over the pending literals (lz4.c:549) */
        while (ip > anchor && cand > 0 && src[ip - 1] == src[cand - 1]) { ip--; cand--; }

        uint8_t *token;
        {
            uint32_t lit = ip - anchor;
            token = op++;
            if (limited && op + lit + (2 + 1 + O_LASTLITERALS) + lit / 255 > olimit) return 0;
            if (lit >= 15) { *token = 15 << 4; op = put_len_tail(op, lit - 15); }
            else *token = (uint8_t)(lit << 4);
            memcpy(op, src + anchor, lit);
            op += lit;
        }
        for (;;) {   /* one match, possibly chained directly into the next (lz4.c:565, 628) */
            uint32_t off = ip - cand;
            *op++ = (uint8_t)off;
            *op++ = (uint8_t)(off >> 8);
            uint32_t extra = common_len(src, ip + O_MINMATCH, cand + O_MINMATCH, matchlimit);
            ip += O_MINMATCH + extra;
            if (limited && op + (1 + O_LASTLITERALS) + (extra >> 8) > olimit) return 0;
            if (extra >= 15) { *token += 15; op = put_len_tail(op, extra - 15); }
            else *token += (uint8_t)extra;

            anchor = ip;
            if (ip > mflimit) goto last_literals;

            pt_put_h(&pt, pt_hash(&pt, src + ip - 2), ip - 2);
            uint32_t h = pt_hash(&pt, src + ip);
            cand = pt_get_h(&pt, h);
            pt_put_h(&pt, h, ip);
            if (cand + O_MAX_DISTANCE >= ip && rd32(src + cand) == rd32(src + ip)) {
                token = op++;
                *token = 0;
                continue;
            }
            break;
        }
        ip++;
        fwd_h = pt_hash(&pt, src + ip);
    }

last_literals: {
        uint32_t run = end - anchor;
        if (limited && (uint32_t)(op - dst) + run + 1 + (run + 255 - 15) / 255 > (uint32_t)cap) return 0;
        if (run >= 15) { *op++ = 15 << 4; op = put_len_tail(op, run - 15); }
        else *op++ = (uint8_t)(run << 4);
        memcpy(op, src + anchor, run);
        op += run;
    }
    return (int)(op - dst);
}

int oracle_lz4_compress_default(const uint8_t *src, uint8_t *dst, int n, int cap) {
    return oracle_lz4_compress(src, dst, n, cap);
}

/* Decoder.  Output bytes of a match are produced with forward byte-copy
 * semantics (what the 8-byte wild copies and dec32/dec64 tables of
 * lz4.c:1209-1236 amount to).  A match with offset 0 reads bytes the
 * reference never defined (uninitialised output memory); here they read as
 * whatever dst already holds at that position. */
int oracle_lz4_decompress_safe(const uint8_t *src, uint8_t *dst, int in_len, int out_cap) {
    /* signed 64-bit positions: the reference compares pointers such as
     * iend-RUN_MASK that may lie before the buffer for tiny inputs */
    const int64_t iend = in_len, oend = out_cap;
    int64_t ip = 0, op = 0;

    if (out_cap == 0) return (in_len == 1 && src[0] == 0) ? 0 : -1;
    if (in_len <= 0) return -1;   /* reference reads past the input here (UB); reported as an error */

    for (;;) {
        uint32_t token = src[ip++];
        int64_t lit = token >> 4;
        if (lit == 15) {
            uint32_t s;
            do {
                /* only a 1..3-byte input can run off the end here; the reference
                 * then reads one stray byte, and every value of it leads to the
                 * same error return below */
                s = ip < iend ? src[ip] : 0;
                ip++;
                lit += s;
            } while (ip < iend - 15 && s == 255);   /* lz4.c:1139-1141 */
        }
        /* terminal literal run, or an error (lz4.c:1147-1163) */
        if (op + lit > oend - O_MFLIMIT || ip + lit > iend - 8) {
            if (ip + lit != iend || op + lit > oend) return (int)(-ip - 1);
            memcpy(dst + op, src + ip, (size_t)lit);
            op += lit;
            return (int)op;
        }
        memcpy(dst + op, src + ip, (size_t)lit);
        ip += lit;
        op += lit;

        int64_t off = (int64_t)src[ip] | ((int64_t)src[ip + 1] << 8);
        ip += 2;
        if (off > op) return (int)(-ip - 1);                     /* lz4.c:1168 */

        int64_t ml = token & 15;
        if (ml == 15) {
            uint32_t s;
            do {
                s = src[ip++];
                if (ip > iend - O_LASTLITERALS) return (int)(-ip - 1);   /* lz4.c:1176 */
                ml += s;
            } while (s == 255);
        }
        ml += O_MINMATCH;
        if (op + ml > oend - O_LASTLITERALS) return (int)(-ip - 1);    /* lz4.c:1225 */
        for (int64_t i = 0; i < ml; i++) dst[op + i] = dst[op - off + i];
        op += ml;
    }
}
