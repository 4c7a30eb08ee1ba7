// lz4_lc_core.h -- the per-lane algorithm of the chunked lane-per-page LZ4
// decoder (lz4_decode_lc.hip): the record parse (stage 1) and the record copies
// (stage 3), shared verbatim by the gfx950 kernel and by the host emulator
// tools/lc_emul.cpp, which runs it page by page against the oracle (the kernel's
// cross-lane parts -- the cooperative line flush -- are plain writes there).
//
// The includer provides: LC_FN (function qualifiers), u128, lq / lb (aligned LDS
// qword / byte), ld16 / sbyte (stream bytes from HBM), funnel8, keep_low,
// kMinMatch / kLastLiterals / kMfLimit / kRunMask (lz4.c:264-281).
#pragma once

#ifndef LC_FN
#define LC_FN __device__ __forceinline__
#endif
#ifndef LC_RCP
#define LC_RCP(x) __builtin_amdgcn_rcpf(x)
#endif
#ifndef LC_BARRIER
#define LC_BARRIER() asm volatile("" ::: "memory")
#endif
// Qword k of a lane's LDS buffer (ring or window) given the lane's base.  The
// kernel interleaves the 64 lanes' buffers qword by qword (qword k of lane L at
// (64 k + L) * 8): a wave-wide qword access then maps lane L to bank pair 2L
// whatever the positions (lanes 0-31 and 32-63 in separate cycles), where
// lane-contiguous buffers collide at random.  The host emulator's buffers are
// plain arrays.
#ifndef LC_Q
#define LC_Q(base, k) ((base) + ((uint32_t)(k) << 9))
#endif
#ifndef LC_PERM
#define LC_PERM(hi, lo, sel) __builtin_amdgcn_perm((hi), (lo), (sel))   // v_perm_b32
#endif
#ifndef LC_UMUL24
#define LC_UMUL24(a, b) __umul24((a), (b))   // v_mul_u32_u24 (full rate; v_mul_hi_u32 is not)
#define LC_MUL24(a, b) __mul24((a), (b))     // v_mul_i32_i24 / v_mad_i32_i24
#endif

// The match-copy table, one entry per offset class c = min(off, 16): the
// v_perm_b32 selectors that turn the 16 bytes at d - off (of which only the
// first off are the match's when off < 16) into the match's first 16 bytes,
// byte i = byte (i mod off) -- dword j = perm(s1, s0, sel[j]) | perm(s3, s2,
// sel[4 + j]), selector 0x0C giving a zero byte -- and e = the smallest multiple
// of off that is >= 16 (the second half's source distance).  Class 16 is the
// identity (no overlap); class 0 (offset 0: a malformed stream the reference
// accepts, undefined bytes) gives zeros.
constexpr int32_t kLutStride = 12;   // u32 per entry: 8 selectors, e, 3 unused (16-byte aligned entries)
constexpr int32_t kLutBytes = 17 * kLutStride * 4;
LC_FN void lc_lut_entry(int32_t c, uint32_t *ent) {
    for (int32_t j = 0; j < 4; j++) {
        uint32_t a = 0, b = 0;
        for (int32_t t = 0; t < 4; t++) {
            const int32_t i = 4 * j + t;
            const int32_t idx = c == 0 ? -1 : (c >= 16 ? i : i % c);
            const uint32_t sa = idx >= 0 && idx < 8 ? (uint32_t)idx : 0x0Cu;
            const uint32_t sb = idx >= 8 ? (uint32_t)(idx - 8) : 0x0Cu;
            a |= sa << (8 * t);
            b |= sb << (8 * t);
        }
        ent[j] = a;
        ent[4 + j] = b;
    }
    ent[8] = (uint32_t)(c >= 16 ? 16 : (c > 0 ? c * ((16 + c - 1) / c) : 16));
    ent[9] = ent[10] = ent[11] = 0;
}
// 16 bytes lo : hi rearranged by an entry's selectors
LC_FN void lc_lut_apply(const uint32_t *sel, uint64_t &lo, uint64_t &hi) {
    const uint32_t s0 = (uint32_t)lo, s1 = (uint32_t)(lo >> 32), s2 = (uint32_t)hi, s3 = (uint32_t)(hi >> 32);
    const uint32_t d0 = LC_PERM(s1, s0, sel[0]) | LC_PERM(s3, s2, sel[4]);
    const uint32_t d1 = LC_PERM(s1, s0, sel[1]) | LC_PERM(s3, s2, sel[5]);
    const uint32_t d2 = LC_PERM(s1, s0, sel[2]) | LC_PERM(s3, s2, sel[6]);
    const uint32_t d3 = LC_PERM(s1, s0, sel[3]) | LC_PERM(s3, s2, sel[7]);
    lo = (uint64_t)d0 | ((uint64_t)d1 << 32);
    hi = (uint64_t)d2 | ((uint64_t)d3 << 32);
}

// LC_FAR16 1: a far match part (source out of the ring, loaded from HBM into registers) takes at
// most 16 bytes, so a record slot needs one 16-byte far register instead of two (32 VGPRs fewer
// per wave); longer far matches continue in the next record
#ifndef LC_FAR16
#define LC_FAR16 1   // round 6: 182 -> 154 VGPRs, 1 % faster at 256K pages, equal at 1M (profiles/r06_*ab.log)
#endif
constexpr int32_t kFarPer = LC_FAR16 ? 1 : 2;   // 16-byte far registers per record slot
#ifndef LC_SLOTS
#define LC_SLOTS 7
#endif
constexpr int32_t kLC = LC_SLOTS;   // record slots per chunk (unrolled)
constexpr int32_t kLW = 64;          // window bytes
// (round 6 tried the window as a ring of rows refilled with only its missing 16-byte pieces, about
// 2 of 4 per chunk: slower, 24.8-24.9 vs 24.3-24.4 ms, profiles/r06_wring_ab.log)
constexpr int32_t kLWS = kLW;   // window bytes per lane in LDS (reads past the end land in later rows: unused bytes)

// 16 bytes at byte position p >= 0 of a lane's window (no wrap), as lo : hi
LC_FN void get16(const uint8_t *base, int32_t p, uint64_t &lo, uint64_t &hi) {
    const int32_t k = p >> 3;
    const uint64_t q0 = lq(LC_Q(base, k)), q1 = lq(LC_Q(base, k + 1)), q2 = lq(LC_Q(base, k + 2));
    const uint32_t s = (uint32_t)p & 7u;
    lo = funnel8(q0, q1, s);
    hi = funnel8(q1, q2, s);
}
// Ring rows (qwords) of a lane: R / 8 of them, R a power of two, 160 or 192 (20 / 24 rows:
// row = k mod 20 / 24 by an exact multiply-high division).  k >= -1 (positions >= -8).
template <int32_t R>
LC_FN int32_t lc_row(int32_t k) {
    constexpr int32_t rows = R / 8;
    if constexpr ((rows & (rows - 1)) == 0) {
        return k & (rows - 1);
    } else if constexpr (rows == 24) {
        // u / 24 = (u * 43691) >> 20 exactly for u < 2^16 (the error u * 3.2e-7 stays under 1/24
        // there; u <= 65535 / 8 + 25), with 24-bit multiplies
        const uint32_t u = (uint32_t)(k + rows);
        const uint32_t q = LC_UMUL24(u, 43691u) >> 20;
        return (int32_t)u + LC_MUL24((int32_t)q, -24);
    } else {
        static_assert(rows == 20, "ring rows: a power of two, 20 or 24");
        // u / 20 = (u * 3277) >> 16 exactly for u < 2^14 (error u * 3.1e-6 < 1/20; u <= 65535 / 8 + 21)
        const uint32_t u = (uint32_t)(k + rows);
        const uint32_t q = LC_UMUL24(u, 3277u) >> 16;
        return (int32_t)u + LC_MUL24((int32_t)q, -20);
    }
}
template <int32_t R>
LC_FN int32_t lc_row_next(int32_t r) { return r + 1 == R / 8 ? 0 : r + 1; }

// the same from a ring of R bytes (page position p >= -8; wraps)
template <int32_t R>
LC_FN void ring16(const uint8_t *ring, int32_t p, uint64_t &lo, uint64_t &hi) {
    const int32_t r0 = lc_row<R>(p >> 3);   // (arithmetic shift: p >= -8 wraps correctly)
    const int32_t r1 = lc_row_next<R>(r0), r2 = lc_row_next<R>(r1);
    const uint64_t q0 = lq(LC_Q(ring, r0)), q1 = lq(LC_Q(ring, r1)), q2 = lq(LC_Q(ring, r2));
    const uint32_t s = (uint32_t)p & 7u;
    lo = funnel8(q0, q1, s);
    hi = funnel8(q1, q2, s);
}
// the first n <= 16 bytes of lo : hi to page position d: the three aligned qwords
// from d & ~7 (bytes below d from the tail, garbage past d + n, which later
// output overwrites); returns the new tail, the qword holding d + n
template <int32_t R>
LC_FN uint64_t put16(uint8_t *ring, int32_t d, uint64_t tail, uint64_t lo, uint64_t hi,
                                          int32_t n) {
    const uint32_t s = (uint32_t)d & 7u;
    const int32_t q0 = d & ~7;
    const uint64_t o0 = keep_low(tail, lo << (8u * s), s);
    const uint64_t o1 = s ? (lo >> (64u - 8u * s)) | (hi << (8u * s)) : hi;
    const uint64_t o2 = s ? hi >> (64u - 8u * s) : 0ull;
    const int32_t r0 = lc_row<R>(q0 >> 3), r1 = lc_row_next<R>(r0), r2 = lc_row_next<R>(r1);
    lq(LC_Q(ring, r0), o0);
    lq(LC_Q(ring, r1), o1);
    lq(LC_Q(ring, r2), o2);
    const uint32_t k = (s + (uint32_t)n) >> 3;
    return k == 0 ? o0 : (k == 1 ? o1 : o2);
}

struct LPage {
    const uint8_t *in;
    uint8_t *out;
    int32_t L, C;
    size_t idx;
    int32_t ip;       // next stream byte the parse reads (a token, or the offset after a literal run)
    int32_t op;       // output bytes emitted into records
    int32_t fl;       // output bytes in HBM (a multiple of 16 until the page ends)
    int32_t wb;       // stream position of window byte 0 (a multiple of 16)
    uint64_t tail;
    int32_t lp, lrem;     // literal run in progress: stream position, bytes left
    int32_t moff, mrem;   // match in progress: offset, bytes left
    int32_t mtok;         // match-length nibble of the token whose header is pending
    int32_t hdr, term;    // offset/length header still to read; the literal run ends the block
};

enum : int32_t { kLParse = 0, kLCut = 1, kLEnd = 2 };

// Ring arithmetic (stage 4 flushes whole 16-byte pieces, so at a chunk's start
// the bytes in HBM reach fl >= op0 - 15; a record part at output position d has
// written at most up to d + 23 before it reads its source: the qwords of put16):
//  * a near source [d - off, d - off + 16) is still in the ring of R bytes while
//    off <= R - 24 (lc_near): larger offsets are far, read from HBM in stage 1;
//  * a far source's used bytes end at d + n2 - off <= op0 + budget - (R - 23),
//    below fl when budget <= R - 39; the chunk's writes (up to op0 + budget + 23)
//    must not reach the unflushed bytes [fl, op0) a ring turn later: the same
//    bound.  So budget = R - 40 (R - 24 - the flush granule, below).
// Flushing whole 64-byte lines instead (LC_LINE 64) leaves up to 63 bytes
// unflushed: budget = R - 23 - 64 = R - 87 by the same two bounds, and every
// flushed line leaves whole (fewer, full-line HBM writes).
#ifndef LC_LINE
#define LC_LINE 16
#endif
constexpr int32_t kLcLine = LC_LINE;   // flush granule: 16 or 64 bytes
static_assert(kLcLine == 16 || kLcLine == 64, "flush granule");
template <int32_t R>
constexpr int32_t lc_near() { return R - 24; }
template <int32_t R>
constexpr int32_t lc_budget() { return R - 24 - kLcLine; }
// a chunk's first record (<= 15 literal + 32 match bytes) must always fit
template <int32_t R>
constexpr bool lc_ring_ok() { return lc_budget<R>() >= 47; }

// record: literal part window position (6 bits) and length (<= 15), match part
// length (<= 32), offset (16 bits)
LC_FN uint32_t lc_rec(int32_t lpr, int32_t n1, int32_t n2, int32_t off) {
    return (uint32_t)lpr | ((uint32_t)n1 << 6) | ((uint32_t)n2 << 10) | ((uint32_t)off << 16);
}

// 8 bytes at byte r (0 <= r < 24) of the 32 bytes q0 : q1 : q2 : q3
LC_FN uint64_t win8(uint64_t q0, uint64_t q1, uint64_t q2, uint64_t q3, uint32_t r) {
    const uint32_t k = r >> 3;
    const uint64_t a = k == 0 ? q0 : (k == 1 ? q1 : q2), b = k == 0 ? q1 : (k == 1 ? q2 : q3);
    return funnel8(a, b, r & 7u);
}

// The common cases of a record in one step, computed for every lane with
// selects: the next part of a split match (its run done, header read), the next
// part of a long literal run that does not end in this part, or a whole new
// sequence (token, literal run < 15 bytes, header with <= 1 length byte, match
// <= 32 bytes) inside the window with none of the reference's checks failing.
// Returns 1 with the record; 0 when the chunk must stop here (the window or the
// output budget: the next chunk takes it); 2 when the lane needs the general
// path (parse_slot: the end of a long literal run and its header, long fields,
// the last literal run, any failing check -- repeated there in the reference's
// order).
// The window qwords q[0..3] at (x & ~7) are read by the caller for the first
// slot and by the slot before for every other one: as soon as a slot knows the
// length of its sequence it reads the next slot's, at the position the next
// slot will have if this one emits its record (the only case in which the next
// one runs), so the read's latency overlaps this slot's checks.
LC_FN void lc_wread(const uint8_t *w16, int32_t x, uint64_t (&q)[4]) {
    const int32_t k = x >> 3;
    q[0] = lq(LC_Q(w16, k));
    q[1] = lq(LC_Q(w16, k + 1));
    q[2] = lq(LC_Q(w16, k + 2));
    q[3] = lq(LC_Q(w16, k + 3));
}
// the window position of the chunk's first token (0 when the parse resumes inside a run)
LC_FN int32_t lc_x0(const LPage &P) {
    return (P.lrem == 0 && P.mrem == 0 && P.hdr == 0) ? min(P.ip - P.wb, kLW) : 0;
}

template <int32_t R>
LC_FN int32_t parse_fast(LPage &P, const uint8_t *w16, int32_t op0, uint32_t &rec, bool &far, int32_t &src,
                         uint64_t (&q)[4]) {
    const int32_t room = op0 + lc_budget<R>() - P.op;   // output bytes the chunk can still take
    // a: the next part of a match
    const bool isA = (P.mrem != 0) & (P.lrem == 0);   // (a budget cut can leave a header read before its run's last bytes)
    const int32_t nA = min(P.mrem, 32);
    // b: the next part of a literal run that goes on after it
    const int32_t nB = min(min(P.lrem, 15), P.wb + kLW - P.lp);
    const bool isB = (P.lrem != 0) & (nB < P.lrem);   // nB <= 0: the run continues past the window
    // c: a new sequence
    const bool fresh = (P.lrem == 0) & (P.mrem == 0) & (P.hdr == 0);
    const int32_t x = fresh ? P.ip - P.wb : 0;   // 0 <= x <= kLW at a token (the window starts at or before it)
    const uint64_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
    const uint32_t s = (uint32_t)x & 7u;
    const uint32_t token = (uint32_t)(win8(q0, q1, q2, q3, s) & 0xFFu);
    const int32_t lit = (int32_t)(token >> 4), mn = (int32_t)(token & 15u);
    const int32_t need = 1 + lit + (mn == 15 ? 3 : 2);   // stream bytes of the sequence
    // the next slot's window qwords: after this sequence, or (a continuation part) at ip; a
    // position past the window (clamped) means the next slot cannot take a fresh sequence
    lc_wread(w16, min(fresh ? x + need : P.ip - P.wb, kLW), q);
    const uint64_t h = win8(q0, q1, q2, q3, s + 1u + (uint32_t)(lit & 15));   // lit < 15 below: s + 1 + lit <= 22
    const int32_t off = (int32_t)(h & 0xFFFFu), ext = (int32_t)((h >> 16) & 0xFFu);
    const int32_t ml = mn == 15 ? 19 + ext : mn + kMinMatch;
    // Every condition below is combined with bitwise & / | on bools and every update is a select:
    // short-circuit && / if chains compile to exec-mask branches (s_and_saveexec / s_cbranch_execz
    // per term) that all 64 lanes walk anyway, since some lane almost always takes each side.
    const bool fitC = x + need <= kLW;
    const bool okC = (lit != 15) & !((mn == 15) & (ext == 255)) &
                     (P.op + lit <= P.C - kMfLimit) & (P.ip + 1 + lit <= P.L - 8) &   // not the last run (lz4.c:1147)
                     (off <= P.op + lit) &                                              // lz4.c:1168
                     !((mn == 15) & (P.ip + need > P.L - kLastLiterals)) &              // lz4.c:1176
                     (P.op + lit + ml <= P.C - kLastLiterals) &                         // lz4.c:1225
                     (ml <= 32);
    const int32_t moff = isA ? P.moff : off;
    const int32_t n1 = isA ? 0 : (isB ? nB : lit);
    const int32_t n2f = isA ? nA : (isB ? 0 : ml);
    const int32_t n2 = (LC_FAR16 && moff > lc_near<R>()) ? min(n2f, 16) : n2f;   // (LC_FAR16: far parts <= 16)
    const bool fits = n1 + n2 <= room;
    // k: 1 the record is emitted; 0 the chunk stops here (window or budget); 2 the general path
    const bool cont = isA | isB;
    const bool stop = !cont & (((P.lrem != 0) & (nB <= 0)) | (fresh & !fitC));
    const bool fast = cont | (fresh & okC);
    const int32_t k = stop ? 0 : (fast ? (fits ? 1 : 0) : 2);
    const bool emit = (k == 1);
    far = emit & (n2 > 0) & (moff > lc_near<R>());
    src = emit ? P.op + n1 - moff : src;
    rec = emit ? lc_rec(n1 > 0 ? (isB ? P.lp - P.wb : x + 1) : 0, n1, n2, moff) : rec;
    P.op += emit ? n1 + n2 : 0;
    P.mrem -= (emit & isA) ? n2 : 0;
    P.lp += (emit & isB) ? n1 : 0;
    P.lrem -= (emit & isB) ? n1 : 0;
    P.ip += (emit & fresh) ? need : 0;
    if (LC_FAR16) {   // a new sequence's far match cut at 16 bytes: the rest is a match in progress
        P.mrem += (emit & fresh) ? ml - n2 : 0;
        P.moff = (emit & fresh) ? off : P.moff;
    }
    return k;
}


// byte p of the stream: from the window when it lies there, else (only when
// `deep`, the chunk's first record: an extension run longer than the window)
// straight from HBM; `miss` reports a byte that neither provides
LC_FN uint32_t lbyte(const LPage &P, const uint8_t *w16, int32_t p, bool deep, bool &miss) {
    if (p < P.wb + kLW) {
        const int32_t i = p - P.wb;
        return lb(LC_Q(w16, i >> 3) + (i & 7));
    }
    if (deep) return sbyte(P.in, p, P.L);
    miss = true;
    return 0;
}

// One record slot of stage 1.  Parses what the next record needs (a token, the
// header after a literal run) and emits up to 16 literal and 16 match bytes.
// Returns the record (valid when emitted), sets `far` when its match part reads
// a source that has left the ring (src: its page position).
template <int32_t R>
LC_FN bool parse_slot(LPage &P, const uint8_t *w16, int32_t op0, bool deep, int32_t &st,
                                           int32_t &rv, uint32_t &rec, bool &far, int32_t &src) {
    constexpr int32_t kBudget = lc_budget<R>();
    const int32_t wend = P.wb + kLW;
    bool miss = false;
    // 1. a new sequence: token and literal length (lz4.c:1134-1163)
    if (P.lrem == 0 && P.mrem == 0 && P.hdr == 0) {
        const int32_t ip = P.ip;
        const uint32_t token = lbyte(P, w16, ip, deep, miss);
        int32_t lit = (int32_t)(token >> 4), pos = 1;
        if (lit == kRunMask) {
            uint32_t s;
            do {
                s = lbyte(P, w16, ip + pos, deep, miss);
                pos++;
                lit += (int32_t)s;
            } while (!miss && ip + pos < P.L - kRunMask && s == 255);
        }
        if (miss) {
            st = kLCut;
            return false;
        }
        const bool last = P.op + lit > P.C - kMfLimit || ip + pos + lit > P.L - 8;   // the last literal run
        if (last && (ip + pos + lit != P.L || P.op + lit > P.C)) {                   // (lz4.c:1155-1163)
            rv = -(ip + pos) - 1;
            st = kLEnd;
            return false;
        }
        // both fields written on both paths: a store of 1 to one or the other through a selected
        // address would put the lane state in scratch memory
        P.term = last ? 1 : 0;
        P.hdr = last ? 0 : 1;
        P.mtok = (int32_t)(token & 15u);
        P.lp = ip + pos;
        P.lrem = lit;
        P.ip = ip + pos + lit;
    }
    // 2. literal bytes of this record (those in the window)
    int32_t n1 = min(P.lrem, 15);
    n1 = min(n1, wend - P.lp);
    if (n1 < 0) n1 = 0;
    if (P.lrem > 0 && n1 == 0) {   // the run continues past the window: next chunk
        st = kLCut;
        return false;
    }
    // 3. the offset / match-length header once the run is done (lz4.c:1166-1182); bytes past the
    // window defer it to the next chunk (the checks are positional and run again there)
    if (P.lrem == n1 && P.hdr) {
        const int32_t ip = P.ip;
        const uint32_t off = lbyte(P, w16, ip, deep, miss) | (lbyte(P, w16, ip + 1, deep, miss) << 8);
        if (!miss) {
            int32_t pos = 2;
            if ((int32_t)off > P.op + n1) {   // lz4.c:1168
                rv = -(ip + pos) - 1;
                st = kLEnd;
                return false;
            }
            int32_t ml = P.mtok;
            if (ml == 15) {
                uint32_t s;
                do {
                    s = lbyte(P, w16, ip + pos, deep, miss);   // a missing byte: its position check still holds
                    pos++;
                    if (ip + pos > P.L - kLastLiterals) {   // lz4.c:1176
                        rv = -(ip + pos) - 1;
                        st = kLEnd;
                        return false;
                    }
                    ml += (int32_t)s;
                } while (!miss && s == 255);
            }
            if (!miss) {
                ml += kMinMatch;
                if (P.op + n1 + ml > P.C - kLastLiterals) {   // lz4.c:1225
                    rv = -(ip + pos) - 1;
                    st = kLEnd;
                    return false;
                }
                P.hdr = 0;
                P.moff = (int32_t)off;
                P.mrem = ml;
                P.ip = ip + pos;
            }
        }
        miss = false;
    }
    // 4. match bytes of this record (after the whole literal run)
    const int32_t n2 = (P.lrem == n1 && P.hdr == 0) ? min(P.mrem, (LC_FAR16 && P.moff > lc_near<R>()) ? 16 : 32) : 0;
    if (P.term && P.lrem == 0) {   // an empty last literal run (a stream the reference accepts)
        rv = P.op;
        st = kLEnd;
        return false;
    }
    if (n1 + n2 == 0) {   // nothing emittable (a header past the window)
        st = kLCut;
        return false;
    }
    if (P.op + n1 + n2 - op0 > kBudget) {
        st = kLCut;
        return false;
    }
    far = n2 > 0 && P.moff > lc_near<R>();
    src = P.op + n1 - P.moff;
    // window position of the literal part (0 without one: a match continuation's lp may lie before the window)
    rec = lc_rec(n1 > 0 ? P.lp - P.wb : 0, n1, n2, P.moff);
    P.lp += n1;
    P.lrem -= n1;
    P.op += n1 + n2;
    P.mrem -= n2;
    if (P.term && P.lrem == 0) {
        rv = P.op;
        st = kLEnd;
    }
    return true;
}

// Stage 3: the chunk's records into the ring, from output position d on.
// farv[kFarPer t] (and farv[2t + 1] when kFarPer is 2) hold the source bytes of record t's match
// part when that part is far (the second only when it is longer than 16 bytes).
// Slots 0..kLC-1 hold the fast path's records (the first nrec of them), slot
// kLC the general path's one (when gen).
template <int32_t R>
LC_FN void copy_records(uint8_t *ring, const uint8_t *w16, int32_t d, uint64_t &tail, const uint32_t *rec,
                        const u128 *farv, int32_t nrec, bool gen, const uint32_t *lut) {
    // the literal source of the record after the current one is read one record ahead (the
    // window is not written here): each record then waits for its match source only
    uint64_t llo, lhi;
    get16(w16, (int32_t)(rec[0] & 63u), llo, lhi);
#pragma unroll
    for (int32_t t = 0; t <= kLC; t++) {
        const uint32_t r = rec[t];
        const bool on = t < kLC ? t < nrec : gen;
        const int32_t n1 = on ? (int32_t)((r >> 6) & 15u) : 0, n2 = on ? (int32_t)((r >> 10) & 63u) : 0,
                      off = (int32_t)(r >> 16);
        uint32_t ent[12];
        lc_lut_load(lut, min(off, 16), ent);
        if (n1 > 0) {
            tail = put16<R>(ring, d, tail, llo, lhi, n1);
            d += n1;
        }
        if (t < kLC) get16(w16, (int32_t)(rec[t + 1] & 63u), llo, lhi);
        if (n2 > 0) {
            const bool far = off > lc_near<R>();
            const int32_t h1 = min(n2, 16);
            uint64_t lo, hi;
            ring16<R>(ring, d - off, lo, hi);
            if (far) {
                lo = (uint64_t)farv[kFarPer * t];
                hi = (uint64_t)(farv[kFarPer * t] >> 64);
            }
            lc_lut_apply(ent, lo, hi);   // the period-off pattern when the match overlaps itself
            tail = put16<R>(ring, d, tail, lo, hi, h1);
            if (n2 > 16) {
                // bytes 16..n2: a plain copy from e bytes back, e the smallest multiple of the offset
                // that is >= 16 (the first half, just written, repeats with that period)
                const int32_t e = off >= 16 ? off : (int32_t)ent[8];
                LC_BARRIER();
                ring16<R>(ring, d + 16 - e, lo, hi);
                if (far && kFarPer == 2) {
                    lo = (uint64_t)farv[kFarPer * t + (kFarPer - 1)];
                    hi = (uint64_t)(farv[kFarPer * t + (kFarPer - 1)] >> 64);
                }
                tail = put16<R>(ring, d + 16, tail, lo, hi, n2 - 16);
            }
            d += n2;
        }
        LC_BARRIER();
    }
}
