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

constexpr int32_t kLC = 7;           // record slots per chunk (unrolled)
constexpr int32_t kLW = 64;          // window bytes
constexpr int32_t kLWS = kLW;   // window stride: reads past a window's end land in the next (unused bytes)

// 16 bytes at byte position p of an 8-aligned LDS buffer (no wrap), as lo : hi
LC_FN void get16(const uint8_t *base, int32_t p, uint64_t &lo, uint64_t &hi) {
    const int32_t a = p & ~7;
    const uint64_t q0 = lq(base + a), q1 = lq(base + a + 8), q2 = lq(base + a + 16);
    const uint32_t s = (uint32_t)p & 7u;
    lo = funnel8(q0, q1, s);
    hi = funnel8(q1, q2, s);
}
// the same from a ring of R bytes (page position p >= -8; wraps)
template <int32_t R>
LC_FN void ring16(const uint8_t *ring, int32_t p, uint64_t &lo, uint64_t &hi) {
    const int32_t a = p & ~7;
    const uint64_t q0 = lq(ring + (a & (R - 1))), q1 = lq(ring + ((a + 8) & (R - 1))),
                   q2 = lq(ring + ((a + 16) & (R - 1)));
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
    lq(ring + (q0 & (R - 1)), o0);
    lq(ring + ((q0 + 8) & (R - 1)), o1);
    lq(ring + ((q0 + 16) & (R - 1)), o2);
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
//    bound.  So budget = R - 40.
template <int32_t R>
constexpr int32_t lc_near() { return R - 24; }
template <int32_t R>
constexpr int32_t lc_budget() { return R - 40; }

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
template <int32_t R>
LC_FN int32_t parse_fast(LPage &P, const uint8_t *w16, int32_t op0, uint32_t &rec, bool &far, int32_t &src) {
    const int32_t room = op0 + lc_budget<R>() - P.op;   // output bytes the chunk can still take
    // a: the next part of a match
    const bool isA = P.mrem != 0 && P.lrem == 0;   // (a budget cut can leave a header read before its run's last bytes)
    const int32_t nA = min(P.mrem, 32);
    // b: the next part of a literal run that goes on after it
    const int32_t nB = min(min(P.lrem, 15), P.wb + kLW - P.lp);
    const bool isB = P.lrem != 0 && nB < P.lrem;   // nB <= 0: the run continues past the window
    // c: a new sequence
    const bool fresh = P.lrem == 0 && P.mrem == 0 && P.hdr == 0;
    const int32_t x = fresh ? P.ip - P.wb : 0;   // 0 <= x <= kLW at a token (the window starts at or before it)
    const int32_t a = x & ~7;
    const uint64_t q0 = lq(w16 + a), q1 = lq(w16 + a + 8), q2 = lq(w16 + a + 16), q3 = lq(w16 + a + 24);
    const uint32_t s = (uint32_t)x & 7u;
    const uint32_t token = (uint32_t)(win8(q0, q1, q2, q3, s) & 0xFFu);
    const int32_t lit = (int32_t)(token >> 4), mn = (int32_t)(token & 15u);
    const uint64_t h = win8(q0, q1, q2, q3, s + 1u + (uint32_t)(lit & 15));   // lit < 15 below: s + 1 + lit <= 22
    const int32_t off = (int32_t)(h & 0xFFFFu), ext = (int32_t)((h >> 16) & 0xFFu);
    const int32_t ml = mn == 15 ? 19 + ext : mn + kMinMatch;
    const int32_t need = 1 + lit + (mn == 15 ? 3 : 2);   // stream bytes of the sequence
    const bool fitC = x + need <= kLW;
    const bool okC = lit != 15 && !(mn == 15 && ext == 255) &&
                     P.op + lit <= P.C - kMfLimit && P.ip + 1 + lit <= P.L - 8 &&   // not the last run (lz4.c:1147)
                     off <= P.op + lit &&                                             // lz4.c:1168
                     !(mn == 15 && P.ip + need > P.L - kLastLiterals) &&              // lz4.c:1176
                     P.op + lit + ml <= P.C - kLastLiterals &&                        // lz4.c:1225
                     ml <= 32;
    const int32_t n1 = isA ? 0 : (isB ? nB : lit);
    const int32_t n2 = isA ? nA : (isB ? 0 : ml);
    int32_t k;
    if (isA || isB)
        k = n1 + n2 <= room ? 1 : 0;
    else if (P.lrem != 0 && nB <= 0)
        k = 0;
    else if (fresh && !fitC)
        k = 0;
    else if (fresh && okC)
        k = n1 + n2 <= room ? 1 : 0;
    else
        k = 2;
    if (k == 1) {
        const int32_t moff = isA ? P.moff : off;
        far = n2 > 0 && moff > lc_near<R>();
        src = P.op + n1 - moff;
        rec = lc_rec(n1 > 0 ? (isB ? P.lp - P.wb : x + 1) : 0, n1, n2, moff);
        P.op += n1 + n2;
        if (isA) P.mrem -= n2;
        if (isB) {
            P.lp += n1;
            P.lrem -= n1;
        }
        if (fresh) P.ip += need;
    }
    return k;
}

// byte p of the stream: from the window when it lies there, else (only when
// `deep`, the chunk's first record: an extension run longer than the window)
// straight from HBM; `miss` reports a byte that neither provides
LC_FN uint32_t lbyte(const LPage &P, const uint8_t *w16, int32_t p, bool deep, bool &miss) {
    if (p < P.wb + kLW) return lb(w16 + (p - P.wb));
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
    const int32_t n2 = (P.lrem == n1 && P.hdr == 0) ? min(P.mrem, 32) : 0;
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
// farv[2t], farv[2t + 1] hold the source bytes of record t's match part when that
// part is far (the second only when it is longer than 16 bytes).
// Slots 0..kLC-1 hold the fast path's records (the first nrec of them), slot
// kLC the general path's one (when gen).
template <int32_t R>
LC_FN void copy_records(uint8_t *ring, const uint8_t *w16, int32_t d, uint64_t &tail, const uint32_t *rec,
                        const u128 *farv, int32_t nrec, bool gen) {
#pragma unroll
    for (int32_t t = 0; t <= kLC; t++) {
        if (t < kLC ? t < nrec : gen) {
            const uint32_t r = rec[t];
            const int32_t lpr = (int32_t)(r & 63u), n1 = (int32_t)((r >> 6) & 15u), n2 = (int32_t)((r >> 10) & 63u),
                          off = (int32_t)(r >> 16);
            if (n1 > 0) {
                uint64_t lo, hi;
                get16(w16, lpr, lo, hi);
                tail = put16<R>(ring, d, tail, lo, hi, n1);
                d += n1;
            }
            if (n2 > 0) {
                const bool far = off > lc_near<R>();
                const int32_t h1 = min(n2, 16);
                uint64_t lo, hi;
                if (far) {
                    lo = (uint64_t)farv[2 * t];
                    hi = (uint64_t)(farv[2 * t] >> 64);
                } else {
                    ring16<R>(ring, d - off, lo, hi);
                    if (off < h1) {
                        // the match overlaps itself: the off bytes below d repeat
                        // (offset 0, a malformed stream the reference accepts: undefined bytes, zeros here)
                        u128 p = 0;
                        if (off > 0) {
                            p = (((u128)hi << 64) | lo) & ((((u128)1) << (8 * off)) - 1);
                            for (int32_t len = off; len < 16; len <<= 1) p |= p << (8 * len);
                        }
                        lo = (uint64_t)p;
                        hi = (uint64_t)(p >> 64);
                    }
                }
                tail = put16<R>(ring, d, tail, lo, hi, h1);
                if (n2 > 16) {
                    // bytes 16..n2: a plain copy from 16 bytes behind a multiple of the offset that
                    // is >= 16 (the first half, just written, repeats with that period)
                    if (far) {
                        lo = (uint64_t)farv[2 * t + 1];
                        hi = (uint64_t)(farv[2 * t + 1] >> 64);
                    } else {
                        // e = off * ceil(16 / off) <= off + 15: the smallest period multiple >= 16 (16/off
                        // has a fraction >= 1/15 unless off divides 16, so +0.999 rounds up exactly)
                        const int32_t e = off >= 16 ? off : (off > 0 ? off * (int32_t)(16.0f * LC_RCP((float)off) + 0.999f) : 16);
                        LC_BARRIER();
                        ring16<R>(ring, d + 16 - e, lo, hi);
                    }
                    tail = put16<R>(ring, d + 16, tail, lo, hi, n2 - 16);
                }
                d += n2;
            }
            LC_BARRIER();
        }
    }
}
