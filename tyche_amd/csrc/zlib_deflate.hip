// zlib_deflate.hip -- gfx950 encoder for zlib streams, the codec behind
// buffer__compress for ZLIB_COMPRESSOR_ID (src/buffer.c:190-200 -> compress2
// level 1, src/zlib/compress.c:22-60 -> deflate_fast, deflate.c:1628).  The
// output is a standard zlib stream that the reference's uncompress()
// (uncompr.c:22-59) restores bit-exactly with the exact length buffer.c:257-260
// requires; it is not required to be the bytes zlib 1.2.8 emits (SURVEY §8a
// A10).
//
// Stream: header 78 01 (compress2 at level 1, deflate.c:781-800), one final
// block holding the page's literals and length/distance pairs -- dynamic
// Huffman (BTYPE 10, trees built per page like _tr_flush_block, trees.c:907)
// or fixed (BTYPE 01, RFC 1951 3.2.6), whichever is smaller -- end-of-block,
// and the adler32 of the page (big-endian).  A page whose stream would not be
// smaller than the stored form is written as stored blocks (BTYPE 00).
//
// Dynamic trees need the page's symbol statistics before the first bit: the
// parse's records go to a per-wave device scratch (or, without one, to the
// tail of the output buffer), the
// hash table's LDS holds the histograms and codes once the parse is done, and
// the symbols are visited twice (count, then code).  When the records do not
// fit below the stream the page is coded in one pass with the fixed codes.
//
// One wave per page, looping over pages.  Matches come from the shared parse
// (lz_parse.h; distances > 32768 are turned back into literals).  Each batch of
// parse records becomes a symbol stream -- every literal byte and every match
// chunk of at most 258 bytes is one symbol -- coded 64 symbols per step: each
// lane builds its symbol's bits (Huffman code bit-reversed, extra bits LSB
// first, <= 31 bits), a DPP prefix sum gives bit offsets, the bits are OR-ed
// into a 128-dword LDS staging area, and complete bytes go to HBM.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "engine.h"
#include "lds_io.h"
#include "huf_enc.h"
#include "lz_parse.h"
#ifndef TYCHE_ZLIB_REP
#define TYCHE_ZLIB_REP 0
#endif
#ifndef TYCHE_ZLIB_MIN3
#define TYCHE_ZLIB_MIN3 1
#endif
// The sinks' page pointer for decode_record: the parse leaves the backward extension to its sinks
// (lz_parse.h kSinkBack) without 3-byte matches -- one-way, or repeat candidates -- so A/B builds of
// those (TYCHE_ZLIB_MIN3=0 with TYCHE_ZLIB_WAYS=1 or TYCHE_ZLIB_REP=1) hand the page over and keep
// the catch-up; the default parse keeps the extension in its records
#define ZLIB_SINK_IN(in) ((!TYCHE_ZLIB_MIN3 && ((TYCHE_ZLIB_WAYS == 1 && !TYCHE_ZLIB_REP) || (TYCHE_SINK_BACK && TYCHE_ZLIB_REP))) ? (in) : nullptr)
#ifndef TYCHE_ZLIB_WAYS
#define TYCHE_ZLIB_WAYS 8   // candidates per hash bucket (lz_parse.h kWays; 4 before round 3)
#endif

namespace tyche {
namespace {

using lzp::kHashSize;
using lzp::kWave;
constexpr int kWays = TYCHE_ZLIB_WAYS;
constexpr uint32_t kTableSlots = lzp::table_slots<kWays>();
constexpr uint32_t kPad = 64;
constexpr uint32_t kStageWords = 128;
constexpr uint32_t kPrefetchVec = 16;

__device__ __forceinline__ uint32_t hb(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }
__device__ __forceinline__ uint32_t rev(uint32_t code, uint32_t len) { return __builtin_bitreverse32(code) >> (32u - len); }

// fixed literal/length code of symbol s (RFC 1951 3.2.6), as stream bits and length
__device__ __forceinline__ void fixed_ll(uint32_t s, uint32_t &bits, uint32_t &len) {
    if (s < 144u) { bits = rev(0x30u + s, 8); len = 8; }
    else if (s < 256u) { bits = rev(0x190u + (s - 144u), 9); len = 9; }
    else if (s < 280u) { bits = rev(s - 256u, 7); len = 7; }
    else { bits = rev(0xC0u + (s - 280u), 8); len = 8; }
}

// bits of a length/distance pair (length 3..258, distance 1..32768): <= 31 bits
__device__ __forceinline__ void match_bits(uint32_t L, uint32_t D, uint32_t &bits, uint32_t &len) {
    uint32_t code, xb, xv;
    const uint32_t l = L - 3u;
    if (l < 8u) { code = 257u + l; xb = 0; xv = 0; }
    else if (l == 255u) { code = 285u; xb = 0; xv = 0; }
    else {
        const uint32_t h = hb(l);
        xb = h - 2u;
        code = 257u + 4u * (h - 1u) + ((l >> xb) & 3u);
        xv = l & ((1u << xb) - 1u);
    }
    uint32_t cb, cl;
    fixed_ll(code, cb, cl);
    bits = cb | (xv << cl);
    len = cl + xb;
    const uint32_t d = D - 1u;
    uint32_t dc, dxb, dxv;
    if (d < 4u) { dc = d; dxb = 0; dxv = 0; }
    else {
        const uint32_t h = hb(d);
        dxb = h - 1u;
        dc = 2u * h + ((d >> dxb) & 1u);
        dxv = d & ((1u << dxb) - 1u);
    }
    bits |= (rev(dc, 5) | (dxv << 5)) << len;
    len += 5u + dxb;
}

// length symbol (257..285) and extra bits of a match length 3..258
__device__ __forceinline__ void len_code(uint32_t L, uint32_t &code, uint32_t &xb, uint32_t &xv) {
    const uint32_t l = L - 3u;
    if (l < 8u) { code = 257u + l; xb = 0; xv = 0; }
    else if (l == 255u) { code = 285u; xb = 0; xv = 0; }
    else {
        const uint32_t h = hb(l);
        xb = h - 2u;
        code = 257u + 4u * (h - 1u) + ((l >> xb) & 3u);
        xv = l & ((1u << xb) - 1u);
    }
}
// distance symbol (0..29) and extra bits of a distance 1..32768
__device__ __forceinline__ void dist_code(uint32_t D, uint32_t &dc, uint32_t &dxb, uint32_t &dxv) {
    const uint32_t d = D - 1u;
    if (d < 4u) { dc = d; dxb = 0; dxv = 0; }
    else {
        const uint32_t h = hb(d);
        dxb = h - 1u;
        dc = 2u * h + ((d >> dxb) & 1u);
        dxv = d & ((1u << dxb) - 1u);
    }
}

// number of <= 258-byte chunks a match is coded as, and the length of chunk c
__device__ __forceinline__ uint32_t n_chunks(uint32_t ml) { return ml ? (ml + 257u) / 258u : 0u; }
__device__ __forceinline__ uint32_t chunk_len(uint32_t ml, uint32_t c) {
    const uint32_t n = n_chunks(ml);
    const uint32_t last = ml - 258u * (n - 1u);
    if (last >= 3u) return c + 1u < n ? 258u : last;
    // a 1- or 2-byte tail borrows from the chunk before it
    if (c + 2u < n) return 258u;
    return c + 2u == n ? 258u - (3u - last) : 3u;
}

struct Out {
    uint8_t *dst;
    uint32_t op;         // bytes written to dst
    uint32_t limit;      // abort once the stream would reach this size (stored form or capacity)
    uint32_t *stage;     // kStageWords dwords of pending bits
    uint32_t nbits;      // pending bits in stage
};

// Writes the complete bytes of the staging area and keeps the partial one.
__device__ __forceinline__ bool drain(Out &o, uint32_t lane) {
    const uint32_t nb = o.nbits >> 3;
    if (o.op + nb + 1u > o.limit) return false;
    const uint8_t *sb = (const uint8_t *)o.stage;
    for (uint32_t j = lane; j < nb; j += kWave) o.dst[o.op + j] = sb[j];
    const uint32_t part = (o.nbits & 7u) ? (uint32_t)sb[nb] : 0u;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t w = lane; w < kStageWords; w += kWave) o.stage[w] = w == 0 ? part : 0u;
    __builtin_amdgcn_wave_barrier();
    o.op += nb;
    o.nbits &= 7u;
    return true;
}

// Appends one symbol's bits per lane (v: up to 48 bits, LSB first) at the
// stream's bit cursor: DPP prefix sum of the lengths, OR into the staging
// dwords, complete bytes out.  Returns false when the stream reaches o.limit.
__device__ __forceinline__ bool put_lanes(Out &o, uint64_t v, uint32_t len, uint32_t lane) {
    const int32_t bi = wave_incl_sum((int32_t)len);
    const uint32_t b = o.nbits + (uint32_t)bi - len;
    if (len) {
        const uint32_t w = b >> 5, sh = b & 31u;
        const uint64_t lo = v << sh;
        atomicOr(&o.stage[w], (uint32_t)lo);
        if (sh + len > 32u) atomicOr(&o.stage[w + 1], (uint32_t)(lo >> 32));
        if (sh + len > 64u) atomicOr(&o.stage[w + 2], (uint32_t)(v >> (64u - sh)));
    }
    __builtin_amdgcn_wave_barrier();
    o.nbits += rdlane((uint32_t)bi, kWave - 1);
    return drain(o, lane);
}
// Appends n <= 32 bits, wave-uniform (header fields); the caller drains.
__device__ __forceinline__ void put_uniform(Out &o, uint32_t v, uint32_t n, uint32_t lane) {
    if (n == 0) return;
    if (lane == 0) {
        const uint32_t w = o.nbits >> 5, sh = o.nbits & 31u;
        const uint64_t x = (uint64_t)(v & (n == 32u ? ~0u : (1u << n) - 1u)) << sh;
        atomicOr(&o.stage[w], (uint32_t)x);
        if (sh + n > 32u) atomicOr(&o.stage[w + 1], (uint32_t)(x >> 32));
    }
    o.nbits += n;
}

// Visits the symbols of a batch of runs (lane i < n: literals in[ls, ls+ll),
// then a match of ml bytes at distance off; ml may be 0), 64 per step: every
// literal byte and every <= 258-byte match chunk is one symbol.  f(valid, lit,
// byte, mlen, dist) runs on all lanes once per step and returns false to stop.
template <typename F>
__device__ bool visit_runs(const uint8_t *in, uint32_t n, uint32_t ls, uint32_t ll, uint32_t ml, uint32_t off,
                           uint8_t *map, uint32_t lane, F &&f) {
    const bool act = lane < n;
    const uint32_t nsym = act ? ll + n_chunks(ml) : 0u;
    const int32_t si = wave_incl_sum((int32_t)nsym);
    const uint32_t s0 = (uint32_t)si - nsym;     // first symbol of this run
    const uint32_t total = rdlane((uint32_t)si, kWave - 1);
    for (uint32_t j0 = 0; j0 < total; j0 += kWave) {
        // owner run of symbol j0 + lane: the last non-empty run starting at or before it
        const uint64_t before = __ballot(act && nsym && s0 <= j0);
        const int32_t owner0 = before ? 63 - (int32_t)__builtin_clzll(before) : 0;
        map[lane] = 0xFF;
        __builtin_amdgcn_wave_barrier();
        if (act && nsym && s0 > j0 && s0 < j0 + kWave) map[s0 - j0] = (uint8_t)lane;
        __builtin_amdgcn_wave_barrier();
        const uint32_t mv = map[lane];
        const uint32_t ow = (uint32_t)max(wave_incl_max(mv == 0xFF ? -1 : (int32_t)mv), owner0);
        const uint32_t os0 = __shfl(s0, ow), ols = __shfl(ls, ow), oll = __shfl(ll, ow), oml = __shfl(ml, ow),
                       ooff = __shfl(off, ow);
        const uint32_t j = j0 + lane;
        const bool valid = j < total;
        bool lit = false;
        uint32_t byte = 0, mlen = 0;
        if (valid) {
            const uint32_t k = j - os0;
            if (k < oll) {
                lit = true;
                byte = in[ols + k];
            } else {
                mlen = chunk_len(oml, k - oll);
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (!f(valid, lit, byte, mlen, ooff)) return false;
    }
    return true;
}

// Codes a batch of runs with the fixed codes.  Returns false when the stream
// reaches o.limit.
__device__ bool code_runs(Out &o, const uint8_t *in, uint32_t n, uint32_t ls, uint32_t ll, uint32_t ml, uint32_t off,
                          uint8_t *map, uint32_t lane) {
    return visit_runs(in, n, ls, ll, ml, off, map, lane, [&](bool valid, bool lit, uint32_t byte, uint32_t mlen,
                                                              uint32_t dist) {
        uint32_t bits = 0, len = 0;
        if (valid) {
            if (lit) fixed_ll(byte, bits, len);
            else match_bits(mlen, dist, bits, len);
        }
        return put_lanes(o, bits, len, lane);
    });
}

// Stored form (RFC 1951 3.2.4): blocks of <= 65535 bytes after the zlib header.
__device__ int32_t emit_stored(const uint8_t *in, uint32_t L, uint8_t *dst, uint32_t cap, uint32_t adler,
                               uint32_t lane) {
    const uint32_t nblk = L ? (L + 65534u) / 65535u : 1u;
    const uint32_t size = 2u + L + 5u * nblk + 4u;
    if (size > cap) return 0;
    if (lane == 0) { dst[0] = 0x78; dst[1] = 0x01; }
    uint32_t op = 2;
    for (uint32_t k = 0; k < nblk; k++) {
        const uint32_t p0 = k * 65535u, bl = min(65535u, L - p0);
        const uint32_t hdr = (k + 1 == nblk ? 1u : 0u) | (bl << 8) | ((~bl & 0xFFFFu) << 24);
        if (lane < 4) dst[op + lane] = (uint8_t)(hdr >> (8u * lane));
        if (lane == 4) dst[op + 4] = (uint8_t)((~bl & 0xFFFFu) >> 8);
        op += 5;
        for (uint32_t j = lane; j < bl; j += kWave) dst[op + j] = in[p0 + j];
        op += bl;
    }
    if (lane < 4) dst[op + lane] = (uint8_t)(adler >> (24u - 8u * lane));
    return (int32_t)(op + 4);
}

// One pass with the fixed codes (the parse codes as it goes).  Returns the
// stream size, or 0 if even the stored form does not fit in cap.
__device__ int32_t encode_fixed1(const uint8_t *in, uint32_t L, uint32_t adler, uint16_t *table, uint8_t *map,
                                 uint2 *rec, uint32_t *stage, uint8_t *dst, uint32_t cap, uint32_t lane) {
    for (uint32_t w = lane; w < kTableSlots / 8; w += kWave) ((u32x4 *)table)[w] = u32x4{0, 0, 0, 0};
    WAVE_SYNC();
    const uint32_t nblk = L ? (L + 65534u) / 65535u : 1u;
    const uint32_t stored = 2u + L + 5u * nblk + 4u;
    Out o;
    o.dst = dst;
    o.op = 2;
    o.limit = min(stored, cap);           // the fixed-code stream must beat the stored form
    o.stage = stage;
    o.nbits = 3;                          // BFINAL = 1, BTYPE = 01
    for (uint32_t w = lane; w < kStageWords; w += kWave) stage[w] = w == 0 ? 3u : 0u;
    __builtin_amdgcn_wave_barrier();
    bool ok = 2u < o.limit;
    if (ok && lane == 0) { dst[0] = 0x78; dst[1] = 0x01; }
    uint32_t anchor = 0;
    if (ok) {
        auto sink = [&](const uint2 *r, uint32_t n, uint32_t anc) -> bool {
            uint32_t ls, ll, ml, off;
            lzp::decode_record(r, n, anc, lane, ls, ll, ml, off, ZLIB_SINK_IN(in));
            if (off > 32768u) { ll += ml; ml = 0; }     // beyond the deflate window: literals
            return code_runs(o, in, n, ls, ll, ml, off, map, lane);
        };
        anchor = lzp::parse_page<TYCHE_ZLIB_REP != 0, TYCHE_ZLIB_MIN3 != 0, kWays>(in, L, table, rec, lane, sink);
        ok = anchor != 0xFFFFFFFFu;
    }
    if (ok) ok = code_runs(o, in, 1, anchor, L - anchor, 0, 1, map, lane);   // last literals
    if (ok) {
        o.nbits += 7;                                   // end of block: symbol 256, 7 zero bits
        o.nbits = (o.nbits + 7u) & ~7u;                 // byte alignment before the trailer
        ok = drain(o, lane) && o.op + 4u < o.limit;
    }
    if (!ok) return emit_stored(in, L, dst, cap, adler, lane);
    if (lane < 4) dst[o.op + lane] = (uint8_t)(adler >> (24u - 8u * lane));
    return (int32_t)(o.op + 4u);
}

// ---- dynamic trees (trees.c build_tree / scan_tree / send_tree, RFC 1951 3.2.7)
constexpr uint32_t kLL = 286, kDist = 30;
__device__ __constant__ uint8_t c_cl_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// length of litlen symbol i / distance symbol i from lane-resident lengths (i uniform)
__device__ __forceinline__ uint32_t len_at(const uint32_t (&l)[5], uint32_t i) { return huf::pick_lane<5>(l, i >> 6, i & 63u); }

// Run-length codes of a code-length sequence (trees.c scan_tree / send_tree):
// emit(sym, extra, nxb) for every code-length symbol, uniform.
template <typename Get, typename Emit>
__device__ void scan_tree(uint32_t n, Get &&get, Emit &&emit) {
    int32_t prevlen = -1;
    uint32_t nextlen = get(0u), count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t curlen = nextlen;
        nextlen = i + 1u < n ? get(i + 1u) : 0xFFFFu;
        if (++count < max_count && curlen == nextlen) continue;
        if (count < min_count) {
            do emit(curlen, 0u, 0u); while (--count);
        } else if (curlen != 0) {
            if ((int32_t)curlen != prevlen) {
                emit(curlen, 0u, 0u);
                count--;
            }
            emit(16u, count - 3u, 2u);
        } else if (count <= 10u) {
            emit(17u, count - 3u, 3u);
        } else {
            emit(18u, count - 11u, 7u);
        }
        count = 0;
        prevlen = (int32_t)curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

// Forces a usable code on alphabets with fewer than two used symbols: symbols
// a and b get length 1 (a complete one-bit code; RFC 1951 needs at least one
// distance code, and inflate rejects an incomplete litlen code).
template <int R>
__device__ __forceinline__ void two_symbol_code(uint32_t (&l)[R], uint32_t a, uint32_t b, uint32_t lane) {
#pragma unroll
    for (int j = 0; j < R; j++) {
        const uint32_t sv = lane + 64u * (uint32_t)j;
        l[j] = (sv == a || sv == b) ? 1u : 0u;
    }
}

// Encodes in[0, L) (LDS, 64 zero bytes after).  Returns the stream size, or 0
// if even the stored form does not fit in cap.
__device__ int32_t encode_page(const uint8_t *in, uint32_t L, uint16_t *table, uint8_t *map, uint2 *rec,
                               uint32_t *stage, uint8_t *dst, uint32_t cap, uint8_t *ws, uint32_t ws_bytes,
                               uint32_t lane) {
    const uint32_t adler = lds_adler32(in, L, lane);
    const uint32_t nblk = L ? (L + 65534u) / 65535u : 1u;
    const uint32_t stored = 2u + L + 5u * nblk + 4u;
    // ---- pass 1: parse; records (ls | ll << 16, ml | off << 16) go down from the
    // end of the wave's scratch (ws: room for L / 3 + 2 records, so every page's
    // records fit and none takes the fixed-code fallback for lack of room), or
    // without scratch from the 8-aligned end of the output buffer
    const bool own = ws != nullptr;
    const uintptr_t base = own ? (uintptr_t)ws : (uintptr_t)dst;
    const uintptr_t top = own ? base + ws_bytes : (base + cap) & ~(uintptr_t)7;
    const uint32_t room = top > base + 8u ? (uint32_t)((top - base - 8u) / 8u) : 0u;   // records that fit above byte 8
    uint2 *recs = (uint2 *)top;        // record i at recs[-1 - i]
    uint32_t nrec = 0;
    for (uint32_t w = lane; w < kTableSlots / 8; w += kWave) ((u32x4 *)table)[w] = u32x4{0, 0, 0, 0};
    WAVE_SYNC();
    auto sink = [&](const uint2 *r, uint32_t n, uint32_t anc) -> bool {
        if (nrec + n > room) return false;
        uint32_t ls, ll, ml, off;
        lzp::decode_record(r, n, anc, lane, ls, ll, ml, off, ZLIB_SINK_IN(in));
        if (off > 32768u) { ll += ml; ml = 0; off = 1; }     // beyond the deflate window: literals
        if (lane < n) recs[-1 - (int32_t)(nrec + lane)] = make_uint2(ls | (ll << 16), ml | (off << 16));
        nrec += n;
        return true;
    };
    const uint32_t anchor = lzp::parse_page<TYCHE_ZLIB_REP != 0, TYCHE_ZLIB_MIN3 != 0, kWays>(in, L, table, rec, lane, sink);
    if (anchor == 0xFFFFFFFFu || nrec + 1u > room)
        return encode_fixed1(in, L, adler, table, map, rec, stage, dst, cap, lane);
    if (lane == 0) recs[-1 - (int32_t)nrec] = make_uint2(anchor | ((L - anchor) << 16), 1u << 16);   // last literals
    nrec += 1;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");   // records visible, L1 invalidated
    __builtin_amdgcn_wave_barrier();
    // reverse them in place: record i at recf[i], the first ones nearest the
    // stream, so the stream may grow over the records already coded (pass 3)
    for (uint32_t i = lane; i < nrec / 2u; i += kWave) {
        const uint2 a = recs[-1 - (int32_t)i], b = recs[-(int32_t)(nrec - i)];
        recs[-1 - (int32_t)i] = b;
        recs[-(int32_t)(nrec - i)] = a;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
    __builtin_amdgcn_wave_barrier();
    const uint2 *recf = (const uint2 *)top - nrec;
    // ---- pass 2: symbol histograms in the hash table's LDS (litlen 0..319, distance 320..351)
    uint32_t *H = (uint32_t *)table;
    for (uint32_t k = lane; k < 352u; k += kWave) H[k] = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t xbits = 0;   // extra bits of lengths and distances (this lane's share)
    for (uint32_t r0 = 0; r0 < nrec; r0 += kWave) {
        const uint32_t cnt = min(nrec - r0, kWave);
        const uint2 rv = lane < cnt ? recf[r0 + lane] : make_uint2(0, 1u << 16);
        visit_runs(in, cnt, rv.x & 0xFFFFu, rv.x >> 16, rv.y & 0xFFFFu, rv.y >> 16, map, lane,
                   [&](bool valid, bool lit, uint32_t byte, uint32_t mlen, uint32_t dist) {
                       if (valid) {
                           if (lit) {
                               atomicAdd(&H[byte], 1u);
                           } else {
                               uint32_t c, xb, xv, dc, dxb, dxv;
                               len_code(mlen, c, xb, xv);
                               dist_code(dist, dc, dxb, dxv);
                               atomicAdd(&H[c], 1u);
                               atomicAdd(&H[320u + dc], 1u);
                               xbits += xb + dxb;
                           }
                       }
                       return true;
                   });
    }
    if (lane == 0) H[256] += 1u;   // end of block
    __builtin_amdgcn_wave_barrier();
    const uint32_t extra = huf::wave_sum(xbits);
    // ---- code lengths (<= 15 bits), fixed-code cost of the same symbols
    uint32_t cll[5], lll[5], cd[1], ld[1];
    uint32_t totl = 0, fixl = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t sv = lane + 64u * (uint32_t)j;
        cll[j] = sv < kLL ? H[sv] : 0u;
        totl += cll[j];
        fixl += cll[j] * (sv < 144u ? 8u : sv < 256u ? 9u : sv < 280u ? 7u : 8u);
    }
    cd[0] = lane < kDist ? H[320u + lane] : 0u;
    totl = huf::wave_sum(totl);
    const uint32_t totd = huf::wave_sum(cd[0]);
    const uint32_t fixed_bits = 3u + huf::wave_sum(fixl) + 5u * totd + extra;
    // (H is free once the counts are in registers: LDS scratch of the Huffman construction)
    __builtin_amdgcn_wave_barrier();
    if (huf::code_lengths<5>(cll, totl, 15, lll, lane, H) == 0) two_symbol_code<5>(lll, 0u, 256u, lane);
    if (huf::code_lengths<1>(cd, totd, 15, ld, lane, H) == 0) {
        const int32_t u = huf::wave_max(cd[0] ? (int32_t)lane : -1);
        two_symbol_code<1>(ld, u > 0 ? 0u : 1u, u > 0 ? (uint32_t)u : 0u, lane);
    }
    int32_t mlit = -1;
#pragma unroll
    for (int j = 0; j < 5; j++)
        if (lll[j]) mlit = (int32_t)(lane + 64u * (uint32_t)j);
    const uint32_t nlit = max(257u, (uint32_t)huf::wave_max(mlit) + 1u);
    const uint32_t ndist = max(1u, (uint32_t)huf::wave_max(ld[0] ? (int32_t)lane : -1) + 1u);
    uint32_t cost = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) cost += cll[j] * lll[j];
    cost += cd[0] * ld[0];
    const uint32_t data_bits = huf::wave_sum(cost) + extra;
    // code-length code: counts of the run-length symbols, then their lengths (<= 7)
    uint32_t clc = 0, clx = 0;
    auto getl = [&](uint32_t i) { return len_at(lll, i); };
    auto getd = [&](uint32_t i) { return rdlane(ld[0], i); };
    auto count_cl = [&](uint32_t sym, uint32_t, uint32_t nxb) {
        if (lane == sym) clc++;
        clx += nxb;
    };
    scan_tree(nlit, getl, count_cl);
    scan_tree(ndist, getd, count_cl);
    uint32_t ccl[1] = {clc}, lcl[1];
    if (huf::code_lengths<1>(ccl, huf::wave_sum(lane < 19u ? clc : 0u), 7, lcl, lane, H) == 0) {
        const int32_t u = huf::wave_max(clc ? (int32_t)lane : -1);
        two_symbol_code<1>(lcl, u > 0 ? 0u : 1u, u > 0 ? (uint32_t)u : 0u, lane);
    }
    uint32_t ncl = 19;
    while (ncl > 4u && rdlane(lcl[0], c_cl_order[ncl - 1u]) == 0u) ncl--;
    const uint32_t dyn_bits = 3u + 14u + 3u * ncl + huf::wave_sum(lane < 19u ? clc * lcl[0] : 0u) + clx + data_bits;
    const bool dyn = dyn_bits < fixed_bits;
    // ---- size checks: below the stored form, below the records still to be read
    const uint32_t bits = dyn ? dyn_bits : fixed_bits;
    const uint32_t size = 2u + (bits + 7u) / 8u + 4u;
    const uint32_t rec_lo = own ? cap : (uint32_t)(top - base) - 8u * nrec;
    if (size >= stored || size > cap) return emit_stored(in, L, dst, cap, adler, lane);
    // (the stream may not reach records still to be read: checked as it grows, o.limit)
    // ---- codes (bit-reversed | length << 16) over the histograms
    uint32_t rll[5], rd[1], rcl[1];
    huf::deflate_codes<5>(lll, rll, lane);
    huf::deflate_codes<1>(ld, rd, lane);
    huf::deflate_codes<1>(lcl, rcl, lane);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t sv = lane + 64u * (uint32_t)j;
        if (sv < 320u) H[sv] = rll[j] | (lll[j] << 16);
    }
    if (lane < 32u) H[320u + lane] = rd[0] | (ld[0] << 16);
    __builtin_amdgcn_wave_barrier();
    // ---- pass 3: header and symbols
    Out o;
    o.dst = dst;
    o.op = 2;
    o.limit = min(rec_lo, cap);
    o.stage = stage;
    o.nbits = 0;
    for (uint32_t w = lane; w < kStageWords; w += kWave) stage[w] = 0;
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) { dst[0] = 0x78; dst[1] = 0x01; }
    if (dyn) {
        put_uniform(o, 1u | (2u << 1), 3, lane);                       // BFINAL, BTYPE 10
        put_uniform(o, (nlit - 257u) | ((ndist - 1u) << 5) | ((ncl - 4u) << 10), 14, lane);
        for (uint32_t i = 0; i < ncl; i++) put_uniform(o, rdlane(lcl[0], c_cl_order[i]), 3, lane);
        __builtin_amdgcn_wave_barrier();
        if (!drain(o, lane)) return encode_fixed1(in, L, adler, table, map, rec, stage, dst, cap, lane);
        auto emit_cl = [&](uint32_t sym, uint32_t x, uint32_t nxb) {
            put_uniform(o, rdlane(rcl[0], sym), rdlane(lcl[0], sym), lane);
            put_uniform(o, x, nxb, lane);
            if (o.nbits > 2048u) {
                __builtin_amdgcn_wave_barrier();
                drain(o, lane);
            }
        };
        scan_tree(nlit, getl, emit_cl);
        scan_tree(ndist, getd, emit_cl);
    } else {
        put_uniform(o, 1u | (1u << 1), 3, lane);                       // BFINAL, BTYPE 01
    }
    __builtin_amdgcn_wave_barrier();
    bool ok = drain(o, lane);
    for (uint32_t r0 = 0; ok && r0 < nrec; r0 += kWave) {
        const uint32_t cnt = min(nrec - r0, kWave);
        const uint2 rv = lane < cnt ? recf[r0 + lane] : make_uint2(0, 1u << 16);
        o.limit = own ? cap : min(cap, rec_lo + 8u * (r0 + cnt));   // this group's records are in registers now
        ok = visit_runs(in, cnt, rv.x & 0xFFFFu, rv.x >> 16, rv.y & 0xFFFFu, rv.y >> 16, map, lane,
                        [&](bool valid, bool lit, uint32_t byte, uint32_t mlen, uint32_t dist) {
                            uint64_t v = 0;
                            uint32_t len = 0;
                            if (valid) {
                                if (!dyn) {
                                    uint32_t b32;
                                    if (lit) fixed_ll(byte, b32, len);
                                    else match_bits(mlen, dist, b32, len);
                                    v = b32;
                                } else if (lit) {
                                    const uint32_t e = H[byte];
                                    v = e & 0xFFFFu;
                                    len = e >> 16;
                                } else {
                                    uint32_t c, xb, xv, dc, dxb, dxv;
                                    len_code(mlen, c, xb, xv);
                                    dist_code(dist, dc, dxb, dxv);
                                    const uint32_t e = H[c], ed = H[320u + dc];
                                    const uint32_t cl = e >> 16, dl = ed >> 16;
                                    v = (uint64_t)(e & 0xFFFFu) | ((uint64_t)xv << cl) |
                                        ((uint64_t)(ed & 0xFFFFu) << (cl + xb)) | ((uint64_t)dxv << (cl + xb + dl));
                                    len = cl + xb + dl + dxb;
                                }
                            }
                            return put_lanes(o, v, len, lane);
                        });
    }
    if (ok) {
        // end of block, byte alignment, trailer
        if (dyn) put_uniform(o, H[256] & 0xFFFFu, H[256] >> 16, lane);
        else put_uniform(o, 0u, 7, lane);
        o.nbits = (o.nbits + 7u) & ~7u;
        __builtin_amdgcn_wave_barrier();
        ok = drain(o, lane) && o.op + 4u <= o.limit;
    }
    if (!ok) return encode_fixed1(in, L, adler, table, map, rec, stage, dst, cap, lane);
    if (lane < 4) dst[o.op + lane] = (uint8_t)(adler >> (24u - 8u * lane));
    return (int32_t)(o.op + 4u);
}

__global__ __launch_bounds__(64) void zlib_deflate_kernel(tyche_batch_t b, uint32_t in_cap, unsigned *ctr, uint8_t *ws,
                                                          uint32_t ws_stride) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint16_t *table = (uint16_t *)smem;
    uint32_t *stage_bits = (uint32_t *)(smem + kTableSlots * sizeof(uint16_t));
    uint8_t *map = (uint8_t *)(stage_bits + kStageWords);
    uint2 *rec = (uint2 *)(map + kWave);
    uint8_t *stage = (uint8_t *)(rec + kWave);
    const size_t stride = gridDim.x;

    size_t page = blockIdx.x;
    if (page >= b.count) return;
    PageRef p = batch_page(b, page);
    uint32_t head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, lane, kWave);
    for (;;) {
        const size_t next = ctr ? claim_page(ctr, lane) : page + stride;   // dynamic assignment (engine.h)
        PageRef pn;
        u32x4 pf[kPrefetchVec];
        uint32_t nhead = 0, nvec = 0;
        if (next < b.count) {
            pn = batch_page(b, next);
            if (pn.src_len <= in_cap && pn.src_len > 0) {
                uintptr_t a = (uintptr_t)pn.src;
                nhead = (uint32_t)(a & 15u);
                nvec = (nhead + pn.src_len + 15u) >> 4;
                const u32x4 *g = (const u32x4 *)(a - nhead);
#pragma unroll
                for (uint32_t k = 0; k < kPrefetchVec; k++) {
                    const uint32_t v = lane + k * kWave;
                    pf[k] = gload_nt(g + min(v, nvec - 1u));   // clamped: no branch, always in bounds
                }
            }
        }
        int32_t rv;
        if (p.src_len > in_cap) {
            rv = kResultTooLarge;
        } else {
            uint8_t *in = stage + head;
            in[p.src_len + lane] = 0;
            WAVE_SYNC();
            rv = encode_page(in, p.src_len, table, map, rec, stage_bits, p.dst, p.dst_cap,
                             ws ? ws + (size_t)blockIdx.x * ws_stride : nullptr, ws_stride, lane);
        }
        if (lane == 0) b.results[page] = rv;
        if (next >= b.count) break;
        WAVE_SYNC();
        page = next;
        p = pn;
        head = nhead;
        if (p.src_len <= in_cap && p.src_len > 0) {
            u32x4 *l = (u32x4 *)stage;
#pragma unroll
            for (uint32_t k = 0; k < kPrefetchVec; k++) {
                const uint32_t v = lane + k * kWave;
                if (v < nvec) l[v] = pf[k];
            }
            const u32x4 *g = (const u32x4 *)((uintptr_t)p.src - nhead);
            for (uint32_t v = lane + kPrefetchVec * kWave; v < nvec; v += kWave) l[v] = gload_nt(g + v);
        }
    }
}

}  // namespace

hipError_t launch_zlib_deflate(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    if (in_cap > 65535u) return hipErrorInvalidValue;    // 16-bit positions in the parse
    const size_t lds = kTableSlots * sizeof(uint16_t) + kStageWords * 4 + kWave + kWave * 8 +
                       ((in_cap + 16u + kPad + 15u) & ~15u);
    const size_t ncu = prepare_launch((const void *)zlib_deflate_kernel);
    const size_t per_cu = waves_per_cu((const void *)zlib_deflate_kernel, lds);
    const size_t grid = std::min<size_t>(b.count, ncu * per_cu);
    WorkCounter ctr(s, grid < b.count);
    if (!ctr.get()) return hipErrorOutOfMemory;
    // per-wave record scratch: L / 3 + 2 records of 8 bytes (each record but the
    // last covers a match of >= 3 bytes)
    const uint32_t ws_stride = ((in_cap / 3u + 3u) * 8u + 255u) & ~255u;
    ScratchLease ws(s, grid * (size_t)ws_stride);
    if (!ws.get()) return hipErrorOutOfMemory;   // the kernel writes its records there
    hipLaunchKernelGGL(zlib_deflate_kernel, dim3((unsigned)grid), dim3(kWave), lds, s, b, in_cap, ctr.get(),
                       (uint8_t *)ws.get(), ws_stride);
    return hipGetLastError();
}

}  // namespace tyche
