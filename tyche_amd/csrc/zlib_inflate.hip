// zlib_inflate.hip -- gfx950 decoder for zlib-wrapped deflate streams, the
// codec behind buffer__decompress for ZLIB_COMPRESSOR_ID (src/buffer.c:256-260
// -> uncompress, src/zlib/uncompr.c:22-59 -> inflate, inflate.c:605,
// inffast.c:67, inftrees.c:32; adler32.c:65).
//
// One wave per page, waves loop over pages.  The serial part of inflate -- the
// Huffman bit stream -- runs on scalar registers:
//   * the compressed stream is read from HBM into a two-register window
//     (2 x 256 B per wave, the next 256 B loaded while the current ones are
//     decoded); 32-bit refills come out of it with v_readlane, so the bit
//     reader never touches LDS;
//   * each Huffman table is a 1024-entry root table held in 16 VGPRs (entry
//     r*64+lane in register r of that lane) and read with v_readlane; codes
//     longer than 10 bits go through a canonical-code slow path;
//   * decoded literals (position, byte) and matches (position, distance,
//     length) are collected in VGPRs with v_writelane and applied 64 at a time:
//     literals with one byte store per lane, matches with the frontier-grouped
//     copy (every pending match whose source ends before the first pending
//     destination is independent; four 16-lane groups copy four of them per
//     instruction).
// Table construction (canonical codes, completeness rules of inflate_table) is
// lane-parallel: ballots count code lengths, rank symbols and fill the root
// table.  The adler32 trailer is checked with a lane-parallel sum over the
// rebuilt page in LDS.
//
// Results follow the repo's restatement oracle/zlib_oracle.c exactly: the
// decoded length, or -3 (Z_DATA_ERROR) / -5 (Z_BUF_ERROR) at the same point of
// the stream.
#include <algorithm>
#include <cstdlib>

#include "engine.h"
#include "lds_io.h"

#ifndef TYCHE_BRIDGE_STEPS
#define TYCHE_BRIDGE_STEPS 4   // token-chain bridge steps per hand-off round (A/B builds)
#endif

namespace tyche {
namespace {

constexpr uint32_t kWave = 64;
constexpr int32_t kZData = -3;   // Z_DATA_ERROR
constexpr int32_t kZBuf = -5;    // Z_BUF_ERROR (output full, input left: uncompr.c:47-53)

// Optional phase profile of the lane-parallel path (diagnostic build only:
// -DTYCHE_PROFILE, tools/zpar_pages.py): shader cycles per phase summed by lane 0.
#ifdef TYCHE_PROFILE
__device__ unsigned long long g_zprof[16];
#define ZPROF_DECL unsigned long long _pt = clock64();
#define ZPROF_MARK(slot)                                                       \
    do {                                                                       \
        unsigned long long _n = clock64();                                     \
        if (lane == 0) atomicAdd(&g_zprof[slot], _n - _pt);                    \
        _pt = _n;                                                              \
    } while (0)
#define ZPROF_ADD(slot, v) do { if (lane == 0) atomicAdd(&g_zprof[slot], (unsigned long long)(v)); } while (0)
#else
#define ZPROF_DECL
#define ZPROF_MARK(slot) do { } while (0)
#define ZPROF_ADD(slot, v) do { } while (0)
#endif

// ---------------------------------------------------------------- table entries
// bits 0-3 code length, 4-6 kind, 8-11 extra bits, 16-31 value
enum : uint32_t { kLit = 0, kLen = 1, kEob = 2, kLong = 3, kBad = 4 };

__device__ __forceinline__ uint32_t mk(uint32_t kind, uint32_t extra, uint32_t val) {
    return (kind << 4) | (extra << 8) | (val << 16);
}
__device__ __forceinline__ uint32_t e_len(uint32_t e) { return e & 15u; }
__device__ __forceinline__ uint32_t e_kind(uint32_t e) { return (e >> 4) & 7u; }
__device__ __forceinline__ uint32_t e_extra(uint32_t e) { return (e >> 8) & 15u; }
__device__ __forceinline__ uint32_t e_val(uint32_t e) { return e >> 16; }

// literal/length alphabet (RFC 1951 3.2.5): 0-255 literal, 256 end of block,
// 257-285 lengths 3..258; 286/287 (fixed code only) are invalid (inflate.c LEN)
__device__ __forceinline__ uint32_t litlen_entry(uint32_t sym) {
    if (sym < 256u) return mk(kLit, 0, sym);
    if (sym == 256u) return mk(kEob, 0, 0);
    const uint32_t i = sym - 257u;
    if (i >= 29u) return mk(kBad, 0, 0);
    if (i == 28u) return mk(kLen, 0, 258);
    if (i < 8u) return mk(kLen, 0, 3u + i);
    const uint32_t x = (i - 4u) >> 2;
    return mk(kLen, x, 3u + ((4u + (i & 3u)) << x));
}
// distance alphabet: 0-29 distances 1..32768; 30/31 invalid
__device__ __forceinline__ uint32_t dist_entry(uint32_t sym) {
    if (sym >= 30u) return mk(kBad, 0, 0);
    if (sym < 4u) return mk(kLen, 0, 1u + sym);
    const uint32_t x = (sym - 2u) >> 1;
    return mk(kLen, x, 1u + ((2u + (sym & 1u)) << x));
}
__device__ __forceinline__ uint32_t sym_entry(uint32_t table_kind, uint32_t sym) {
    if (table_kind == 1) return litlen_entry(sym);
    if (table_kind == 2) return dist_entry(sym);
    return mk(kLit, 0, sym);   // code-length alphabet
}

// A decoder: 1024-entry root table in registers plus the canonical-code
// limits used by the slow path (lane k holds the value for code length k).
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));   // one register tuple, indexed with v_movrels

struct Table {
    u32x16 root;
    uint32_t lim;   // (first[k] + count[k]) << (15 - k): left-justified end of the length-k codes
    uint32_t dlt;   // offs[k] - first[k]: sorted-symbol index of code c of length k is dlt + c
};

__device__ __forceinline__ uint32_t lookup(const Table &t, uint32_t idx) {
    // index a register copy, not the struct: instcombine would turn rt[i] on a plain load back into
    // an indexed load from the Table's stack slot, which SROA cannot split -- the table then lives
    // in scratch memory
    u32x16 rt = t.root;
    asm volatile("" : "+v"(rt));
    return rdlane(rt[idx >> 6], idx & 63u);
}

// Canonical decode of a code longer than the root (the bits are LSB-first in bb).
__device__ __forceinline__ uint32_t slow_entry(const Table &t, const uint16_t *sorted, uint32_t table_kind,
                                               uint64_t bb, uint32_t lane) {
    const uint32_t v15 = __builtin_bitreverse32((uint32_t)bb) >> 17;
    const uint64_t m = __ballot(lane >= 1u && lane <= 15u && t.lim <= v15);
    const uint32_t l = (uint32_t)__builtin_popcountll(m) + 1u;
    if (l > 15u) return mk(kBad, 0, 0);
    const uint32_t idx = rdlane(t.dlt, l) + (v15 >> (15u - l));
    const uint32_t sym = rfl(sorted[idx]);
    return sym_entry(table_kind, sym) | l;
}

// Builds the decoder for code lengths lens[0..n) (LDS).  table_kind 0 = code
// lengths (must be complete), 1 = literal/length, 2 = distance (an incomplete
// code is accepted only when it is a single 1-bit code; an empty one decodes
// nothing).  Same acceptance as oracle build() / inflate_table (inftrees.c:32).
__device__ __forceinline__ bool build_table(const uint8_t *lens, uint32_t n, uint32_t table_kind, Table &t, uint16_t *sorted,
                            uint32_t lane) {
    uint32_t cnt[16];
#pragma unroll
    for (int l = 0; l < 16; l++) cnt[l] = 0;
    for (uint32_t c = 0; c < n; c += kWave) {
        const uint32_t s = c + lane;
        const uint32_t len = s < n ? lens[s] : 0u;
#pragma unroll
        for (uint32_t l = 1; l <= 15; l++) cnt[l] += (uint32_t)__builtin_popcountll(__ballot(len == l));
    }
    uint32_t maxl = 0;
#pragma unroll
    for (uint32_t l = 1; l <= 15; l++) if (cnt[l]) maxl = l;
    if (maxl == 0 && table_kind == 0) return false;
    int32_t left = 1;
#pragma unroll
    for (uint32_t l = 1; l <= 15; l++) {
        left = left * 2 - (int32_t)cnt[l];
        if (left < 0) return false;                              // over-subscribed
    }
    if (left > 0 && (table_kind == 0 || maxl != 1)) return false;   // incomplete
    // canonical first codes, sorted-symbol offsets, left-justified limits
    uint32_t run[16], lim_s[16], dlt_s[16];
    {
        uint32_t first = 0, offs = 0;
#pragma unroll
        for (uint32_t l = 1; l <= 15; l++) {
            run[l] = offs;
            dlt_s[l] = offs - first;
            lim_s[l] = (first + cnt[l]) << (15 - l);
            offs += cnt[l];
            first = (first + cnt[l]) << 1;
        }
    }
    t.lim = 0xFFFFFFFFu;
    t.dlt = 0;
#pragma unroll
    for (uint32_t l = 1; l <= 15; l++)
        if (lane == l) { t.lim = lim_s[l]; t.dlt = dlt_s[l]; }
    // symbols sorted by (length, value)
    for (uint32_t c = 0; c < n; c += kWave) {
        const uint32_t s = c + lane;
        const uint32_t len = s < n ? lens[s] : 0u;
        uint32_t pos = 0;
#pragma unroll
        for (uint32_t l = 1; l <= 15; l++) {
            const uint64_t m = __ballot(len == l);
            if (len == l) pos = run[l] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            run[l] += (uint32_t)__builtin_popcountll(m);
        }
        if (len) sorted[pos] = (uint16_t)s;
    }
    // root table: entry idx holds the code whose first 10 bits (LSB-first) are idx
    uint32_t sidx[16], l_of[16];
#pragma unroll
    for (uint32_t r = 0; r < 16; r++) {
        const uint32_t v = __builtin_bitreverse32(r * kWave + lane) >> 22;
        const uint32_t vlj = v << 5;
        uint32_t l = 1, d = dlt_s[1];
#pragma unroll
        for (uint32_t k = 1; k <= 15; k++) {
            if (lim_s[k] <= vlj) {
                l = k + 1;
                d = k < 15 ? dlt_s[k < 15 ? k + 1 : 15] : 0u;
            }
        }
        l_of[r] = l;
        sidx[r] = l <= 10 ? d + (v >> (10 - l)) : 0u;
    }
    u32x16 rt;   // assembled as a value and stored whole: element stores into t.root get
                 // merged into sub-vector stores that keep the table out of registers
#pragma unroll
    for (uint32_t r = 0; r < 16; r++) {
        const uint32_t l = l_of[r];
        uint32_t e;
        if (l <= 10) e = sym_entry(table_kind, sorted[sidx[r]]) | l;
        else if (l <= 15) e = mk(kLong, 0, 0);
        else e = mk(kBad, 0, 0);
        rt[r] = e;
    }
    t.root = rt;
    return true;
}

// The fixed codes of RFC 1951 3.2.6, computed per entry.
__device__ __forceinline__ void fixed_tables(Table &L, Table &D, uint32_t lane) {
    u32x16 lr, dr;
#pragma unroll
    for (uint32_t r = 0; r < 16; r++) {
        const uint32_t v = __builtin_bitreverse32(r * kWave + lane) >> 22;
        uint32_t sym, len;
        if ((v >> 3) < 24u) { sym = 256u + (v >> 3); len = 7; }
        else if ((v >> 2) < 192u) { sym = (v >> 2) - 48u; len = 8; }
        else if ((v >> 2) < 200u) { sym = 280u + (v >> 2) - 192u; len = 8; }
        else { sym = 144u + (v >> 1) - 400u; len = 9; }
        lr[r] = litlen_entry(sym) | len;
        dr[r] = dist_entry(v >> 5) | 5u;
    }
    L.root = lr;
    D.root = dr;
    L.lim = D.lim = 0xFFFFFFFFu;
    L.dlt = D.dlt = 0;
}

// ---------------------------------------------------------------- bit reader
struct BitReader {
    uint64_t bb;         // bit buffer, next bit at bit 0
    uint32_t bc;         // valid bits in bb (may run past the end of the stream: avail guards)
    uint32_t inpos;      // stream byte that enters bb next
    int32_t avail;       // stream bits not yet consumed
    const uint32_t *s4;  // stream start rounded down to 4 bytes
    uint32_t h;          // stream start & 3
    uint32_t nd;         // dwords of s4 that hold stream bytes
    uint32_t wbase;      // byte offset (from s4) of window A
    uint32_t wa, wb;     // window A = s4 bytes [wbase, wbase+256), B = the next 256
};

__device__ __forceinline__ uint32_t load_win(const BitReader &r, uint32_t base, uint32_t lane) {
    const uint32_t q = (base >> 2) + lane;
    return q < r.nd ? gload_nt(r.s4 + q) : 0u;
}

__device__ __forceinline__ void refill(BitReader &r, uint32_t lane) {
    if (r.bc >= 32) return;
    uint32_t rel = r.inpos + r.h - r.wbase;
    if (rel >= 256u) {
        r.wa = r.wb;
        r.wbase += 256u;
        r.wb = load_win(r, r.wbase + 256u, lane);
        rel -= 256u;
    }
    const uint32_t q = rel >> 2, sh = (rel & 3u) * 8u;
    const uint32_t d0 = rdlane(r.wa, q);
    const uint32_t d1 = q + 1 < 64u ? rdlane(r.wa, q + 1) : rdlane(r.wb, 0);
    const uint32_t w = (uint32_t)((((uint64_t)d1 << 32) | d0) >> sh);
    r.bb |= (uint64_t)w << r.bc;
    r.bc += 32;
    r.inpos += 4;
}

__device__ __forceinline__ uint32_t take(BitReader &r, uint32_t n) {
    const uint32_t v = (uint32_t)(r.bb & ((1ull << n) - 1ull));
    r.bb >>= n;
    r.bc -= n;
    r.avail -= (int32_t)n;
    return v;
}

// restart the reader at stream byte pos (after a stored block)
__device__ __forceinline__ void seek(BitReader &r, uint32_t pos, uint32_t lane) {
    r.bb = 0;
    r.bc = 0;
    r.inpos = pos;
    r.wbase = (pos + r.h) & ~255u;
    r.wa = load_win(r, r.wbase, lane);
    r.wb = load_win(r, r.wbase + 256u, lane);
}

// v_writelane: lane j of v takes the (uniform) value x
__device__ __forceinline__ uint32_t put_lane(uint32_t v, uint32_t j, uint32_t x, uint32_t lane) {
    return lane == j ? x : v;
}


// ------------------------------------------------------------- batched output
struct Pending {
    uint32_t lit;    // lane j: (position << 8) | byte of the j-th pending literal
    uint32_t md;     // lane j: destination of the j-th pending match
    uint32_t mx;     // lane j: distance | length << 16
    uint32_t nlit, nmat;
};

__device__ __forceinline__ void flush_literals(Pending &q, uint8_t *out, uint32_t lane) {
    if (lane < q.nlit) out[q.lit >> 8] = (uint8_t)q.lit;
    q.nlit = 0;
}

// Applies the pending matches in stream order semantics (RFC 1951 3.2.3: a copy
// may overlap its own output).  Literals must have been flushed.
__device__ __forceinline__ void flush_matches(Pending &q, uint8_t *out, uint32_t lane) {
    const bool act = lane < q.nmat;
    const int32_t d = (int32_t)q.md;
    const int32_t off = (int32_t)(q.mx & 0xFFFFu);
    const int32_t ml = (int32_t)(q.mx >> 16);
    const int32_t src_end = d - off + min(ml, off);
    uint64_t pending = __ballot(act);
    const uint64_t shortm = __ballot(act && ml <= 64);
    const uint32_t dpk = (uint32_t)d | ((uint32_t)off << 16);
    const uint32_t grp = lane >> 4, gl = lane & 15u;
    q.nmat = 0;
    while (pending) {
        const uint32_t f = (uint32_t)__builtin_ctzll(pending);
        const int32_t F = (int32_t)rdlane((uint32_t)d, f);
        if (!((shortm >> f) & 1ull)) {
            const int32_t mlf = (int32_t)rdlane((uint32_t)ml, f);
            const int32_t fo = (int32_t)rdlane((uint32_t)off, f);
            const int32_t fs = F - fo;
            if (fo >= (int32_t)kWave) {
                for (int32_t i = (int32_t)lane; i < mlf; i += kWave) out[F + i] = out[fs + i];
            } else {
                for (int32_t i = (int32_t)lane; i < mlf; i += kWave)
                    out[F + i] = out[fs + (int32_t)mod_small((uint32_t)i, (uint32_t)fo)];
            }
            pending &= ~(1ull << f);
            continue;
        }
        uint64_t ready = pending & shortm & __ballot(src_end <= F);
        uint32_t gpk = 0, gml = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            if (ready) {
                const uint32_t r = (uint32_t)__builtin_ctzll(ready);
                ready &= ready - 1;
                pending &= ~(1ull << r);
                const uint32_t pk = rdlane(dpk, r), mlr = rdlane((uint32_t)ml, r);
                if (grp == k) { gpk = pk; gml = mlr; }
            }
        }
        const int32_t md = (int32_t)(gpk & 0xFFFFu), mo = (int32_t)(gpk >> 16), mm = (int32_t)gml;
        const int32_t ms = md - mo;
        for (int32_t i = (int32_t)gl; i < mm; i += 16) {
            const int32_t si = (mo >= 16 || mo >= mm) ? i : (int32_t)mod_small((uint32_t)i, (uint32_t)mo);
            out[md + i] = out[ms + si];
        }
    }
}

// code-length code order (RFC 1951 3.2.7), 5 bits per entry
__device__ __forceinline__ uint32_t cl_order(uint32_t i) {
    // 16 17 18 0 8 7 9 6 10 5 11 4 | 12 3 13 2 14 1 15
    const uint64_t lo = 16ull | 17ull << 5 | 18ull << 10 | 0ull << 15 | 8ull << 20 | 7ull << 25 | 9ull << 30 |
                        6ull << 35 | 10ull << 40 | 5ull << 45 | 11ull << 50 | 4ull << 55;
    const uint64_t hi = 12ull | 3ull << 5 | 13ull << 10 | 2ull << 15 | 14ull << 20 | 1ull << 25 | 15ull << 30;
    return (uint32_t)((i < 12 ? lo >> (5 * i) : hi >> (5 * (i - 12))) & 31u);
}

// zlib header (RFC 1950: CMF/FLG, inflate.c HEAD); 0 or kZData
__device__ __forceinline__ int32_t zlib_header(BitReader &r, uint32_t lane) {
    refill(r, lane);
    if (r.avail < 16) return kZData;
    const uint32_t cmf = take(r, 8), flg = take(r, 8);
    if (((cmf << 8) | flg) % 31u) return kZData;
    if ((cmf & 15u) != 8u) return kZData;
    if ((cmf >> 4) + 8u > 15u) return kZData;
    if (flg & 0x20u) return kZData;
    return 0;
}

// One block header (BFINAL, BTYPE; inflate.c TYPE/TABLE/LENLENS/CODELENS).
// Returns 1 for a stored block (reader just past BTYPE), 0 when L and D hold
// the block's fixed or dynamic codes, kZData on error.
__device__ __forceinline__ int32_t block_head(BitReader &r, uint32_t &last, Table &L, Table &D, uint8_t *lens,
                                              uint16_t *sortL, uint16_t *sortD, uint32_t lane) {
    refill(r, lane);
    if (r.avail < 3) return kZData;
    last = take(r, 1);
    const uint32_t type = take(r, 2);
    if (type == 0) return 1;
    if (type == 3) return kZData;
    if (type == 1) {
        fixed_tables(L, D, lane);
        return 0;
    }
    refill(r, lane);
    if (r.avail < 14) return kZData;
    const uint32_t nlen = take(r, 5) + 257u, ndist = take(r, 5) + 1u, ncode = take(r, 4) + 4u;
    if (nlen > 286u || ndist > 30u) return kZData;
    if (r.avail < (int32_t)(3u * ncode)) return kZData;
    uint32_t clv = 0;
    for (uint32_t i = 0; i < ncode; i++) {
        refill(r, lane);
        clv = put_lane(clv, cl_order(i), take(r, 3), lane);
    }
    if (lane < 19u) lens[lane] = (uint8_t)clv;
    if (!build_table(lens, 19, 0, L, sortL, lane)) return kZData;
    const uint32_t total = nlen + ndist;
    uint32_t n = 0, prev = 0;
    while (n < total) {
        refill(r, lane);
        const uint32_t e = lookup(L, (uint32_t)r.bb & 1023u);
        const uint32_t l = e_len(e);
        if (e_kind(e) != kLit || (int32_t)l > r.avail) return kZData;
        take(r, l);
        const uint32_t sym = e_val(e);
        if (sym < 16u) {
            if (lane == 0) lens[n] = (uint8_t)sym;
            prev = sym;
            n++;
            continue;
        }
        uint32_t rep, val = 0;
        if (sym == 16u) {
            if (n == 0) return kZData;
            if (r.avail < 2) return kZData;
            val = prev;
            rep = 3u + take(r, 2);
        } else if (sym == 17u) {
            if (r.avail < 3) return kZData;
            rep = 3u + take(r, 3);
        } else {
            if (r.avail < 7) return kZData;
            rep = 11u + take(r, 7);
        }
        if (n + rep > total) return kZData;
        for (uint32_t j = lane; j < rep; j += kWave) lens[n + j] = (uint8_t)val;
        prev = val;
        n += rep;
    }
    if (rfl(lens[256]) == 0) return kZData;
    if (!build_table(lens, nlen, 1, L, sortL, lane)) return kZData;
    if (!build_table(lens + nlen, ndist, 2, D, sortD, lane)) return kZData;
    return 0;
}

// Decodes one zlib stream into out (LDS, cap bytes).  Returns the decoded
// length or kZData / kZBuf, as oracle_zlib_uncompress.
__device__ __forceinline__ int32_t inflate_page(BitReader &r, const uint8_t *src, uint8_t *out, int32_t cap, uint8_t *lens,
                                uint16_t *sortL, uint16_t *sortD, uint32_t lane) {
    if (zlib_header(r, lane)) return kZData;
    Table L, D;
    Pending q;
    q.lit = q.md = q.mx = 0;
    q.nlit = q.nmat = 0;
    int32_t op = 0;
    uint32_t last;
    do {
        const int32_t hr = block_head(r, last, L, D, lens, sortL, sortD, lane);
        if (hr < 0) return hr;
        if (hr == 1) {
            // stored block (inflate.c STORED/COPY)
            take(r, r.bc & 7u);
            refill(r, lane);
            if (r.avail < 32) return kZData;
            const uint32_t len = take(r, 16), nlen = take(r, 16);
            if (len != (~nlen & 0xFFFFu)) return kZData;
            const uint32_t A = (uint32_t)r.avail >> 3;
            const uint32_t P = r.inpos - (r.bc >> 3);
            const uint32_t R = (uint32_t)(cap - op);
            if (len > min(A, R)) return A <= R ? kZData : kZBuf;
            for (uint32_t j = lane; j < len; j += kWave) out[op + (int32_t)j] = src[P + j];
            op += (int32_t)len;
            r.avail -= (int32_t)(len * 8u);
            seek(r, P + len, lane);
            continue;
        }
        // ---- compressed data (inflate.c LEN/DIST; inffast.c)
        for (;;) {
            refill(r, lane);
            uint32_t e = lookup(L, (uint32_t)r.bb & 1023u);
            if (e_kind(e) == kLong) e = slow_entry(L, sortL, 1, r.bb, lane);
            uint32_t l = e_len(e), kind = e_kind(e);
            if (kind == kBad || (int32_t)l > r.avail) return kZData;
            take(r, l);
            if (kind == kLit) {
                if (op >= cap) return kZBuf;
                q.lit = put_lane(q.lit, q.nlit, ((uint32_t)op << 8) | e_val(e), lane);
                op++;
                if (++q.nlit == kWave) flush_literals(q, out, lane);
                continue;
            }
            if (kind == kEob) break;
            uint32_t x = e_extra(e);
            if ((int32_t)x > r.avail) return kZData;
            const uint32_t len = e_val(e) + take(r, x);
            refill(r, lane);
            e = lookup(D, (uint32_t)r.bb & 1023u);
            if (e_kind(e) == kLong) e = slow_entry(D, sortD, 2, r.bb, lane);
            l = e_len(e);
            if (e_kind(e) == kBad || (int32_t)l > r.avail) return kZData;
            take(r, l);
            x = e_extra(e);
            if ((int32_t)x > r.avail) return kZData;
            const uint32_t dist = e_val(e) + take(r, x);
            if ((int32_t)dist > op) return kZData;
            if (op + (int32_t)len > cap) return kZBuf;
            q.md = put_lane(q.md, q.nmat, (uint32_t)op, lane);
            q.mx = put_lane(q.mx, q.nmat, dist | (len << 16), lane);
            op += (int32_t)len;
            if (++q.nmat == kWave) {
                flush_literals(q, out, lane);
                flush_matches(q, out, lane);
            }
        }
    } while (!last);
    // adler32 trailer, big-endian, byte aligned (inflate.c CHECK)
    take(r, r.bc & 7u);
    refill(r, lane);
    if (r.avail < 32) return kZData;
    const uint32_t want = __builtin_bswap32(take(r, 32));
    flush_literals(q, out, lane);
    flush_matches(q, out, lane);
    if (lds_adler32(out, (uint32_t)op, lane) != want) return kZData;
    return op;
}

// ------------------------------------------------- lane-parallel block decode
// inflate_par: the latency path.  The serial decoder above spends ~1.3 ms of
// one wave on a 16 KiB page (one Huffman symbol after another, every step a
// chain of scalar/readlane dependencies); a restore that waits for its page
// waits for that.  Here the 64 lanes decode the block's symbol stream
// together, the way lz4_decode.hip splits LZ4's token chain:
//   1. the stream is staged in LDS and its bits cut into 64 segments (32-bit
//      aligned); lane k decodes compound symbols (a literal, or length +
//      distance with their extra bits, or end-of-block) from the start of its
//      segment to its end, setting the bit of every symbol start in a bitmap
//      (V).  Only lane 0 starts at a true symbol boundary; a Huffman code
//      resynchronises after a few symbols, so the others usually join the
//      true chain quickly;
//   2. from its exit each lane keeps decoding ("bridge") until it reaches a
//      bit set by a later lane, end-of-block, an invalid code or the stream end;
//   3. the true chain is lane 0's walk followed by the hand-offs (<= 64 steps of
//      scalar code), which gives every on-chain lane its entry;
//   4. on-chain lanes re-decode entry -> hand-off to count output bytes; a
//      prefix sum places them; a third pass writes literals and leaves each
//      match's (distance, length) in the first three bytes of its own output
//      range, marking its start in a second bitmap (M);
//   5. after the last block the matches are applied in order, 64 at a time,
//      with the serial path's frontier-grouped copy (flush_matches).
// Anything the happy path does not cover -- an invalid code or a stream that
// ends early on the true chain, a distance beyond the output, output past the
// capacity, stored blocks, a stream longer than the staging area -- returns
// kFallback and the page is decoded again by inflate_page, so results and
// error verdicts are exactly the serial decoder's.
constexpr int32_t kFallback = INT32_MIN + 1;

struct ParTabs {
    const uint32_t *LT, *DT;          // 1024-entry root tables (LDS), entry format of Table
    const uint16_t *sortL, *sortD;    // sorted symbols (slow path)
    uint32_t limL[5], dltL[5], limD[5], dltD[5];   // lengths 11..15
};

__device__ __forceinline__ uint32_t peek32(const uint32_t *S32, uint32_t p) {
    const uint32_t i = p >> 5;
    return __builtin_amdgcn_alignbit(S32[i + 1], S32[i], p & 31u);
}

// per-lane canonical decode of a code longer than 10 bits (slow_entry's rule)
__device__ __forceinline__ uint32_t slow_lane(const uint32_t *lim, const uint32_t *dlt, const uint16_t *sorted,
                                              uint32_t table_kind, uint32_t w) {
    const uint32_t v15 = __builtin_bitreverse32(w) >> 17;
    if (v15 >= lim[4]) return mk(kBad, 0, 0);
    const uint32_t i = (uint32_t)(v15 >= lim[0]) + (uint32_t)(v15 >= lim[1]) + (uint32_t)(v15 >= lim[2]) +
                       (uint32_t)(v15 >= lim[3]);
    const uint32_t l = 11u + i;
    const uint32_t d = i == 0 ? dlt[0] : i == 1 ? dlt[1] : i == 2 ? dlt[2] : i == 3 ? dlt[3] : dlt[4];
    return sym_entry(table_kind, sorted[d + (v15 >> (15u - l))]) | l;
}

enum : uint32_t { kSymLit = 0, kSymMatch = 1, kSymEob = 2, kSymBad = 3 };

// one compound symbol at bit p: a literal (val = byte), a match (val =
// length, dist), end-of-block, or an invalid code; advances p
__device__ __forceinline__ uint32_t par_sym(const ParTabs &t, const uint32_t *S32, uint32_t &p, uint32_t &val,
                                            uint32_t &dist) {
    uint32_t w = peek32(S32, p);
    uint32_t e = t.LT[w & 1023u];
    if (e_kind(e) == kLong) e = slow_lane(t.limL, t.dltL, t.sortL, 1, w);
    const uint32_t l = e_len(e), k = e_kind(e);
    if (k == kLit) {
        p += l;
        val = e_val(e);
        return kSymLit;
    }
    if (k == kEob) {
        p += l;
        return kSymEob;
    }
    if (k != kLen) return kSymBad;
    const uint32_t x = e_extra(e);
    val = e_val(e) + ((w >> l) & ((1u << x) - 1u));
    p += l + x;
    w = peek32(S32, p);
    e = t.DT[w & 1023u];
    if (e_kind(e) == kLong) e = slow_lane(t.limD, t.dltD, t.sortD, 2, w);
    if (e_kind(e) != kLen) return kSymBad;
    const uint32_t l2 = e_len(e), x2 = e_extra(e);
    dist = e_val(e) + ((w >> l2) & ((1u << x2) - 1u));
    p += l2 + x2;
    return kSymMatch;
}

__device__ __forceinline__ void par_tables(ParTabs &t, const Table &L, const Table &D, uint32_t *LT, uint32_t *DT,
                                           const uint16_t *sortL, const uint16_t *sortD, uint32_t lane) {
#pragma unroll
    for (uint32_t r = 0; r < 16; r++) {
        LT[r * kWave + lane] = L.root[r];
        DT[r * kWave + lane] = D.root[r];
    }
    t.LT = LT;
    t.DT = DT;
    t.sortL = sortL;
    t.sortD = sortD;
#pragma unroll
    for (uint32_t i = 0; i < 5; i++) {
        t.limL[i] = rdlane(L.lim, 11 + i);
        t.dltL[i] = rdlane(L.dlt, 11 + i);
        t.limD[i] = rdlane(D.lim, 11 + i);
        t.dltD[i] = rdlane(D.dlt, 11 + i);
    }
}

// Decodes one block's symbols [P0, end-of-block) of the staged stream (bit
// positions in stage coordinates, E = stream end) into out at op.  Returns the
// new output length and the bit position after end-of-block (yend), or
// kFallback.  V: bitmap scratch inside the output window (out + vo, above op);
// M: match-start bitmap.
// items (optional, the jump path's cells region, rows per lane): every symbol a
// lane visits is recorded (bit position - base | output bytes before it << 17),
// so an on-chain lane's output count is its total minus the count at its entry
// (a binary search) instead of a second decode pass; lanes whose walks leave
// the items or 15 bits of output take the counting pass.
__device__ __forceinline__ int32_t par_block(const ParTabs &t, const uint32_t *S32, uint32_t P0, uint32_t E, uint8_t *out, int32_t op,
                             int32_t cap, uint32_t W, uint32_t *M, uint32_t lane, uint32_t &yend,
                             uint32_t *items = nullptr, uint32_t rows = 0) {
    if (P0 >= E) return kFallback;
    ZPROF_DECL
    const uint32_t base = P0 & ~31u;
    const uint32_t S = ((E - base + kWave - 1) / kWave + 31u) & ~31u;   // bits per segment
    const uint32_t nv = (E - base + 31u) / 32u + 1u;                        // bitmap words
    const uint32_t vo = ((uint32_t)op + 3u) & ~3u;
    if (vo + 4u * nv > W) return kFallback;
    uint32_t *V = (uint32_t *)(out + vo);
    for (uint32_t w = lane; w < nv; w += kWave) V[w] = 0;
    WAVE_SYNC();
    // 1. walk the own segment
    const uint32_t a = base + lane * S, b = min(a + S, E);
    uint32_t y = lane == 0 ? P0 : a, stop = 0, val, dist;
    uint32_t ni = 0, cum = 0;   // items recorded, output bytes so far (items)
    const bool rec = items && E - base < (1u << 17);
    if (a < E) {
        while (y < b) {
            atomicOr(&V[(y - base) >> 5], 1u << (y & 31u));
            if (rec) {
                if (ni < rows) items[ni * kWave + lane] = (y - base) | (min(cum, 0x7FFFu) << 17);
                ni++;
            }
            const uint32_t k = par_sym(t, S32, y, val, dist);
            cum += k == kSymLit ? 1u : k == kSymMatch ? val : 0u;
            if (k >= kSymEob) {
                stop = k;
                break;
            }
        }
    }
    WAVE_SYNC();
    ZPROF_MARK(2);
    // 2. bridge to a later lane's walk, and 3. follow the hand-offs from lane 0.
    // Bridges advance in rounds of kBridgeSteps symbols, each followed by the
    // hand-off walk as far as the finished bridges reach; lanes behind it stop
    // (a lane off the true chain may bridge for a long way before it meets a
    // later lane's walk, and one loop for all lanes waited for the longest).
    constexpr uint32_t kBridgeSteps = TYCHE_BRIDGE_STEPS;
    uint32_t o = 0;   // owner lane + 1 of the hand-off position, 0 = chain ends here
    bool done = !(a < E && stop == 0) || y >= E;
    uint32_t entry = 0xFFFFFFFFu;
    uint32_t cur = 0, e = P0;
    for (bool fin = false; !fin;) {
        for (uint32_t it = 0; it < kBridgeSteps; it++) {
            if (!done) {
                if ((V[(y - base) >> 5] >> (y & 31u)) & 1u) {
                    o = (y - base) / S + 1u;
                    done = true;
                } else {
                    if (rec) {
                        if (ni < rows) items[ni * kWave + lane] = (y - base) | (min(cum, 0x7FFFu) << 17);
                        ni++;
                    }
                    const uint32_t k = par_sym(t, S32, y, val, dist);
                    cum += k == kSymLit ? 1u : k == kSymMatch ? val : 0u;
                    if (k >= kSymEob) stop = k;
                    done = k >= kSymEob || y >= E;
                }
            }
        }
        for (;;) {
            if (lane == cur) entry = e;
            if (!rdlane((uint32_t)done, cur)) break;   // cur's hand-off not found yet
            e = rdlane(y, cur);
            const uint32_t nx = rdlane(o, cur);
            if (nx == 0) { fin = true; break; }
            cur = nx - 1;
        }
        if (lane < cur) done = true;
    }
    ZPROF_MARK(3);
    ZPROF_ADD(10, cur);
    if (rdlane(stop, cur) != kSymEob || e > E) return kFallback;
    yend = e;
    // 4. count, place, write
    const bool on = entry != 0xFFFFFFFFu;
    uint32_t nout = 0;
    bool counted = false;
    if (on && rec && ni <= rows && cum < 0x8000u) {
        // the entry is a symbol start this lane's walk visited: its item
        uint32_t lo = 0, hi = ni;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((items[mid * kWave + lane] & 0x1FFFFu) < entry - base) lo = mid + 1;
            else hi = mid;
        }
        if (lo < ni && (items[lo * kWave + lane] & 0x1FFFFu) == entry - base) {
            // the lane's part ends at its hand-off (or at end-of-block, which adds no output)
            nout = cum - (items[lo * kWave + lane] >> 17);
            counted = true;
        }
    }
    if (on && !counted) {
        for (uint32_t q = entry; q < y;) {
            const uint32_t k = par_sym(t, S32, q, val, dist);
            if (k == kSymLit) nout++;
            else if (k == kSymMatch) nout += val;
            else break;
        }
    }
    ZPROF_MARK(4);
    const int32_t incl = wave_incl_sum((int32_t)nout);
    const int32_t total = op + (int32_t)rdlane((uint32_t)incl, kWave - 1);
    if (total > cap) return kFallback;
    WAVE_SYNC();   // V is dead from here on; the output overwrites it
    bool bad = false;
    if (on) {
        uint32_t o2 = (uint32_t)(op + incl) - nout;
        for (uint32_t q = entry; q < y;) {
            const uint32_t k = par_sym(t, S32, q, val, dist);
            if (k == kSymLit) {
                out[o2++] = (uint8_t)val;
            } else if (k == kSymMatch) {
                if (dist > o2) bad = true;
                out[o2] = (uint8_t)dist;
                out[o2 + 1] = (uint8_t)(dist >> 8);
                out[o2 + 2] = (uint8_t)(val - 3u);
                atomicOr(&M[o2 >> 5], 1u << (o2 & 31u));
                o2 += val;
            } else {
                break;
            }
        }
    }
    ZPROF_MARK(5);
    if (__ballot(bad)) return kFallback;
    return total;
}

// Applies the matches recorded by par_block, in output order.  pos: scratch
// for one chunk's match positions (<= 683 u16).
__device__ __forceinline__ void par_matches(uint8_t *out, uint32_t total, const uint32_t *M, uint16_t *pos, uint32_t lane) {
    const uint32_t nw = (total + 31u) >> 5;
    Pending q;
    q.lit = 0;
    q.nlit = 0;
    for (uint32_t w0 = 0; w0 < nw; w0 += kWave) {
        uint32_t word = w0 + lane < nw ? M[w0 + lane] : 0u;
        const uint32_t c = (uint32_t)__builtin_popcount(word);
        const int32_t incl = wave_incl_sum((int32_t)c);
        const uint32_t T = rdlane((uint32_t)incl, kWave - 1);
        uint32_t at = (uint32_t)incl - c;
        while (word) {
            const uint32_t bit = (uint32_t)__builtin_ctz(word);
            word &= word - 1u;
            pos[at++] = (uint16_t)((w0 + lane) * 32u + bit);
        }
        WAVE_SYNC();
        for (uint32_t i0 = 0; i0 < T; i0 += kWave) {
            const uint32_t n = min(T - i0, kWave);
            uint32_t d = 0, dist = 0, len = 0;
            if (lane < n) {
                d = pos[i0 + lane];
                dist = (uint32_t)out[d] | ((uint32_t)out[d + 1] << 8);
                len = (uint32_t)out[d + 2] + 3u;
            }
            q.md = d;
            q.mx = dist | (len << 16);
            q.nmat = n;
            ZPROF_ADD(12, 1);
            ZPROF_ADD(13, n);
            WAVE_SYNC();
            flush_matches(q, out, lane);
            WAVE_SYNC();
        }
    }
}

// The same matches resolved by pointer jumping (small batches, pages <= 32 KiB;
// lz4_decode.hip's jump decoder describes the cells).  One 16-bit cell per
// output byte: a literal is final (0x8000 | byte), a match byte holds the
// position it copies, d - dist + (j mod dist), which always lies below its own
// match; cell = cells[cell] until every cell is a literal gives inflate's
// forward byte copies (inffast.c:263-307) in log2(chain depth) rounds.  Each
// lane classifies a contiguous span of bytes, carrying in the last match start
// before it (a max-scan over the lanes' last starts in M).  The frontier copy
// above needs ~1,000 dependent rounds on a 16 KiB page of deflate's short
// matches; the byte-level variant tried before it (one byte per step, 9 full
// passes) was slower than the frontier.
__device__ void par_matches_jump(uint8_t *out, uint32_t total, const uint32_t *M, uint16_t *cells, uint32_t lane) {
    ZPROF_DECL
    const uint32_t n8 = (total + 7u) & ~7u;
    const uint32_t span = (((n8 + 63u) / 64u + kWave - 1u) / kWave) * 64u;   // bytes per lane, a multiple of 64
    const uint32_t x0 = min(lane * span, n8), x1 = min(x0 + span, n8);
    uint32_t last = 0;   // match starts are >= 1 (dist <= position)
    for (uint32_t w = x0 >> 5; w < (x1 + 31u) >> 5; w++) {
        const uint32_t m = M[w];
        if (m) last = 32u * w + 31u - (uint32_t)__builtin_clz(m);
    }
    const int32_t incl = wave_incl_max((int32_t)last);
    const int32_t before = __shfl_up(incl, 1);
    const uint32_t carry = lane ? (uint32_t)before : 0u;
    uint32_t d = 0, dist = 1, end = 0, k = 0;
    if (carry) {
        const uint32_t r = lds_ld32(out + carry);
        d = carry;
        dist = r & 0xFFFFu;
        end = d + ((r >> 16) & 0xFFu) + 3u;
        k = x0 < end ? mod_small(x0 - d, dist) : 0u;
    }
    for (uint32_t x = x0; x < x1; x += 8u) {
        const uint32_t o0 = *(const uint32_t *)(out + x), o1 = *(const uint32_t *)(out + x + 4u);
        const uint32_t mb = (M[x >> 5] >> (x & 31u)) & 0xFFu;
        uint32_t c[4];
#pragma unroll
        for (uint32_t h = 0; h < 8; h++) {
            const uint32_t xb = x + h;
            if ((mb >> h) & 1u) {
                const uint32_t r = lds_ld32(out + xb);   // the match's record: dist, len - 3
                d = xb;
                dist = r & 0xFFFFu;
                end = xb + ((r >> 16) & 0xFFu) + 3u;
                k = 0;
            }
            const uint32_t byte = ((h < 4 ? o0 : o1) >> (8u * (h & 3u))) & 0xFFu;
            const bool in_match = xb < end;
            const uint32_t v = in_match ? d - dist + k : (0x8000u | byte);
            if (in_match) {
                k++;
                if (k == dist) k = 0;
            }
            if (h & 1u) c[h >> 1] |= v << 16;
            else c[h >> 1] = v;
        }
        *(u32x4 *)(cells + x) = u32x4{c[0], c[1], c[2], c[3]};
    }
    WAVE_SYNC();
    ZPROF_MARK(14);
    u32x4 *c4 = (u32x4 *)cells;
    const uint32_t ng = n8 / 8u;
    for (;;) {
        uint32_t open = 0;
        for (uint32_t g = lane; g < ng; g += 2u * kWave) {
            const uint32_t g2 = g + kWave;
            const u32x4 fin = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
            u32x4 v = c4[g], u = g2 < ng ? c4[g2] : fin;
            const bool dv = ((v.x & v.y & v.z & v.w) & 0x80008000u) != 0x80008000u;
            const bool du = ((u.x & u.y & u.z & u.w) & 0x80008000u) != 0x80008000u;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (dv) {
                    uint32_t lo = v[j] & 0xFFFFu, hi = v[j] >> 16;
                    if (!(lo & 0x8000u)) lo = cells[lo];
                    if (!(hi & 0x8000u)) hi = cells[hi];
                    open |= ~(lo & hi) & 0x8000u;
                    v[j] = lo | (hi << 16);
                }
                if (du) {
                    uint32_t lo = u[j] & 0xFFFFu, hi = u[j] >> 16;
                    if (!(lo & 0x8000u)) lo = cells[lo];
                    if (!(hi & 0x8000u)) hi = cells[hi];
                    open |= ~(lo & hi) & 0x8000u;
                    u[j] = lo | (hi << 16);
                }
            }
            if (dv) c4[g] = v;
            if (du) c4[g2] = u;
        }
        ZPROF_ADD(15, 1);
        if (!__ballot(open != 0)) break;
        WAVE_SYNC();
    }
    WAVE_SYNC();
    for (uint32_t g = lane; g < ng; g += kWave) {
        const u32x4 a = c4[g];
        uint32_t *o = (uint32_t *)(out + 8u * g);
        o[0] = __builtin_amdgcn_perm(a.y, a.x, 0x06040200u);
        o[1] = __builtin_amdgcn_perm(a.w, a.z, 0x06040200u);
    }
}

__device__ __forceinline__ void seek_bits(BitReader &r, uint32_t bitpos, uint32_t src_len, uint32_t lane) {
    seek(r, bitpos >> 3, lane);
    r.avail = (int32_t)(src_len * 8u - (bitpos & ~7u));
    refill(r, lane);
    take(r, bitpos & 7u);
}

// The page's stream is staged at stage + head (head = src & 15), zero-padded.
// Returns the decoded length, kZData, or kFallback.
__device__ __forceinline__ int32_t inflate_par(BitReader &r, const PageRef &p, const uint8_t *stage, uint32_t head, uint8_t *out,
                               int32_t cap, uint32_t W, uint32_t *M, uint32_t *LT, uint32_t *DT, uint8_t *lens,
                               uint16_t *sortL, uint16_t *sortD, uint16_t *cells, uint32_t lane,
                               uint32_t *want_out = nullptr) {
    ZPROF_DECL
    if (zlib_header(r, lane)) return kFallback;
    const uint32_t *S32 = (const uint32_t *)stage;
    const uint32_t h8 = head * 8u, E = h8 + p.src_len * 8u;
    for (uint32_t w = lane; w < ((uint32_t)cap + 31u) / 32u; w += kWave) M[w] = 0;
    int32_t op = 0;
    uint32_t last = 0, yend = 0;
    Table L, D;
    do {
        const int32_t hr = block_head(r, last, L, D, lens, sortL, sortD, lane);
        if (hr != 0) return kFallback;   // errors and stored blocks: the serial decoder
        ParTabs t;
        par_tables(t, L, D, LT, DT, sortL, sortD, lane);
        WAVE_SYNC();
        ZPROF_MARK(1);
        const uint32_t P0 = h8 + (uint32_t)p.src_len * 8u - (uint32_t)r.avail;
        op = par_block(t, S32, P0, E, out, op, cap, W, M, lane, yend, (uint32_t *)cells,
                       cells ? (uint32_t)(((cap + 7) & ~7) * 2 / (4 * kWave)) : 0u);
        if (op < 0) return kFallback;
        WAVE_SYNC();
        if (!last) seek_bits(r, yend - h8, p.src_len, lane);
    } while (!last);
    // adler32 trailer: big-endian, byte aligned after the last block
    const uint32_t tb = (yend - h8 + 7u) >> 3;
    if (tb + 4u > p.src_len) return kFallback;
    const uint8_t *tp = stage + head + tb;
    const uint32_t want = ((uint32_t)tp[0] << 24) | ((uint32_t)tp[1] << 16) | ((uint32_t)tp[2] << 8) | tp[3];
    if (want_out) {
        // the workgroup kernel applies the matches and checks the trailer itself
        if (lane == 0) *want_out = want;
        return op;
    }
    WAVE_SYNC();
    if (cells) par_matches_jump(out, (uint32_t)op, M, cells, lane);
    else par_matches(out, (uint32_t)op, M, (uint16_t *)stage, lane);   // the stage is free now
    WAVE_SYNC();
    ZPROF_MARK(6);
    if (lds_adler32(out, (uint32_t)op, lane) != want) return kZData;
    ZPROF_MARK(8);
    ZPROF_ADD(0, 1);
    return op;
}

__device__ __forceinline__ void reader_init(BitReader &r, const PageRef &p, uint32_t lane) {
    const uintptr_t a = (uintptr_t)p.src;
    r.h = (uint32_t)(a & 3u);
    r.s4 = (const uint32_t *)(a - r.h);
    r.nd = (r.h + p.src_len + 3u) >> 2;
    r.avail = (int32_t)(p.src_len * 8u);
    r.bb = 0;
    r.bc = 0;
    r.inpos = 0;
    r.wbase = 0;
    (void)lane;
}

__global__ __launch_bounds__(64) void zlib_inflate_kernel(tyche_batch_t b, uint32_t out_cap, uint32_t off_lens,
                                                          unsigned *ctr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint8_t *out = smem;
    uint8_t *lens = smem + off_lens;
    uint16_t *sortL = (uint16_t *)(lens + 320);
    uint16_t *sortD = sortL + 320;
    const size_t stride = gridDim.x;
    size_t page = blockIdx.x;
    if (page >= b.count) return;
    PageRef p = batch_page(b, page);
    BitReader r;
    reader_init(r, p, lane);
    r.wa = load_win(r, 0, lane);
    r.wb = load_win(r, 256, lane);
    for (;;) {
        const size_t next = ctr ? claim_page(ctr, lane) : page + stride;   // dynamic assignment (engine.h)
        // the next page's first 512 stream bytes are loaded behind this page's decode
        PageRef pn;
        BitReader rn;
        if (next < b.count) {
            pn = batch_page(b, next);
            reader_init(rn, pn, lane);
            rn.wa = load_win(rn, 0, lane);
            rn.wb = load_win(rn, 256, lane);
        }
        int32_t rv;
        if (p.dst_cap > out_cap || p.src_len > 0x0FFFFFFFu) {
            rv = kResultTooLarge;
        } else {
            rv = inflate_page(r, p.src, out, (int32_t)p.dst_cap, lens, sortL, sortD, lane);
            WAVE_SYNC();
            if (rv > 0) stage_out(p.dst, out, (uint32_t)rv, lane, kWave);
        }
        if (lane == 0) b.results[page] = rv;
        if (next >= b.count) break;
        WAVE_SYNC();
        page = next;
        p = pn;
        r = rn;
    }
}

// The latency kernel: inflate_par per page (stream staged in LDS), the serial
// decoder when it falls back.  LDS: output window | lens/sorted | LT | DT | M |
// stage.
__global__ __launch_bounds__(64) void zlib_inflate_par_kernel(tyche_batch_t b, uint32_t out_cap, uint32_t off_lens,
                                                              uint32_t off_lt, uint32_t off_m, uint32_t off_stage,
                                                              uint32_t stage_cap, int32_t no_fallback, uint32_t off_cells,
                                                              unsigned *ctr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint8_t *out = smem;
    uint8_t *lens = smem + off_lens;
    uint16_t *sortL = (uint16_t *)(lens + 320);
    uint16_t *sortD = sortL + 320;
    uint32_t *LT = (uint32_t *)(smem + off_lt);
    uint32_t *DT = LT + 1024;
    uint32_t *M = (uint32_t *)(smem + off_m);
    uint8_t *stage = smem + off_stage;
    uint16_t *cells = off_cells ? (uint16_t *)(smem + off_cells) : nullptr;
    size_t page = blockIdx.x;
    while (page < b.count) {
        const PageRef p = batch_page(b, page);
        int32_t rv;
        if (p.dst_cap > out_cap || p.src_len > 0x0FFFFFFFu) {
            rv = kResultTooLarge;
        } else {
            rv = kFallback;
            const uint32_t head = (uint32_t)((uintptr_t)p.src & 15u);
            if (head + p.src_len + 48u <= stage_cap) {
                stage_in(p.src, p.src_len, stage, lane, kWave);
                // zero the 32 bytes after the stream (symbol reads run past its end)
                if (lane < 8u) lds_st32(stage + ((head + p.src_len + 15u) & ~15u) + 4u * lane, 0u);
                WAVE_SYNC();
                BitReader r;
                reader_init(r, p, lane);
                r.wa = load_win(r, 0, lane);
                r.wb = load_win(r, 256, lane);
                rv = inflate_par(r, p, stage, head, out, (int32_t)p.dst_cap, off_lens, M, LT, DT, lens, sortL, sortD,
                                 cells, lane);
                WAVE_SYNC();
            }
            if (rv == kFallback && !no_fallback) {
                BitReader r;
                reader_init(r, p, lane);
                r.wa = load_win(r, 0, lane);
                r.wb = load_win(r, 256, lane);
                rv = inflate_page(r, p.src, out, (int32_t)p.dst_cap, lens, sortL, sortD, lane);
                WAVE_SYNC();
            }
            if (rv > 0) stage_out(p.dst, out, (uint32_t)rv, lane, kWave);
        }
        if (lane == 0) b.results[page] = rv;
        WAVE_SYNC();
        page = claim_page(ctr, lane);
    }
}

// ------------------------------------------------------------ small batches
// The restore path's zlib kernel: a workgroup of kZThreads per page.  Wave 0
// decodes the page exactly as zlib_inflate_par_kernel (inflate_par up to the
// match records); then every wave resolves the matches by pointer jumping
// (par_matches_jump's cells, spread over the workgroup: the one-wave version
// spent ~250 k cycles of a 16 KiB page there); wave 0 checks the adler32
// trailer and takes the serial decoder on any fallback; all waves store the page.
// 256 threads per page, 512 when the batch has no more pages than the device has
// CUs (at 211 VGPRs a CU holds 8 waves: two 256-thread pages or one 512-thread one)

// wg: 32 scratch words (round flags [0..2], wave maxima [16..16 + waves))
template <uint32_t kZThreads>
__device__ void par_matches_jump_wg(uint8_t *out, uint32_t total, const uint32_t *M, uint16_t *cells, uint32_t *wg,
                                    uint32_t tid) {
    const uint32_t lane = tid & (kWave - 1), wave = tid / kWave;
    const uint32_t n8 = (total + 7u) & ~7u;
    const uint32_t span = (((n8 + 63u) / 64u + kZThreads - 1u) / kZThreads) * 64u;
    const uint32_t x0 = min(tid * span, n8), x1 = min(x0 + span, n8);
    uint32_t last = 0;
    for (uint32_t w = x0 >> 5; w < (x1 + 31u) >> 5; w++) {
        const uint32_t m = M[w];
        if (m) last = 32u * w + 31u - (uint32_t)__builtin_clz(m);
    }
    const int32_t incl = wave_incl_max((int32_t)last);
    if (lane == kWave - 1) wg[16 + wave] = (uint32_t)incl;
    if (tid == 0) wg[0] = 0;
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t w = 0; w < wave; w++) carry = max(carry, wg[16 + w]);
    const int32_t before = __shfl_up(incl, 1);
    if (lane) carry = max(carry, (uint32_t)before);
    uint32_t d = 0, dist = 1, end = 0, k = 0;
    if (carry) {
        const uint32_t r = lds_ld32(out + carry);
        d = carry;
        dist = r & 0xFFFFu;
        end = d + ((r >> 16) & 0xFFu) + 3u;
        k = x0 < end ? mod_small(x0 - d, dist) : 0u;
    }
    for (uint32_t x = x0; x < x1; x += 8u) {
        const uint32_t o0 = *(const uint32_t *)(out + x), o1 = *(const uint32_t *)(out + x + 4u);
        const uint32_t mb = (M[x >> 5] >> (x & 31u)) & 0xFFu;
        uint32_t c[4];
#pragma unroll
        for (uint32_t h = 0; h < 8; h++) {
            const uint32_t xb = x + h;
            if ((mb >> h) & 1u) {
                const uint32_t r = lds_ld32(out + xb);
                d = xb;
                dist = r & 0xFFFFu;
                end = xb + ((r >> 16) & 0xFFu) + 3u;
                k = 0;
            }
            const uint32_t byte = ((h < 4 ? o0 : o1) >> (8u * (h & 3u))) & 0xFFu;
            const bool in_match = xb < end;
            const uint32_t v = in_match ? d - dist + k : (0x8000u | byte);
            if (in_match) {
                k++;
                if (k == dist) k = 0;
            }
            if (h & 1u) c[h >> 1] |= v << 16;
            else c[h >> 1] = v;
        }
        *(u32x4 *)(cells + x) = u32x4{c[0], c[1], c[2], c[3]};
    }
    __syncthreads();
    u32x4 *c4 = (u32x4 *)cells;
    const uint32_t ng = n8 / 8u;
    for (uint32_t rd = 0;; rd++) {
        if (tid == 0) wg[(rd + 1) % 3] = 0;   // cleared one round ahead (its readers passed a barrier since)
        uint32_t open = 0;
        for (uint32_t g = tid; g < ng; g += 2u * kZThreads) {
            const uint32_t g2 = g + kZThreads;
            const u32x4 fin = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
            u32x4 v = c4[g], u = g2 < ng ? c4[g2] : fin;
            const bool dv = ((v.x & v.y & v.z & v.w) & 0x80008000u) != 0x80008000u;
            const bool du = ((u.x & u.y & u.z & u.w) & 0x80008000u) != 0x80008000u;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (dv) {
                    uint32_t lo = v[j] & 0xFFFFu, hi = v[j] >> 16;
                    if (!(lo & 0x8000u)) lo = cells[lo];
                    if (!(hi & 0x8000u)) hi = cells[hi];
                    open |= ~(lo & hi) & 0x8000u;
                    v[j] = lo | (hi << 16);
                }
                if (du) {
                    uint32_t lo = u[j] & 0xFFFFu, hi = u[j] >> 16;
                    if (!(lo & 0x8000u)) lo = cells[lo];
                    if (!(hi & 0x8000u)) hi = cells[hi];
                    open |= ~(lo & hi) & 0x8000u;
                    u[j] = lo | (hi << 16);
                }
            }
            if (dv) c4[g] = v;
            if (du) c4[g2] = u;
        }
        if (open) atomicOr(&wg[rd % 3], 1u);
        __syncthreads();
        if (wg[rd % 3] == 0) break;
    }
    for (uint32_t g = tid; g < ng; g += kZThreads) {
        const u32x4 a = c4[g];
        uint32_t *o = (uint32_t *)(out + 8u * g);
        o[0] = __builtin_amdgcn_perm(a.y, a.x, 0x06040200u);
        o[1] = __builtin_amdgcn_perm(a.w, a.z, 0x06040200u);
    }
    __syncthreads();
}

// LDS: output window | lens/sorted | LT | DT | M | stage | cells | wg (32 words)
template <uint32_t kZThreads>
__global__ __launch_bounds__(kZThreads) void zlib_inflate_jump_kernel(tyche_batch_t b, uint32_t out_cap,
                                                                       uint32_t off_lens, uint32_t off_lt,
                                                                       uint32_t off_m, uint32_t off_stage,
                                                                       uint32_t stage_cap, uint32_t off_cells,
                                                                       uint32_t off_wg, unsigned *ctr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
    uint8_t *out = smem;
    uint8_t *lens = smem + off_lens;
    uint16_t *sortL = (uint16_t *)(lens + 320);
    uint16_t *sortD = sortL + 320;
    uint32_t *LT = (uint32_t *)(smem + off_lt);
    uint32_t *DT = LT + 1024;
    uint32_t *M = (uint32_t *)(smem + off_m);
    uint8_t *stage = smem + off_stage;
    uint16_t *cells = (uint16_t *)(smem + off_cells);
    uint32_t *wg = (uint32_t *)(smem + off_wg);   // [0..2] flags, [8] rv, [9] want, [10] page, [16..] wave maxima
    size_t page = blockIdx.x;
    while (page < b.count) {
        const PageRef p = batch_page(b, page);
        const bool fits = p.dst_cap <= out_cap && p.src_len <= 0x0FFFFFFFu;
        const uint32_t head = (uint32_t)((uintptr_t)p.src & 15u);
        const bool staged = fits && head + p.src_len + 48u <= stage_cap;
        if (staged) stage_in(p.src, p.src_len, stage, tid, kZThreads);
        __syncthreads();
        if (wave == 0) {
            int32_t rv = fits ? kFallback : kResultTooLarge;
            if (staged) {
                if (lane < 8u) lds_st32(stage + ((head + p.src_len + 15u) & ~15u) + 4u * lane, 0u);
                WAVE_SYNC();
                BitReader r;
                reader_init(r, p, lane);
                r.wa = load_win(r, 0, lane);
                r.wb = load_win(r, 256, lane);
                rv = inflate_par(r, p, stage, head, out, (int32_t)p.dst_cap, off_lens, M, LT, DT, lens, sortL, sortD,
                                 cells, lane, &wg[9]);
            }
            if (lane == 0) wg[8] = (uint32_t)rv;
        }
        __syncthreads();
        int32_t rv = (int32_t)wg[8];
        if (rv > 0) par_matches_jump_wg<kZThreads>(out, (uint32_t)rv, M, cells, wg, tid);
        if (wave == 0) {
            if (rv >= 0 && lds_adler32(out, (uint32_t)rv, lane) != wg[9]) rv = kZData;
            if (rv == kFallback) {
                BitReader r;
                reader_init(r, p, lane);
                r.wa = load_win(r, 0, lane);
                r.wb = load_win(r, 256, lane);
                rv = inflate_page(r, p.src, out, (int32_t)p.dst_cap, lens, sortL, sortD, lane);
            }
            WAVE_SYNC();
            if (lane == 0) wg[8] = (uint32_t)rv;
        }
        __syncthreads();
        rv = (int32_t)wg[8];
        if (rv > 0) stage_out(p.dst, out, (uint32_t)rv, tid, kZThreads);
        if (tid == 0) b.results[page] = rv;
        if (ctr) {
            if (tid == 0) wg[10] = (uint32_t)claim_page(ctr, 0);
            __syncthreads();
            page = wg[10];
        } else {
            page += gridDim.x;
        }
        __syncthreads();
    }
}

}  // namespace

#ifdef TYCHE_PROFILE
extern "C" int tyche_debug_zlib_profile(unsigned long long *host16, int reset) {
    if (reset) {
        unsigned long long z[16] = {0};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_zprof), z, sizeof(z)) == hipSuccess ? 0 : 1;
    }
    return hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_zprof), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : 1;
}
#endif

// TYCHE_ZLIB_PAR: 1 (default) the lane-parallel kernel, 0 the serial one (A/B timing), 2 the
// parallel path without its fallback (diagnostics: such pages report INT32_MIN + 1)
hipError_t launch_zlib_inflate(const tyche_batch_t &b, uint32_t out_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    const long par = knob("ZLIB_PAR", 1);   // per call: the parity tests switch it in-process
    const uint32_t off_lens = (out_cap + 64u + 15u) & ~15u;
    if (par && out_cap <= 65535u) {
        const uint32_t off_lt = (off_lens + 320u + 2u * 320u + 2u * 32u + 15u) & ~15u;
        const uint32_t off_m = off_lt + 2u * 4096u;
        const uint32_t off_stage = off_m + ((((out_cap + 31u) / 32u) * 4u + 15u) & ~15u);
        const uint32_t stage_cap = (std::max(2048u, out_cap / 2u) + 63u) & ~15u;
        // small batches (restores) resolve matches by pointer jumping: 2 bytes of LDS per
        // output byte more (below TYCHE_ZLIB_JUMP_MAX pages, default 1,024: on the workgroup
        // kernel 512-page batches still gain, 459 vs 698 us at 16 KiB; 0 = never)
        const long jmax = knob("ZLIB_JUMP_MAX", 1024);
        const uint32_t off_cells = (long)b.count < jmax && out_cap <= 32768u ? off_stage + stage_cap : 0u;
        const size_t lds = (size_t)off_stage + stage_cap + (off_cells ? 2u * ((out_cap + 7u) & ~7u) : 0u);
        // the jump path on a workgroup of kZThreads per page (TYCHE_ZLIB_JUMP_WG=0: one wave)
        if (off_cells && par == 1 && knob("ZLIB_JUMP_WG", 1) && lds + 128u <= 160 * 1024) {
            const void *k256 = (const void *)zlib_inflate_jump_kernel<256>;
            const void *k512 = (const void *)zlib_inflate_jump_kernel<512>;
            const size_t ncu = prepare_launch(k256);
            const bool wide = b.count <= ncu;
            const void *k = wide ? k512 : k256;
            const uint32_t threads = wide ? 512u : 256u;
            if (wide) (void)prepare_launch(k512);
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, (int)threads, lds + 128u) != hipSuccess ||
                per_cu < 1)
                per_cu = 1;
            const size_t grid = std::min<size_t>(b.count, ncu * (size_t)per_cu);
            WorkCounter ctr(s, grid < b.count);
            if (grid < b.count && !ctr.get()) return hipErrorOutOfMemory;
            unsigned *cp = grid < b.count ? ctr.get() : nullptr;
            const uint32_t off_wg = (uint32_t)lds;
            void *args[] = {(void *)&b, &out_cap, (void *)&off_lens, (void *)&off_lt, (void *)&off_m, (void *)&off_stage,
                            (void *)&stage_cap, (void *)&off_cells, (void *)&off_wg, &cp};
            (void)hipLaunchKernel(k, dim3((unsigned)grid), dim3(threads), args, lds + 128u, s);
            return hipGetLastError();
        }
        if (lds <= 160 * 1024) {
            const size_t ncu = prepare_launch((const void *)zlib_inflate_par_kernel);
            const size_t per_cu = waves_per_cu((const void *)zlib_inflate_par_kernel, lds);
            const size_t grid = std::min<size_t>(b.count, ncu * per_cu);
            WorkCounter ctr(s, grid < b.count);
            if (!ctr.get()) return hipErrorOutOfMemory;
            hipLaunchKernelGGL(zlib_inflate_par_kernel, dim3((unsigned)grid), dim3(kWave), lds, s, b, out_cap,
                               off_lens, off_lt, off_m, off_stage, stage_cap, (int32_t)(par == 2), off_cells, ctr.get());
            return hipGetLastError();
        }
    }
    const size_t lds = off_lens + 320 + 2 * 320 + 2 * 32;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const size_t ncu = prepare_launch((const void *)zlib_inflate_kernel);
    const size_t per_cu = waves_per_cu((const void *)zlib_inflate_kernel, lds);
    const size_t grid = std::min<size_t>(b.count, ncu * per_cu);
    WorkCounter ctr(s, grid < b.count);
    if (!ctr.get()) return hipErrorOutOfMemory;
    hipLaunchKernelGGL(zlib_inflate_kernel, dim3((unsigned)grid), dim3(kWave), lds, s, b, out_cap, off_lens,
                       ctr.get());
    return hipGetLastError();
}

}  // namespace tyche
