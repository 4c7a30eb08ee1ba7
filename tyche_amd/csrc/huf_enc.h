// huf_enc.h -- entropy-coder construction for the gfx950 encoders: Huffman code
// lengths under a length limit, zstd's canonical Huffman codes and weight
// header, and the small FSE encoder that header needs.
//
// Everything here runs on one 64-lane wave.  Alphabets are at most 256 symbols,
// four per lane (symbol lane + 64 j in register j).
//
// Code lengths: Shannon lengths ceil(log2(total / count)) clamped to
// [1, maxbits], then the Kraft sum is repaired to exactly 2^maxbits units: while
// over-subscribed the least frequent symbol below the limit is lengthened, while
// under-subscribed the most frequent symbol whose shortening still fits is
// shortened.  The result is a complete prefix code (zstd's implied last weight
// requires one, entropy_common.c HUF_readStats) within a fraction of a percent
// of Huffman's lengths on page literals, without the serial tree build.
#pragma once
#include <hip/hip_runtime.h>

#include "engine.h"
#include "lds_io.h"

namespace tyche {
namespace huf {

constexpr uint32_t kWave = 64;

__device__ __forceinline__ uint32_t hb(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return rdlane((uint32_t)wave_incl_sum((int32_t)v), kWave - 1); }
__device__ __forceinline__ int32_t wave_max(int32_t v) { return (int32_t)rdlane((uint32_t)wave_incl_max(v), kWave - 1); }

// Element (j, lane) of an R-register per-lane array, j and lane uniform: every
// register is read and the scalar result selected (a dynamically indexed
// register array would go through scratch memory).
template <int R>
__device__ __forceinline__ uint32_t pick_lane(const uint32_t (&r)[R], uint32_t j, uint32_t ln) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < R; k++) {
        const uint32_t t = rdlane(r[k], ln);
        v = j == (uint32_t)k ? t : v;
    }
    return v;
}

// Smallest l >= 0 with c << l >= total (c >= 1, total < 2^24).
__device__ __forceinline__ uint32_t shannon_len(uint32_t c, uint32_t total) {
    uint32_t l = hb(total) > hb(c) + 1u ? hb(total) - hb(c) - 1u : 0u;
#pragma unroll
    for (int k = 0; k < 3; k++) l += ((uint64_t)c << l) < (uint64_t)total ? 1u : 0u;
    return l;
}

// Optimal (Huffman) code lengths of the used symbols, unlimited (at most 63).
// Counts are ranked by (count, symbol) lane-parallel and placed in LDS in
// ascending order, then the in-place minimum-redundancy construction of Moffat
// and Katajainen runs on that array as wave-uniform code: pass 1 pairs the two
// lightest items left to right (leaf or earlier internal node), storing parent
// indices; pass 2 turns them into internal-node depths; pass 3 hands out leaf
// depths from the heaviest leaf down.  Lengths are then limited to maxbits
// (<= 15) on the per-length counts.  sc: 128 R words of LDS scratch.  Returns
// false if the lengths could not be made (the caller falls back to Shannon's).
template <int R>
__device__ bool huffman_lengths(const uint32_t (&c)[R], uint32_t maxbits, uint32_t (&l)[R], uint32_t *sc,
                                uint32_t lane) {
    uint32_t key[R], rank[R];
#pragma unroll
    for (int j = 0; j < R; j++) {
        key[j] = c[j] ? (c[j] << 9) | (lane + 64u * (uint32_t)j) : 0xFFFFFFFFu;
        rank[j] = 0;
    }
    uint32_t n = 0;
#pragma unroll
    for (int jj = 0; jj < R; jj++) {
        uint64_t m = __ballot(key[jj] != 0xFFFFFFFFu);
        n += (uint32_t)__popcll(m);
        while (m) {
            const uint32_t ln = (uint32_t)__builtin_ctzll(m);
            m &= m - 1ull;
            const uint32_t k = rdlane(key[jj], ln);
#pragma unroll
            for (int j = 0; j < R; j++) rank[j] += k < key[j] ? 1u : 0u;
        }
    }
#pragma unroll
    for (int j = 0; j < R; j++)
        if (c[j]) sc[rank[j]] = c[j];
    __builtin_amdgcn_wave_barrier();
    auto rd = [&](uint32_t i) { return __builtin_amdgcn_readfirstlane(sc[i]); };
    auto wr = [&](uint32_t i, uint32_t v) {
        if (lane == 0) sc[i] = v;
        __builtin_amdgcn_wave_barrier();
    };
    if (n >= 2u) {
        // pass 1: weights then parents
        // (at the start of step nx, root <= nx - 1 and leaf >= nx + 1, so the
        // cached leaf weight vl stays valid and A[nx] is written last)
        wr(0, rd(0) + rd(1));
        uint32_t root = 0, leaf = 2;
        uint32_t vl = n > 2u ? rd(2) : 0u;
        for (uint32_t nx = 1; nx < n - 1u; nx++) {
            uint32_t vr = rd(root), w;
            if (leaf >= n || vr < vl) {
                w = vr;
                wr(root, nx);
                root++;
                if (root < nx) vr = rd(root);
            } else {
                w = vl;
                leaf++;
                if (leaf < n) vl = rd(leaf);
            }
            if (leaf >= n || (root < nx && vr < vl)) {
                w += vr;
                wr(root, nx);
                root++;
            } else {
                w += vl;
                leaf++;
                if (leaf < n) vl = rd(leaf);
            }
            wr(nx, w);
        }
        // pass 2: internal depths by pointer jumping (lane-parallel, 9 rounds
        // cover any depth < 512): D[t] = depth so far, P[t] = ancestor
        uint32_t *D = sc + 64u * R;
        uint32_t d[R], pp[R];
#pragma unroll
        for (int k = 0; k < R; k++) {
            const uint32_t t = lane + 64u * (uint32_t)k;
            const bool in = t < n - 2u;                 // internal, not the root
            pp[k] = in ? sc[t] : t;
            d[k] = in ? 1u : 0u;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < R; k++) {
            const uint32_t t = lane + 64u * (uint32_t)k;
            if (t < n - 1u) {
                D[t] = d[k];
                sc[t] = pp[k];
            }
        }
        __builtin_amdgcn_wave_barrier();
        for (int round = 0; round < 9; round++) {
            uint32_t nd[R], np[R];
#pragma unroll
            for (int k = 0; k < R; k++) {
                const uint32_t t = lane + 64u * (uint32_t)k;
                const uint32_t a = t < n - 1u ? pp[k] : 0u;
                nd[k] = d[k] + (t < n - 1u ? D[a] : 0u);
                np[k] = t < n - 1u ? sc[a] : 0u;
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < R; k++) {
                const uint32_t t = lane + 64u * (uint32_t)k;
                d[k] = nd[k];
                pp[k] = np[k];
                if (t < n - 1u) {
                    D[t] = d[k];
                    sc[t] = pp[k];
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        // pass 3: leaves per depth from internal nodes per depth (a node at
        // depth x has two children at x + 1), folded at maxbits
        uint32_t *hist = D;                            // 64 words, D is read out
        hist[lane] = 0;
        __builtin_amdgcn_wave_barrier();
        bool deep = false;
#pragma unroll
        for (int k = 0; k < R; k++) {
            const uint32_t t = lane + 64u * (uint32_t)k;
            if (t < n - 1u) {
                deep |= d[k] > 62u;
                atomicAdd(&hist[min(d[k], 62u)], 1u);
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (__ballot(deep)) return false;
        const uint32_t ci = hist[lane];
        const uint32_t cprev = (uint32_t)__shfl((int)ci, (int)(lane ? lane - 1u : 0u));
        const uint32_t leaves = lane ? 2u * cprev - ci : 0u;  // leaves at depth = lane
        uint32_t bl[16];
        uint32_t over = 0;
        {
            uint32_t ov = lane > maxbits ? leaves : 0u;
            over = (uint32_t)wave_sum(ov);
        }
#pragma unroll
        for (int L = 0; L < 16; L++) bl[L] = (uint32_t)L <= maxbits ? rdlane(leaves, (uint32_t)L) : 0u;
#pragma unroll
        for (int L = 0; L < 16; L++)
            if ((uint32_t)L == maxbits) bl[L] += over;
        if (over) {
            // Kraft repair on the per-length counts: lengthen a code of the deepest
            // level below maxbits while over-subscribed, then shorten the deepest
            // one whose gain fits while under-subscribed
            const uint32_t T = 1u << maxbits;
            uint32_t K = 0;
#pragma unroll
            for (int L = 1; L < 16; L++)
                if ((uint32_t)L <= maxbits) K += bl[L] << (maxbits - (uint32_t)L);
            for (uint32_t it = 0; K > T && it < 4096u; it++) {
                int lv = -1;
#pragma unroll
                for (int L = 1; L < 16; L++)
                    if ((uint32_t)L < maxbits && bl[L]) lv = L;
                if (lv < 0) return false;
#pragma unroll
                for (int L = 1; L < 16; L++) {
                    if (L == lv) bl[L]--;
                    if (L == lv + 1) bl[L]++;
                }
                K -= 1u << (maxbits - (uint32_t)lv - 1u);
            }
            for (uint32_t it = 0; K < T && it < 4096u; it++) {
                int lv = -1;
#pragma unroll
                for (int L = 2; L < 16; L++)
                    if ((uint32_t)L <= maxbits && bl[L] && (1u << (maxbits - (uint32_t)L)) <= T - K) lv = L;
                if (lv < 0) return false;
#pragma unroll
                for (int L = 1; L < 16; L++) {
                    if (L == lv) bl[L]--;
                    if (L == lv - 1) bl[L]++;
                }
                K += 1u << (maxbits - (uint32_t)lv);
            }
            if (K != T) return false;
        }
        // lengths by rank: the least frequent symbols take the longest codes
#pragma unroll
        for (int j = 0; j < R; j++) {
            uint32_t r = rank[j], len = 0;
#pragma unroll
            for (int L = 15; L >= 1; L--) {
                if (len == 0u && (uint32_t)L <= maxbits) {
                    if (r < bl[L]) len = (uint32_t)L;
                    else r -= bl[L];
                }
            }
            l[j] = c[j] ? len : 0u;
        }
    } else {
#pragma unroll
        for (int j = 0; j < R; j++) l[j] = c[j] ? 1u : 0u;
    }
    __builtin_amdgcn_wave_barrier();
    return true;
}

// Code lengths for counts c[j] (symbol lane + 64 j; 0 = unused) of `total`
// symbols, limited to maxbits (64 R symbols must fit in 2^maxbits; R <= 8 and
// total < 2^22, so a count and a symbol share one 31-bit selection key).  Returns the
// longest length, or 0 when fewer than two symbols are used (no code needed).
template <int R>
__device__ uint32_t code_lengths(const uint32_t (&c)[R], uint32_t total, uint32_t maxbits, uint32_t (&l)[R],
                                 uint32_t lane, uint32_t *sc = nullptr) {
    uint32_t units = 0, used = 0;
    // start from the optimal lengths when LDS scratch is given (the loops below
    // then only run when some length exceeds maxbits), else from Shannon's
    const bool huff = sc && huffman_lengths<R>(c, maxbits, l, sc, lane);
#pragma unroll
    for (int j = 0; j < R; j++) {
        l[j] = c[j] ? min(max(huff ? l[j] : shannon_len(c[j], total), 1u), maxbits) : 0u;
        units += c[j] ? 1u << (maxbits - l[j]) : 0u;
        used += c[j] ? 1u : 0u;
    }
    if (wave_sum(used) < 2u) return 0;
    uint32_t K = wave_sum(units);
    const uint32_t T = 1u << maxbits;
    // over-subscribed: lengthen the least frequent symbol below the limit (each
    // step frees at least one unit; the caps only guard against a logic error)
    for (uint32_t it = 0; K > T; it++) {
        if (it >= 4096u) return 0;
        int32_t best = -1;
#pragma unroll
        for (int j = 0; j < R; j++)
            if (c[j] && l[j] < maxbits) best = max(best, (int32_t)(0x7FFFFFFFu - ((c[j] << 9) | (lane + 64u * j))));
        const int32_t bk = wave_max(best);
        if (bk < 0) return 0;
        const uint32_t s = (0x7FFFFFFFu - (uint32_t)bk) & 511u;
        const uint32_t js = s >> 6, lo = pick_lane<R>(l, js, s & 63u);
        K -= 1u << (maxbits - lo - 1u);
        if (lane == (s & 63u)) {
#pragma unroll
            for (int j = 0; j < R; j++)
                if ((uint32_t)j == js) l[j]++;
        }
    }
    // under-subscribed: shorten the most frequent symbol whose shortening fits
    // (the longest codes always do: every unit count divides the slack)
    for (uint32_t it = 0; K < T; it++) {
        if (it >= 4096u) return 0;
        const uint32_t slack = T - K;
        int32_t best = -1;
#pragma unroll
        for (int j = 0; j < R; j++)
            if (c[j] && l[j] > 1u && (1u << (maxbits - l[j])) <= slack)
                best = max(best, (int32_t)((c[j] << 9) | (lane + 64u * j)));
        const int32_t bk = wave_max(best);
        if (bk < 0) return 0;
        const uint32_t s = (uint32_t)bk & 511u;
        const uint32_t js = s >> 6, lo = pick_lane<R>(l, js, s & 63u);
        K += 1u << (maxbits - lo);
        if (lane == (s & 63u)) {
#pragma unroll
            for (int j = 0; j < R; j++)
                if ((uint32_t)j == js) l[j]--;
        }
    }
    int32_t m = 0;
#pragma unroll
    for (int j = 0; j < R; j++) m = max(m, (int32_t)l[j]);
    return (uint32_t)wave_max(m);
}

// zstd's canonical Huffman codes (huf_compress.c HUF_buildCTable, 1.1.2): the
// starting value of each length walks down from the longest, then codes are
// handed out in symbol order within a length.
__device__ void canonical_codes(const uint32_t (&l)[4], uint32_t maxlen, uint32_t (&code)[4], uint32_t lane) {
    uint32_t start[16];
    {
        uint32_t nb[16];
#pragma unroll
        for (int L = 0; L < 16; L++) nb[L] = 0;
#pragma unroll
        for (int L = 1; L <= 12; L++) {
            uint32_t k = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) k += (uint32_t)__popcll(__ballot(l[j] == (uint32_t)L));
            nb[L] = k;
        }
        uint32_t mn = 0;
#pragma unroll
        for (int L = 12; L >= 1; L--) {
            start[L] = (uint32_t)L <= maxlen ? mn : 0u;
            if ((uint32_t)L <= maxlen) mn = (mn + nb[L]) >> 1;
        }
    }
    const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        code[j] = 0;
#pragma unroll
        for (int L = 1; L <= 12; L++) {
            const uint64_t m = __ballot(l[j] == (uint32_t)L);
            if (l[j] == (uint32_t)L) code[j] = start[L] + (uint32_t)__popcll(m & lt);
            start[L] += (uint32_t)__popcll(m);
        }
    }
}

// Deflate's canonical codes (RFC 1951 3.2.2): shorter codes first, symbol
// order within a length; returned bit-reversed (deflate sends codes MSB first
// into an LSB-first stream).
template <int R>
__device__ void deflate_codes(const uint32_t (&l)[R], uint32_t (&rcode)[R], uint32_t lane) {
    uint32_t next[16];
    {
        uint32_t code = 0, prev = 0;
#pragma unroll
        for (int L = 1; L <= 15; L++) {
            code = (code + prev) << 1;
            next[L] = code;
            uint32_t k = 0;
#pragma unroll
            for (int j = 0; j < R; j++) k += (uint32_t)__popcll(__ballot(l[j] == (uint32_t)L));
            prev = k;
        }
    }
    const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
#pragma unroll
    for (int j = 0; j < R; j++) {
        uint32_t c = 0;
#pragma unroll
        for (int L = 1; L <= 15; L++) {
            const uint64_t m = __ballot(l[j] == (uint32_t)L);
            if (l[j] == (uint32_t)L) c = next[L] + (uint32_t)__popcll(m & lt);
            next[L] += (uint32_t)__popcll(m);
        }
        rcode[j] = l[j] ? __builtin_bitreverse32(c) >> (32u - l[j]) : 0u;
    }
}

// ------------------------------------------------------------ small FSE encoder (Huffman weights)
// Backward-readable bit writer (bitstream.h BIT_CStream): bits accumulate LSB
// first, whole bytes go out through lanes 0-7.
struct BitW {
    uint64_t c;
    uint32_t pos;
    uint32_t ptr;
};
__device__ __forceinline__ void bw_add(BitW &b, uint32_t v, uint32_t nb) {
    b.c |= (uint64_t)(v & ((1u << nb) - 1u)) << b.pos;
    b.pos += nb;
}
__device__ __forceinline__ void bw_flush(BitW &b, uint8_t *dst, uint32_t lane) {
    const uint32_t nbytes = b.pos >> 3;
    if (lane < nbytes) dst[b.ptr + lane] = (uint8_t)(b.c >> (8u * lane));
    b.ptr += nbytes;
    b.pos &= 7u;
    b.c = nbytes >= 8u ? 0ull : b.c >> (8u * nbytes);
}

// An FSE table of log <= 7 (at most 64 symbols) held in lanes: lane u has
// stateTable[u] (state) and stateTable[64 + u] (state_hi); lane s has the
// symbol transform of symbol s.
struct SmallCT {
    uint32_t state;      // stateTable entry u of this lane
    uint32_t state_hi;   // stateTable entry 64 + u (log 7)
    uint32_t dnb;        // deltaNbBits of symbol `lane`
    int32_t dfs;         // deltaFindState of symbol `lane`
    uint32_t log;
};

// FSE_buildCTable_wksp (fse_compress.c) for norm[], log <= 7; -1 entries
// (low-probability symbols) take one cell each at the top of the table.
// norm_l: lane s holds norm[s] (0 beyond max_sv).  A log-7 table goes through
// scr (128 LDS bytes of the caller's scratch) for its state scatter.
__device__ SmallCT build_small_ct(int32_t norm_l, uint32_t max_sv, uint32_t log, uint32_t lane, uint8_t *scr = nullptr) {
    const uint32_t size = 1u << log, mask = size - 1u, step = (size >> 1) + (size >> 3) + 3u;
    // low-probability cells from the top, then the spread (uniform serial walk);
    // lane u ends up with tableSymbol[u] (tsym) and tableSymbol[64 + u] (tsym_hi)
    uint32_t tsym = 0, tsym_hi = 0, pos = 0, high = size - 1u;
    auto put = [&](uint32_t cell, uint32_t s) {   // selects, not stores: keeps tsym / tsym_hi in VGPRs
        tsym = lane == cell ? s : tsym;
        tsym_hi = lane + 64u == cell ? s : tsym_hi;
    };
    for (uint32_t s = 0; s <= max_sv; s++)
        if ((int32_t)rdlane((uint32_t)norm_l, s) == -1) {
            put(high, s);
            high--;
        }
    for (uint32_t s = 0; s <= max_sv; s++) {
        const int32_t n = (int32_t)rdlane((uint32_t)norm_l, s);
        for (int32_t i = 0; i < n; i++) {
            put(pos, s);
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    }
    // cumul of norm (exclusive, -1 counting as 1), per symbol, in lanes
    const int32_t cells = lane <= max_sv ? (norm_l == -1 ? 1 : norm_l) : 0;
    const int32_t incl = wave_incl_sum(cells);
    const uint32_t cum_l = (uint32_t)(incl - cells);
    // stateTable[cumul[s] + rank of cell u among the cells of s] = size + u
    const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
    const bool lo_ok = lane < size, hi_ok = 64u + lane < size;
    uint32_t idx = lane, idx_hi = 0;   // lanes past the table permute onto themselves
    for (uint32_t s = 0; s <= max_sv; s++) {
        const uint64_t m = __ballot(lo_ok && tsym == s);
        const uint64_t mh = __ballot(hi_ok && tsym_hi == s);
        if (lo_ok && tsym == s) idx = rdlane(cum_l, s) + (uint32_t)__popcll(m & lt);
        if (hi_ok && tsym_hi == s) idx_hi = rdlane(cum_l, s) + (uint32_t)__popcll(m) + (uint32_t)__popcll(mh & lt);
    }
    SmallCT t;
    if (size <= 64u) {
        // scatter: lane idx receives size + u (ds_permute: the value goes to lane `addr / 4`)
        t.state = (uint32_t)__builtin_amdgcn_ds_permute((int32_t)(idx * 4u), (int32_t)(size + lane));
        if (lane >= size) t.state = 0;
        t.state_hi = 0;
    } else {
        __builtin_amdgcn_wave_barrier();
        scr[idx] = (uint8_t)(size + lane);
        scr[idx_hi] = (uint8_t)(size + 64u + lane);
        __builtin_amdgcn_wave_barrier();
        t.state = scr[lane];
        t.state_hi = scr[64u + lane];
        __builtin_amdgcn_wave_barrier();
    }
    // symbol transforms
    t.dnb = 0;
    t.dfs = 0;
    if (lane <= max_sv && norm_l != 0) {
        if (norm_l == 1 || norm_l == -1) {
            t.dnb = (log << 16) - (1u << log);
            t.dfs = (int32_t)cum_l - 1;
        } else {
            const uint32_t mbo = log - hb((uint32_t)norm_l - 1u);
            const uint32_t msp = (uint32_t)norm_l << mbo;
            t.dnb = (mbo << 16) - msp;
            t.dfs = (int32_t)cum_l - norm_l;
        }
    }
    t.log = log;
    return t;
}

// stateTable[i] for a wave-uniform i
__device__ __forceinline__ uint32_t ct_state(const SmallCT &t, uint32_t i) {
    return i < 64u ? rdlane(t.state, i) : rdlane(t.state_hi, i - 64u);
}
__device__ __forceinline__ uint32_t ct_init2(const SmallCT &t, uint32_t sym) {
    const uint32_t dnb = rdlane(t.dnb, sym);
    const uint32_t nbo = (dnb + (1u << 15)) >> 16;
    const uint32_t v = (nbo << 16) - dnb;
    return ct_state(t, (uint32_t)((int32_t)(v >> nbo) + (int32_t)rdlane((uint32_t)t.dfs, sym)));
}
__device__ __forceinline__ void ct_encode(BitW &b, uint32_t &st, const SmallCT &t, uint32_t sym) {
    const uint32_t nbo = (st + rdlane(t.dnb, sym)) >> 16;
    bw_add(b, st, nbo);
    st = ct_state(t, (uint32_t)((int32_t)(st >> nbo) + (int32_t)rdlane((uint32_t)t.dfs, sym)));
}

// FSE_optimalTableLog_internal (fse_compress.c:479-498) for n >= 2 symbols
// coded, max_sv the largest, the accuracy capped at max_log
__device__ __forceinline__ uint32_t optimal_log(uint32_t max_log, uint32_t n, uint32_t max_sv, uint32_t minus) {
    uint32_t log = max_log;
    const uint32_t max_bits_src = hb(n - 1u) - minus;
    const uint32_t min_bits = min(hb(n - 1u) + 1u, hb(max_sv ? max_sv : 1u) + 2u);
    if (max_bits_src < log) log = max_bits_src;
    if (min_bits > log) log = min_bits;
    return min(max(log, 5u), 12u);
}

// FSE_writeNCount (fse_compress.c, generic path) for norm_l (lane s = norm[s],
// all >= 0) at dst + o.  Returns the header size.
__device__ uint32_t write_ncount(int32_t norm_l, uint32_t max_sv, uint32_t log, uint8_t *dst, uint32_t o,
                                 uint32_t lane) {
    const uint32_t size = 1u << log;
    uint32_t bits = log - 5u, nbits = 4;    // FSE_MIN_TABLELOG 5
    uint32_t out = o;
    int32_t remaining = (int32_t)size + 1, threshold = (int32_t)size;
    uint32_t nb = log + 1u, s = 0;
    bool prev0 = false;
    auto put16 = [&]() {
        if (lane < 2) dst[out + lane] = (uint8_t)(bits >> (8u * lane));
        out += 2;
        bits >>= 16;
        nbits -= 16;
    };
    while (remaining > 1) {
        if (prev0) {
            uint32_t start = s;
            while (s <= max_sv && rdlane((uint32_t)norm_l, s) == 0u) s++;
            while (s >= start + 24u) {
                start += 24u;
                bits += 0xFFFFu << nbits;
                nbits += 16;
                put16();
            }
            while (s >= start + 3u) {
                start += 3u;
                bits += 3u << nbits;
                nbits += 2;
            }
            bits += (s - start) << nbits;
            nbits += 2;
            if (nbits > 16) put16();
        }
        int32_t count = (int32_t)rdlane((uint32_t)norm_l, s);
        s++;
        const int32_t mx = (2 * threshold - 1) - remaining;
        remaining -= count;
        count++;
        if (count >= threshold) count += mx;
        bits += (uint32_t)count << nbits;
        nbits += nb;
        nbits -= count < mx ? 1u : 0u;
        prev0 = count == 1;
        while (remaining < threshold) {
            nb--;
            threshold >>= 1;
        }
        if (nbits > 16) put16();
    }
    if (lane < 2) dst[out + lane] = (uint8_t)(bits >> (8u * lane));
    out += (nbits + 7u) / 8u;
    return out - o;
}

// Normalized counts for an FSE table of 2^log cells (FSE_normalizeCount's
// contract, simpler rounding): lane s holds count cnt of `total`; each used
// symbol gets >= 1 cell, the rest is proportional, and the rounding remainder
// goes to (or is taken from) the largest entries.  At most 64 symbols, and no
// more used symbols than cells.  Returns false only on a logic error.
__device__ bool normalize(uint32_t cnt, uint32_t total, uint32_t log, int32_t &norm, uint32_t lane) {
    const uint32_t size = 1u << log;
    norm = cnt ? max(1, (int32_t)(((uint64_t)cnt * size + total / 2u) / total)) : 0;
    int32_t diff = (int32_t)size - (int32_t)wave_sum((uint32_t)norm);
    for (uint32_t it = 0; diff != 0; it++) {
        if (it >= 64u) return false;
        // give to / take from the symbol with the largest normalized count (> 1 when taking)
        const int32_t key = (norm > (diff < 0 ? 1 : 0)) ? (norm << 8) | (int32_t)lane : -1;
        const int32_t bk = wave_max(key);
        if (bk < 0) return false;
        const uint32_t s = (uint32_t)bk & 255u;
        const int32_t have = (int32_t)rdlane((uint32_t)norm, s);
        const int32_t d = diff > 0 ? diff : max(diff, 1 - have);
        if (lane == s) norm += d;
        diff -= d;
    }
    return true;
}

// HUF_compressWeights (huf_compress.c, 1.1.2): FSE table log 6 at most,
// FSE_optimalTableLog, normalized counts, NCount header, two interleaved states
// (FSE_compress_usingCTable_generic).  w[0, n) are the weights (LDS bytes,
// values <= 11).  Writes at dst + o; returns the size, 0 when not compressible,
// 1 when every weight is equal (the caller then stores weights raw).
__device__ uint32_t compress_weights(const uint8_t *w, uint32_t n, uint8_t *dst, uint32_t o, uint32_t lane) {
    if (n <= 1u) return 0;
    // histogram of the weights in lanes: lane v counts weight v
    uint32_t cnt = 0;
    for (uint32_t i0 = 0; i0 < n; i0 += kWave) {
        const uint32_t i = i0 + lane;
        const uint32_t v = i < n ? w[i] : 0xFFu;
#pragma unroll
        for (uint32_t s = 0; s < 12; s++) {
            const uint32_t k = (uint32_t)__popcll(__ballot(v == s));
            if (lane == s) cnt += k;
        }
    }
    const uint32_t max_sv = (uint32_t)wave_max(cnt ? (int32_t)lane : -1);
    const uint32_t max_cnt = (uint32_t)wave_max((int32_t)cnt);
    if (max_cnt == n) return 1;
    if (max_cnt == 1u) return 0;
    const uint32_t log = optimal_log(6, n, max_sv, 2);   // FSE_optimalTableLog(6, n, max_sv)
    int32_t norm;
    if (!normalize(cnt, n, log, norm, lane)) return 0;
    uint32_t op = o + write_ncount(norm, max_sv, log, dst, o, lane);
    const SmallCT t = build_small_ct(norm, max_sv, log, lane);
    // FSE_compress_usingCTable_generic, 64-bit container (4 symbols per flush)
    if (n <= 2u) return 0;
    BitW b;
    b.c = 0;
    b.pos = 0;
    b.ptr = op;
    uint32_t s1, s2;
    int32_t ip = (int32_t)n;
    auto sym = [&](int32_t i) -> uint32_t { return rfl(w[i]); };
    if (n & 1u) {
        s1 = ct_init2(t, sym(--ip));
        s2 = ct_init2(t, sym(--ip));
        ct_encode(b, s1, t, sym(--ip));
        bw_flush(b, dst, lane);
    } else {
        s2 = ct_init2(t, sym(--ip));
        s1 = ct_init2(t, sym(--ip));
    }
    if ((n - 2u) & 2u) {
        ct_encode(b, s2, t, sym(--ip));
        ct_encode(b, s1, t, sym(--ip));
        bw_flush(b, dst, lane);
    }
    while (ip > 0) {
        ct_encode(b, s2, t, sym(--ip));
        ct_encode(b, s1, t, sym(--ip));
        ct_encode(b, s2, t, sym(--ip));
        ct_encode(b, s1, t, sym(--ip));
        bw_flush(b, dst, lane);
    }
    bw_add(b, s2, log);     // FSE_flushCState x2
    bw_flush(b, dst, lane);
    bw_add(b, s1, log);
    bw_flush(b, dst, lane);
    bw_add(b, 1u, 1u);      // BIT_closeCStream: end mark
    bw_flush(b, dst, lane);
    const uint32_t end = b.ptr + (b.pos > 0 ? 1u : 0u);
    if (b.pos > 0 && lane == 0) dst[b.ptr] = (uint8_t)b.c;
    return end - o;
}

}  // namespace huf
}  // namespace tyche
