// zstd_decode.hip -- gfx950 decoder for zstd frames, the codec behind
// buffer__decompress for ZSTD_COMPRESSOR_ID (src/buffer.c:263-266 ->
// ZSTD_decompress, src/zstd/zstd_decompress.c:1459; vendored zstd v1.1.2).
//
// One wave per page, waves loop over pages.  Per wave, LDS holds the rebuilt
// page (the match window), the staged frame, the Huffman table (4096 x 16 bit)
// and the three sequence FSE tables.  The decode follows the restatement in
// oracle/zstd_oracle.c step by step:
//
//   * frame / block headers, FSE_readNCount, FSE table spreading and the
//     sequence FSE chain are inherently serial: they run as wave-uniform code
//     (every lane computes the same value; loads are LDS broadcasts);
//   * Huffman tables are built lane-parallel (a ballot-ranked fill of the
//     X2 single-symbol table, huf_decompress.c:86-131);
//   * the four Huffman literal streams of a 4X section decode in four lanes at
//     once; the literals land at the tail of the page window [cap-litSize, cap):
//     every literal's output position is at or below its buffer position, so
//     sequences executed in order never overwrite a literal before it is read
//     (the "literals in dst" layout), and no separate literal buffer is needed;
//   * sequences are decoded 64 at a time (v_writelane into one register per
//     field) and executed like the LZ4 decoder's batches: output positions from
//     a DPP prefix sum, the reference's per-sequence checks in parallel
//     (zstd_decompress.c:940-954), literal runs placed in parallel, matches
//     copied in dependency (frontier) order.  The prefix of a batch whose output
//     stays below the first unread literal runs in parallel; the rest (the last
//     sequences of a block, when the window has no slack left) runs in order.
//
// The backward bit reader uses the reference's container (64 bits, the same
// BIT_lookBits / BIT_lookBitsFast / BIT_reloadDStream arithmetic) wherever the
// number of symbols depends on it (FSE-compressed Huffman weights, the
// sequence loop); Huffman literal streams reload whenever fewer than 12 bits
// remain, which yields the same symbols and the same exact-end verdict.
//
// Result per page: decoded size, or a negative value (any ZSTD_isError).
#include <algorithm>

#include "engine.h"
#include "lane_ring.h"
#include "lds_io.h"

namespace tyche {
namespace {

// Optional phase profile (diagnostic build only: -DTYCHE_PROFILE,
// tools/zstd_phases.py): shader cycles per phase summed by lane 0.
#ifdef TYCHE_PROFILE
__device__ unsigned long long g_sdprof[16];
#define SPROF_DECL unsigned long long _pt = clock64();
#define SPROF_MARK(slot)                                                       \
    do {                                                                       \
        unsigned long long _n = clock64();                                     \
        if (lane == 0) atomicAdd(&g_sdprof[slot], _n - _pt);                   \
        _pt = _n;                                                              \
    } while (0)
#define SPROF_ADD(slot, v) do { if (lane == 0) atomicAdd(&g_sdprof[slot], (unsigned long long)(v)); } while (0)
#else
#define SPROF_DECL
#define SPROF_MARK(slot) do { } while (0)
#define SPROF_ADD(slot, v) do { } while (0)
#endif

constexpr uint32_t kWave = 64;
#ifndef TYCHE_ZABLATE
#define TYCHE_ZABLATE 0
#endif
constexpr int32_t kErr = -20;          // corruption_detected (any error: buffer.c only tests ZSTD_isError)
constexpr int32_t kErrDst = -70;       // dstSize_tooSmall
constexpr uint32_t kBlockMax = 128u * 1024u;
constexpr uint32_t kStreamPad = 32;    // zero bytes after the staged frame (8-byte container reads)
constexpr uint32_t kWinPad = 32;       // slack after the window (4X streams may run 3 bytes past)

// ------------------------------------------------------------ constant tables
__device__ __constant__ uint32_t c_ll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                                 1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12,
                                                 13, 14, 15, 16};
__device__ __constant__ uint32_t c_ml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                                 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                                 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11,
                                                 12, 13, 14, 15, 16};
__device__ __constant__ uint32_t c_ll_base[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
                                                  16, 18, 20, 22, 24, 28, 32, 40, 48, 64, 0x80, 0x100, 0x200, 0x400,
                                                  0x800, 0x1000, 0x2000, 0x4000, 0x8000, 0x10000};
__device__ __constant__ uint32_t c_ml_base[53] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18,
                                                  19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34,
                                                  35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 0x83, 0x103, 0x203,
                                                  0x403, 0x803, 0x1003, 0x2003, 0x4003, 0x8003, 0x10003};
__device__ __constant__ uint32_t c_of_base[29] = {0, 1, 1, 5, 0xD, 0x1D, 0x3D, 0x7D, 0xFD, 0x1FD, 0x3FD, 0x7FD,
                                                  0xFFD, 0x1FFD, 0x3FFD, 0x7FFD, 0xFFFD, 0x1FFFD, 0x3FFFD, 0x7FFFD,
                                                  0xFFFFD, 0x1FFFFD, 0x3FFFFD, 0x7FFFFD, 0xFFFFFD, 0x1FFFFFD,
                                                  0x3FFFFFD, 0x7FFFFFD, 0xFFFFFFD};
// Base value and extra-bit count of a code (LL_base/LL_bits, ML_base/ML_bits,
// OF_base of zstd_decompress.c:864-879, zstd_internal.h:115-127), computed
// instead of loaded so the serial sequence chain carries no memory waits.
__device__ __forceinline__ uint32_t of_base(uint32_t c) { return c < 2u ? c : (1u << c) - 3u; }
// The middle codes of both tables share one shape: k < 4 -> base step 2, 1 bit;
// then pairs j = k - 4: base step (4 | 6) << (j / 2), 2 + j / 2 bits.  Written as
// selects so the scalar chain has no branches.
__device__ __forceinline__ void mid_code(uint32_t k, uint32_t &f, uint32_t &bits) {
    const uint32_t j = k - 4u, h = j >> 1;
    const uint32_t fj = ((j & 1u) ? 6u : 4u) << (h & 7u);
    f = k < 4u ? k : fj;
    bits = k < 4u ? 1u : 2u + h;
}
__device__ __forceinline__ void ll_code(uint32_t c, uint32_t &base, uint32_t &bits) {
    // 0..15: base c; 16..24: bases 16 18 20 22 24 28 32 40 48, bits 1 1 1 1 2 2 3 3 4;
    // 25..35: bits c - 19, base 1 << bits
    uint32_t f, mb;
    mid_code(c - 16u, f, mb);
    const uint32_t hb = c - 19u;
    bits = c < 16u ? 0u : (c < 25u ? mb : hb);
    base = c < 16u ? c : (c < 25u ? 16u + 2u * f : 1u << (hb & 31u));
}
__device__ __forceinline__ void ml_code(uint32_t c, uint32_t &base, uint32_t &bits) {
    // 0..31: base c + 3; 32..42: bases 35 37 39 41 43 47 51 59 67 83 99,
    // bits 1 1 1 1 2 2 3 3 4 4 5; 43..52: bits c - 36, base (1 << bits) + 3
    uint32_t f, mb;
    mid_code(c - 32u, f, mb);
    const uint32_t hb = c - 36u;
    bits = c < 32u ? 0u : (c < 43u ? mb : hb);
    base = c < 32u ? c + 3u : (c < 43u ? 35u + 2u * f : (1u << (hb & 31u)) + 3u);
}

// The same as branches: the wave-uniform chain below runs faster on SALU
// branches than on selects (2,087 vs 2,294 ms per 1M C3 pages, fused kernel)
__device__ __forceinline__ void ll_code_s(uint32_t c, uint32_t &base, uint32_t &bits) {
    if (c < 16u) { base = c; bits = 0; return; }
    if (c < 24u) {
        // codes 16..23: bases 16 18 20 22 24 28 32 40, bits 1 1 1 1 2 2 3 3
        const uint32_t k = c - 16u;
        bits = k < 4u ? 1u : (k < 6u ? 2u : 3u);
        base = k < 4u ? 16u + 2u * k : (k < 6u ? 24u + 4u * (k - 4u) : 32u + 8u * (k - 6u));
        return;
    }
    if (c == 24u) { base = 48u; bits = 4u; return; }
    bits = c - 19u;
    base = 1u << bits;
}
__device__ __forceinline__ void ml_code_s(uint32_t c, uint32_t &base, uint32_t &bits) {
    if (c < 32u) { base = c + 3u; bits = 0; return; }
    if (c < 43u) {
        // codes 32..42: bases 35 37 39 41 43 47 51 59 67 83 99, bits 1 1 1 1 2 2 3 3 4 4 5
        const uint32_t k = c - 32u;
        bits = k < 4u ? 1u : (k < 6u ? 2u : (k < 8u ? 3u : (k < 10u ? 4u : 5u)));
        base = k < 4u ? 35u + 2u * k : (k < 6u ? 43u + 4u * (k - 4u) : (k < 8u ? 51u + 8u * (k - 6u)
                                                                          : (k < 10u ? 67u + 16u * (k - 8u) : 99u)));
        return;
    }
    bits = c - 36u;
    base = (1u << bits) + 3u;
}

// The predefined decoding tables (ZSTD_buildSeqTable set_basic ->
// LL/OF/ML_defaultDTable, zstd_decompress.c:517-687) are FSE_buildDTable over
// the default distributions; built here at compile time.
constexpr int8_t kLLNormH[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1,
                                 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int8_t kMLNormH[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int8_t kOFNormH[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1,
                                 -1, -1};
struct DTab {
    uint32_t cell[64];   // newState | symbol << 16 | nbBits << 24
};
constexpr uint32_t ce_hb(uint32_t v) {
    uint32_t r = 0;
    while (v >>= 1) r++;
    return r;
}
constexpr DTab make_dtab(const int8_t *norm, uint32_t max_sv, uint32_t log) {
    DTab t{};
    const uint32_t size = 1u << log, mask = size - 1u, step = (size >> 1) + (size >> 3) + 3u;
    uint32_t high = size - 1u;
    uint32_t next[64] = {};
    uint32_t sym[64] = {};
    for (uint32_t s = 0; s <= max_sv; s++) {
        if (norm[s] == -1) {
            sym[high--] = s;
            next[s] = 1;
        } else {
            next[s] = (uint32_t)norm[s];
        }
    }
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= max_sv; s++)
        for (int i = 0; i < norm[s]; i++) {
            sym[pos] = s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t sy = sym[u], ns = next[sy]++;
        const uint32_t nb = log - ce_hb(ns);
        t.cell[u] = ((ns << nb) - size) | (sy << 16) | (nb << 24);
    }
    return t;
}
__device__ __constant__ DTab c_ll_def = make_dtab(kLLNormH, 35, 6);
__device__ __constant__ DTab c_of_def = make_dtab(kOFNormH, 28, 5);
__device__ __constant__ DTab c_ml_def = make_dtab(kMLNormH, 52, 6);

// ------------------------------------------------------------ LDS workspace
struct Work {
    uint8_t *win;        // page window (cap + kWinPad)
    const uint8_t *in;   // staged frame (len + kStreamPad zero bytes)
    uint16_t *huf;       // 2048 entries: symbol | nbBits << 8, indexed by the next min(tableLog, 11) bits
    uint8_t *hpair;      // tableLog 12 only: the symbols of the 12-bit codes, by 12-bit index
    uint32_t *ll, *of, *ml;   // FSE cells: newState | symbol << 16 | nbBits << 24
    uint32_t *wt;        // 64 cells for the Huffman-weight FSE table
    int16_t *norm;       // 256 normalized counts
    uint16_t *next;      // 256 symbolNext counters
    uint8_t *w;          // 256 Huffman weights
    // Pass 1 (zstd_entropy_kernel, round 6) stages the frame lazily: only the byte ranges its parse
    // reads (stage_range), so the literal streams and sequence bitstreams it hands to
    // zstd_lit_kernel and zstd_seqexec_kernel cross HBM once.  gsrc == nullptr: the whole frame was
    // staged up front (the other kernels).
    const uint8_t *gsrc;   // the frame in global memory
    uint32_t ghead;        // gsrc & 15 (in = 16-byte-aligned stage + ghead)
    int32_t gL;            // frame bytes
    mutable int32_t wlo, whi;   // [wlo, whi): the staged window the parse is in
};

// 8 bytes at any LDS byte address from three aligned dwords: an unaligned LDS
// read is replayed at ~64 LDS cycles per wave instruction (this file builds
// without the IR load/store vectorizer, so the dwords are not re-fused into a
// misaligned ds_read_b96; _build.py)
__device__ __forceinline__ uint64_t ld64(const uint8_t *p) {
    const uint32_t s = (uint32_t)(uintptr_t)p & 3u;
    const uint32_t *A = (const uint32_t *)(p - s);
    const uint32_t d0 = A[0], d1 = A[1], d2 = A[2];
    return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32);
}
__device__ __forceinline__ uint32_t highbit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// Makes frame bytes [a, e) readable in W.in (lazy staging, Work::gsrc; the whole wave).  The parse
// reads forward only: a range starting inside the current window extends it, one starting past
// it opens a new window (the bytes skipped -- deferred sections -- are never read in pass 1).
// Bytes at and past L read as the kStreamPad zeros, as with the whole frame staged.
__device__ __forceinline__ void stage_range(const Work &W, int32_t a, int32_t e, uint32_t lane) {
    if (!W.gsrc) return;
    a = max(a, 0);
    e = min(e, W.gL);
    if (e <= a || (a >= W.wlo && e <= W.whi)) return;
    const bool extend = a >= W.wlo && a <= W.whi;
    const int32_t from = extend ? W.whi : a;
    const uint32_t v0 = (W.ghead + (uint32_t)from) >> 4, v1 = (W.ghead + (uint32_t)e + 15u) >> 4;
    const u32x4 *g = (const u32x4 *)((uintptr_t)W.gsrc - W.ghead);
    u32x4 *l = (u32x4 *)(const_cast<uint8_t *>(W.in) - W.ghead);
    for (uint32_t v = v0 + lane; v < v1; v += kWave) l[v] = gload_nt(g + v);
    __builtin_amdgcn_wave_barrier();
    const int32_t top = (int32_t)(v1 * 16u - W.ghead);   // staged through here (the last vector whole)
    if (top > W.gL) {   // that vector carried bytes past L over the zero pad: restore it
        if (lane < kStreamPad / 4) lds_st32(const_cast<uint8_t *>(W.in) + W.gL + lane * 4, 0u);
        __builtin_amdgcn_wave_barrier();
    }
    if (!extend) W.wlo = a;
    W.whi = min(top, W.gL);
}

// Wave-uniform reads of the staged frame: the value goes through
// v_readfirstlane so everything computed from it stays in SGPRs.
__device__ __forceinline__ uint32_t u8u(const uint8_t *in, int32_t i) { return rfl(in[i]); }
__device__ __forceinline__ uint32_t u16u(const uint8_t *in, int32_t i) { return rfl(lds_ld16(in + i)); }
__device__ __forceinline__ uint32_t u32u(const uint8_t *in, int32_t i) { return rfl(lds_ld32(in + i)); }
__device__ __forceinline__ int32_t ru(int32_t v) { return (int32_t)rfl((uint32_t)v); }

// ------------------------------------------------------------ bit reader (bitstream.h:260-408)
enum : uint32_t { kUnfinished = 0, kEndOfBuffer = 1, kCompleted = 2, kOverflow = 3 };

struct BitD {
    uint64_t c;
    uint32_t used;
    int32_t ptr, start;   // byte offsets into the staged frame
};

// Returns false when BIT_initDStream fails (empty stream or no end mark).
__device__ __forceinline__ bool bitd_init(BitD &b, const uint8_t *in, int32_t start, int32_t n) {
    b.start = start;
    b.c = 0;
    b.used = 0;
    b.ptr = start;
    if (n < 1) return false;
    const uint32_t last = in[start + n - 1];
    if (last == 0) return false;
    const uint32_t mark = 8u - highbit(last);
    if (n >= 8) {
        b.ptr = start + n - 8;
        b.c = ld64(in + b.ptr);
        b.used = mark;
    } else {
        uint64_t c = in[start];
        for (int32_t k = 1; k < n; k++) {
            const uint32_t sh = k <= 3 ? 8u * (uint32_t)k : 64u - 8u * (8u - (uint32_t)k);
            c += (uint64_t)in[start + k] << sh;
        }
        b.c = c;
        b.used = mark + (uint32_t)(8 - n) * 8u;
    }
    return true;
}
// Wave-uniform variants: the loaded container goes through v_readfirstlane so
// the whole reader (and every table index derived from it) lives in SGPRs and
// constant-table lookups become scalar loads.
__device__ __forceinline__ uint64_t ld64u(const uint8_t *p) {
    const uint64_t v = ld64(p);
    return (uint64_t)rfl((uint32_t)v) | ((uint64_t)rfl((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ bool bitd_init_u(BitD &b, const uint8_t *in, int32_t start, int32_t n) {
    start = ru(start);
    n = ru(n);
    b.start = start;
    b.c = 0;
    b.used = 0;
    b.ptr = start;
    if (n < 1) return false;
    const uint32_t last = rfl(in[start + n - 1]);
    if (last == 0) return false;
    const uint32_t mark = 8u - highbit(last);
    if (n >= 8) {
        b.ptr = start + n - 8;
        b.c = ld64u(in + b.ptr);
        b.used = mark;
    } else {
        uint64_t c = rfl(in[start]);
        for (int32_t k = 1; k < n; k++) {
            const uint32_t sh = k <= 3 ? 8u * (uint32_t)k : 64u - 8u * (8u - (uint32_t)k);
            c += (uint64_t)rfl(in[start + k]) << sh;
        }
        b.c = c;
        b.used = mark + (uint32_t)(8 - n) * 8u;
    }
    return true;
}

__device__ __forceinline__ uint64_t bitd_look(const BitD &b, uint32_t nb) {
    return ((b.c << (b.used & 63u)) >> 1) >> ((63u - nb) & 63u);
}
__device__ __forceinline__ uint64_t bitd_look_fast(const BitD &b, uint32_t nb) {
    return (b.c << (b.used & 63u)) >> ((64u - nb) & 63u);
}
__device__ __forceinline__ uint32_t bitd_read(BitD &b, uint32_t nb) {
    const uint32_t v = (uint32_t)bitd_look(b, nb);
    b.used += nb;
    return v;
}
__device__ __forceinline__ uint32_t bitd_read_fast(BitD &b, uint32_t nb) {
    const uint32_t v = (uint32_t)bitd_look_fast(b, nb);
    b.used += nb;
    return v;
}
__device__ __forceinline__ uint32_t bitd_reload(BitD &b, const uint8_t *in) {
    if (b.used > 64u) return kOverflow;
    if (b.ptr >= b.start + 8) {
        b.ptr -= (int32_t)(b.used >> 3);
        b.used &= 7u;
        b.c = ld64(in + b.ptr);
        return kUnfinished;
    }
    if (b.ptr == b.start) return b.used < 64u ? kEndOfBuffer : kCompleted;
    int32_t nbytes = (int32_t)(b.used >> 3);
    uint32_t r = kUnfinished;
    if (b.ptr - nbytes < b.start) {
        nbytes = b.ptr - b.start;
        r = kEndOfBuffer;
    }
    b.ptr -= nbytes;
    b.used -= (uint32_t)nbytes * 8u;
    b.c = ld64(in + b.ptr);
    return r;
}

__device__ __forceinline__ uint32_t bitd_reload_u(BitD &b, const uint8_t *in) {
    if (b.used > 64u) return kOverflow;
    if (b.ptr >= b.start + 8) {
        b.ptr -= (int32_t)(b.used >> 3);
        b.used &= 7u;
        b.c = ld64u(in + b.ptr);
        return kUnfinished;
    }
    if (b.ptr == b.start) return b.used < 64u ? kEndOfBuffer : kCompleted;
    int32_t nbytes = (int32_t)(b.used >> 3);
    uint32_t r = kUnfinished;
    if (b.ptr - nbytes < b.start) {
        nbytes = b.ptr - b.start;
        r = kEndOfBuffer;
    }
    b.ptr -= nbytes;
    b.used -= (uint32_t)nbytes * 8u;
    b.c = ld64u(in + b.ptr);
    return r;
}

// ------------------------------------------------------------ FSE (uniform code)
// FSE_readNCount (entropy_common.c:65-157) over in[ip0, ip0+n).  Returns header
// bytes or < 0; max_sv in/out, table_log out.
__device__ int32_t read_ncount(const uint8_t *in, int32_t ip0, int32_t n, int16_t *norm, uint32_t &max_sv,
                               uint32_t &table_log) {
    if (n < 4) return kErr;
    const int32_t iend = ip0 + n;
    int32_t ip = ip0;
    uint32_t bits = rfl(lds_ld32(in + ip));
    int32_t nb = (int32_t)(bits & 0xFu) + 5;
    if (nb > 15) return kErr;
    bits >>= 4;
    int32_t bitcount = 4;
    table_log = (uint32_t)nb;
    int32_t remaining = (1 << nb) + 1, threshold = 1 << nb;
    nb++;
    uint32_t charnum = 0;
    bool prev0 = false;
    while ((remaining > 1) & (charnum <= max_sv)) {
        if (prev0) {
            uint32_t n0 = charnum;
            while ((bits & 0xFFFFu) == 0xFFFFu) {
                n0 += 24;
                if (ip < iend - 5) {
                    ip += 2;
                    bits = rfl(lds_ld32(in + ip)) >> (bitcount & 31);
                } else {
                    bits >>= 16;
                    bitcount += 16;
                }
            }
            while ((bits & 3u) == 3u) {
                n0 += 3;
                bits >>= 2;
                bitcount += 2;
            }
            n0 += bits & 3u;
            bitcount += 2;
            if (n0 > max_sv) return kErr;
            while (charnum < n0) norm[charnum++] = 0;
            if ((ip <= iend - 7) || (ip + (bitcount >> 3) <= iend - 4)) {
                ip += bitcount >> 3;
                bitcount &= 7;
                bits = rfl(lds_ld32(in + ip)) >> bitcount;
            } else {
                bits >>= 2;
            }
        }
        const int32_t mx = (2 * threshold - 1) - remaining;
        int32_t count;
        if ((bits & (uint32_t)(threshold - 1)) < (uint32_t)mx) {
            count = (int32_t)(bits & (uint32_t)(threshold - 1));
            bitcount += nb - 1;
        } else {
            count = (int32_t)(bits & (uint32_t)(2 * threshold - 1));
            if (count >= threshold) count -= mx;
            bitcount += nb;
        }
        count--;
        remaining -= count < 0 ? -count : count;
        norm[charnum++] = (int16_t)count;
        prev0 = count == 0;
        while (remaining < threshold) {
            nb--;
            threshold >>= 1;
        }
        if ((ip <= iend - 7) || (ip + (bitcount >> 3) <= iend - 4)) {
            ip += bitcount >> 3;
            bitcount &= 7;
        } else {
            bitcount -= 8 * (iend - 4 - ip);
            ip = iend - 4;
        }
        bits = rfl(lds_ld32(in + ip)) >> (bitcount & 31);
    }
    if (remaining != 1) return kErr;
    if (bitcount > 32) return kErr;
    max_sv = charnum - 1;
    ip += (bitcount + 7) >> 3;
    return ip - ip0;
}

__device__ __forceinline__ uint32_t cell(uint32_t new_state, uint32_t sym, uint32_t nb) {
    return new_state | (sym << 16) | (nb << 24);
}
__device__ __forceinline__ uint32_t cell_state(uint32_t c) { return c & 0xFFFFu; }
__device__ __forceinline__ uint32_t cell_sym(uint32_t c) { return (c >> 16) & 0xFFu; }
__device__ __forceinline__ uint32_t cell_nb(uint32_t c) { return c >> 24; }

// FSE_buildDTable (fse_decompress.c:113-168) from norm[0..max_sv]; cells[] gets
// 1 << table_log entries.  The symbol spread is lane-parallel (a serial,
// wave-uniform walk for alphabets over 64 symbols or tables over 512 cells);
// lanes then finish the cells of each 64-entry chunk with per-symbol ranks.
// Returns false on the reference's GENERIC error (spread did not close).
__device__ bool dtable_states(uint32_t *cells, uint16_t *next, uint32_t table_log, uint32_t lane);
__device__ bool build_dtable(uint32_t *cells, const int16_t *norm, uint32_t max_sv, uint32_t table_log,
                             uint16_t *next, uint32_t lane) {
    const uint32_t size = 1u << table_log, mask = size - 1u;
    const uint32_t step = (size >> 1) + (size >> 3) + 3u;
    if (max_sv < kWave && size <= 512u) {
        // Round 3: the spread lane-parallel.  The serial walk visits positions (k * step) & mask
        // (k = 0, 1, ...) skipping those above `high`, and the i-th valid position takes the i-th
        // occurrence in symbol order -- so each lane takes a k, ranks the valid ones with a ballot,
        // and looks its occurrence's symbol up in an occurrence -> symbol map (in next's bytes
        // until next is filled).  read_ncount guarantees the counts fill the table; a table that
        // does not is rejected as the serial walk's `position != 0` rejects it.
        const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
        const bool sym = lane <= max_sv;
        const int32_t c = sym ? (int32_t)norm[lane] : 0;
        const bool low = sym && c == -1;
        const uint64_t mlow = __ballot(low);
        if (low) cells[size - 1u - (uint32_t)__popcll(mlow & below)] = lane << 16;
        const uint32_t high = size - 1u - (uint32_t)__popcll(mlow);
        const int32_t cnt = low || c < 0 ? 0 : c;
        const int32_t incl = wave_incl_sum(cnt), excl = incl - cnt;
        if ((uint32_t)rdlane((uint32_t)incl, kWave - 1) != high + 1u) return false;
        uint8_t *occ = (uint8_t *)next;   // <= 512 entries: next's 256 x 16 bit
        __builtin_amdgcn_wave_barrier();
        for (int32_t i = 0; i < cnt; i++) occ[excl + i] = (uint8_t)lane;
        __builtin_amdgcn_wave_barrier();
        uint32_t taken = 0;
        for (uint32_t k0 = 0; k0 < size; k0 += kWave) {
            const uint32_t k = k0 + lane, p = (k * step) & mask;
            const bool v = k < size && p <= high;
            const uint64_t mv = __ballot(v);
            if (v) cells[p] = (uint32_t)occ[taken + (uint32_t)__popcll(mv & below)] << 16;
            taken += (uint32_t)__popcll(mv);
        }
        __builtin_amdgcn_wave_barrier();
        if (sym) next[lane] = (uint16_t)(low ? 1 : c);
        __builtin_amdgcn_wave_barrier();
        return dtable_states(cells, next, table_log, lane);
    }
    uint32_t high = size - 1u;
    // symbols are written into bits 16..23 first (cell = sym << 16)
    for (uint32_t s = 0; s <= max_sv; s++) {
        const int32_t c = norm[s];
        if (c == -1) {
            if (lane == 0) cells[high] = s << 16;
            high--;
        }
        if (lane == 0) next[s] = (uint16_t)(c == -1 ? 1 : c);
    }
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= max_sv; s++) {
        const int32_t c = norm[s];
        // occurrences of s go 64 at a time: lane i takes the i-th next valid position
        for (int32_t i0 = 0; i0 < c; i0 += (int32_t)kWave) {
            const uint32_t take = (uint32_t)min((int32_t)kWave, c - i0);
            // walk serially (positions above `high` are skipped)
            uint32_t mine = 0;
            for (uint32_t k = 0; k < take; k++) {
                if (lane == k) mine = pos;
                pos = (pos + step) & mask;
                while (pos > high) pos = (pos + step) & mask;
            }
            if (lane < take) cells[mine] = s << 16;
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (pos != 0) return false;
    return dtable_states(cells, next, table_log, lane);
}

// nextState = symbolNext[s]++ in cell order (FSE_buildDTable): per 64-cell chunk, rank lanes by
// symbol; cells hold their symbol in bits 16..23, next[s] the symbol's count (-1 as 1).
__device__ bool dtable_states(uint32_t *cells, uint16_t *next, uint32_t table_log, uint32_t lane) {
    const uint32_t size = 1u << table_log;
    for (uint32_t u0 = 0; u0 < size; u0 += kWave) {
        const uint32_t u = u0 + lane;
        const bool act = u < size;
        const uint32_t s = act ? cell_sym(cells[u]) : 0xFFFFu;
        uint64_t todo = __ballot(act);
        uint32_t ns = 0;
        while (todo) {
            const uint32_t l = (uint32_t)__builtin_ctzll(todo);
            const uint32_t sl = rdlane(s, l);
            const uint64_t m = __ballot(act && s == sl);
            const uint32_t base = next[sl];
            if (s == sl && act) ns = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            __builtin_amdgcn_wave_barrier();
            if (lane == l) next[sl] = (uint16_t)(base + (uint32_t)__builtin_popcountll(m));
            __builtin_amdgcn_wave_barrier();
            todo &= ~m;
        }
        if (act) {
            const uint32_t nb = table_log - highbit(ns);
            cells[u] = cell((ns << nb) - size, s, nb);
        }
    }
    __builtin_amdgcn_wave_barrier();
    return true;
}

// ------------------------------------------------------------ Huffman (HUF_readStats + HUF_readDTableX2)
// Reads the table description at in[ip, ip+n).  Returns header bytes or < 0;
// fills W.huf and sets tlog.
// HUF_readDTableX2's fill (huf_decompress.c): symbol s of weight w takes (1 << w) >> 1 entries after
// the earlier symbols of that weight, entry = s | nbBits << 8 (nbBits = tlog + 1 - w); rank[k] is the
// number of symbols of weight k (the last, implied weight included).  The whole wave; hpair only for
// tlog 12 (see below).
__device__ void huf_fill(const uint8_t *w, uint32_t nsym, uint32_t tlog, const uint32_t (&rank)[13], uint16_t *huf,
                         uint8_t *hpair, uint32_t lane) {
    // rank starts (HUF_readDTableX2 "Prepare ranks")
    uint32_t start[13];
    {
        uint32_t nx = 0;
#pragma unroll
        for (uint32_t k = 1; k < 13; k++) {
            start[k] = nx;
            if (k < tlog + 1u) nx += rank[k] << (k - 1);
        }
    }
    for (uint32_t s0 = 0; s0 < nsym; s0 += kWave) {
        const uint32_t s = s0 + lane;
        const uint32_t wv = s < nsym ? w[s] : 0u;
        uint32_t at = 0;
#pragma unroll
        for (uint32_t k = 1; k < 13; k++) {
            const uint64_t m = __ballot(s < nsym && wv == k);
            if (wv == k) at = start[k] + (__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0)) << (k - 1));
            start[k] += (uint32_t)__builtin_popcountll(m) << (k - 1);
        }
        // tableLog 12: the table is indexed by 11 bits.  Symbols of weight >= 2
        // start at even 12-bit positions and cover an even number of them, so
        // they halve exactly; the weight-1 symbols (12-bit codes, an even number
        // of them, first in the table) go to hpair and their 11-bit entries say
        // "12 bits, see hpair".
        const bool t12 = tlog == 12u;
        uint32_t len = s < nsym && wv ? (1u << wv) >> 1 : 0u;
        const uint16_t e = (uint16_t)(s | ((tlog + 1u - wv) << 8));
        if (t12) {
            if (len == 1u) {
                hpair[at] = (uint8_t)s;
                huf[at >> 1] = (uint16_t)(12u << 8);
                len = 0;
            }
            at >>= 1;
            len >>= 1;
        }
        if (len <= 16) {
            for (uint32_t i = 0; i < len; i++) huf[at + i] = e;
        }
        uint64_t big = __ballot(len > 16);
        while (big) {
            const uint32_t l = (uint32_t)__builtin_ctzll(big);
            big &= big - 1;
            const uint32_t bat = rdlane(at, l), blen = rdlane(len, l), be = rdlane((uint32_t)e, l);
            for (uint32_t i = lane; i < blen; i += kWave) huf[bat + i] = (uint16_t)be;
        }
    }
}

__device__ int32_t huf_read_table(const Work &W, int32_t ip, int32_t n, uint32_t &tlog, uint32_t &nsym_out, uint32_t lane) {
    const uint8_t *in = W.in;
    if (n < 1) return kErr;
    int32_t isize = (int32_t)u8u(in, ip);
    uint32_t osize;
    if (isize >= 128) {
        osize = (uint32_t)isize - 127u;
        isize = (int32_t)((osize + 1) / 2);
        if (isize + 1 > n) return kErr;
        if (osize >= 256) return kErr;
        for (uint32_t k = lane; k < (osize + 1) / 2 * 2; k += kWave) {
            const uint32_t b = in[ip + 1 + (int32_t)(k / 2)];
            W.w[k] = (uint8_t)((k & 1) ? (b & 15u) : (b >> 4));
        }
    } else {
        if (isize + 1 > n) return kErr;
        // FSE_decompress_wksp(w, 255, ip+1, isize, ws, 6)
        uint32_t max_sv = 255, flog;
        const int32_t hs = read_ncount(in, ip + 1, isize, W.norm, max_sv, flog);
        if (hs < 0) return hs;
        if (hs > isize) return kErr;
        if (flog > 6) return kErr;
        if (!build_dtable(W.wt, W.norm, max_sv, flog, W.next, lane)) return kErr;
        bool fast = true;
        const int32_t large = 1 << (flog - 1);
        for (uint32_t s = 0; s <= max_sv; s++)
            if (W.norm[s] >= large) fast = false;
        // FSE_decompress_usingDTable_generic (fse_decompress.c:218-275)
        BitD b;
        if (!bitd_init_u(b, in, ip + 1 + hs, isize - hs)) return kErr;
        uint32_t s1 = bitd_read(b, flog);
        bitd_reload_u(b, in);
        uint32_t s2 = bitd_read(b, flog);
        bitd_reload_u(b, in);
        uint32_t op = 0;
        const uint32_t omax = 255, olimit = omax - 3;
        auto sym = [&](uint32_t &st) -> uint32_t {
            const uint32_t c = rfl(W.wt[st]);
            const uint32_t nbb = cell_nb(c);
            const uint32_t low = fast ? bitd_read_fast(b, nbb) : bitd_read(b, nbb);
            st = cell_state(c) + low;
            return cell_sym(c);
        };
        for (;;) {
            const uint32_t st = bitd_reload_u(b, in);
            if (!((st == kUnfinished) & (op < olimit))) break;
            const uint32_t a0 = sym(s1), a1 = sym(s2), a2 = sym(s1), a3 = sym(s2);
            if (lane == 0) {
                W.w[op] = (uint8_t)a0;
                W.w[op + 1] = (uint8_t)a1;
                W.w[op + 2] = (uint8_t)a2;
                W.w[op + 3] = (uint8_t)a3;
            }
            op += 4;
        }
        for (;;) {
            if (op > omax - 2) return kErr;
            uint32_t a = sym(s1);
            if (lane == 0) W.w[op] = (uint8_t)a;
            op++;
            if (bitd_reload_u(b, in) == kOverflow) {
                a = sym(s2);
                if (lane == 0) W.w[op] = (uint8_t)a;
                op++;
                break;
            }
            if (op > omax - 2) return kErr;
            a = sym(s2);
            if (lane == 0) W.w[op] = (uint8_t)a;
            op++;
            if (bitd_reload_u(b, in) == kOverflow) {
                a = sym(s1);
                if (lane == 0) W.w[op] = (uint8_t)a;
                op++;
                break;
            }
        }
        osize = op;
    }
    __builtin_amdgcn_wave_barrier();
    // weight statistics (ballots over 64-symbol chunks)
    uint32_t rank[13];
#pragma unroll
    for (int k = 0; k < 13; k++) rank[k] = 0;
    uint32_t total = 0;
    bool bad = false;
    for (uint32_t s0 = 0; s0 < osize; s0 += kWave) {
        const uint32_t s = s0 + lane;
        const uint32_t wv = s < osize ? W.w[s] : 0u;
        if (__ballot(s < osize && wv >= 12u)) bad = true;
        const uint32_t part = s < osize && wv < 12u ? (1u << wv) >> 1 : 0u;
        total += rdlane((uint32_t)wave_incl_sum((int32_t)part), kWave - 1);
#pragma unroll
        for (uint32_t k = 1; k < 12; k++) rank[k] += (uint32_t)__builtin_popcountll(__ballot(s < osize && wv == k));
    }
    if (bad) return kErr;
    if (total == 0) return kErr;
    tlog = highbit(total) + 1u;
    if (tlog > 12u) return kErr;
    {
        const uint32_t rest = (1u << tlog) - total;
        const uint32_t lastw = highbit(rest) + 1u;
        if ((1u << highbit(rest)) != rest) return kErr;
        if (lane == 0) W.w[osize] = (uint8_t)lastw;
#pragma unroll
        for (uint32_t k = 1; k < 13; k++)
            if (k == lastw) rank[k]++;
    }
    if (rank[1] < 2 || (rank[1] & 1u)) return kErr;
    __builtin_amdgcn_wave_barrier();
    const uint32_t nsym = osize + 1u;
    nsym_out = nsym;
    huf_fill(W.w, nsym, tlog, rank, W.huf, W.hpair, lane);
    __builtin_amdgcn_wave_barrier();
    return isize + 1;
}

// Decodes the Huffman stream(s) of a literals section: 1 or 4 streams, lanes 0-3
// each take one.  Literal k is written to out[k].  Returns false on error.
// kGlobal: out is the pass-1 literal buffer in HBM; each stream's lane gathers
// its symbols into 8-byte words and stores whole aligned words (bytes only at the
// two ends of its segment).
template <bool kGlobal>
__device__ bool huf_decode(const Work &W, int32_t cs, int32_t n, bool single, uint32_t lsize, uint32_t tlog,
                           uint8_t *out, uint32_t lane) {
    const uint8_t *in = W.in;
    int32_t s_start = 0, s_len = 0;
    uint32_t o0 = 0, cnt = 0;
    bool ok = true;
    if (single) {
        s_start = cs;
        s_len = n;
        cnt = lane == 0 ? lsize : 0u;
    } else {
        if (n < 10) return false;
        const int32_t l1 = (int32_t)lds_ld16(in + cs), l2 = (int32_t)lds_ld16(in + cs + 2),
                      l3 = (int32_t)lds_ld16(in + cs + 4);
        const int32_t l4 = n - (l1 + l2 + l3 + 6);
        if (l4 < 0 || l4 > n) return false;
        const uint32_t seg = (lsize + 3u) / 4u;
        const uint32_t n4 = lsize > 3u * seg ? lsize - 3u * seg : 0u;
        const int32_t st[4] = {cs + 6, cs + 6 + l1, cs + 6 + l1 + l2, cs + 6 + l1 + l2 + l3};
        const int32_t ln[4] = {l1, l2, l3, l4};
        if (lane < 4) {
            s_start = st[lane];
            s_len = ln[lane];
            o0 = seg * lane;
            cnt = lane < 3 ? seg : n4;
        }
    }
    BitD b;
    if (lane < (single ? 1u : 4u)) ok = bitd_init(b, in, s_start, s_len);
    if (__ballot(lane < (single ? 1u : 4u) && !ok)) return false;
    const uint32_t act_n = single ? 1u : 4u;
    const uint32_t mc = rdlane(cnt, 0);   // stream 1 holds the most symbols
    const uint32_t hsh = tlog == 12u ? 1u : 0u;   // the table is indexed by at most 11 bits
    uint64_t acc = 0;
    uint32_t lo = (uint32_t)((uintptr_t)(out + o0) & 7u);   // first valid byte of the current word
    for (uint32_t i = 0; i < mc; i++) {
        if (lane < act_n && i < cnt) {
            if (b.used > 52u) bitd_reload(b, in);
            const uint32_t v = (uint32_t)bitd_look_fast(b, tlog);
            // branch-free: both reads go out together; hpair only matters for a
            // 12-bit code (tableLog 12), the mask keeps the other reads in bounds
            const uint32_t e0 = W.huf[v >> hsh], ep = W.hpair[v & 255u];
            const uint32_t e = (e0 >> 8) == 12u ? (ep | (12u << 8)) : e0;
            b.used += e >> 8;
            if (!kGlobal) {
                out[o0 + i] = (uint8_t)e;
            } else {
                uint8_t *at = out + o0 + i;
                const uint32_t k = (uint32_t)((uintptr_t)at & 7u);
                acc |= (uint64_t)(e & 255u) << (8u * k);
                if (k == 7u || i + 1u == cnt) {
                    uint8_t *word = at - k;
                    if (lo == 0u && k == 7u) {
                        *(uint64_t *)word = acc;
                    } else {
                        for (uint32_t j = lo; j <= k; j++) word[j] = (uint8_t)(acc >> (8u * j));
                    }
                    acc = 0;
                    lo = 0;
                }
            }
        }
    }
    // exact end of every stream (BIT_endOfDStream); a reload settles ptr/used
    bool end_ok = true;
    if (lane < act_n) {
        if (b.used <= 64u) bitd_reload(b, in);
        end_ok = b.ptr == b.start && b.used == 64u;
    }
    return __ballot(lane < act_n && !end_ok) == 0;
}

// ------------------------------------------------------------ sequence execution

// whole-wave forward copy out[d, d+ml) <- out[d-off, ...) (overlap semantics)
__device__ __forceinline__ void wave_match(uint8_t *out, int32_t d, int32_t off, int32_t ml, uint32_t lane) {
    const int32_t s = d - off;
    if (off >= (int32_t)kWave || off >= ml) {
        for (int32_t i = (int32_t)lane; i < ml; i += (int32_t)kWave) out[d + i] = out[s + i];
    } else {
        for (int32_t i = (int32_t)lane; i < ml; i += (int32_t)kWave) out[d + i] = out[s + (int32_t)mod_small((uint32_t)i, (uint32_t)off)];
    }
}

// Applies n <= 64 decoded sequences (lane j: ll, ml, off) in order.  op: output
// position (frame offset); lp: literal cursor (literal k lives at lit[k]).
// Returns false on a reference exec error.
__device__ bool exec_batch(uint8_t *out, const uint8_t *lit, bool lit_in_window, int32_t lit_win_base, uint32_t n,
                           uint32_t ll, uint32_t ml, uint32_t off, int32_t &op, int32_t &lp, int32_t lsize,
                           int32_t cap, uint32_t lane) {
    const bool act = lane < n;
    const int32_t olen = act ? (int32_t)(ll + ml) : 0;
    const int32_t llen = act ? (int32_t)ll : 0;
    const int32_t oi = wave_incl_sum(olen), li = wave_incl_sum(llen);
    const int32_t o = op + oi - olen;     // this sequence's output position
    const int32_t l0 = lp + li - llen;    // its first literal
    const int32_t d = o + (int32_t)ll;    // match destination
    // ZSTD_execSequence checks (zstd_decompress.c:940-954)
    const bool bad = act && (o + olen > cap || l0 + llen > lsize || (int32_t)off > d);
    if (__ballot(bad)) return false;
    const int32_t out_end = op + (int32_t)rdlane((uint32_t)oi, kWave - 1);
    const int32_t lit_end = lp + (int32_t)rdlane((uint32_t)li, kWave - 1);
    // parallel prefix: sequences whose output ends at or below the first unread literal
    uint32_t npar = n;
    if (lit_in_window) {
        const int32_t first_buf = lit_win_base + lp;
        const uint64_t unsafe = __ballot(act && o + olen > first_buf);
        npar = unsafe ? (uint32_t)__builtin_ctzll(unsafe) : n;
    }
    // ---- literals of the parallel prefix
    const bool pl = lane < npar;
    const bool short_lit = pl && ll <= 32u;
    if (short_lit)
        for (int32_t i = 0; i < (int32_t)ll; i += 4) lds_st32(out + o + i, lds_ld32(lit + l0 + i));
    uint64_t longl = __ballot(pl && !short_lit);
    while (longl) {
        const uint32_t k = (uint32_t)__builtin_ctzll(longl);
        longl &= longl - 1;
        const int32_t kl = (int32_t)rdlane(ll, k), ko = (int32_t)rdlane((uint32_t)o, k), ks = (int32_t)rdlane((uint32_t)l0, k);
        for (int32_t i = (int32_t)lane; i < kl; i += (int32_t)kWave) out[ko + i] = lit[ks + i];
    }
    // ---- matches of the parallel prefix, frontier order
    const int32_t src_end = d - (int32_t)off + min((int32_t)ml, (int32_t)off);
    uint64_t pending = __ballot(pl && ml > 0);
    const uint64_t shortm = __ballot(pl && ml <= 64u);
    const uint32_t grp = lane >> 4, gl = lane & 15u;
    while (pending) {
        const uint32_t f = (uint32_t)__builtin_ctzll(pending);
        const int32_t F = (int32_t)rdlane((uint32_t)d, f);
        if (!((shortm >> f) & 1ull)) {
            wave_match(out, F, (int32_t)rdlane(off, f), (int32_t)rdlane(ml, f), lane);
            pending &= ~(1ull << f);
            continue;
        }
        uint64_t ready = pending & shortm & __ballot(src_end <= F);
        int32_t gd = 0, go = 1, gm = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            if (ready) {
                const uint32_t r = (uint32_t)__builtin_ctzll(ready);
                ready &= ready - 1;
                pending &= ~(1ull << r);
                const int32_t rd = (int32_t)rdlane((uint32_t)d, r), ro = (int32_t)rdlane(off, r), rm = (int32_t)rdlane(ml, r);
                if (grp == k) { gd = rd; go = ro; gm = rm; }
            }
        }
        const int32_t gs = gd - go;
        for (int32_t i = (int32_t)gl; i < gm; i += 16) {
            const int32_t si = (go >= 16 || go >= gm) ? i : (int32_t)mod_small((uint32_t)i, (uint32_t)go);
            out[gd + i] = out[gs + si];
        }
    }
    // ---- the rest in stream order, one sequence at a time
    for (uint32_t j = npar; j < n; j++) {
        const int32_t jo = (int32_t)rdlane((uint32_t)o, j), jl = (int32_t)rdlane(ll, j), js = (int32_t)rdlane((uint32_t)l0, j);
        // chunked so that a chunk's reads precede its writes (output position <= buffer position)
        for (int32_t c = 0; c < jl; c += (int32_t)kWave) {
            const int32_t i = c + (int32_t)lane;
            const uint8_t v = i < jl ? lit[js + i] : 0;
            __builtin_amdgcn_wave_barrier();
            if (i < jl) out[jo + i] = v;
            __builtin_amdgcn_wave_barrier();
        }
        wave_match(out, jo + jl, (int32_t)rdlane(off, j), (int32_t)rdlane(ml, j), lane);
        __builtin_amdgcn_wave_barrier();
    }
    op = out_end;
    lp = lit_end;
    return true;
}

// ------------------------------------------------------------ XXH64 of out[0, n) (checksum frames)
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
constexpr uint64_t kP1 = 11400714785074694791ull, kP2 = 14029467366897019727ull, kP3 = 1609587929392839161ull,
                   kP4 = 9650029242287828579ull, kP5 = 2870177450012600261ull;
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t v) { return rotl64(acc + v * kP2, 31) * kP1; }

__device__ uint32_t xxh64_lds(const uint8_t *p, uint32_t len, uint32_t lane) {
    uint64_t h;
    uint32_t i = 0;
    if (len >= 32) {
        // lanes 0-3 run the four accumulators over all stripes
        uint64_t v = lane == 0 ? kP1 + kP2 : lane == 1 ? kP2 : lane == 2 ? 0ull : (uint64_t)0 - kP1;
        const uint32_t nst = len / 32;
        if (lane < 4)
            for (uint32_t s = 0; s < nst; s++) v = xround(v, ld64(p + s * 32 + lane * 8));
        const uint64_t v1 = ((uint64_t)rdlane((uint32_t)(v >> 32), 0) << 32) | rdlane((uint32_t)v, 0);
        const uint64_t v2 = ((uint64_t)rdlane((uint32_t)(v >> 32), 1) << 32) | rdlane((uint32_t)v, 1);
        const uint64_t v3 = ((uint64_t)rdlane((uint32_t)(v >> 32), 2) << 32) | rdlane((uint32_t)v, 2);
        const uint64_t v4 = ((uint64_t)rdlane((uint32_t)(v >> 32), 3) << 32) | rdlane((uint32_t)v, 3);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = (h ^ xround(0, v1)) * kP1 + kP4;
        h = (h ^ xround(0, v2)) * kP1 + kP4;
        h = (h ^ xround(0, v3)) * kP1 + kP4;
        h = (h ^ xround(0, v4)) * kP1 + kP4;
        i = nst * 32;
    } else {
        h = kP5;
    }
    h += (uint64_t)len;
    for (; i + 8 <= len; i += 8) h = rotl64(h ^ xround(0, ld64(p + i)), 27) * kP1 + kP4;
    if (i + 4 <= len) {
        h ^= (uint64_t)lds_ld32(p + i) * kP1;
        h = rotl64(h, 23) * kP2 + kP3;
        i += 4;
    }
    for (; i < len; i++) h = rotl64(h ^ (uint64_t)p[i] * kP5, 11) * kP1;
    h ^= h >> 33;
    h *= kP2;
    h ^= h >> 29;
    h *= kP3;
    h ^= h >> 32;
    return (uint32_t)h;
}

// ------------------------------------------------------------ block / frame
struct SeqTables {
    uint32_t ll_log, of_log, ml_log;
    bool fse_entropy, lit_entropy;
    uint32_t huf_log;
    uint32_t rep0, rep1, rep2;
    // pass 1 with sequence jobs (the FSE chains run lane-per-page in zstd_seq_kernel):
    // the tables in force (byte offsets into the page's table area; kTabDefault:
    // none yet), jobs written, table bytes used
    bool jobs;
    uint32_t ll_off, of_off, ml_off, njobs, tb_used;
    // pass 1 with literal jobs (the Huffman streams run lane-per-stream in zstd_lit_kernel):
    // the published Huffman table in force (offset in the page's Huffman region, or -1 when
    // the table in W.huf was not published), tables published, literal jobs written
    int32_t huf_pub;
    uint32_t nhuf, nlj;
    uint32_t huf_nsym;   // symbols (weights) of the Huffman table in force
};

// ZSTD_buildSeqTable (zstd_decompress.c:693-724).  Returns bytes read or < 0.
__device__ int32_t seq_table(const Work &W, uint32_t *cells, uint32_t &log, uint32_t type, uint32_t max,
                             uint32_t max_log, int32_t ip, int32_t n, const DTab &def, uint32_t def_log,
                             bool flag_repeat, uint32_t lane) {
    // an RLE byte, or a normalized-count header: its reader stops after at most ~80 bytes (53
    // symbols of <= 10 bits and the repeat flags, FSE_readNCount)
    if (type == 1 || type == 2) stage_range(W, ip, ip + min(n, 256), lane);
    if (type == 1) {   // set_rle
        if (n < 1) return kErr;
        const uint32_t sym = u8u(W.in, ip);
        if (sym > max) return kErr;
        if (lane == 0) cells[0] = cell(0, sym, 0);
        log = 0;
        return 1;
    }
    if (type == 0) {   // set_basic
        if (lane < (1u << def_log)) cells[lane] = def.cell[lane];
        log = def_log;
        return 0;
    }
    if (type == 3) return flag_repeat ? 0 : kErr;
    uint32_t tl, mx = max;
    const int32_t hs = read_ncount(W.in, ip, n, W.norm, mx, tl);
    if (hs < 0) return kErr;
    if (tl > max_log) return kErr;
    build_dtable(cells, W.norm, mx, tl, W.next, lane);   // its result is ignored by the reference (:720)
    log = tl;
    return hs;
}

// ------------------------------------------------------------ two-pass decode
// The fused kernel holds window + staged frame + tables in LDS (~51 KiB for a
// 32 KiB page: 3 waves per CU), and the serial FSE chain -- two thirds of its
// time -- runs at that residency.  The split decode runs the same walk twice:
//
//   pass 1 (entropy, decode_frame<true>): frame and block structure, Huffman
//     literals and the FSE sequence chain.  LDS = staged frame + tables, no
//     window.  Output per page, in HBM: a stream of entries (three u32 planes)
//     -- one command per block, each compressed block's command followed by its
//     sequences (litLength, matchLength, offset after repeat resolution) -- and
//     a literal buffer (raw blocks and literal sections, decoded).
//   pass 2 (execution, exec_page): LDS = the window only.  Replays the entries:
//     raw / RLE blocks, literal placement at the window tail, exec_batch.
//
// Every check the reference makes stays in one of the two passes; a page fails
// when either does (callers compare success/failure, buffer.c only tests
// ZSTD_isError).  Pass 1 also fails a page early where the reference would fail
// later in any case: a block whose literals or whose output (literals + match
// lengths) exceed the remaining capacity.  The entry and literal capacities
// below are bounds no successful page reaches: every block has a 3-byte header,
// every executed sequence writes >= 3 bytes, literals are part of the output.
enum : uint32_t { kCmdRaw = 0, kCmdRle = 1, kCmdBlk = 2, kCmdEnd = 3 };

struct Ent {
    uint32_t *ll, *ml, *of;   // entry planes
    uint8_t *lit;             // literal buffer
    uint32_t ecap, lcap;      // entries, literal bytes
    uint32_t *jobs;           // [0] = job count, then kJobWords words per job
    uint32_t *tabs;           // FSE cells of the tables the jobs use
    bool fused;               // zstd_seqexec_kernel's layout: commands only, no sequence entries
    int32_t over;             // pass 1's result when the planes are full (fused: kRetryFused)
    bool defer_lit;           // Huffman literal streams left to zstd_lit_kernel (fused layout)
    uint32_t *litjobs;        // [0] = literal job count, then kLitJobWords words per job
    uint16_t *hufs;           // published Huffman decoding tables, kHufCells entries each
};
// Sequence jobs: one per compressed block with sequences, decoded by
// zstd_seq_kernel one page per lane -- the chain is serial within a page, so the
// parallelism comes from the pages.  A page that needs more jobs or table space
// than its area holds is redone with the chains inline (decode_frame, jobs off).
constexpr uint32_t kJobWords = 8;   // start, length, nbSeq, first entry, ll/of/ml table, logs
constexpr uint32_t kMaxJobs = 31;
constexpr uint32_t kJobBytes = 4u * (4u + kMaxJobs * kJobWords);   // 1008
constexpr uint32_t kTabBytes = 12u * 1024u;                       // two full LL+OF+ML sets and more
// Literal jobs (round 3, fused layout): one per Huffman-compressed literals section whose
// table has at most kHufCells entries (tableLog <= 11), decoded by zstd_lit_kernel one stream
// per lane; the table is published to the area (at most kMaxHuf per page).  Pages with more
// sections or tables decode the rest in pass 1 as before.
constexpr uint32_t kLitJobWords = 8;   // streams' start and length, lsize, literal-buffer position, table, log | single << 8
constexpr uint32_t kMaxLitJobs = 31;
constexpr uint32_t kLitJobBytes = 4u * (4u + kMaxLitJobs * kLitJobWords);   // 1008
constexpr uint32_t kHufCells = 2048;
constexpr uint32_t kMaxHuf = 4;
constexpr uint32_t kAreaJobs = 13312u;                            // seq jobs + FSE tables
constexpr uint32_t kAreaBytes = kAreaJobs + kLitJobBytes + kMaxHuf * kHufCells * 2u + 16u;   // 256-aligned: 30720
constexpr uint32_t kTabDefault = 0xFFFFFFFFu;
constexpr int32_t kRetryInline = -1000;
// fused layout: a page with more than kFusedCmds block commands, or whose jobs do not fit
// (kRetryInline), is decoded by the fused one-wave kernel after pass 2 (kRetryFused)
constexpr int32_t kRetryFused = -1001;
constexpr uint32_t kFusedCmds = 64;
__host__ __device__ inline uint32_t ent_cap(uint32_t in_cap, uint32_t out_cap, bool fused) {
    if (fused) return kFusedCmds;
    return ((in_cap / 3u + out_cap / 3u + 72u) + 15u) & ~15u;   // multiple of 16: planes and literals 64-aligned
}
__host__ __device__ inline uint32_t lit_cap(uint32_t out_cap) { return out_cap + 16u * (out_cap / 64u + 2u) + 64u; }
__host__ __device__ inline size_t ent_page_bytes(uint32_t in_cap, uint32_t out_cap, bool fused) {
    return kAreaBytes + (((size_t)ent_cap(in_cap, out_cap, fused) * 12u + lit_cap(out_cap) + 255u) & ~(size_t)255u);
}
__device__ inline Ent ent_of(uint8_t *area, uint32_t in_cap, uint32_t out_cap, bool fused) {
    Ent E;
    E.jobs = (uint32_t *)area;
    E.tabs = (uint32_t *)(area + kJobBytes);
    E.litjobs = (uint32_t *)(area + kAreaJobs);
    E.hufs = (uint16_t *)(area + kAreaJobs + kLitJobBytes);
    E.defer_lit = false;
    E.fused = fused;
    E.over = fused ? kRetryFused : kErr;
    uint8_t *base = area + kAreaBytes;
    E.ecap = ent_cap(in_cap, out_cap, fused);
    E.lcap = lit_cap(out_cap);
    E.ll = (uint32_t *)base;
    E.ml = E.ll + E.ecap;
    E.of = E.ml + E.ecap;
    E.lit = base + (size_t)E.ecap * 12u;
    return E;
}
__device__ __forceinline__ void put_cmd(const Ent &E, uint32_t at, uint32_t a, uint32_t b, uint32_t c, uint32_t lane) {
    if (lane == 0) {
        E.ll[at] = a;
        E.ml[at] = b;
        E.of[at] = c;
    }
}
// Literal-buffer position for n bytes that pass 2 copies to LDS offset `to`: runs
// of 64+ bytes keep to's 16-byte phase, so the copy moves 16-byte vectors.
__device__ __forceinline__ uint32_t lit_place(uint32_t litc, uint32_t to, uint32_t n) {
    return n >= 64u ? litc + ((to - litc) & 15u) : litc;
}
// in[src, src+n) (LDS) -> the literal buffer at `at`
__device__ __forceinline__ void lds_to_lit(uint8_t *dst, const uint8_t *in, int32_t src, int32_t n, uint32_t lane) {
    for (int32_t i = (int32_t)lane; i < n; i += (int32_t)kWave) dst[i] = in[src + i];
}

// Copies a table just built in LDS to the page's table area (jobs mode).  mode:
// the block's compression mode for it (set_repeat keeps the one in force).
// Returns false when the area is full.
__device__ bool publish_table(const Ent &E, SeqTables &T, const uint32_t *cells, uint32_t mode, uint32_t log,
                              uint32_t &off, uint32_t lane) {
    if (mode == 3u) return true;
    // set_basic: seq_table left the predefined cells in LDS like any other table
    const uint32_t n = mode == 1u ? 1u : 1u << log;
    if (T.tb_used + n * 4u > kTabBytes) return false;
    uint32_t *g = E.tabs + T.tb_used / 4u;
    for (uint32_t i = lane; i < n; i += kWave) g[i] = cells[i];
    off = T.tb_used;
    T.tb_used += n * 4u;
    return true;
}

// One compressed block at in[ip, ip+n); output from op (frame offset) up to cap.
// Returns bytes written or < 0.  kSplit: pass 1 (entries and literals to E;
// ecur / litc are the page's entry and literal cursors).
template <bool kSplit>
__device__ int32_t decode_block(const Work &W, SeqTables &T, const Ent &E, uint32_t &ecur, uint32_t &litc,
                                int32_t ip, int32_t n, int32_t op, int32_t cap, uint32_t lane) {
    const uint8_t *in = W.in;
    SPROF_DECL
    ip = ru(ip);
    n = ru(n);
    op = ru(op);
    cap = ru(cap);
    if (n >= (int32_t)kBlockMax) return kErr;
    // ---- literals section (ZSTD_decodeLiteralsBlock)
    if (n < 3) return kErr;
    stage_range(W, ip, ip + 5, lane);   // the section header (<= 5 bytes)
    const uint32_t b0 = u8u(in, ip);
    const uint32_t ltype = b0 & 3u, lhl = (b0 >> 2) & 3u;
    const uint8_t *lit;
    bool lit_in_window;
    int32_t lsize, lcons, lit_win_base = 0;
    uint32_t lat = 0;   // kSplit: literal-buffer position of this block's literals
    if (ltype >= 2u) {
        if (ltype == 3u && !T.lit_entropy) return kErr;
        if (n < 5) return kErr;
        const uint32_t lhc = u32u(in, ip);
        int32_t lh, csize;
        bool single = false;
        if (lhl <= 1u) { single = lhl == 0; lh = 3; lsize = (int32_t)((lhc >> 4) & 0x3FFu); csize = (int32_t)((lhc >> 14) & 0x3FFu); }
        else if (lhl == 2u) { lh = 4; lsize = (int32_t)((lhc >> 4) & 0x3FFFu); csize = (int32_t)(lhc >> 18); }
        else { lh = 5; lsize = (int32_t)((lhc >> 4) & 0x3FFFFu); csize = (int32_t)((lhc >> 22) + (u8u(in, ip + 4) << 10)); }
        if (lsize > (int32_t)kBlockMax) return kErr;
        if (csize + lh > n) return kErr;
        // the block's output is lsize + sum(ml) bytes: a section that cannot fit the
        // remaining capacity makes the reference fail later in any case
        if (op + lsize > cap) return kErrDst;
        uint8_t *dst = W.win + (cap - lsize);
        if constexpr (kSplit) {
            lat = lit_place(litc, (uint32_t)(cap - lsize), (uint32_t)lsize);
            if (lat + (uint32_t)lsize > E.lcap) return kErr;
            dst = E.lit + lat;
        }
        const int32_t cs = ip + lh;
        bool ok;
        // defer: the streams go to zstd_lit_kernel when the table is (or can be) published
        auto defer = [&](int32_t at, int32_t len) -> bool {
            if (!(kSplit && E.defer_lit && T.huf_pub >= 0 && T.nlj < kMaxLitJobs)) return false;
            if (lane == 0) {
                uint32_t *J = E.litjobs + 4u + T.nlj * kLitJobWords;
                J[0] = (uint32_t)at;
                J[1] = (uint32_t)len;
                J[2] = (uint32_t)lsize;
                J[3] = lat;
                J[4] = (uint32_t)T.huf_pub;
                J[5] = T.huf_log | ((single ? 1u : 0u) << 8) | (T.huf_nsym << 16);
            }
            T.nlj++;
            return true;
        };
        // after a new table: publish it if it fits a slot -- its symbols' weights (round 6: at most 256
        // bytes instead of the 2^tl-entry decoding table, which zstd_lit_kernel rebuilds in LDS)
        auto publish = [&](uint32_t tl, uint32_t nsym) {
            T.huf_pub = -1;
            T.huf_nsym = nsym;
            if (!(kSplit && E.defer_lit) || tl > 11u || T.nhuf >= kMaxHuf) return;
            uint8_t *g = (uint8_t *)(E.hufs + T.nhuf * kHufCells);
            for (uint32_t i = lane; i < nsym; i += kWave) g[i] = W.w[i];
            T.huf_pub = (int32_t)(T.nhuf * kHufCells);
            T.nhuf++;
        };
        // streams decoded here are staged first; deferred ones never are (lazy staging).  One
        // decode site for the three cases: the stream's range and table log
        int32_t hat = cs, hlen = csize;
        uint32_t htl = T.huf_log;
        bool here = false;
        if (ltype == 3u) {
            ok = true;
            here = !defer(cs, csize);
        } else {
            ok = single || (lsize != 0 && csize < lsize && csize > 1);
            if (ok) {
                uint32_t tl, nsym = 0;
                stage_range(W, cs, cs + min(csize, 144), lane);   // the table description: <= 1 + 128 bytes
                const int32_t hs = huf_read_table(W, cs, csize, tl, nsym, lane);
                SPROF_MARK(7);
                ok = hs >= 0 && hs < csize;
                if (ok) {
                    T.huf_log = tl;
                    publish(tl, nsym);
                    hat = cs + hs;
                    hlen = csize - hs;
                    htl = tl;
                    here = !defer(hat, hlen);
                }
            }
        }
        if (ok && here) {
            stage_range(W, hat, hat + hlen, lane);
            ok = huf_decode<kSplit>(W, hat, hlen, single, (uint32_t)lsize, htl, dst, lane);
        }
        if (!ok) return kErr;
        T.lit_entropy = true;
        lit = dst;
        lit_in_window = true;
        lit_win_base = cap - lsize;
        lcons = lh + csize;
    } else {
        int32_t lh;
        if (lhl == 1u) { lh = 2; lsize = (int32_t)(u16u(in, ip) >> 4); }
        else if (lhl == 3u) { lh = 3; lsize = (int32_t)((u32u(in, ip) & 0xFFFFFFu) >> 4); }
        else { lh = 1; lsize = (int32_t)(b0 >> 3); }
        if (ltype == 0u) {   // raw
            if (lh + lsize > n) return kErr;
            stage_range(W, ip + lh, ip + lh + lsize, lane);
            lit = in + ip + lh;
            lit_in_window = false;
            lcons = lh + lsize;
            if constexpr (kSplit) {
                // pass 2 places every literal section at the window tail; a section
                // that cannot fit makes the reference fail later in any case
                if (op + lsize > cap) return kErrDst;
                lat = lit_place(litc, (uint32_t)(cap - lsize), (uint32_t)lsize);
                if (lat + (uint32_t)lsize > E.lcap) return kErr;
                lds_to_lit(E.lit + lat, in, ip + lh, lsize, lane);
            }
        } else {             // RLE
            if (lhl == 3u && n < 4) return kErr;
            if (lsize > (int32_t)kBlockMax) return kErr;
            if (op + lsize > cap) return kErrDst;
            uint8_t *dst = W.win + (cap - lsize);
            if constexpr (kSplit) {
                lat = lit_place(litc, (uint32_t)(cap - lsize), (uint32_t)lsize);
                if (lat + (uint32_t)lsize > E.lcap) return kErr;
                dst = E.lit + lat;
            }
            stage_range(W, ip + lh, ip + lh + 1, lane);
            const uint8_t v = in[ip + lh];
            for (int32_t i = (int32_t)lane; i < lsize; i += (int32_t)kWave) dst[i] = v;
            lit = dst;
            lit_in_window = true;
            lit_win_base = cap - lsize;
            lcons = lh + 1;
        }
    }
    __builtin_amdgcn_wave_barrier();
    SPROF_MARK(2);
    // ---- sequences section (ZSTD_decodeSeqHeaders)
    int32_t sp = ip + lcons;
    const int32_t send = ip + n;
    if (send - sp < 1) return kErr;
    stage_range(W, sp, sp + 4, lane);   // nbSeq (<= 3 bytes) and the modes byte
    int32_t nbseq = (int32_t)u8u(in, sp++);
    int32_t op0 = op, lp = 0;
    uint32_t cmd_at = 0, nseq_all = 0;
    int32_t mlsum = 0;   // kSplit: sum of match lengths (the block's output is lsize + mlsum)
    if constexpr (kSplit) {
        litc = lat + (uint32_t)lsize;
        if (ecur >= E.ecap) return E.over;
        cmd_at = ecur++;
    }
    if (nbseq) {
        if (nbseq > 0x7F) {
            if (nbseq == 0xFF) {
                if (sp + 2 > send) return kErr;
                nbseq = (int32_t)u16u(in, sp) + 0x7F00;
                sp += 2;
            } else {
                if (sp >= send) return kErr;
                nbseq = ((nbseq - 0x80) << 8) + (int32_t)u8u(in, sp++);
            }
        }
        if (sp + 4 > send) return kErr;
        nseq_all = (uint32_t)nbseq;
        const uint32_t modes = u8u(in, sp++);
        int32_t r = seq_table(W, W.ll, T.ll_log, modes >> 6, 35, 9, sp, send - sp, c_ll_def, 6, T.fse_entropy, lane);
        if (r < 0) return kErr;
        sp += r;
        r = seq_table(W, W.of, T.of_log, (modes >> 4) & 3u, 28, 8, sp, send - sp, c_of_def, 5, T.fse_entropy, lane);
        if (r < 0) return kErr;
        sp += r;
        r = seq_table(W, W.ml, T.ml_log, (modes >> 2) & 3u, 52, 9, sp, send - sp, c_ml_def, 6, T.fse_entropy, lane);
        if (r < 0) return kErr;
        sp += r;
        __builtin_amdgcn_wave_barrier();
        SPROF_MARK(3);
        if constexpr (kSplit) {
            if (T.jobs) {
                // hand the chain to zstd_seq_kernel; the block's output size is
                // checked in pass 2 (K1 only counts the literals toward op)
                if (!publish_table(E, T, W.ll, modes >> 6, T.ll_log, T.ll_off, lane) ||
                    !publish_table(E, T, W.of, (modes >> 4) & 3u, T.of_log, T.of_off, lane) ||
                    !publish_table(E, T, W.ml, (modes >> 2) & 3u, T.ml_log, T.ml_off, lane) || T.njobs >= kMaxJobs)
                    return kRetryInline;
                if (!E.fused && (uint32_t)nbseq > E.ecap - ecur) return kErr;
                if (lane == 0) {
                    uint32_t *J = E.jobs + 4u + T.njobs * kJobWords;
                    J[0] = (uint32_t)sp;
                    J[1] = (uint32_t)(send - sp);
                    J[2] = (uint32_t)nbseq;
                    J[3] = ecur;
                    J[4] = T.ll_off;
                    J[5] = T.of_off;
                    J[6] = T.ml_off;
                    J[7] = T.ll_log | (T.of_log << 8) | (T.ml_log << 16);
                }
                T.njobs++;
                if (!E.fused) ecur += (uint32_t)nbseq;   // entry slots for zstd_seq_kernel
                T.fse_entropy = true;
                put_cmd(E, cmd_at, kCmdBlk | (lat << 2), (uint32_t)lsize, nseq_all, lane);
                return lsize;
            }
        }
        // ---- sequence loop (ZSTD_decompressSequences)
        T.fse_entropy = true;
        stage_range(W, sp, send, lane);
        BitD b;
        if (!bitd_init_u(b, in, sp, send - sp)) return kErr;
        uint32_t sll = bitd_read(b, T.ll_log);
        bitd_reload_u(b, in);
        uint32_t sof = bitd_read(b, T.of_log);
        bitd_reload_u(b, in);
        uint32_t sml = bitd_read(b, T.ml_log);
        bitd_reload_u(b, in);
        uint32_t rep0 = T.rep0, rep1 = T.rep1, rep2 = T.rep2;
        bool more = true;
        while (more) {
            // decode up to 64 sequences into lanes
            uint32_t vll = 0, vml = 0, voff = 0, k = 0;
            for (; k < kWave; k++) {
                if (!((bitd_reload_u(b, in) <= kCompleted) && nbseq)) { more = false; break; }
                nbseq--;
                const uint32_t cl = rfl(W.ll[sll]), cm = rfl(W.ml[sml]), co = rfl(W.of[sof]);
                const uint32_t llc = cell_sym(cl), mlc = cell_sym(cm), ofc = cell_sym(co);
                uint32_t offv;
                if (!ofc) offv = 0;
                else offv = of_base(ofc) + bitd_read_fast(b, ofc);
                if (ofc <= 1u) {
                    offv += llc == 0;
                    if (offv) {
                        uint32_t t = offv == 3u ? rep0 - 1u : (offv == 1u ? rep1 : rep2);
                        t += t == 0;
                        if (offv != 1u) rep2 = rep1;
                        rep1 = rep0;
                        rep0 = offv = t;
                    } else {
                        offv = rep0;
                    }
                } else {
                    rep2 = rep1;
                    rep1 = rep0;
                    rep0 = offv;
                }
                uint32_t mlbase, mlb, llbase, llb;
                ml_code_s(mlc, mlbase, mlb);
                ll_code_s(llc, llbase, llb);
                const uint32_t mlv = mlbase + (mlc > 31u ? bitd_read_fast(b, mlb) : 0u);
                const uint32_t llv = llbase + (llc > 15u ? bitd_read_fast(b, llb) : 0u);
                if (llb + mlb + ofc > 31u) bitd_reload_u(b, in);
                sll = cell_state(cl) + bitd_read(b, cell_nb(cl));
                sml = cell_state(cm) + bitd_read(b, cell_nb(cm));
                sof = cell_state(co) + bitd_read(b, cell_nb(co));

                if (lane == k) {
                    vll = llv;
                    vml = mlv;
                    voff = offv;
                }
            }
            SPROF_MARK(4);
            SPROF_ADD(9, k);
            if (k == 0) break;
            if constexpr (kSplit) {
                if (ecur + k > E.ecap) return E.over;
                if (lane < k) {
                    E.ll[ecur + lane] = vll;
                    E.ml[ecur + lane] = vml;
                    E.of[ecur + lane] = voff;
                }
                ecur += k;
                // match lengths are < 2^18: a batch sums below 2^24
                mlsum += (int32_t)rdlane((uint32_t)wave_incl_sum(lane < k ? (int32_t)vml : 0), kWave - 1);
                if (mlsum > cap) return kErrDst;
            } else {
#if TYCHE_ZABLATE & 1
                // timing-only: skip execution (output wrong), keep the positions moving
                op += (int32_t)rdlane((uint32_t)wave_incl_sum(lane < k ? (int32_t)(vll + vml) : 0), kWave - 1);
                lp += (int32_t)rdlane((uint32_t)wave_incl_sum(lane < k ? (int32_t)vll : 0), kWave - 1);
#else
                if (!exec_batch(W.win, lit, lit_in_window, lit_win_base, k, vll, vml, voff, op, lp, lsize, cap, lane))
                    return kErr;
#endif
            }
            SPROF_MARK(5);
        }
        if (nbseq) return kErr;
        T.rep0 = rep0;
        T.rep1 = rep1;
        T.rep2 = rep2;
    }
    if constexpr (kSplit) {
        if (op + lsize + mlsum > cap) return kErrDst;
        put_cmd(E, cmd_at, kCmdBlk | (lat << 2), (uint32_t)lsize, nseq_all, lane);
        return lsize + mlsum;
    }
    // ---- last literals
    const int32_t last = lsize - lp;
    if (last > cap - op) return kErrDst;
    for (int32_t c = 0; c < last; c += (int32_t)kWave) {
        const int32_t i = c + (int32_t)lane;
        const uint8_t v = i < last ? lit[lp + i] : 0;
        __builtin_amdgcn_wave_barrier();
        if (i < last) W.win[op + i] = v;
        __builtin_amdgcn_wave_barrier();
    }
    op += last;
    SPROF_MARK(6);
    return op - op0;
}

// ZSTD_decompressFrame (zstd_decompress.c:1369-1436) for the frame staged at
// W.in[0, L).  Returns the decoded size or < 0.
// kSplit: pass 1 -- returns 0 or < 0 and leaves the page's entries in E.
template <bool kSplit>
__device__ int32_t decode_frame(const Work &W, const Ent &E, int32_t L, int32_t cap, uint32_t lane, bool jobs = false) {
    const uint8_t *in = W.in;
    if (L < 9) return kErr;
    stage_range(W, 0, 18, lane);   // the frame header (<= 18 bytes)
    const uint32_t magic = u32u(in, 0);
    const uint32_t fhd = u8u(in, 4);
    const uint32_t did = fhd & 3u, single = (fhd >> 5) & 1u, fcs_id = fhd >> 6;
    bool checksum = (fhd >> 2) & 1u;
    const int32_t fh = 5 + (int32_t)!single + (int32_t)(did == 3 ? 4 : did) + (int32_t)(fcs_id == 0 ? 0 : 1u << fcs_id) +
                       (int32_t)(single && !fcs_id);
    if (L < fh + 3) return kErr;
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
        if (fh < 8) return kErr;
        checksum = false;
    } else if (magic != 0xFD2FB528u) {
        return kErr;
    } else {
        if (fhd & 0x08u) return kErr;
        int32_t pos = 5;
        uint64_t window = 0, fcs = 0;
        uint32_t dict_id = 0;
        if (!single) {
            const uint32_t wl = u8u(in, pos++);
            const uint32_t wlog = (wl >> 3) + 10u;
            if (wlog > 27u) return kErr;
            window = 1ull << wlog;
            window += (window >> 3) * (wl & 7u);
        }
        if (did == 1) { dict_id = u8u(in, pos); pos += 1; }
        else if (did == 2) { dict_id = u16u(in, pos); pos += 2; }
        else if (did == 3) { dict_id = u32u(in, pos); pos += 4; }
        if (fcs_id == 0) { if (single) fcs = u8u(in, pos); }
        else if (fcs_id == 1) fcs = (uint64_t)u16u(in, pos) + 256u;
        else if (fcs_id == 2) fcs = u32u(in, pos);
        else fcs = ld64u(in + pos);
        if (!window) window = (uint32_t)fcs;
        if (window > (1ull << 27)) return kErr;
        if (dict_id) return kErr;
    }
    SeqTables T;
    T.ll_log = T.of_log = T.ml_log = 0;
    T.fse_entropy = T.lit_entropy = false;
    T.huf_log = 0;
    T.rep0 = 1;
    T.rep1 = 4;
    T.rep2 = 8;
    T.jobs = jobs;
    T.ll_off = T.of_off = T.ml_off = kTabDefault;
    T.njobs = 0;
    T.tb_used = 0;
    T.huf_pub = -1;
    T.nhuf = 0;
    T.nlj = 0;
    int32_t ip = fh, remaining = L - fh, op = 0;
    uint32_t ecur = 0, litc = 0;
    for (;;) {
        if (remaining < 3) return kErr;
        stage_range(W, ip, ip + 3, lane);
        const uint32_t bh = u8u(in, ip) | (u8u(in, ip + 1) << 8) | (u8u(in, ip + 2) << 16);
        const uint32_t last = bh & 1u, btype = (bh >> 1) & 3u, csize0 = bh >> 3;
        if (btype == 3u) return kErr;
        const int32_t csize = btype == 1u ? 1 : (int32_t)csize0;
        ip += 3;
        remaining -= 3;
        if (csize > remaining) return kErr;
        int32_t dec;
        if (btype == 2u) {
            dec = decode_block<kSplit>(W, T, E, ecur, litc, ip, csize, op, cap, lane);
        } else if (btype == 0u) {
            if (csize > cap - op) return kErrDst;
            if constexpr (kSplit) {
                const uint32_t at = lit_place(litc, (uint32_t)op, (uint32_t)csize);
                if (at + (uint32_t)csize > E.lcap) return kErr;
                if (ecur >= E.ecap) return E.over;
                stage_range(W, ip, ip + csize, lane);
                lds_to_lit(E.lit + at, in, ip, csize, lane);
                put_cmd(E, ecur++, kCmdRaw | (at << 2), (uint32_t)csize, 0u, lane);
                litc = at + (uint32_t)csize;
            } else {
                for (int32_t i = (int32_t)lane; i < csize; i += (int32_t)kWave) W.win[op + i] = in[ip + i];
            }
            dec = csize;
        } else {
            if ((int64_t)csize0 > (int64_t)(cap - op)) return kErrDst;
            stage_range(W, ip, ip + 1, lane);
            const uint8_t v = in[ip];
            if constexpr (kSplit) {
                if (ecur >= E.ecap) return E.over;
                put_cmd(E, ecur++, kCmdRle, csize0, v, lane);
            } else {
                for (int32_t i = (int32_t)lane; i < (int32_t)csize0; i += (int32_t)kWave) W.win[op + i] = v;
            }
            dec = (int32_t)csize0;
        }
        if (dec < 0) return dec;
        op += dec;
        ip += csize;
        remaining -= csize;
        __builtin_amdgcn_wave_barrier();
        if (last) break;
    }
    uint32_t sum = 0;
    if (checksum) {
        if (remaining < 4) return kErr;
        stage_range(W, ip, ip + 4, lane);
        sum = lds_ld32(in + ip);
        if constexpr (!kSplit)
            if (sum != xxh64_lds(W.win, (uint32_t)op, lane)) return kErr;
        remaining -= 4;
    }
    if (remaining) return kErr;
    if constexpr (kSplit) {
        if (ecur >= E.ecap) return E.over;
        put_cmd(E, ecur, kCmdEnd | ((uint32_t)checksum << 2), 0u, sum, lane);
        if (lane == 0) {
            E.jobs[0] = T.njobs;
            E.litjobs[0] = T.nlj;
        }
        return 0;
    }
    return op;
}

struct Layout {
    uint32_t off_in, off_huf, off_ll, off_of, off_ml, off_wt, off_norm, off_next, off_w, off_hp, total;
};

// with_window false: pass 1 (no window)
__host__ __device__ inline Layout make_layout(uint32_t in_cap, uint32_t out_cap, bool with_window = true) {
    Layout l;
    l.off_in = with_window ? (out_cap + kWinPad + 15u) & ~15u : 0u;
    l.off_huf = l.off_in + ((in_cap + 16u + kStreamPad + 15u) & ~15u);
    l.off_ll = l.off_huf + 2048u * 2u;
    l.off_of = l.off_ll + 512u * 4u;
    l.off_ml = l.off_of + 256u * 4u;
    l.off_wt = l.off_ml + 512u * 4u;
    l.off_norm = l.off_wt + 64u * 4u;
    l.off_next = l.off_norm + 256u * 2u;
    l.off_w = l.off_next + 256u * 2u;
    l.off_hp = l.off_w + 256u + 16u;
    l.total = l.off_hp + 256u;
    return l;
}

// only (optional): decode just the pages of [first, first + count) whose pass-1 status
// only[j] is kRetryFused (the fused-layout split decode's leftovers)
__global__ __launch_bounds__(64) void zstd_decode_kernel(tyche_batch_t b, size_t first, size_t count, uint32_t in_cap,
                                                         uint32_t out_cap, Layout lay, unsigned *ctr,
                                                         const int32_t *only) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    Work W;
    W.gsrc = nullptr;
    W.ghead = 0;
    W.gL = 0;
    W.wlo = W.whi = 0;
    W.win = smem;
    W.huf = (uint16_t *)(smem + lay.off_huf);
    W.hpair = smem + lay.off_hp;
    W.ll = (uint32_t *)(smem + lay.off_ll);
    W.of = (uint32_t *)(smem + lay.off_of);
    W.ml = (uint32_t *)(smem + lay.off_ml);
    W.wt = (uint32_t *)(smem + lay.off_wt);
    W.norm = (int16_t *)(smem + lay.off_norm);
    W.next = (uint16_t *)(smem + lay.off_next);
    W.w = smem + lay.off_w;
    uint8_t *stage = smem + lay.off_in;
    auto do_page = [&](size_t j) {
        const size_t page = first + j;
        const PageRef p = batch_page(b, page);
        int32_t rv;
        if (p.src_len > in_cap || p.dst_cap > out_cap) {
            rv = kResultTooLarge;
        } else {
            WAVE_SYNC();
            const uint32_t head = stage_in(p.src, p.src_len, stage, lane, kWave);
            uint8_t *in = stage + head;
            WAVE_SYNC();
            if (lane < kStreamPad / 4) lds_st32(in + p.src_len + lane * 4, 0u);
            WAVE_SYNC();
            W.in = in;
            SPROF_DECL
            rv = decode_frame<false>(W, Ent{}, (int32_t)p.src_len, (int32_t)p.dst_cap, lane);
            SPROF_MARK(1);
            SPROF_ADD(0, 1);
            WAVE_SYNC();
            if (rv > 0) stage_out(p.dst, W.win, (uint32_t)rv, lane, kWave);
        }
        if (lane == 0) b.results[page] = rv;
    };
    if (only) {
        // 64 statuses per read; the flagged pages in order
        for (size_t g = (size_t)blockIdx.x * kWave; g < count; g += (size_t)gridDim.x * kWave) {
            uint64_t m = __ballot(g + lane < count && only[g + lane] == kRetryFused);
            while (m) {
                const uint32_t k = (uint32_t)__builtin_ctzll(m);
                m &= m - 1ull;
                do_page(g + k);
            }
        }
        return;
    }
    for (size_t j = blockIdx.x; j < count; j = ctr ? claim_page(ctr, lane) : j + gridDim.x) do_page(j);   // engine.h
}

// ---- sequence jobs: one page per lane

// 8 bytes at any global address from aligned dwords that hold needed bytes only
// (an aligned dword never crosses a page, so none of these reads can fault)
__device__ __forceinline__ uint64_t ld64g(const uint8_t *p) {
    const uint32_t s = (uint32_t)(uintptr_t)p & 3u;
    const uint32_t *A = (const uint32_t *)(p - s);
    const uint32_t d0 = A[0], d1 = A[1];
    const uint32_t d2 = s ? A[2] : 0u;
    return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32);
}
__device__ __forceinline__ uint32_t gld(const uint32_t *p) { return *(const __attribute__((address_space(1))) uint32_t *)(uintptr_t)p; }
// A container reload in two halves: issue computes the reference's new ptr/used
// and sends the load, finish takes the bytes.  Stores placed between the two do
// not delay the wait for the load (in-order vmcnt).
struct PendLoad {
    uint32_t d0, d1, d2, s;
    bool take;
};
__device__ __forceinline__ uint32_t gbitd_reload_issue(BitD &b, const uint8_t *in, PendLoad &L) {
    uint32_t r = kUnfinished;
    L.take = false;
    if (b.used > 64u) {
        r = kOverflow;
    } else if (b.ptr >= b.start + 8) {
        b.ptr -= (int32_t)(b.used >> 3);
        b.used &= 7u;
        L.take = true;
    } else if (b.ptr == b.start) {
        r = b.used < 64u ? kEndOfBuffer : kCompleted;
    } else {
        int32_t nbytes = (int32_t)(b.used >> 3);
        if (b.ptr - nbytes < b.start) {
            nbytes = b.ptr - b.start;
            r = kEndOfBuffer;
        }
        b.ptr -= nbytes;
        b.used -= (uint32_t)nbytes * 8u;
        L.take = true;
    }
    // every lane loads (at ptr, always inside the stream); a dword past the needed
    // bytes is never touched (index 1 again when the address is aligned)
    const uint8_t *p = in + b.ptr;
    L.s = (uint32_t)(uintptr_t)p & 3u;
    const uint32_t *A = (const uint32_t *)(p - L.s);
    L.d0 = gld(A);
    L.d1 = gld(A + 1);
    L.d2 = gld(A + (L.s ? 2 : 1));
    return r;
}
__device__ __forceinline__ void gbitd_reload_finish(BitD &b, const PendLoad &L) {
    if (L.take)
        b.c = (uint64_t)__builtin_amdgcn_alignbyte(L.d1, L.d0, L.s) |
              ((uint64_t)__builtin_amdgcn_alignbyte(L.d2, L.d1, L.s) << 32);
}
// BIT_initDStream / BIT_reloadDStream over global memory (the per-lane reader above, other loads)
__device__ __forceinline__ bool gbitd_init(BitD &b, const uint8_t *in, int32_t start, int32_t n) {
    b.start = start;
    b.c = 0;
    b.used = 0;
    b.ptr = start;
    if (n < 1) return false;
    const uint32_t last = in[start + n - 1];
    if (last == 0) return false;
    const uint32_t mark = 8u - highbit(last);
    if (n >= 8) {
        b.ptr = start + n - 8;
        b.c = ld64g(in + b.ptr);
        b.used = mark;
    } else {
        uint64_t c = in[start];
        for (int32_t k = 1; k < n; k++) c += (uint64_t)in[start + k] << (8u * (uint32_t)k);
        b.c = c;
        b.used = mark + (uint32_t)(8 - n) * 8u;
    }
    return true;
}
__device__ __forceinline__ uint32_t gbitd_reload(BitD &b, const uint8_t *in) {
    if (b.used > 64u) return kOverflow;
    if (b.ptr >= b.start + 8) {
        b.ptr -= (int32_t)(b.used >> 3);
        b.used &= 7u;
        b.c = ld64g(in + b.ptr);
        return kUnfinished;
    }
    if (b.ptr == b.start) return b.used < 64u ? kEndOfBuffer : kCompleted;
    int32_t nbytes = (int32_t)(b.used >> 3);
    uint32_t r = kUnfinished;
    if (b.ptr - nbytes < b.start) {
        nbytes = b.ptr - b.start;
        r = kEndOfBuffer;
    }
    b.ptr -= nbytes;
    b.used -= (uint32_t)nbytes * 8u;
    b.c = ld64g(in + b.ptr);
    return r;
}

// Sequence chains, one page per lane (zstd_seq_kernel, zstd_seqexec_kernel).
//
// kLog 7 / 6 (a job whose table logs are <= kLog / kLog - 1 / kLog: every frame
// of this encoder at TYCHE_ZSTD_FSE_LOG 7 / 6, the predefined tables): the lane's
// three tables are copied into its LDS slot as 16-bit cells (newState | symbol <<
// 7 | nbBits << 13); kLog 0: cells are gathered from the table area.  The
// sequence kernel also stages its entries in LDS 16 at a time, so each plane
// gets whole 64-byte lines (kLog 0: stored one by one).
template <uint32_t kLog>
struct Slots {
    static constexpr uint32_t LL = 0u, OF = 1u << kLog, ML = (1u << kLog) + (1u << kLog >> 1);
    static constexpr uint32_t cells = 2u * (1u << kLog) + (1u << kLog >> 1);
};
template <uint32_t kLog>
__device__ __forceinline__ bool job_fits(uint32_t logs) {
    return (logs & 255u) <= kLog && ((logs >> 8) & 255u) + 1u <= kLog && ((logs >> 16) & 255u) <= kLog;
}
constexpr uint32_t kSlotCells = Slots<7>::cells;   // zstd_seq_kernel
constexpr uint32_t kSeqLds = kWave * (kSlotCells * 2u + 3u * 16u * 4u);
__device__ __forceinline__ uint32_t cell16(uint32_t c) { return (c & 127u) | (((c >> 7) & 63u) << 16) | ((c >> 13) << 24); }
__device__ __forceinline__ uint16_t pack16(uint32_t c) {   // area cell: newState | symbol << 16 | nbBits << 24
    return (uint16_t)((c & 0xFFFFu) | (((c >> 16) & 0xFFu) << 7) | ((c >> 24) << 13));
}
// The chain of one job: pre(i) runs right after step i's bitstream load is
// issued (the plane stores of step i - 1 go there: loads and stores share
// vmcnt and complete in order, so waiting for the load never waits for them),
// emit(i, litLength, matchLength, offset) after step i's sequence is decoded
// (false: the page fails).
template <uint32_t kLog, typename Pre, typename Emit>
__device__ __forceinline__ bool seq_chain(const Ent &E, const uint8_t *src, const uint32_t *J, uint32_t &rep0,
                                          uint32_t &rep1, uint32_t &rep2, uint16_t *lt, Pre &&pre, Emit &&emit) {
    const int32_t start = (int32_t)J[0], len = (int32_t)J[1];
    const uint32_t nbseq = J[2];
    const uint32_t *LL = E.tabs + J[4] / 4u, *OF = E.tabs + J[5] / 4u, *ML = E.tabs + J[6] / 4u;
    const uint32_t lls = J[7] & 255u, ofs = (J[7] >> 8) & 255u, mls = (J[7] >> 16) & 255u;
    using S = Slots<kLog ? kLog : 7u>;
    if (kLog) {
        for (uint32_t u = 0; u < (1u << lls); u++) lt[S::LL + u] = pack16(gld(LL + u));
        for (uint32_t u = 0; u < (1u << ofs); u++) lt[S::OF + u] = pack16(gld(OF + u));
        for (uint32_t u = 0; u < (1u << mls); u++) lt[S::ML + u] = pack16(gld(ML + u));
    }
    BitD b;
    if (!gbitd_init(b, src, start, len)) return false;
    uint32_t sll = bitd_read(b, lls);
    gbitd_reload(b, src);
    uint32_t sof = bitd_read(b, ofs);
    gbitd_reload(b, src);
    uint32_t sml = bitd_read(b, mls);
    gbitd_reload(b, src);
    for (uint32_t i = 0; i < nbseq; i++) {
        uint32_t cl_v, cm_v, co_v;
        if (kLog) {
            cl_v = cell16(lt[S::LL + sll]);
            cm_v = cell16(lt[S::ML + sml]);
            co_v = cell16(lt[S::OF + sof]);
        } else {
            cl_v = gld(LL + sll);
            cm_v = gld(ML + sml);
            co_v = gld(OF + sof);
        }
        PendLoad pl;
        const uint32_t rs = gbitd_reload_issue(b, src, pl);
        pre(i);
        if (rs > kCompleted) return false;
        gbitd_reload_finish(b, pl);
        const uint32_t cl = cl_v, cm = cm_v, co = co_v;
        const uint32_t llc = cell_sym(cl), mlc = cell_sym(cm), ofc = cell_sym(co);
        const uint32_t ofx = (uint32_t)bitd_look_fast(b, ofc);
        b.used += ofc;
        uint32_t offv = ofc ? of_base(ofc) + ofx : 0u;
        {
            const bool small = ofc <= 1u;
            const uint32_t adj = offv + (llc == 0u);
            uint32_t t = adj == 3u ? rep0 - 1u : (adj == 1u ? rep1 : rep2);
            t += t == 0u;
            const uint32_t n0 = small ? (adj ? t : rep0) : offv;
            const uint32_t n1 = small ? (adj ? rep0 : rep1) : rep0;
            const uint32_t n2 = small ? (adj ? (adj != 1u ? rep1 : rep2) : rep2) : rep1;
            offv = n0;
            rep0 = n0;
            rep1 = n1;
            rep2 = n2;
        }
        uint32_t mlbase, mlb, llbase, llb;
        ml_code(mlc, mlbase, mlb);
        ll_code(llc, llbase, llb);
        const uint32_t mlx = (uint32_t)bitd_look_fast(b, mlb);
        b.used += mlb;
        const uint32_t mlv = mlbase + (mlb ? mlx : 0u);
        const uint32_t llx = (uint32_t)bitd_look_fast(b, llb);
        b.used += llb;
        const uint32_t llv = llbase + (llb ? llx : 0u);
        if (llb + mlb + ofc > 31u) gbitd_reload(b, src);
        sll = cell_state(cl) + bitd_read(b, cell_nb(cl));
        sml = cell_state(cm) + bitd_read(b, cell_nb(cm));
        sof = cell_state(co) + bitd_read(b, cell_nb(co));
        if (!emit(i, llv, mlv, offv)) return false;
    }
    return true;
}

// ZSTD_decompressSequences (zstd_decompress.c:1010-1060) for one job, this lane's
// page: the decoded (litLength, matchLength, offset) triples go to the entry planes.
template <bool kSmall>   // kSmall: Slots<7> tables in LDS
__device__ bool seq_job(const Ent &E, const uint8_t *src, const uint32_t *J, uint32_t &rep0, uint32_t &rep1,
                        uint32_t &rep2, uint16_t *lt, uint32_t *sg) {
    const uint32_t nbseq = J[2], e0 = J[3];
    uint32_t pll = 0, pml = 0, pof = 0;
    auto pre = [&](uint32_t i) {
        if (!kSmall && i) {
            E.ll[e0 + i - 1] = pll;
            E.ml[e0 + i - 1] = pml;
            E.of[e0 + i - 1] = pof;
        }
    };
    auto emit = [&](uint32_t i, uint32_t llv, uint32_t mlv, uint32_t offv) -> bool {
        if (kSmall) {
            // stage; a full 16-entry line (or the job's last entry) goes out
            const uint32_t e = e0 + i, k = e & 15u;
            sg[k] = llv;
            sg[16u + k] = mlv;
            sg[32u + k] = offv;
            if (k == 15u || i + 1u == nbseq) {
                const uint32_t lo = e - k < e0 ? e0 & 15u : 0u, base = e - k;
                if (lo == 0u && k == 15u) {
#pragma unroll
                    for (uint32_t q = 0; q < 4u; q++) {
                        ((u32x4 *)(E.ll + base))[q] = ((const u32x4 *)sg)[q];
                        ((u32x4 *)(E.ml + base))[q] = ((const u32x4 *)(sg + 16u))[q];
                        ((u32x4 *)(E.of + base))[q] = ((const u32x4 *)(sg + 32u))[q];
                    }
                } else {
                    for (uint32_t q = lo; q <= k; q++) {
                        E.ll[base + q] = sg[q];
                        E.ml[base + q] = sg[16u + q];
                        E.of[base + q] = sg[32u + q];
                    }
                }
            }
        } else {
            pll = llv;
            pml = mlv;
            pof = offv;
        }
        return true;
    };
    if (!seq_chain<kSmall ? 7u : 0u>(E, src, J, rep0, rep1, rep2, lt, pre, emit)) return false;
    if (!kSmall && nbseq) {
        E.ll[e0 + nbseq - 1] = pll;
        E.ml[e0 + nbseq - 1] = pml;
        E.of[e0 + nbseq - 1] = pof;
    }
    return true;
}

// One lane per page of the chunk: runs the page's jobs in order (repeat offsets
// carry across blocks); a failed chain fails the page.
__global__ __launch_bounds__(64) void zstd_seq_kernel(tyche_batch_t b, size_t first, size_t count, uint32_t in_cap,
                                                      uint32_t out_cap, uint8_t *ws, size_t ws_page, int32_t *st) {
    const size_t j = (size_t)blockIdx.x * kWave + threadIdx.x;
    if (j >= count || st[j] < 0) return;
    const Ent E = ent_of(ws + j * ws_page, in_cap, out_cap, false);
    const uint32_t njobs = E.jobs[0];
    if (njobs == 0) return;
    const PageRef p = batch_page(b, first + j);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint16_t *lt = (uint16_t *)smem + threadIdx.x * kSlotCells;
    uint32_t *sg = (uint32_t *)(smem + kWave * kSlotCells * 2u) + threadIdx.x * 48u;
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;
    for (uint32_t q = 0; q < njobs; q++) {
        const uint32_t *J = E.jobs + 4u + q * kJobWords;
        const uint32_t logs = J[7];
        const bool small = job_fits<7>(logs);
        const bool ok = small ? seq_job<true>(E, p.src, J, rep0, rep1, rep2, lt, sg)
                              : seq_job<false>(E, p.src, J, rep0, rep1, rep2, lt, sg);
        if (!ok) {
            st[j] = kErr;
            return;
        }
    }
}

// ---- pass 2

// global src -> LDS dst, n bytes.  Equal 16-byte phases (pass 1 arranges that for
// runs of 64+ bytes, lit_place) copy 16-byte vectors; anything else goes bytewise.
__device__ __forceinline__ void lit_to_lds(uint8_t *dst, const uint8_t *src, int32_t n, uint32_t lane) {
    int32_t i0 = 0;
    if (n >= 64 && (((uintptr_t)dst ^ (uintptr_t)src) & 15u) == 0) {
        const int32_t head = (int32_t)((16u - ((uint32_t)(uintptr_t)dst & 15u)) & 15u);
        if ((int32_t)lane < head) dst[lane] = src[lane];
        const int32_t nv = (n - head) >> 4;
        const u32x4 *g = (const u32x4 *)(src + head);
        u32x4 *l = (u32x4 *)(dst + head);
        int32_t v = (int32_t)lane;
        for (; v + 3 * (int32_t)kWave < nv; v += 4 * (int32_t)kWave) {
            const u32x4 x0 = g[v], x1 = g[v + kWave], x2 = g[v + 2 * kWave], x3 = g[v + 3 * kWave];
            l[v] = x0;
            l[v + kWave] = x1;
            l[v + 2 * kWave] = x2;
            l[v + 3 * kWave] = x3;
        }
        for (; v < nv; v += (int32_t)kWave) l[v] = g[v];
        i0 = head + (nv << 4);
    }
    for (int32_t i = i0 + (int32_t)lane; i < n; i += (int32_t)kWave) dst[i] = src[i];
}

// Replays a page's entries into the window.  Returns the decoded size or < 0.
__device__ int32_t exec_page(uint8_t *win, const Ent &E, int32_t cap, uint32_t lane) {
    uint32_t cur = 0;
    int32_t op = 0;
    for (;;) {
        if (cur >= E.ecap) return kErr;
        const uint32_t a = rfl(E.ll[cur]), bsz = rfl(E.ml[cur]), c = rfl(E.of[cur]);
        cur++;
        const uint32_t kind = a & 3u;
        if (kind == kCmdEnd) {
            if (((a >> 2) & 1u) && c != xxh64_lds(win, (uint32_t)op, lane)) return kErr;
            return op;
        }
        const int32_t sz = (int32_t)bsz;
        if (kind == kCmdRaw) {
            if (sz > cap - op) return kErrDst;
            lit_to_lds(win + op, E.lit + (a >> 2), sz, lane);
            op += sz;
        } else if (kind == kCmdRle) {
            if (sz > cap - op) return kErrDst;
            for (int32_t i = (int32_t)lane; i < sz; i += (int32_t)kWave) win[op + i] = (uint8_t)c;
            op += sz;
        } else {
            const int32_t lsize = sz;
            if (op + lsize > cap) return kErrDst;
            uint8_t *lit = win + (cap - lsize);
            lit_to_lds(lit, E.lit + (a >> 2), lsize, lane);
            __builtin_amdgcn_wave_barrier();
            int32_t lp = 0;
            const uint32_t nseq = c;
            if (nseq > E.ecap - cur) return kErr;
            // the next batch's loads go out before this batch executes
            uint32_t nll = 0, nml = 0, nof = 0;
            if (lane < min(nseq, kWave)) {
                nll = E.ll[cur + lane];
                nml = E.ml[cur + lane];
                nof = E.of[cur + lane];
            }
            for (uint32_t done = 0; done < nseq; done += kWave) {
                const uint32_t k = min(nseq - done, kWave);
                const uint32_t vll = nll, vml = nml, voff = nof;
                const uint32_t nx = done + kWave;
                if (nx < nseq && lane < min(nseq - nx, kWave)) {
                    nll = E.ll[cur + nx + lane];
                    nml = E.ml[cur + nx + lane];
                    nof = E.of[cur + nx + lane];
                }
                if (!exec_batch(win, lit, true, cap - lsize, k, vll, vml, voff, op, lp, lsize, cap, lane)) return kErr;
            }
            cur += nseq;
            const int32_t last = lsize - lp;
            if (last > cap - op) return kErrDst;
            for (int32_t c0 = 0; c0 < last; c0 += (int32_t)kWave) {
                const int32_t i = c0 + (int32_t)lane;
                const uint8_t v = i < last ? lit[lp + i] : 0;
                __builtin_amdgcn_wave_barrier();
                if (i < last) win[op + i] = v;
                __builtin_amdgcn_wave_barrier();
            }
            op += last;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- pass 2, one page per lane (default for batches of >= TYCHE_ZSTD_EXEC_LANE_MIN pages)
//
// exec_page runs a page's sequences 64 at a time across the wave, but a batch's
// matches depend on each other (the frontier loop above serialises most of
// them) and the 32 KiB window holds a CU to 4 waves.  Here one lane replays one
// page's entries in order -- the reference's ZSTD_execSequence loop
// (zstd_decompress.c:940-1003) -- through a per-lane LDS ring (lane_ring.h):
// entries and literals stream from the pass-1 buffer in HBM, near matches read
// the ring, far ones the page's flushed lines.  Results and checks are
// exec_page's, in the same order.

// A page's entries in order, four at a time: aligned 16-byte loads of each plane
// (planes are 64-byte aligned), the next quad in flight while this one is used.
struct EntRd {
    const uint32_t *ll, *ml, *of;
    uint32_t q;   // index of quad 0's first entry
    u32x4 a0, b0, c0, a1, b1, c1;
};
__device__ __forceinline__ u32x4 gquad(const uint32_t *p) { return *(g_u32x4 *)(uintptr_t)p; }
__device__ __forceinline__ uint32_t pick(u32x4 v, uint32_t i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
__device__ __forceinline__ void er_init(EntRd &r, const Ent &E) {
    r.ll = E.ll;
    r.ml = E.ml;
    r.of = E.of;
    r.q = 0;
    r.a0 = gquad(r.ll);
    r.b0 = gquad(r.ml);
    r.c0 = gquad(r.of);
    r.a1 = gquad(r.ll + 4);
    r.b1 = gquad(r.ml + 4);
    r.c1 = gquad(r.of + 4);
}
// entry i < ecap (i never decreases; the prefetch may read up to 7 entries past
// a plane's end: the next plane, or for `of` the literal buffer)
__device__ __forceinline__ void er_get(EntRd &r, uint32_t i, uint32_t &a, uint32_t &b, uint32_t &c) {
    while (i >= r.q + 4) {
        r.q += 4;
        r.a0 = r.a1;
        r.b0 = r.b1;
        r.c0 = r.c1;
        r.a1 = gquad(r.ll + r.q + 4);
        r.b1 = gquad(r.ml + r.q + 4);
        r.c1 = gquad(r.of + r.q + 4);
    }
    const uint32_t k = i - r.q;
    a = pick(r.a0, k);
    b = pick(r.b0, k);
    c = pick(r.c0, k);
}

// n bytes from the literal buffer to page position op through the ring (reads
// up to 15 bytes past the run: inside the page's area, or the lease's slack)
template <int32_t kRing>
__device__ __forceinline__ void lit_run(uint8_t *rb, uint8_t *__restrict__ out, int32_t &fl, int32_t op,
                                        const uint8_t *__restrict__ src, int32_t n) {
    for (int32_t k = 0; k < n; k += 16) {
        ring_wr<kRing>(rb, op + k, ld16(src + k));
        ring_flush<kRing>(rb, out, fl, op + min(k + 16, n));
    }
}

// XXH64 (low 32 bits) of out[0, len) in HBM, one lane
__device__ uint32_t xxh64_lane(const uint8_t *p, uint32_t len) {
    uint64_t h;
    uint32_t i = 0;
    if (len >= 32) {
        uint64_t v1 = kP1 + kP2, v2 = kP2, v3 = 0, v4 = (uint64_t)0 - kP1;
        for (; i + 32 <= len; i += 32) {
            v1 = xround(v1, ld8(p + i));
            v2 = xround(v2, ld8(p + i + 8));
            v3 = xround(v3, ld8(p + i + 16));
            v4 = xround(v4, ld8(p + i + 24));
        }
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = (h ^ xround(0, v1)) * kP1 + kP4;
        h = (h ^ xround(0, v2)) * kP1 + kP4;
        h = (h ^ xround(0, v3)) * kP1 + kP4;
        h = (h ^ xround(0, v4)) * kP1 + kP4;
    } else {
        h = kP5;
    }
    h += (uint64_t)len;
    for (; i + 8 <= len; i += 8) h = rotl64(h ^ xround(0, ld8(p + i)), 27) * kP1 + kP4;
    if (i + 4 <= len) {
        const uint64_t w = ld1(p + i) | (ld1(p + i + 1) << 8) | (ld1(p + i + 2) << 16) | ((uint64_t)ld1(p + i + 3) << 24);
        h ^= w * kP1;
        h = rotl64(h, 23) * kP2 + kP3;
        i += 4;
    }
    for (; i < len; i++) h = rotl64(h ^ (uint64_t)ld1(p + i) * kP5, 11) * kP1;
    h ^= h >> 33;
    h *= kP2;
    h ^= h >> 29;
    h *= kP3;
    h ^= h >> 32;
    return (uint32_t)h;
}

// A lane's page on its way out through the ring
struct LaneOut {
    uint8_t *rb;                 // the lane's LDS ring (lane_ring.h)
    uint8_t *__restrict__ out;   // the page's destination
    int32_t fl, op, cap;         // bytes already in HBM, bytes decoded, capacity
};

// One sequence: exec_batch's checks (ZSTD_execSequence, zstd_decompress.c:940-954),
// ll literals from lit + lp, then ml bytes from off back.  False: the page fails.
template <int32_t kRing>
__device__ __forceinline__ bool exec_seq(LaneOut &o, const uint8_t *__restrict__ lit, int32_t &lp, int32_t lsize,
                                         uint32_t ll, uint32_t ml, uint32_t off) {
    if ((uint64_t)ll + ml > (uint64_t)(o.cap - o.op) || ll > (uint32_t)(lsize - lp) || off > (uint64_t)o.op + ll)
        return false;
    const int32_t d = o.op + (int32_t)ll;   // match destination
    lit_run<kRing>(o.rb, o.out, o.fl, o.op, lit + lp, (int32_t)ll);
    lp += (int32_t)ll;
    // the unflushed tail is < kLine bytes here and the ring holds every position above
    // d + 16 - kRing, so a source more than kRing - 32 back is already in HBM
    const int32_t f = (int32_t)off, n = (int32_t)ml;
    const bool far = f > kRing - 32;
    u128 m = far ? ld16(o.out + d - f) : ring_rd<kRing>(o.rb, d - f);
    if (f >= 16) {
        ring_wr<kRing>(o.rb, d, m);
        for (int32_t k = 16; k < n; k += 16) {
            ring_flush<kRing>(o.rb, o.out, o.fl, d + k);
            m = far ? ld16(o.out + d + k - f) : ring_rd<kRing>(o.rb, d + k - f);
            ring_wr<kRing>(o.rb, d + k, m);
        }
    } else {
        int32_t step;
        const u128 p = period_pattern(m, f, step);
        for (int32_t k = 0; k < n; k += step) {
            ring_flush<kRing>(o.rb, o.out, o.fl, d + k);
            ring_wr<kRing>(o.rb, d + k, p);
        }
    }
    o.op = d + n;
    ring_flush<kRing>(o.rb, o.out, o.fl, o.op);
    return true;
}

// exec_page for one lane: the page's commands into out[0, cap) through the ring
// rb.  blk_seqs(r, cur, nseq, lit, lp, lsize, o) runs a compressed block's nseq
// sequences (cur: the entry after the block's command; the entry source advances
// it past what it consumes) and returns false when the page fails.
template <int32_t kRing, typename BlkSeqs>
__device__ __forceinline__ int32_t exec_cmds(const Ent &E, uint8_t *__restrict__ out, int32_t cap, uint8_t *rb,
                                             BlkSeqs &&blk_seqs) {
    EntRd r;
    er_init(r, E);
    uint32_t cur = 0;
    LaneOut o{rb, out, 0, 0, cap};
    for (;;) {
        if (cur >= E.ecap) return kErr;
        uint32_t a, bsz, c;
        er_get(r, cur, a, bsz, c);
        cur++;
        const uint32_t kind = a & 3u;
        if (kind == kCmdEnd) {
            ring_flush_all<kRing>(rb, out, o.fl, o.op);
            if (((a >> 2) & 1u) && c != xxh64_lane(out, (uint32_t)o.op)) return kErr;
            return o.op;
        }
        const int32_t sz = (int32_t)bsz;
        if (kind == kCmdRaw) {
            if (sz > cap - o.op) return kErrDst;
            lit_run<kRing>(rb, out, o.fl, o.op, E.lit + (a >> 2), sz);
            o.op += sz;
            continue;
        }
        if (kind == kCmdRle) {
            if (sz > cap - o.op) return kErrDst;
            const u128 p = (u128)(c & 0xFFu) * (~(u128)0 / 255u);
            for (int32_t k = 0; k < sz; k += 16) {
                ring_flush<kRing>(rb, out, o.fl, o.op + k);
                ring_wr<kRing>(rb, o.op + k, p);
            }
            o.op += sz;
            ring_flush<kRing>(rb, out, o.fl, o.op);
            continue;
        }
        const int32_t lsize = sz;
        if (o.op + lsize > cap) return kErrDst;
        const uint8_t *__restrict__ lit = E.lit + (a >> 2);
        int32_t lp = 0;
        if (!blk_seqs(r, cur, c, lit, lp, lsize, o)) return kErr;
        const int32_t last = lsize - lp;
        if (last > cap - o.op) return kErrDst;
        lit_run<kRing>(rb, out, o.fl, o.op, lit + lp, last);
        o.op += last;
    }
}

// The page's sequences from the entry planes (zstd_seq_kernel's output)
template <int32_t kRing>
__device__ int32_t exec_lane(const Ent &E, uint8_t *__restrict__ out, int32_t cap, uint8_t *rb) {
    return exec_cmds<kRing>(E, out, cap, rb,
                            [&](EntRd &r, uint32_t &cur, uint32_t nseq, const uint8_t *lit, int32_t &lp, int32_t lsize,
                                LaneOut &o) -> bool {
                                if (nseq > E.ecap - cur) return false;
                                for (uint32_t q = 0; q < nseq; q++) {
                                    uint32_t ll, ml, off;
                                    er_get(r, cur + q, ll, ml, off);
                                    if (!exec_seq<kRing>(o, lit, lp, lsize, ll, ml, off)) return false;
                                }
                                cur += nseq;
                                return true;
                            });
}

template <int32_t kRing>
__global__ __launch_bounds__(64) void zstd_exec_lane_kernel(tyche_batch_t b, size_t first, size_t count,
                                                            uint32_t in_cap, uint32_t out_cap, const uint8_t *ws,
                                                            size_t ws_page, const int32_t *st, unsigned *ctr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *rb = smem + threadIdx.x * (kRing + 48) + 16;
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    while (j < count) {
        const size_t i = first + j;
        int32_t rv = st[j];
        if (rv >= 0) {
            const uint64_t dof = b.dst_offsets ? b.dst_offsets[i] : (uint64_t)i * b.dst_stride;
            const uint32_t C = b.dst_capacities ? b.dst_capacities[i] : b.dst_capacity;
            const Ent E = ent_of(const_cast<uint8_t *>(ws) + j * ws_page, in_cap, out_cap, false);
            rv = exec_lane<kRing>(E, (uint8_t *)b.dst + dof, (int32_t)C, rb);
        }
        b.results[i] = rv;
        j = (size_t)atomicAdd(ctr, 1u) + nthreads;
    }
}

// ---- pass 2, chains and execution fused (default): one page per lane runs each
// compressed block's sequence chain (the job pass 1 left) and executes every
// sequence as it is decoded -- the reference's own order (ZSTD_decompressSequences
// decodes and executes one sequence at a time, zstd_decompress.c:1037-1047).  No
// entries go through HBM: the pass-1 area holds commands only (kFusedCmds), so a
// chunk of pages needs ~50 KiB per 32 KiB page instead of ~310 KiB.  Tables of up
// to kLog / kLog - 1 / kLog are copied to the lane's LDS slot, larger ones gathered.
template <int32_t kRing, uint32_t kLog>
__device__ int32_t seqexec_page(const Ent &E, const uint8_t *src, uint8_t *__restrict__ out, int32_t cap, uint8_t *rb,
                                uint16_t *lt) {
    const uint32_t njobs = E.jobs[0];
    uint32_t q = 0, rep0 = 1, rep1 = 4, rep2 = 8;
    return exec_cmds<kRing>(E, out, cap, rb,
                            [&](EntRd &, uint32_t &, uint32_t nseq, const uint8_t *lit, int32_t &lp, int32_t lsize,
                                LaneOut &o) -> bool {
                                if (nseq == 0) return true;
                                if (q >= njobs) return false;
                                const uint32_t *J = E.jobs + 4u + q * kJobWords;
                                q++;
                                if (J[2] != nseq) return false;
                                auto nopre = [](uint32_t) {};
                                auto run = [&](uint32_t, uint32_t ll, uint32_t ml, uint32_t off) -> bool {
                                    return exec_seq<kRing>(o, lit, lp, lsize, ll, ml, off);
                                };
                                return job_fits<kLog>(J[7]) ? seq_chain<kLog>(E, src, J, rep0, rep1, rep2, lt, nopre, run)
                                                            : seq_chain<0u>(E, src, J, rep0, rep1, rep2, lt, nopre, run);
                            });
}

template <int32_t kRing, uint32_t kLog>
__global__ __launch_bounds__(64) void zstd_seqexec_kernel(tyche_batch_t b, size_t first, size_t count,
                                                          uint32_t in_cap, uint32_t out_cap, const uint8_t *ws,
                                                          size_t ws_page, const int32_t *st, unsigned *ctr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *rb = smem + threadIdx.x * (kRing + 48) + 16;
    uint16_t *lt = (uint16_t *)(smem + 64u * (kRing + 48)) + threadIdx.x * Slots<kLog>::cells;
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    while (j < count) {
        const size_t i = first + j;
        int32_t rv = st[j];
        if (rv >= 0) {
            const uint64_t so = b.src_offsets ? b.src_offsets[i] : (uint64_t)i * b.src_stride;
            const uint64_t dof = b.dst_offsets ? b.dst_offsets[i] : (uint64_t)i * b.dst_stride;
            const uint32_t C = b.dst_capacities ? b.dst_capacities[i] : b.dst_capacity;
            const Ent E = ent_of(const_cast<uint8_t *>(ws) + j * ws_page, in_cap, out_cap, true);
            rv = seqexec_page<kRing, kLog>(E, (const uint8_t *)b.src + so, (uint8_t *)b.dst + dof, (int32_t)C, rb, lt);
        }
        if (rv != kRetryFused) b.results[i] = rv;
        j = (size_t)atomicAdd(ctr, 1u) + nthreads;
    }
}

// ---- literal streams, one per lane (fused layout, TYCHE_ZSTD_LIT_LANES; between pass 1 and
// zstd_seqexec_kernel).
//
// Pass 1 decoded a section's 1 or 4 Huffman streams in lanes 0-3 of its wave, ~480 cycles per
// symbol (the whole wave's instruction stream for 4 lanes: 60 % of pass 1, tools/zstd_phases.py).
// Here lane 4g + s decodes stream s of page g of the workgroup, kGroups pages per wave: the
// page's decoding table is rebuilt from its published weights in its group's LDS slot (kHufCells
// x 16 bit) and each lane
// walks its stream from global memory (huf_decode's reader, checks and end test), writing
// whole aligned 8-byte words of the literal buffer.  A failed stream fails the page.
template <uint32_t kGroups>
__global__ __launch_bounds__(64) void zstd_lit_kernel(tyche_batch_t b, size_t first, size_t count, uint32_t in_cap,
                                                      uint32_t out_cap, uint8_t *ws, size_t ws_page, int32_t *st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x, g = lane >> 2, s = lane & 3u;
    uint16_t *tab = (uint16_t *)smem + min(g, kGroups - 1u) * kHufCells;
    uint8_t *wbuf = smem + kGroups * kHufCells * 2u;   // a table's weights (<= 256 bytes)
    const size_t j = (size_t)blockIdx.x * kGroups + g;
    const bool act = g < kGroups && j < count && st[j] >= 0;
    Ent E;
    const uint8_t *src = nullptr;
    uint32_t njobs = 0;
    if (act) {
        E = ent_of(ws + j * ws_page, in_cap, out_cap, true);
        njobs = E.litjobs[0];
        const size_t i = first + j;
        src = (const uint8_t *)b.src + (b.src_offsets ? b.src_offsets[i] : (uint64_t)i * b.src_stride);
    }
    uint32_t maxj = njobs;
#pragma unroll
    for (uint32_t m = 1; m < kWave; m <<= 1) maxj = max(maxj, (uint32_t)__shfl_xor((int)maxj, (int)m));
    bool ok = true;
    for (uint32_t q = 0; q < maxj; q++) {
        const bool has = act && q < njobs;
        uint32_t cs = 0, n = 0, lsize = 0, lat = 0, toff = 0, tlog = 0, nsym = 0;
        bool single = false;
        if (has) {
            const uint32_t *J = E.litjobs + 4u + q * kLitJobWords;
            cs = J[0];
            n = J[1];
            lsize = J[2];
            lat = J[3];
            toff = J[4];
            tlog = J[5] & 255u;
            single = ((J[5] >> 8) & 1u) != 0u;
            nsym = J[5] >> 16;
        }
        // each group's decoding table from its published weights, the whole wave per group (the
        // weights through the wave's LDS scratch, then HUF_readDTableX2's fill, huf_fill): 256
        // bytes read per table instead of the 2^tlog-entry table
        const uint64_t gmask = __ballot(has && s == 0u);
        for (uint64_t gm = gmask; gm; gm &= gm - 1) {
            const uint32_t l = (uint32_t)__builtin_ctzll(gm), gg = l >> 2;
            const uint32_t gn = rdlane(nsym, l), glog = rdlane(tlog, l), gtoff = rdlane(toff, l);
            const uint32_t lo = rdlane((uint32_t)(uintptr_t)E.hufs, l), hi = rdlane((uint32_t)((uintptr_t)E.hufs >> 32), l);
            const uint8_t *gw = (const uint8_t *)((const uint16_t *)(uintptr_t)(((uint64_t)hi << 32) | lo) + gtoff);
            for (uint32_t i = lane; i < gn; i += kWave) wbuf[i] = gw[i];
            __builtin_amdgcn_wave_barrier();
            uint32_t rank[13];
#pragma unroll
            for (uint32_t k = 0; k < 13; k++) rank[k] = 0;
            for (uint32_t s0 = 0; s0 < gn; s0 += kWave) {
                const uint32_t wv = s0 + lane < gn ? wbuf[s0 + lane] : 0u;
#pragma unroll
                for (uint32_t k = 1; k < 12; k++) rank[k] += (uint32_t)__builtin_popcountll(__ballot(s0 + lane < gn && wv == k));
            }
            huf_fill(wbuf, gn, glog, rank, (uint16_t *)smem + gg * kHufCells, nullptr, lane);
            __builtin_amdgcn_wave_barrier();
        }
        if (has && ok) {
            int32_t sstart = 0, slen = 0;
            uint32_t o0 = 0, cnt = 0;
            bool good = true;
            if (single) {
                sstart = (int32_t)cs;
                slen = (int32_t)n;
                cnt = s == 0 ? lsize : 0u;
            } else {
                good = n >= 10u;
                if (good) {
                    const int32_t l1 = (int32_t)(src[cs] | (src[cs + 1] << 8)), l2 = (int32_t)(src[cs + 2] | (src[cs + 3] << 8)),
                                  l3 = (int32_t)(src[cs + 4] | (src[cs + 5] << 8));
                    const int32_t l4 = (int32_t)n - (l1 + l2 + l3 + 6);
                    good = l4 >= 0 && l4 <= (int32_t)n;
                    const uint32_t seg = (lsize + 3u) / 4u;
                    const uint32_t n4 = lsize > 3u * seg ? lsize - 3u * seg : 0u;
                    sstart = (int32_t)cs + 6 + (s > 0 ? l1 : 0) + (s > 1 ? l2 : 0) + (s > 2 ? l3 : 0);
                    slen = s == 0 ? l1 : s == 1 ? l2 : s == 2 ? l3 : l4;
                    o0 = seg * s;
                    cnt = s < 3u ? seg : n4;
                }
            }
            if (good && (!single || s == 0u)) {
                BitD bd;
                good = gbitd_init(bd, src, sstart, slen);
                uint8_t *out = E.lit + lat;
                uint64_t acc = 0;
                uint32_t lo = (uint32_t)((uintptr_t)(out + o0) & 7u);   // first valid byte of the current word
                for (uint32_t i = 0; good && i < cnt; i++) {
                    if (bd.used > 52u) gbitd_reload(bd, src);
                    const uint32_t e = tab[(uint32_t)bitd_look_fast(bd, tlog)];
                    bd.used += e >> 8;
                    uint8_t *at = out + o0 + i;
                    const uint32_t k = (uint32_t)((uintptr_t)at & 7u);
                    acc |= (uint64_t)(e & 255u) << (8u * k);
                    if (k == 7u || i + 1u == cnt) {
                        uint8_t *word = at - k;
                        if (lo == 0u && k == 7u) {
                            *(uint64_t *)word = acc;
                        } else {
                            for (uint32_t t = lo; t <= k; t++) word[t] = (uint8_t)(acc >> (8u * t));
                        }
                        acc = 0;
                        lo = 0;
                    }
                }
                if (good) {   // BIT_endOfDStream
                    if (bd.used <= 64u) gbitd_reload(bd, src);
                    good = bd.ptr == bd.start && bd.used == 64u;
                }
            }
            ok = good;
        }
        __builtin_amdgcn_wave_barrier();   // the slot is reused by the next job's table
    }
    // a stream that failed fails its page (all four lanes of the group agree on the verdict)
    const uint32_t grp_bad = (uint32_t)(__ballot(act && !ok) >> (4u * min(g, 15u))) & 15u;
    if (act && s == 0u && grp_bad) st[j] = kErr;
}

// Pass 1 over pages [first, first + count) of b; page j's entries at ws + j * ws_page.
__global__ __launch_bounds__(64) void zstd_entropy_kernel(tyche_batch_t b, size_t first, size_t count, uint32_t in_cap,
                                                          uint32_t out_cap, Layout lay, uint8_t *ws, size_t ws_page,
                                                          int32_t *st, unsigned *ctr, bool use_jobs, bool fused,
                                                          bool defer_lit, bool lazy_stage) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    Work W;
    W.gsrc = nullptr;
    W.ghead = 0;
    W.gL = 0;
    W.wlo = W.whi = 0;
    W.win = nullptr;
    W.huf = (uint16_t *)(smem + lay.off_huf);
    W.hpair = smem + lay.off_hp;
    W.ll = (uint32_t *)(smem + lay.off_ll);
    W.of = (uint32_t *)(smem + lay.off_of);
    W.ml = (uint32_t *)(smem + lay.off_ml);
    W.wt = (uint32_t *)(smem + lay.off_wt);
    W.norm = (int16_t *)(smem + lay.off_norm);
    W.next = (uint16_t *)(smem + lay.off_next);
    W.w = smem + lay.off_w;
    uint8_t *stage = smem + lay.off_in;
    for (size_t j = blockIdx.x; j < count; j = ctr ? claim_page(ctr, lane) : j + gridDim.x) {
        const PageRef p = batch_page(b, first + j);
        int32_t rv;
        if (p.src_len > in_cap || p.dst_cap > out_cap) {
            rv = kResultTooLarge;
        } else {
            WAVE_SYNC();
            // (lazy staging, Work::gsrc: nothing staged yet but the zero pad)
            const uint32_t head = (uint32_t)((uintptr_t)p.src & 15u);
            uint8_t *in = stage + head;
            if (lane < kStreamPad / 4) lds_st32(in + p.src_len + lane * 4, 0u);
            WAVE_SYNC();
            W.in = in;
            W.gsrc = lazy_stage ? p.src : nullptr;
            W.ghead = head;
            W.gL = (int32_t)p.src_len;
            if (!lazy_stage) {
                (void)stage_in(p.src, p.src_len, stage, lane, kWave);
                WAVE_SYNC();
                if (lane < kStreamPad / 4) lds_st32(in + p.src_len + lane * 4, 0u);
                WAVE_SYNC();
            }
            Ent E = ent_of(ws + j * ws_page, in_cap, out_cap, fused);
            E.defer_lit = fused && defer_lit;
            SPROF_DECL
            // jobs first; a page whose jobs do not fit is redone with the chains inline (fused
            // layout: by the one-wave kernel after pass 2)
            for (bool jobs = use_jobs || fused;; jobs = false) {
                W.wlo = W.whi = 0;   // (a redo parses from the frame's start again)
                rv = decode_frame<true>(W, E, (int32_t)p.src_len, (int32_t)p.dst_cap, lane, jobs);
                if (rv == kRetryInline && fused) rv = kRetryFused;
                if (!(rv == kRetryInline && jobs)) break;
            }
            SPROF_MARK(1);
            SPROF_ADD(0, 1);
        }
        if (lane == 0) st[j] = rv;
    }
}

// Pass 2: window in LDS, entries from pass 1.
__global__ __launch_bounds__(64) void zstd_exec_kernel(tyche_batch_t b, size_t first, size_t count, uint32_t in_cap,
                                                       uint32_t out_cap, const uint8_t *ws, size_t ws_page,
                                                       const int32_t *st, unsigned *ctr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    for (size_t j = blockIdx.x; j < count; j = ctr ? claim_page(ctr, lane) : j + gridDim.x) {
        const PageRef p = batch_page(b, first + j);
        int32_t rv = st[j];
        if (rv >= 0) {
            const Ent E = ent_of(const_cast<uint8_t *>(ws) + j * ws_page, in_cap, out_cap, false);
            WAVE_SYNC();
#ifdef TYCHE_PROFILE
            unsigned long long _pt = clock64();
#endif
            rv = exec_page(smem, E, (int32_t)p.dst_cap, lane);
#ifdef TYCHE_PROFILE
            if (lane == 0) atomicAdd(&g_sdprof[5], clock64() - _pt);
#endif
            WAVE_SYNC();
            if (rv > 0) stage_out(p.dst, smem, (uint32_t)rv, lane, kWave);
        }
        if (lane == 0) b.results[first + j] = rv;
    }
}

}  // namespace

#ifdef TYCHE_PROFILE
extern "C" int tyche_debug_zstd_decode_profile(unsigned long long *host16, int reset) {
    if (reset) {
        unsigned long long z[16] = {0};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_sdprof), z, sizeof(z)) == hipSuccess ? 0 : 1;
    }
    return hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_sdprof), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : 1;
}
#endif

// TYCHE_ZSTD_SPLIT: 1 (default) two-pass decode where it fits and the batch has at
// least TYCHE_ZSTD_SPLIT_MIN (4096) pages, 0 the fused kernel.
// TYCHE_ZSTD_JOBS: 1 (default) sequence chains lane-per-page (zstd_seq_kernel), 0 inline.
// TYCHE_ZSTD_SCRATCH_MB bounds the pass-1 buffer; batches go through it in chunks.
static hipError_t launch_fused(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s) {
    const Layout lay = make_layout(in_cap, out_cap);
    if (lay.total > 160u * 1024u) return hipErrorInvalidValue;
    const size_t ncu = prepare_launch((const void *)zstd_decode_kernel);
    const size_t per_cu = waves_per_cu((const void *)zstd_decode_kernel, lay.total);
    const size_t grid = std::min<size_t>(b.count, ncu * per_cu);
    WorkCounter ctr(s, grid < b.count);
    if (!ctr.get()) return hipErrorOutOfMemory;
    hipLaunchKernelGGL(zstd_decode_kernel, dim3((unsigned)grid), dim3(kWave), lay.total, s, b, (size_t)0, b.count, in_cap,
                       out_cap, lay, ctr.get(), (const int32_t *)nullptr);
    return hipGetLastError();
}

// Pass 2 runs one page per lane from this many pages per batch (lane-per-page
// kernels need ~512 pages per CU in flight; below that the wave kernel's window
// in LDS wins).
constexpr long kExecLaneMin = 16384;

// TYCHE_ZSTD_SEQEXEC: 1 (default) pass 2 = zstd_seqexec_kernel (chains and
// execution fused, commands-only areas); 0 = zstd_seq_kernel + an execution kernel
// over sequence entries (lane per page: zstd_exec_lane_kernel, TYCHE_ZSTD_EXEC_RING
// 128 / 256; wave per page below TYCHE_ZSTD_EXEC_LANE_MIN pages: zstd_exec_kernel).
// TYCHE_ZSTD_SEQ_SLOTS 7 (default) / 6: the largest table logs pass 2 keeps in LDS
// (7: LL/ML 7, OF 6, 3 waves per CU; 6: 6 / 5, 5 waves per CU).
hipError_t launch_zstd_decode(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    // small batches (restores) take the one-launch kernel: the split's extra
    // launches cost more latency than its throughput gains on a few pages
    const long mn = knob("ZSTD_SPLIT_MIN", 4096);
    const size_t split_min = mn > 0 ? (size_t)mn : 4096;
    const bool split = knob("ZSTD_SPLIT", 1) != 0 && b.count >= split_min;
    const Layout l1 = make_layout(in_cap, out_cap, false);
    const Layout lf = make_layout(in_cap, out_cap);   // the one-wave kernel (leftovers of the fused layout)
    const bool use_jobs = knob("ZSTD_JOBS", 1) != 0;   // 0: sequence chains inline in pass 1
    const uint32_t lds2 = (out_cap + kWinPad + 15u) & ~15u;
    const long lmin = knob("ZSTD_EXEC_LANE_MIN", kExecLaneMin);
    const bool lane_exec = lmin >= 0 && b.count >= (size_t)lmin;
    const bool seqexec = lane_exec && use_jobs && knob("ZSTD_SEQEXEC", 1) != 0 && lf.total <= 160u * 1024u;
    const long ring = knob("ZSTD_EXEC_RING", 128);
    const bool slots6 = knob("ZSTD_SEQ_SLOTS", 7) == 6;
    // literal streams lane-per-stream (zstd_lit_kernel) between pass 1 and zstd_seqexec_kernel
    const long lit_groups = knob("ZSTD_LIT_LANES", 8);   // pages per wave: 8 / 16; 0 = streams in pass 1
    // TYCHE_ZSTD_LAZY_STAGE 0: pass 1 stages every frame whole (A/B; default 1: only the ranges it reads)
    const bool lazy_stage = knob("ZSTD_LAZY_STAGE", 1) != 0;
    const bool lit_lanes = seqexec && lit_groups > 0;
    const void *kl = lit_groups == 16 ? (const void *)zstd_lit_kernel<16> : (const void *)zstd_lit_kernel<8>;
    const uint32_t kgroups = lit_groups == 16 ? 16u : 8u;
    const void *kx = seqexec ? (slots6 ? (const void *)zstd_seqexec_kernel<128, 6> : (const void *)zstd_seqexec_kernel<128, 7>)
                     : ring == 256 ? (const void *)zstd_exec_lane_kernel<256>
                                   : (const void *)zstd_exec_lane_kernel<128>;
    const size_t lds_lane = seqexec ? 64u * (128u + 48u + 2u * (slots6 ? Slots<6>::cells : Slots<7>::cells))
                                    : 64u * ((ring == 256 ? 256u : 128u) + 48u);
    if (!split || l1.total > 160u * 1024u || (!lane_exec && lds2 > 160u * 1024u))
        return launch_fused(b, in_cap, out_cap, s);
    const size_t page_bytes = ent_page_bytes(in_cap, out_cap, seqexec);
    // pass 2's time per chunk is a page's chain (latency-bound, one lane per
    // page), so chunks are made as large as memory allows: 16 GiB or a quarter
    // of the free memory, whichever is less
    const long mb = knob("ZSTD_SCRATCH_MB", 0);
    size_t budget = (size_t)16 << 30;
    size_t free_b = 0, total_b = 0;
    if (b.count * page_bytes > ((size_t)1 << 30) && hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
        ((free_b += scratch_idle_bytes()), true) && free_b / 4 < budget)
        budget = free_b / 4;
    if (mb > 0) budget = (size_t)mb << 20;
    const size_t chunk = std::max<size_t>(1, std::min<size_t>(b.count, budget / page_bytes));
    const size_t st_bytes = (chunk * 4u + 255u) & ~(size_t)255u;
    ScratchLease ws(s, st_bytes + chunk * page_bytes + 64u);   // + the lane pass's literal over-read
    if (!ws.get()) return launch_fused(b, in_cap, out_cap, s);
    int32_t *st = (int32_t *)ws.get();
    uint8_t *ent = (uint8_t *)ws.get() + st_bytes;
    const size_t ncu = prepare_launch((const void *)zstd_entropy_kernel);
    (void)prepare_launch(lane_exec ? kx : (const void *)zstd_exec_kernel);
    // the leftovers launch of the one-wave kernel below runs at lf.total bytes of dynamic LDS
    // (~70 KiB at 32 KiB pages, above the 64 KiB default): its limit must be raised here too, and
    // before cuf is sized, whether or not launch_fused ran earlier in this process
    if (seqexec) (void)prepare_launch((const void *)zstd_decode_kernel);
    const size_t cu1 = waves_per_cu((const void *)zstd_entropy_kernel, l1.total);
    const size_t cu2 = lane_exec ? waves_per_cu(kx, lds_lane) : waves_per_cu((const void *)zstd_exec_kernel, lds2);
    const size_t cuf = seqexec ? waves_per_cu((const void *)zstd_decode_kernel, lf.total) : 0;
    for (size_t first = 0; first < b.count; first += chunk) {
        const size_t n = std::min(chunk, b.count - first);
        const size_t g1 = std::min<size_t>(n, ncu * cu1);
        {
            WorkCounter ctr(s, g1 < n);
            if (!ctr.get()) return hipErrorOutOfMemory;
            hipLaunchKernelGGL(zstd_entropy_kernel, dim3((unsigned)g1), dim3(kWave), l1.total, s, b, first, n, in_cap,
                               out_cap, l1, ent, page_bytes, st, ctr.get(), use_jobs, seqexec, lit_lanes, lazy_stage);
        }
        if (lit_lanes) {
            (void)prepare_launch(kl);
            size_t f = first, nn = n, pb = page_bytes;
            uint8_t *wsp = ent;
            int32_t *stp = st;
            void *args[] = {(void *)&b, &f, &nn, &in_cap, &out_cap, &wsp, &pb, &stp};
            (void)hipLaunchKernel(kl, dim3((unsigned)((n + kgroups - 1) / kgroups)), dim3(64), args,
                                  (size_t)kgroups * kHufCells * 2u + 256u, s);
        }
        if (!seqexec)
            hipLaunchKernelGGL(zstd_seq_kernel, dim3((unsigned)((n + kWave - 1) / kWave)), dim3(kWave), kSeqLds, s, b,
                               first, n, in_cap, out_cap, ent, page_bytes, st);
        if (lane_exec) {
            const size_t g2 = std::min<size_t>((n + 63) / 64, ncu * cu2);
            WorkCounter ctr(s, true);
            unsigned *cp = ctr.get();
            if (!cp) return hipErrorOutOfMemory;
            const uint8_t *wsp = ent;
            const int32_t *stp = st;
            size_t f = first, nn = n, pb = page_bytes;
            void *args[] = {(void *)&b, &f, &nn, &in_cap, &out_cap, &wsp, &pb, &stp, &cp};
            (void)hipLaunchKernel(kx, dim3((unsigned)g2), dim3(64), args, lds_lane, s);
        } else {
            const size_t g2 = std::min<size_t>(n, ncu * cu2);
            WorkCounter ctr(s, g2 < n);
            if (!ctr.get()) return hipErrorOutOfMemory;
            hipLaunchKernelGGL(zstd_exec_kernel, dim3((unsigned)g2), dim3(kWave), lds2, s, b, first, n, in_cap,
                               out_cap, (const uint8_t *)ent, page_bytes, (const int32_t *)st, ctr.get());
        }
        if (seqexec) {
            // the pages pass 1 left to the one-wave kernel (too many blocks or jobs for the
            // fused layout): every wave skips the others after one status read
            const size_t gf = std::min<size_t>((n + kWave - 1) / kWave, ncu * cuf);
            hipLaunchKernelGGL(zstd_decode_kernel, dim3((unsigned)gf), dim3(kWave), lf.total, s, b, first, n, in_cap,
                               out_cap, lf, (unsigned *)nullptr, (const int32_t *)st);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace tyche
