// zstd_encode.hip -- gfx950 encoder for zstd frames, the codec behind
// buffer__compress for ZSTD_COMPRESSOR_ID (src/buffer.c:203-212 -> ZSTD_compress
// level 1, src/zstd/zstd_compress.c:2721).  The output is a standard zstd frame
// that the reference's ZSTD_decompress (zstd_decompress.c:1459) restores
// bit-exactly; it is not required to be the bytes zstd 1.1.2 emits (SURVEY §8a
// A8).  Literals are Huffman-coded, the sequences get per-block FSE tables and
// all three repeat offsets (§8f rank 4); the parse (lz_parse.h) tries both
// leading repeat offsets beside the hash candidate.
//
// Frame layout (zstd_compress.c:2334-2376): magic, a single-segment frame
// header with the content size (no checksum, no dictionary), then blocks of at
// most kSeqCap sequences each (the last flagged).  Per block:
//   literals section   Huffman-compressed (1 or 4 streams, FSE-compressed
//                      weights; huf_literals below), else RLE or raw
//                      (ZSTD_noCompressLiterals, zstd_compress.c:406-428)
//   sequences section  nbSeq, the mode byte (per-block FSE tables from 64
//                      sequences on, predefined below) with their NCount
//                      headers, and the FSE bitstream written exactly as
//                      ZSTD_compressSequences does
//                      (zstd_compress.c:695-735): last sequence first through
//                      FSE_initCState2, the rest backwards with
//                      FSE_encodeSymbol OF, ML, LL then the LL, ML, OF extra
//                      bits, the three final states, the end mark
//                      (bitstream.h BIT_addBits / BIT_flushBits / BIT_closeCStream)
// A block whose encoding would not be smaller than its input is stored raw.
//
// One wave per page, looping over pages with the next page prefetched into
// registers.  The match finder is the shared parse (lz_parse.h).  Sequence
// codes and extra-bit values are computed lane-parallel; the FSE state chain
// is serial, so it runs as wave-uniform code over 64 sequences held in lanes
// (v_readlane), with each table held in one VGPR (huf::SmallCT), flushing each
// sequence's bytes with one 8-lane byte store.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "engine.h"
#include "lds_io.h"
#include "huf_enc.h"
#include "lz_parse.h"

namespace tyche {
namespace {

// Optional phase profile (diagnostic build only: -DTYCHE_PROFILE,
// tools/zstd_prof.py): shader cycles per phase summed by lane 0.
#ifdef TYCHE_PROFILE
__device__ unsigned long long g_seprof[16];
#define SPROF_DECL unsigned long long _pt = clock64();
#define SPROF_MARK(slot)                                                       \
    do {                                                                       \
        unsigned long long _n = clock64();                                     \
        if (lane == 0) atomicAdd(&g_seprof[slot], _n - _pt);                  \
        _pt = _n;                                                              \
    } while (0)
#define SPROF_ADD(slot, v) do { if (lane == 0) atomicAdd(&g_seprof[slot], (unsigned long long)(v)); } while (0)
#else
#define SPROF_DECL
#define SPROF_MARK(slot) do { } while (0)
#define SPROF_ADD(slot, v) do { } while (0)
#endif

using lzp::kHashSize;
#ifndef TYCHE_ZSTD_WAYS
#define TYCHE_ZSTD_WAYS 2   // candidates per hash bucket (lz_parse.h kWays)
#endif
constexpr int kZWays = TYCHE_ZSTD_WAYS;
constexpr uint32_t kTableSlots = lzp::table_slots<kZWays, true>();
using lzp::kWave;
constexpr uint32_t kPad = 64;
constexpr uint32_t kSeqCap = 1024;       // sequences buffered per block
constexpr uint32_t kHtab = 512;          // htab words
constexpr uint32_t kPrefetchVec = 16;

// ------------------------------------------------------------ predefined distributions
// zstd_internal.h:118-136 (LL, ML: log 6; OF: log 5), used below 64 sequences
__device__ __constant__ int16_t c_ll_norm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2,
                                                 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__device__ __constant__ int16_t c_ml_norm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__device__ __constant__ int16_t c_of_norm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1,
                                                 -1, -1};
__device__ __forceinline__ uint32_t hb(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// (code, extra bits) of one sequence -- ZSTD_seqToCodes (zstd_compress.c:535-556).
// LL_Code / ML_Code are evaluated with compares against the code bases
// (zstd_decompress.c:864-873) instead of table gathers.
struct SeqCode {
    uint32_t llc, mlc, ofc;          // codes
    uint32_t llv, mlv, ofv;          // extra-bit values (masked by BIT_addBits)
    uint32_t llb, mlb;               // extra-bit counts (ofc for offsets)
};
__device__ __forceinline__ SeqCode seq_code(uint32_t ll, uint32_t ml, uint32_t ofcode) {
    SeqCode c;
    const uint32_t m = ml - 3u;
    if (ll < 16u) {
        c.llc = ll;
        c.llb = 0;
    } else if (ll < 64u) {
        c.llc = 16u + (ll >= 18u) + (ll >= 20u) + (ll >= 22u) + (ll >= 24u) + (ll >= 28u) + (ll >= 32u) +
                (ll >= 40u) + (ll >= 48u);
        c.llb = 1u + (ll >= 24u) + (ll >= 32u) + (ll >= 48u);
    } else {
        c.llb = hb(ll);
        c.llc = c.llb + 19u;
    }
    if (m < 32u) {
        c.mlc = m;
        c.mlb = 0;
    } else if (m < 128u) {
        c.mlc = 32u + (m >= 34u) + (m >= 36u) + (m >= 38u) + (m >= 40u) + (m >= 44u) + (m >= 48u) + (m >= 56u) +
                (m >= 64u) + (m >= 80u) + (m >= 96u);
        c.mlb = 1u + (m >= 40u) + (m >= 48u) + (m >= 64u) + (m >= 96u);
    } else {
        c.mlb = hb(m);
        c.mlc = c.mlb + 36u;
    }
    c.ofc = hb(ofcode);
    c.llv = ll & ((1u << c.llb) - 1u);
    c.mlv = m & ((1u << c.mlb) - 1u);
    c.ofv = ofcode & ((1u << c.ofc) - 1u);
    return c;
}

// ------------------------------------------------------------ block emission
// The sequence map of a page's sequence region (split encode; seq_slot below)
struct SeqMap {
    uint32_t c1, c2, c3, slice;
};
// The literal map of a page's literal region (split encode; lit_pos below)
struct LitMap {
    uint32_t w[5];
};

// Sequences of the current block live in LDS: seq[i] = (ll | off << 16, ml | rc << 16),
// rc = the repeat code chosen at emission (0: the offset is sent as off + 3).
struct Enc {
    const uint8_t *in;   // page (LDS)
    uint8_t *dst;        // output (global)
    uint32_t cap, op;    // capacity, bytes written
    uint2 *seq;          // kSeqCap sequences
    uint32_t nseq;       // sequences in the current block
    uint32_t bstart;     // first page byte of the current block
    uint32_t cursor;     // end of the last buffered sequence's match
    uint8_t *map;        // 64-byte owner map
    uint32_t *htab;      // 512 entries: literal histogram, then Huffman code | length << 16 (all 512:
                         // scratch of the Huffman construction)
    uint8_t *wts;        // 256 Huffman weights
    uint32_t *stage;     // 128 dwords of pending stream bits (the parse's record area, free here)
    uint32_t r0, r1, r2; // the decoder's repeat offsets after the blocks emitted so far (initial {1, 4, 8},
                         // zstd_internal.h:73); raw blocks leave them unchanged
    bool fail;
    uint8_t *area;       // split encode: the page's work area (nullptr: the chain runs here)
    uint32_t nblk, nrec; // blocks and sequence records written to the area
    uint32_t rec_cap;
    uint32_t logcap;     // 7: LL / OF / ML table logs FSE_optimalTableLog's, capped at 7 / 6 / 7; 6: fixed 6 / 5 / 6
    const uint32_t *psum;   // split encode: the parse block's literal bytes, span and extra bits (nullptr: summed here)
    const uint8_t *lit;     // split encode: the literal region from pass A1 (nullptr: literals gathered from in);
    LitMap lmap;            //   literal j of the block at lit[lit_pos(lmap, lofs + j)]
    uint32_t lofs;
    uint2 *sreg;            // split encode: the sequence region, sequence `sfirst + i` of the block at
    SeqMap smap;            //   sreg[seq_slot(smap, sfirst + i)] (e.seq is not used)
    uint32_t sfirst;
    __device__ uint32_t nrec_cap() const { return rec_cap; }
};

// ------------------------------------------------------------ split encode
// The FSE chain of a block is serial, and at one wave per page it ran as
// wave-uniform code at the parse's residency (3 waves per CU for 32 KiB pages).
// Split: pass A1 (zstd_parse_kernel) runs the parse alone -- LDS = page + hash
// table, 4 waves per CU at 32 KiB -- and writes the sequences and the block
// boundaries to the page's area; pass A2 (zstd_block_kernel, a few KiB of LDS)
// emits each block with the FSE bitstream's upper bound left open, plus the
// sequences' codes and the block's three tables; pass B (zstd_fse_kernel, one
// page per lane) writes the bitstreams into the gaps; pass C (zstd_pack_kernel)
// closes the gaps and patches the block headers.  Capacity decisions use the
// bounds, so a page that pass A2 accepts always fits.
constexpr uint32_t kMaxBlk = 24;                 // blocks per page (> 65535 / 4 / 960 + 1; kZBlk below)
constexpr uint32_t kBlkWords = 8;                // g_start, g_len, pre, fse (bound, then actual), n, rec, tab, flags
// Sequence table logs: FSE_optimalTableLog capped at these (emit_block)
constexpr uint32_t kStateBits = 7u + 6u + 7u;   // bits one sequence's three states emit at most (LL, OF, ML logs <= 7 / 6 / 7)
// one table, packed for pass B's LDS copy: per symbol deltaNbBits | (deltaFindState + 128) << 19
// (dnb < 2^19: log <= 7, every symbol's maxBitsOut >= 1; dfs in [-128, 127]), word 63 the
// table log, then the 128 stateTable bytes (values < 256)
constexpr uint32_t kCtWords = 64u + 32u;
constexpr uint32_t kTabBytes = 3u * kCtWords * 4u;   // 1152
// parse blocks: page start, page end, first sequence, sequences, then the block's literal bytes,
// sequence span (page bytes) and extra bits at raw offsets, which pass A2 would otherwise read the
// sequence list again for (emit_block's sizes; round 6), one word spare
constexpr uint32_t kPblkWords = 8;
constexpr uint32_t kAreaHdr = 48u;   // [0] emitted blocks, [1] parse blocks, [2..3] sequence map, [4..8] literal map
constexpr uint32_t kAreaHead = kAreaHdr + kMaxBlk * kBlkWords * 4u + kMaxBlk * kPblkWords * 4u;
// area: [0] emitted blocks, [1] parse blocks, [2..3] the sequence map | block records | parse
//       blocks | tables | the parse's sequences (16 B per sequence of room: the split parse's
//       per-part slices, where they stay -- the map below; pass A2 overwrites each with its
//       record for pass B as it reads it) | the page's literals in page order (8 B per
//       sequence of room).  Round 6: pass A1 copies the literals out of the page it holds in
//       LDS, so that pass A2 reads them once and contiguously instead of gathering them from
//       the page in HBM, and leaves its parts' sequences where it wrote them instead of
//       joining them into one list (one write and one read of every sequence less).
__host__ __device__ inline uint32_t enc_rec_cap(uint32_t in_cap) { return in_cap / 4u + 64u; }
__host__ __device__ inline size_t enc_area_bytes(uint32_t in_cap) {
    return ((size_t)kAreaHead + (size_t)kMaxBlk * kTabBytes + (size_t)enc_rec_cap(in_cap) * 24u + 255u) & ~(size_t)255u;
}
__device__ __forceinline__ uint32_t *area_blk(uint8_t *a, uint32_t k) { return (uint32_t *)(a + kAreaHdr) + k * kBlkWords; }
__device__ __forceinline__ uint32_t *area_pblk(uint8_t *a, uint32_t k) {
    return (uint32_t *)(a + kAreaHdr + kMaxBlk * kBlkWords * 4u) + k * kPblkWords;
}
__device__ __forceinline__ uint32_t *area_tab(uint8_t *a, uint32_t k) {
    return (uint32_t *)(a + kAreaHead + (size_t)k * kTabBytes);
}
__device__ __forceinline__ uint4 *area_rec(uint8_t *a) { return (uint4 *)(a + kAreaHead + (size_t)kMaxBlk * kTabBytes); }
__device__ __forceinline__ uint2 *area_seq(uint8_t *a, uint32_t rec_cap) { return (uint2 *)(area_rec(a) + rec_cap); }
__device__ __forceinline__ uint8_t *area_lit(uint8_t *a, uint32_t rec_cap) { return (uint8_t *)area_seq(a, rec_cap); }   // (8 rec_cap > in_cap)
// Sequence i of a page (in page order) lives in part k's slice of the sequence region: parts
// 0..3 start at 0, slice, 2 slice, 3 slice and hold [0, c1), [c1, c2), [c2, c3), [c3, ...)
// (one-wave parse: one part, c1 = c2 = c3 = 0xFFFF).  Kept in area words 2..3 as 16-bit fields.
__device__ __forceinline__ SeqMap seq_map(const uint8_t *a, bool uniform) {   // uniform: one page per wave
    uint32_t w2 = ((const uint32_t *)a)[2], w3 = ((const uint32_t *)a)[3];
    if (uniform) {
        w2 = __builtin_amdgcn_readfirstlane(w2);
        w3 = __builtin_amdgcn_readfirstlane(w3);
    }
    return SeqMap{w2 & 0xFFFFu, w2 >> 16, w3 & 0xFFFFu, w3 >> 16};
}
__device__ __forceinline__ void put_seq_map(uint8_t *a, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t slice) {
    ((uint32_t *)a)[2] = c1 | (c2 << 16);
    ((uint32_t *)a)[3] = c3 | (slice << 16);
}
// The page's literals (in page order: literal j of the page) lie in the literal region in up to
// five runs (split parse: each part's own literals where its part starts, behind the bytes its
// first run was extended back over, then the literals after the last match): run k starts at
// literal c_k and region byte s_k; area words 4..8 hold c_k | s_k << 16 (c_k = 0xFFFF: unused).
__device__ __forceinline__ LitMap lit_map(const uint8_t *a) {
    LitMap m;
#pragma unroll
    for (int k = 0; k < 5; k++) m.w[k] = __builtin_amdgcn_readfirstlane(((const uint32_t *)a)[4 + k]);
    return m;
}
__device__ __forceinline__ uint32_t lit_pos(const LitMap &m, uint32_t j) {
    uint32_t p = j;
#pragma unroll
    for (int k = 0; k < 5; k++)
        if (j >= (m.w[k] & 0xFFFFu)) p = j - (m.w[k] & 0xFFFFu) + (m.w[k] >> 16);
    return p;
}
__device__ __forceinline__ uint32_t seq_slot(const SeqMap &m, uint32_t i) {
    return i >= m.c3 ? i - m.c3 + 3u * m.slice : i >= m.c2 ? i - m.c2 + 2u * m.slice : i >= m.c1 ? i - m.c1 + m.slice : i;
}

// Copies the literal runs [ls, ls + ll) of the wave's lanes, in lane order, from the page in
// LDS to dst[0, sum of ll), 64 bytes a step; returns the sum of ll.  Byte j's run is the last
// one starting at or before j.  With `map` (64 dwords of LDS): the runs starting in the step
// mark their position there with their source delta (page position - literal position), and a
// prefix max over the map gives each byte its run -- one LDS round trip a step; without it, a
// binary search over the lanes' exclusive prefix (six dependent lane permutes a step; it cost
// the split parse 9 % of its time, round 6).  Lanes with ll = 0 are never a byte's run.
__device__ __forceinline__ uint32_t copy_runs(const uint8_t *in, uint32_t ls, uint32_t ll, uint8_t *dst, uint32_t lane,
                                              uint32_t *map) {
    const uint32_t inc = (uint32_t)wave_incl_sum((int32_t)ll), excl = inc - ll;
    const uint32_t total = rdlane(inc, kWave - 1);
    if (map) {
        uint32_t carry = 0;   // the delta of the run the previous step ended in
        for (uint32_t j0 = 0; j0 < total; j0 += kWave) {
            map[lane] = 0;
            __builtin_amdgcn_wave_barrier();
            if (ll && excl >= j0 && excl < j0 + kWave) map[excl - j0] = ((excl - j0 + 1u) << 16) | (ls - excl);
            __builtin_amdgcn_wave_barrier();
            const uint32_t k = (uint32_t)wave_incl_max((int32_t)map[lane]);
            const uint32_t d = k ? (k & 0xFFFFu) : carry;
            const uint32_t j = j0 + lane;
            if (j < total) dst[j] = in[j + d];
            carry = rdlane(d, kWave - 1);
            __builtin_amdgcn_wave_barrier();
        }
        return total;
    }
    for (uint32_t j0 = 0; j0 < total; j0 += kWave) {
        const uint32_t j = j0 + lane;
        uint32_t o = 0;
#pragma unroll
        for (uint32_t step = kWave / 2; step; step >>= 1) {
            const uint32_t c = o + step;
            if ((uint32_t)__shfl((int)excl, (int)c) <= j) o = c;
        }
        const uint32_t src = (uint32_t)__shfl((int)ls, (int)o) + j - (uint32_t)__shfl((int)excl, (int)o);
        if (j < total) dst[j] = in[src];
    }
    return total;
}
// a block record (lane 0)
__device__ __forceinline__ void put_blk(Enc &e, uint32_t g_start, uint32_t g_len, uint32_t pre, uint32_t fse, uint32_t n,
                                        uint32_t rec, uint32_t flags, uint32_t lane) {
    if (lane == 0) {
        uint32_t *B = area_blk(e.area, e.nblk);
        B[0] = g_start;
        B[1] = g_len;
        B[2] = pre;
        B[3] = fse;
        B[4] = n;
        B[5] = rec;
        B[6] = e.nblk;
        B[7] = flags;
    }
    e.nblk++;
}

// Codes of sequence i of the block, after resolve_repeats.
__device__ __forceinline__ SeqCode seq_code_at(const Enc &e, uint32_t i) {
    const uint2 r = e.seq[i];
    const uint32_t ll = r.x & 0xFFFFu, off = r.x >> 16, rc = r.y >> 16;
    return seq_code(ll, r.y & 0xFFFFu, rc ? rc : off + 3u);
}

// Pass A2's record of a sequence for pass B, 8 bytes (round 6; 16-byte records of codes and
// extra-bit values before, 2x the HBM bytes between the passes; in place of the sequence since
// round 6): the literal length, the match
// length - 3 and the offset code (pages < 64 KiB: 16, 16 and 17 bits) with the LL and ML codes,
//   x = ll | llc << 16 | mlc << 22 | (ofcode >> 16) << 28,  y = (ml - 3) | (ofcode & 0xFFFF) << 16;
// pass B derives the extra-bit counts and values as seq_code does (ZSTD_seqToCodes,
// zstd_compress.c:535-556).  Written by resolve_repeats.
__device__ __forceinline__ SeqCode seq_record_codes(uint2 r) {
    SeqCode c;
    const uint32_t ll = r.x & 0xFFFFu, m = r.y & 0xFFFFu, ofcode = (r.y >> 16) | ((r.x >> 28) << 16);
    c.llc = (r.x >> 16) & 63u;
    c.mlc = (r.x >> 22) & 63u;
    c.llb = ll < 16u ? 0u : ll < 64u ? 1u + (ll >= 24u) + (ll >= 32u) + (ll >= 48u) : hb(ll);
    c.mlb = m < 32u ? 0u : m < 128u ? 1u + (m >= 40u) + (m >= 48u) + (m >= 64u) + (m >= 96u) : hb(m);
    c.ofc = hb(ofcode);
    c.llv = ll & ((1u << c.llb) - 1u);
    c.mlv = m & ((1u << c.mlb) - 1u);
    c.ofv = ofcode & ((1u << c.ofc) - 1u);
    return c;
}

// Offset_Value of every sequence of the block against the repeat history
// (ZSTD_decodeSequence's rules, zstd_decompress.c:897-915): with a literal
// length, 1/2/3 name repeat offsets 1/2/3; without one, 1/2 name repeat offsets
// 2/3 (zstd's "immediate repcode", zstd_compress.c:985-994).  Using repeat
// offset 1 with a literal length changes nothing (event E), repeat 2 swaps the
// first two, anything else shifts the history.  The scan is lane-parallel:
//   r0 before i = off[i-1] (every case leaves the offset just used in front);
//   r1 before i = off[p-1] for the last p < i that is not an E event (E keeps
//                 r1, every other case sets it to the previous r0);
//   r2 before i = r1 before q for the last q < i that shifted (!E and
//                 off[q] != r1 before q; swaps and E keep r2).
// Returns the history after the block through h0..h2 (committed only if the
// block is emitted compressed: raw blocks leave the decoder's history alone).
// The same pass counts the LL / ML / OF codes into e.htab (0 / 64 / 128, zeroed by the
// caller) and hands each sequence on: split encode (R = e.sreg), its 8-byte record for pass B
// in the sequence's own slot; one-kernel encode, its repeat code into e.seq[i].y for the
// bitstream below
// (round 6: one pass over the block's sequences instead of three -- the repeat codes
// written back, the histogram and the records each read the list again)
__device__ __forceinline__ void resolve_repeats(const Enc &e, uint32_t n, uint32_t lane, uint32_t &h0, uint32_t &h1,
                                                uint32_t &h2, uint2 *R) {
    uint32_t c0 = e.r0, c1 = e.r1, c2 = e.r2;
    const uint64_t below = (1ull << lane) - 1ull;
    for (uint32_t g = 0; g < n; g += kWave) {
        const uint32_t i = g + lane;
        uint2 *sp = R ? e.sreg + seq_slot(e.smap, e.sfirst + min(i, n - 1u)) : e.seq + i;
        const uint2 r = i < n ? *sp : make_uint2(0u, 0u);
        const uint32_t ll = r.x & 0xFFFFu, off = r.x >> 16;
        const uint32_t up = (uint32_t)__shfl((int)off, (int)(lane ? lane - 1u : 0u));
        const uint32_t r0b = lane ? up : c0;
        const bool ev = ll > 0u && off == r0b;
        const uint64_t ne = __ballot(!ev) & below;
        const int p = ne ? 63 - __builtin_clzll(ne) : 0;
        const uint32_t tp = (uint32_t)__shfl((int)r0b, p);
        const uint32_t r1b = ne ? tp : c1;
        const bool sh = !ev && off != r1b;
        const uint64_t sm = __ballot(sh) & below;
        const int q = sm ? 63 - __builtin_clzll(sm) : 0;
        const uint32_t tq = (uint32_t)__shfl((int)r1b, q);
        const uint32_t r2b = sm ? tq : c2;
        uint32_t rc;
        if (ll) rc = off == r0b ? 1u : off == r1b ? 2u : off == r2b ? 3u : 0u;
        else rc = off == r1b ? 1u : off == r2b ? 2u : 0u;
#ifdef TYCHE_NO_RESOLVE
        rc = 0;   // timing ablation: raw offsets only
#endif
        if (i < n) {
            const uint32_t ml = r.y & 0xFFFFu, ofcode = rc ? rc : off + 3u;
            const SeqCode c = seq_code(ll, ml, ofcode);
            atomicAdd(&e.htab[c.llc], 1u);
            atomicAdd(&e.htab[64u + c.mlc], 1u);
            atomicAdd(&e.htab[128u + c.ofc], 1u);
            if (R) *sp = make_uint2(ll | (c.llc << 16) | (c.mlc << 22) | ((ofcode >> 16) << 28), (ml - 3u) | (ofcode << 16));
            else sp->y = ml | (rc << 16);
        }
        // the history after the group's last sequence
        const uint32_t last = min(n - g, kWave) - 1u;
        const uint32_t o_l = rdlane(off, last), r0_l = rdlane(r0b, last), r1_l = rdlane(r1b, last),
                       r2_l = rdlane(r2b, last);
        const bool ev_l = rdlane((uint32_t)ev, last) != 0u, sh_l = rdlane((uint32_t)sh, last) != 0u;
        c0 = o_l;
        c1 = ev_l ? r1_l : r0_l;
        c2 = sh_l ? r1_l : r2_l;
    }
    h0 = c0;
    h1 = c1;
    h2 = c2;
}

// Calls f(j, byte) for every literal j of the block (literal-section order),
// 64 per step: literal j belongs to the last run starting at or before it
// (sequences 0..n-1, then the trailing literals as run n).
template <typename F>
__device__ void for_each_literal(const Enc &e, uint32_t n, uint32_t trail, uint32_t lane, F &&f) {
    uint32_t lo = 0, pstart = e.bstart;   // literal-section offset / page position of this group
    for (uint32_t g = 0; g <= n; g += kWave) {
        const uint32_t i = g + lane;
        uint32_t ll = 0, ml = 0;
        if (i < n) {
            const uint2 r = e.seq[i];
            ll = r.x & 0xFFFFu;
            ml = r.y & 0xFFFFu;
        } else if (i == n) {
            ll = trail;
        }
        const bool run = i <= n;
        const int32_t li = wave_incl_sum((int32_t)ll), si = wave_incl_sum((int32_t)(ll + ml));
        const uint32_t rlo = lo + (uint32_t)li - ll;                   // run start in the literal section
        const uint32_t rsrc = pstart + (uint32_t)si - (ll + ml);       // run start in the page
        const uint32_t glen = rdlane((uint32_t)li, kWave - 1);
        for (uint32_t j0 = 0; j0 < glen; j0 += kWave) {
            const uint32_t j = lo + j0 + lane;
            const uint64_t before = __ballot(run && ll && rlo <= lo + j0);
            const int32_t owner0 = before ? 63 - (int32_t)__builtin_clzll(before) : 0;
            e.map[lane] = 0xFF;
            __builtin_amdgcn_wave_barrier();
            if (run && ll && rlo > lo + j0 && rlo < lo + j0 + kWave) e.map[rlo - lo - j0] = (uint8_t)lane;
            __builtin_amdgcn_wave_barrier();
            const uint32_t mv = e.map[lane];
            const uint32_t owner = (uint32_t)max(wave_incl_max(mv == 0xFF ? -1 : (int32_t)mv), owner0);
            const uint32_t orlo = __shfl(rlo, owner), orsrc = __shfl(rsrc, owner);
            if (j0 + lane < glen) f(j, (uint32_t)e.in[orsrc + (j - orlo)]);
            __builtin_amdgcn_wave_barrier();
        }
        lo += glen;
        pstart += rdlane((uint32_t)si, kWave - 1);
    }
}

constexpr uint32_t kHufMinLit = 64;      // fewer literals stay raw (ZSTD_compressLiterals' minimum is 63)
constexpr uint32_t kHufMaxBits = 11;     // HUF_TABLELOG_DEFAULT

// Huffman-compressed literals section (ZSTD_compressLiterals, zstd_compress.c:459-514,
// with HUF_compress4X / 1X_usingCTable): the literals are first scattered to
// the tail of the output buffer as scratch while an LDS histogram is built;
// after the code is chosen the streams are written at o, below the scratch.
// Returns the section size, or 0 when raw literals are to be used instead.
__device__ uint32_t huf_literals(Enc &e, uint32_t n, uint32_t trail, uint32_t lit_total, uint32_t o, uint32_t lane) {
    const uint32_t lh = 3u + (lit_total >= 1024u) + (lit_total >= 16384u);
    const bool single = lit_total < 256u;
    if (e.cap < lit_total || e.cap - lit_total < o + lh + 272u) return 0;   // room for header + weights below the scratch
    const uint32_t scr = e.cap - lit_total;
    SPROF_DECL
    // ---- pass 1: scatter to scratch, histogram
    for (uint32_t k = lane; k < 256u; k += kWave) e.htab[k] = 0;
    __builtin_amdgcn_wave_barrier();
    uint8_t *dst = e.dst;
    uint32_t *hist = e.htab;
    if (e.lit) {   // split encode: the literals are in the area already (no scratch copy)
        for (uint32_t j = lane; j < lit_total; j += kWave) atomicAdd(&hist[e.lit[lit_pos(e.lmap, e.lofs + j)]], 1u);
    } else {
        for_each_literal(e, n, trail, lane, [&](uint32_t j, uint32_t v) {
            dst[scr + j] = (uint8_t)v;
            atomicAdd(&hist[v], 1u);
        });
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");   // scratch stores visible, L1 invalidated
    __builtin_amdgcn_wave_barrier();
    uint32_t c[4], l[4], code[4];
#pragma unroll
    for (int j = 0; j < 4; j++) c[j] = e.htab[lane + 64u * j];
    __builtin_amdgcn_wave_barrier();   // htab (now in c) is the Huffman construction's scratch
    SPROF_MARK(10);   // scatter + histogram
    const uint32_t maxlen = huf::code_lengths(c, lit_total, kHufMaxBits, l, lane, e.htab);
    SPROF_MARK(11);   // code lengths
    if (maxlen == 0) {
        // a single distinct byte: RLE literals (set_rle)
        const uint32_t fl = 1u + (lit_total > 31u) + (lit_total > 4095u);
        uint32_t h;
        if (fl == 1u) h = 1u | (lit_total << 3);
        else if (fl == 2u) h = 1u | (1u << 2) | (lit_total << 4);
        else h = 1u | (3u << 2) | (lit_total << 4);
        int32_t sym = -1;
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (c[j]) sym = (int32_t)(lane + 64u * j);
        sym = huf::wave_max(sym);
        if (lane < fl) e.dst[o + lane] = (uint8_t)(h >> (8u * lane));
        if (lane == 0) e.dst[o + fl] = (uint8_t)sym;
        return fl + 1u;
    }
    int32_t msv = -1;
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (c[j]) msv = (int32_t)(lane + 64u * j);
    const uint32_t max_sv = (uint32_t)huf::wave_max(msv);
    // ---- weights of symbols 0..max_sv-1 (the last one is implied), HUF_writeCTable
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t sv = lane + 64u * j;
        e.wts[sv] = (uint8_t)(l[j] ? maxlen + 1u - l[j] : 0u);
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t wpos = o + lh;
    uint32_t whdr;
    const uint32_t hs = huf::compress_weights(e.wts, max_sv, e.dst, wpos + 1u, lane);
    if (hs > 1u && hs < 128u) {
        if (lane == 0) e.dst[wpos] = (uint8_t)hs;
        whdr = hs + 1u;
    } else if (max_sv <= 128u) {
        // raw 4-bit weights
        if (lane == 0) e.dst[wpos] = (uint8_t)(127u + max_sv);
        for (uint32_t k = lane; 2u * k < max_sv; k += kWave) {
            const uint32_t a = e.wts[2u * k], b = 2u * k + 1u < max_sv ? e.wts[2u * k + 1u] : 0u;
            e.dst[wpos + 1u + k] = (uint8_t)((a << 4) | b);
        }
        whdr = (max_sv + 1u) / 2u + 1u;
    } else {
        return 0;
    }
    // ---- size check against the raw form and the scratch
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) bits += c[j] * l[j];
    const uint32_t total_bits = huf::wave_sum(bits);
    const uint32_t nst = single ? 1u : 4u;
    const uint32_t bound = whdr + (single ? 0u : 6u) + total_bits / 8u + 2u * nst;
    const uint32_t min_gain = (lit_total >> 6) + 2u;
    if (bound + min_gain >= lit_total || o + lh + bound > scr) return 0;
    // ---- codes: htab[s] = code | length << 16
    huf::canonical_codes(l, maxlen, code, lane);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 4; j++) e.htab[lane + 64u * j] = code[j] | (l[j] << 16);
    __builtin_amdgcn_wave_barrier();
    SPROF_MARK(12);   // weights, size check, codes
    // ---- streams: symbols last to first, bits LSB first (HUF_compress1X_usingCTable), end mark
    uint32_t sp = wpos + whdr + (single ? 0u : 6u);
    const uint32_t seg = (lit_total + 3u) / 4u;
    auto lit_at = [&](uint32_t j) -> uint32_t { return e.lit ? e.lit[lit_pos(e.lmap, e.lofs + j)] : e.dst[scr + j]; };
    for (uint32_t st = 0; st < nst; st++) {
        const uint32_t a = single ? 0u : st * seg;
        const uint32_t bnd = single ? lit_total : (st == 3u ? lit_total : min(lit_total, (st + 1u) * seg));
        const uint32_t s0 = sp;
        uint32_t nbits = 0;
        for (uint32_t k = lane; k < 128u; k += kWave) e.stage[k] = 0;
        __builtin_amdgcn_wave_barrier();
        for (uint32_t k0 = 0; a + k0 < bnd; k0 += kWave) {
            const bool act = a + k0 + lane < bnd;
            uint32_t ent = 0;
            if (act) ent = e.htab[lit_at(bnd - 1u - (k0 + lane))];
            const uint32_t len = ent >> 16, cv = ent & 0xFFFFu;
            const int32_t bi = wave_incl_sum((int32_t)len);
            const uint32_t b = nbits + (uint32_t)bi - len;
            if (len) {
                const uint32_t w = b >> 5, sh = b & 31u;
                atomicOr(&e.stage[w], cv << sh);
                if (sh + len > 32u) atomicOr(&e.stage[w + 1u], cv >> (32u - sh));
            }
            __builtin_amdgcn_wave_barrier();
            nbits += rdlane((uint32_t)bi, kWave - 1);
            // drain the complete bytes, keep the partial one in word 0
            const uint32_t nb = nbits >> 3;
            const uint8_t *sb = (const uint8_t *)e.stage;
            for (uint32_t j = lane; j < nb; j += kWave) e.dst[sp + j] = sb[j];
            const uint32_t part = (nbits & 7u) ? (uint32_t)sb[nb] : 0u;
            __builtin_amdgcn_wave_barrier();
            const uint32_t used = (nbits + 31u) >> 5;
            for (uint32_t w = lane; w <= used && w < 128u; w += kWave) e.stage[w] = w == 0 ? part : 0u;
            __builtin_amdgcn_wave_barrier();
            sp += nb;
            nbits &= 7u;
        }
        // BIT_closeCStream: end mark, last partial byte
        const uint32_t last = (e.stage[0] & ((1u << nbits) - 1u)) | (1u << nbits);
        if (lane == 0) e.dst[sp] = (uint8_t)last;
        sp += 1u;
        if (!single && st < 3u) {
            const uint32_t ssz = sp - s0;
            if (lane < 2) e.dst[wpos + whdr + 2u * st + lane] = (uint8_t)(ssz >> (8u * lane));
        }
        __builtin_amdgcn_wave_barrier();
    }
    SPROF_MARK(13);   // streams
    const uint32_t clit = sp - (o + lh);
    // ---- literals section header (set_compressed)
    if (lh == 3u) {
        const uint32_t h = 2u | ((single ? 0u : 1u) << 2) | (lit_total << 4) | (clit << 14);
        if (lane < 3) e.dst[o + lane] = (uint8_t)(h >> (8u * lane));
    } else if (lh == 4u) {
        const uint32_t h = 2u | (2u << 2) | (lit_total << 4) | (clit << 18);
        if (lane < 4) e.dst[o + lane] = (uint8_t)(h >> (8u * lane));
    } else {
        const uint64_t h = 2ull | (3ull << 2) | ((uint64_t)lit_total << 4) | ((uint64_t)clit << 22);
        if (lane < 5) e.dst[o + lane] = (uint8_t)(h >> (8u * lane));
    }
    return sp - o;
}

// Writes one block covering page bytes [s.bstart, bend) with the buffered
// sequences; `last` sets Last_Block.  Returns false if it does not fit.
__device__ __forceinline__ bool emit_block(Enc &e, uint32_t bend, bool last, uint32_t lane) {
    SPROF_DECL
    const uint32_t n = e.nseq, blen = bend - e.bstart;
    // ---- per-sequence sizes (lane-parallel over 64-sequence groups; the split parse sums them)
    uint32_t lit_sum = 0, span = 0, xbits = 0;
    if (e.psum) {
        lit_sum = __builtin_amdgcn_readfirstlane(e.psum[0]);
        span = __builtin_amdgcn_readfirstlane(e.psum[1]);
        xbits = __builtin_amdgcn_readfirstlane(e.psum[2]);
    }
    for (uint32_t g = 0; !e.psum && g < n; g += kWave) {
        const uint32_t i = g + lane;
        uint32_t ll = 0, ml = 0, xb = 0;
        if (i < n) {
            const uint2 r = e.seq[i];
            ll = r.x & 0xFFFFu;
            ml = r.y & 0xFFFFu;
            const SeqCode c = seq_code(ll, ml, (r.x >> 16) + 3u);   // bound: no repeat offsets
            xb = c.llb + c.mlb + c.ofc;
        }
        lit_sum += rdlane((uint32_t)wave_incl_sum((int32_t)ll), kWave - 1);
        span += rdlane((uint32_t)wave_incl_sum((int32_t)(ll + ml)), kWave - 1);
        xbits += rdlane((uint32_t)wave_incl_sum((int32_t)xb), kWave - 1);
    }
    const uint32_t trail = bend - (e.bstart + span);       // literals after the last match
    const uint32_t lit_total = lit_sum + trail;
    const uint32_t fl = 1u + (lit_total > 31u) + (lit_total > 4095u);
    const uint32_t nsh = n < 0x7Fu ? 1u : (n < 0x7F00u ? 2u : 3u);
    // upper bound of the FSE bitstream: every state emits at most its table log
    const uint32_t fse_bound = n ? (n * kStateBits + xbits + kStateBits + 8u + 7u) / 8u + 1u : 0u;
    const uint32_t comp_bound = fl + lit_total + nsh + (n ? 1u + 3u * 48u : 0u) + fse_bound;   // + NCount headers
    const uint32_t hdr = e.op;                              // block header position
    if (comp_bound >= blen) {
        // ---- raw block (Block_Type 0): header + the page bytes
        if (e.op + 3u + blen > e.cap) return false;
        if (e.area && e.nblk >= kMaxBlk) return false;
        const uint32_t bh = (last ? 1u : 0u) | (0u << 1) | (blen << 3);
        if (lane < 3) e.dst[hdr + lane] = (uint8_t)(bh >> (8u * lane));
        for (uint32_t j = lane; j < blen; j += kWave) e.dst[hdr + 3u + j] = e.in[e.bstart + j];
        if (e.area) put_blk(e, hdr, 3u + blen, blen, 0u, 0u, 0u, last ? 1u : 0u, lane);
        e.op += 3u + blen;
        return true;
    }
    if (e.op + 3u + comp_bound > e.cap) return false;
    if (e.area && (e.nblk >= kMaxBlk || e.nrec + n > e.nrec_cap())) return false;
    uint32_t o = hdr + 3u;
    // ---- literals section: Huffman-compressed when it pays, else raw (ZSTD_noCompressLiterals)
    SPROF_MARK(2);
    uint32_t lsec = lit_total >= kHufMinLit ? huf_literals(e, n, trail, lit_total, o, lane) : 0u;
    if (lsec == 0) {
        uint32_t h;
        if (fl == 1u) h = lit_total << 3;
        else if (fl == 2u) h = (1u << 2) | (lit_total << 4);
        else h = (3u << 2) | (lit_total << 4);
        if (lane < fl) e.dst[o + lane] = (uint8_t)(h >> (8u * lane));
        uint8_t *dst = e.dst;
        const uint32_t lo0 = o + fl;
        if (e.lit) {
            for (uint32_t j = lane; j < lit_total; j += kWave) dst[lo0 + j] = e.lit[lit_pos(e.lmap, e.lofs + j)];
        } else {
            for_each_literal(e, n, trail, lane, [&](uint32_t j, uint32_t v) { dst[lo0 + j] = (uint8_t)v; });
        }
        lsec = fl + lit_total;
    }
    o += lsec;
    SPROF_MARK(3);
    // ---- sequences section header
    if (lane < nsh) {
        uint32_t h;
        if (nsh == 1u) h = n;
        else if (nsh == 2u) h = ((n >> 8) + 0x80u) | ((n & 0xFFu) << 8);
        else h = 0xFFu | ((n - 0x7F00u) << 8);
        e.dst[o + lane] = (uint8_t)(h >> (8u * lane));
    }
    o += nsh;
    uint32_t h0 = e.r0, h1 = e.r1, h2 = e.r2;
    if (n) {
        // ---- repeat codes, code histograms (htab is free once the literals are out: LL at 0, ML at
        // 64, OF at 128) and, split encode, the sequences' records for pass B
        for (uint32_t k = lane; k < 192u; k += kWave) e.htab[k] = 0;
        __builtin_amdgcn_wave_barrier();
        resolve_repeats(e, n, lane, h0, h1, h2, e.area ? e.sreg : nullptr);   // (split: records in place)
        __builtin_amdgcn_wave_barrier();
        // ---- tables: per-block distributions from 64 sequences on (MIN_SEQ_FOR_DYNAMIC_FSE)
        // at FSE_optimalTableLog's accuracy capped at LL 7 / OF 6 / ML 7 (the reference caps at
        // 9 / 8 / 9; a log-7 table is two cells per lane -- tools/parse_sim.c zfse: the cap costs
        // 0.3 % of ratio at 32 KiB pages, the old fixed 6 / 5 / 6 cost 1.6 %), the predefined
        // ones below (ZSTD_compressSequences, zstd_compress.c:595-680); NCount headers follow
        // the mode byte in LL, OF, ML order
        const uint32_t mpos = o;
        o += 1u;
        const bool dyn = n >= 64u;
        huf::SmallCT tll, tof, tml;
        {
            int32_t nll, nof, nml;
            uint32_t mll, mof, mml, gll = 6, gof = 5, gml = 6;
            if (dyn) {
                const uint32_t cll = e.htab[lane], cml = e.htab[64u + lane], cof = lane < 32u ? e.htab[128u + lane] : 0u;
                mll = (uint32_t)huf::wave_max(cll ? (int32_t)lane : -1);
                mml = (uint32_t)huf::wave_max(cml ? (int32_t)lane : -1);
                mof = (uint32_t)huf::wave_max(cof ? (int32_t)lane : -1);
                if (e.logcap == 7u) {
                    gll = huf::optimal_log(7u, n, mll, 2);
                    gof = huf::optimal_log(6u, n, mof, 2);
                    gml = huf::optimal_log(7u, n, mml, 2);
                }
                if (!huf::normalize(cll, n, gll, nll, lane) || !huf::normalize(cof, n, gof, nof, lane) ||
                    !huf::normalize(cml, n, gml, nml, lane))
                    return false;
                o += huf::write_ncount(nll, mll, gll, e.dst, o, lane);
                o += huf::write_ncount(nof, mof, gof, e.dst, o, lane);
                o += huf::write_ncount(nml, mml, gml, e.dst, o, lane);
            } else {
                nll = lane <= 35u ? (int32_t)c_ll_norm[min(lane, 35u)] : 0;
                nml = lane <= 52u ? (int32_t)c_ml_norm[min(lane, 52u)] : 0;
                nof = lane <= 28u ? (int32_t)c_of_norm[min(lane, 28u)] : 0;
                mll = 35;
                mml = 52;
                mof = 28;
            }
            uint8_t *scr = (uint8_t *)(e.htab + 256u);   // past the code histograms
            tll = huf::build_small_ct(nll, mll, gll, lane, scr);
            tof = huf::build_small_ct(nof, mof, gof, lane, scr);
            tml = huf::build_small_ct(nml, mml, gml, lane, scr);
        }
        if (lane == 0) e.dst[mpos] = dyn ? (uint8_t)((2u << 6) | (2u << 4) | (2u << 2)) : 0u;
        SPROF_MARK(4);
        SPROF_ADD(9, n);
        if (e.area) {
            // pass A: the tables go to the area (the records went with resolve_repeats), the
            // bitstream's bound stays open
            uint32_t *T = area_tab(e.area, e.nblk);
            const huf::SmallCT *ts[3] = {&tll, &tof, &tml};
#pragma unroll
            for (uint32_t t = 0; t < 3; t++) {
                // word 63 (no symbol 63 in any of the three alphabets) holds the table log
                T[t * kCtWords + lane] = lane == 63u ? ts[t]->log : ts[t]->dnb | ((uint32_t)(ts[t]->dfs + 128) << 19);
                ((uint8_t *)(T + t * kCtWords + 64u))[lane] = (uint8_t)ts[t]->state;
                ((uint8_t *)(T + t * kCtWords + 64u))[64u + lane] = (uint8_t)ts[t]->state_hi;
            }
            const uint32_t pre = o - (hdr + 3u);
            const uint32_t glen = 3u + pre + fse_bound;
            const uint32_t bh = (last ? 1u : 0u) | (2u << 1) | ((glen - 3u) << 3);
            if (lane < 3) e.dst[hdr + lane] = (uint8_t)(bh >> (8u * lane));
            put_blk(e, hdr, glen, pre, fse_bound, n, e.nrec, (last ? 1u : 0u) | 2u, lane);
            e.nrec += n;
            e.op = hdr + glen;
            e.r0 = h0;
            e.r1 = h1;
            e.r2 = h2;
            SPROF_MARK(5);
            return true;
        }
        // ---- FSE bitstream: groups of 64 sequences from the last, serial inside a group
        huf::BitW b;
        b.c = 0;
        b.pos = 0;
        b.ptr = o;
        uint32_t sll = 0, sml = 0, sof = 0;
        const uint32_t ng = (n + kWave - 1) / kWave;
        for (uint32_t gi = ng; gi-- > 0;) {
            const uint32_t g = gi * kWave;
            const uint32_t i = g + lane;
            uint32_t pk_code = 0, pk_ll = 0, pk_ml = 0, pk_of = 0;
            if (i < n) {
                const SeqCode c = seq_code_at(e, i);
                pk_code = c.llc | (c.mlc << 8) | (c.ofc << 16);
                pk_ll = c.llv | (c.llb << 24);
                pk_ml = c.mlv | (c.mlb << 24);
                pk_of = c.ofv;
            }
            const uint32_t top = min(n - g, kWave);
            for (uint32_t k = top; k-- > 0;) {
                const uint32_t code = rdlane(pk_code, k), xl = rdlane(pk_ll, k), xm = rdlane(pk_ml, k),
                               xo = rdlane(pk_of, k);
                const uint32_t llc = code & 0xFFu, mlc = (code >> 8) & 0xFFu, ofc = code >> 16;
                const uint32_t llb = xl >> 24, mlb = xm >> 24;
                if (g + k == n - 1) {
                    // first symbols (zstd_compress.c:700-708)
                    sml = huf::ct_init2(tml, mlc);
                    sof = huf::ct_init2(tof, ofc);
                    sll = huf::ct_init2(tll, llc);
                } else {
                    huf::ct_encode(b, sof, tof, ofc);
                    huf::ct_encode(b, sml, tml, mlc);
                    huf::ct_encode(b, sll, tll, llc);
                    if (ofc + mlb + llb >= 64u - 7u - (9u + 9u + 8u)) huf::bw_flush(b, e.dst, lane);
                }
                huf::bw_add(b, xl & 0xFFFFFFu, llb);
                huf::bw_add(b, xm & 0xFFFFFFu, mlb);
                huf::bw_add(b, xo, ofc);
                huf::bw_flush(b, e.dst, lane);
            }
        }
        // FSE_flushCState x3, BIT_closeCStream (end mark)
        huf::bw_add(b, sml, tml.log);
        huf::bw_flush(b, e.dst, lane);
        huf::bw_add(b, sof, tof.log);
        huf::bw_flush(b, e.dst, lane);
        huf::bw_add(b, sll, tll.log);
        huf::bw_flush(b, e.dst, lane);
        huf::bw_add(b, 1u, 1u);
        huf::bw_flush(b, e.dst, lane);
        o = b.ptr + (b.pos > 0 ? 1u : 0u);
        if (b.pos > 0 && lane == 0) e.dst[b.ptr] = (uint8_t)b.c;
    }
    SPROF_MARK(5);
    const uint32_t csize = o - (hdr + 3u);
    const uint32_t bh = (last ? 1u : 0u) | (2u << 1) | (csize << 3);
    if (lane < 3) e.dst[hdr + lane] = (uint8_t)(bh >> (8u * lane));
    if (e.area) put_blk(e, hdr, 3u + csize, csize, 0u, 0u, 0u, last ? 1u : 0u, lane);
    e.op = o;
    e.r0 = h0;
    e.r1 = h1;
    e.r2 = h2;
    return true;
}

// Encodes one page held in LDS (in[0, L), 64 zero bytes after).  Returns the
// frame size, or 0 if it does not fit in cap.
__device__ __forceinline__ int32_t encode_page(const uint8_t *in, uint32_t L, uint16_t *table, uint8_t *map, uint2 *rec, uint2 *seq,
                               uint32_t *htab, uint8_t *wts, uint8_t *dst, uint32_t cap, uint32_t logcap, uint32_t lane) {
    // ---- frame header: magic, single-segment descriptor with the content size
    const uint32_t fcs_id = L < 256u ? 0u : (L < 65536u + 256u ? 1u : 2u);
    const uint32_t fcs_len = fcs_id == 0u ? 1u : (fcs_id == 1u ? 2u : 4u);
    const uint32_t fh = 5u + fcs_len;
    if (fh + 3u > cap) return 0;
    {
        const uint32_t fcs = fcs_id == 1u ? L - 256u : L;
        uint32_t v = 0;
        if (lane < 4) v = 0xFD2FB528u >> (8u * lane);
        else if (lane == 4) v = 0x20u | (fcs_id << 6);
        else if (lane < 5u + fcs_len) v = fcs >> (8u * (lane - 5u));
        if (lane < fh) dst[lane] = (uint8_t)v;
    }
    Enc e;
    e.in = in;
    e.dst = dst;
    e.cap = cap;
    e.op = fh;
    e.seq = seq;
    e.nseq = 0;
    e.bstart = 0;
    e.cursor = 0;
    e.map = map;
    e.r0 = 1u;
    e.r1 = 4u;
    e.r2 = 8u;
    e.htab = htab;
    e.wts = wts;
    e.stage = (uint32_t *)rec;
    e.fail = false;
    e.area = nullptr;
    e.nblk = 0;
    e.nrec = 0;
    e.rec_cap = 0;
    e.logcap = logcap;
    e.psum = nullptr;
    e.lit = nullptr;
    auto sink = [&](const uint2 *r, uint32_t n, uint32_t anchor) -> bool {
        uint32_t ls, ll, ml, off;
        lzp::decode_record(r, n, anchor, lane, ls, ll, ml, off, TYCHE_SINK_BACK ? in : nullptr);
        if (lane < n) seq[e.nseq + lane] = make_uint2(ll | (off << 16), ml);
        e.nseq += n;
        const uint2 lastr = r[n - 1];
        e.cursor = (lastr.x & 0xFFFFu) + (lastr.y & 0xFFFFu);
        __builtin_amdgcn_wave_barrier();
        if (e.nseq > kSeqCap - kWave) {
            if (!emit_block(e, e.cursor, false, lane)) return false;
            e.bstart = e.cursor;
            e.nseq = 0;
        }
        return true;
    };
    SPROF_DECL
    const uint32_t anchor = lzp::parse_page<true, false, kZWays>(in, L, table, rec, lane, sink);
    if (anchor == 0xFFFFFFFFu) return 0;
    if (!emit_block(e, L, true, lane)) return 0;
    SPROF_MARK(1);   // whole page (parse + every block)
    SPROF_ADD(0, 1);
    return (int32_t)e.op;
}

// Sequences per block of the split encode.  Its blocks live in the area, not in LDS, so
// they are not held to the one-kernel encode's kSeqCap: 4096 makes a 32 KiB page one
// block, which halves pass A2's per-block Huffman and FSE table work (1M x 32 KiB:
// encode 855 -> 793 ms, decode 308 -> 296 ms, ratio 4.946 -> 4.940; 16 KiB pages,
// mostly one block already, unchanged -- profiles/r03_zstd_block_size_ab.log)
#ifndef TYCHE_ZSTD_AREA_BLK
#define TYCHE_ZSTD_AREA_BLK 4096
#endif
constexpr uint32_t kZBlk = TYCHE_ZSTD_AREA_BLK;
static_assert(kZBlk >= kWave && (65536u / 4u + kZBlk - 1u) / kZBlk + 1u <= kMaxBlk, "area blocks");

// Pass A1: the parse of one page (LDS, 64 zero bytes after) into the area: the
// sequences, and blocks cut where encode_page's sink cuts them.  Returns 1, or
// 0 when a bound is exceeded (the page is then stored uncompressed by the caller).
// parse(sink) runs the parse over the page and returns its last anchor.  The literals go
// to the area's literal region as the sequences come (copy_runs from the page `in`).
template <typename Parse>
__device__ __forceinline__ int32_t parse_to_area_with(const uint8_t *in, uint32_t L, uint8_t *area, uint32_t rec_cap,
                                                      uint32_t lane, Parse &&parse, const uint8_t *sink_in,
                                                      uint32_t *map) {
    uint2 *S = (uint2 *)area_rec(area);   // one part: the sequence map below is the identity
    uint8_t *lits = area_lit(area, rec_cap);
    uint32_t nseq = 0, bseq = 0, bstart = 0, cursor = 0, npb = 0;
    uint32_t a_lit = 0, a_span = 0, a_xb = 0;   // this lane's share of the block's sums
    uint32_t lpos = 0, blit = 0;                // literals copied; the block's first
    auto put_pblk = [&](uint32_t bend) {
        const uint32_t lit = huf::wave_sum(a_lit), span = huf::wave_sum(a_span), xb = huf::wave_sum(a_xb);
        if (lane == 0) {
            uint32_t *P = area_pblk(area, npb);
            P[0] = bstart;
            P[1] = bend;
            P[2] = bseq;
            P[3] = nseq - bseq;
            P[4] = lit;
            P[5] = span;
            P[6] = xb;
            P[7] = blit;
        }
        a_lit = a_span = a_xb = 0;
        blit = lpos;
        npb++;
    };
    auto sink = [&](const uint2 *r, uint32_t n, uint32_t anchor) -> bool {
        uint32_t ls, ll, ml, off;
        lzp::decode_record(r, n, anchor, lane, ls, ll, ml, off, sink_in);   // (sink_in: lz_parse.h back_at)
        if (nseq + n > rec_cap) return false;
        if (lane < n) {
            S[nseq + lane] = make_uint2(ll | (off << 16), ml);
            const SeqCode c = seq_code(ll, ml, off + 3u);   // emit_block's bound: no repeat offsets
            a_lit += ll;
            a_span += ll + ml;
            a_xb += c.llb + c.mlb + c.ofc;
        }
        lpos += copy_runs(in, ls, ll, lits + lpos, lane, map);
        nseq += n;
        const uint2 lastr = r[n - 1];
        cursor = (lastr.x & 0xFFFFu) + (lastr.y & 0xFFFFu);
        __builtin_amdgcn_wave_barrier();
        if (nseq - bseq > kZBlk) {
            if (npb + 1u >= kMaxBlk) return false;
            put_pblk(cursor);
            bstart = cursor;
            bseq = nseq;
        }
        return true;
    };
    const uint32_t anchor = parse(sink);
    if (anchor == 0xFFFFFFFFu) return 0;
    for (uint32_t j = lane; anchor + j < L; j += kWave) lits[lpos + j] = in[anchor + j];   // the last literals
    put_pblk(L);
    if (lane == 0) {
        ((uint32_t *)area)[1] = npb;
        put_seq_map(area, 0xFFFFu, 0xFFFFu, 0xFFFFu, 0u);
        ((uint32_t *)area)[4] = 0u;   // one literal run from region byte 0
        for (int k = 1; k < 5; k++) ((uint32_t *)area)[4 + k] = 0xFFFFu;
    }
    return 1;
}
template <int kW>
__device__ __forceinline__ int32_t parse_to_area(const uint8_t *in, uint32_t L, uint16_t *table, uint2 *rec,
                                                 uint8_t *area, uint32_t rec_cap, uint32_t lane, uint32_t *map) {
    return parse_to_area_with(
        in, L, area, rec_cap, lane,
        [&](auto &sink) { return lzp::parse_page<true, false, kW>(in, L, table, rec, lane, sink); },
        TYCHE_SINK_BACK ? in : nullptr, map);
}

// Pass A2: frame header and every block of the page from the area (the page
// itself is read from global memory).  Returns the gapped frame size or 0.
__device__ __forceinline__ int32_t emit_page(const uint8_t *src, uint32_t L, uint8_t *area, uint32_t rec_cap,
                                             uint8_t *map, uint2 *stage, uint32_t *htab, uint8_t *wts, uint8_t *dst,
                                             uint32_t cap, uint32_t logcap, uint32_t lane) {
    const uint32_t fcs_id = L < 256u ? 0u : (L < 65536u + 256u ? 1u : 2u);
    const uint32_t fcs_len = fcs_id == 0u ? 1u : (fcs_id == 1u ? 2u : 4u);
    const uint32_t fh = 5u + fcs_len;
    if (fh + 3u > cap) return 0;
    {
        const uint32_t fcs = fcs_id == 1u ? L - 256u : L;
        uint32_t v = 0;
        if (lane < 4) v = 0xFD2FB528u >> (8u * lane);
        else if (lane == 4) v = 0x20u | (fcs_id << 6);
        else if (lane < 5u + fcs_len) v = fcs >> (8u * (lane - 5u));
        if (lane < fh) dst[lane] = (uint8_t)v;
    }
    Enc e;
    e.in = src;
    e.dst = dst;
    e.cap = cap;
    e.op = fh;
    e.map = map;
    e.r0 = 1u;
    e.r1 = 4u;
    e.r2 = 8u;
    e.htab = htab;
    e.wts = wts;
    e.stage = (uint32_t *)stage;
    e.fail = false;
    e.area = area;
    e.nblk = 0;
    e.nrec = 0;
    e.rec_cap = rec_cap;
    e.logcap = logcap;
    e.cursor = 0;
    const uint32_t npb = __builtin_amdgcn_readfirstlane(((const uint32_t *)area)[1]);
    e.sreg = (uint2 *)area_rec(area);
    e.smap = seq_map(area, true);
    e.seq = nullptr;
    e.lit = area_lit(area, rec_cap);
    e.lmap = lit_map(area);
    for (uint32_t k = 0; k < npb; k++) {
        const uint32_t *P = area_pblk(area, k);
        e.bstart = __builtin_amdgcn_readfirstlane(P[0]);
        const uint32_t bend = __builtin_amdgcn_readfirstlane(P[1]);
        e.nrec = __builtin_amdgcn_readfirstlane(P[2]);   // the block's records replace its sequences
        e.sfirst = e.nrec;
        e.nseq = __builtin_amdgcn_readfirstlane(P[3]);
        e.psum = P + 4;
        e.lofs = __builtin_amdgcn_readfirstlane(P[7]);
        if (!emit_block(e, bend, k + 1u == npb, lane)) return 0;
    }
    if (lane == 0) ((uint32_t *)area)[0] = e.nblk;
    return (int32_t)e.op;
}

// The one-kernel encode of pages [first, first + count) of b (TYCHE_ZSTD_ENC_SPLIT=0).
// kParse: pass A1 of the split encode instead (the parse only, into ws; status to st), its
// buckets of kW ways (2 or 4: the same 3,712 table slots, lz_parse.h)
template <bool kParse, int kW = kZWays>
__global__ __launch_bounds__(64) void zstd_encode_kernel(tyche_batch_t b, size_t first, size_t count, uint32_t in_cap,
                                                         unsigned *ctr, uint8_t *ws, size_t ws_page, int32_t *st,
                                                         uint32_t logcap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint16_t *table = (uint16_t *)smem;
    uint8_t *map = smem + kTableSlots * sizeof(uint16_t);               // 64-byte owner map
    uint2 *rec = (uint2 *)(map + kWave);                               // 64 parse records
    uint2 *seq = rec + kWave;                                          // kSeqCap block sequences
    uint32_t *htab = (uint32_t *)(seq + kSeqCap);                      // literal histogram / Huffman codes
    uint8_t *wts = (uint8_t *)(htab + kHtab);                          // Huffman weights
    uint32_t *lmap = (uint32_t *)seq;                                   // A1: no block buffers, a copy map
    uint8_t *stage = kParse ? (uint8_t *)seq + kWave * 4 : wts + 256;   // (A1: lds1 has room for it)
    const size_t stride = gridDim.x;

    size_t page = blockIdx.x;   // chunk-local
    if (page >= count) return;
    PageRef p = batch_page(b, first + page);
    uint32_t head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, lane, kWave);
    for (;;) {
        const size_t next = ctr ? claim_page(ctr, lane) : page + stride;   // dynamic assignment (engine.h)
        PageRef pn;
        u32x4 pf[kPrefetchVec];
        uint32_t nhead = 0, nvec = 0;
        if (next < count) {
            pn = batch_page(b, first + next);
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
            for (uint32_t w = lane; w < kTableSlots / 8; w += kWave) ((u32x4 *)table)[w] = u32x4{0, 0, 0, 0};
            WAVE_SYNC();
            in[p.src_len + lane] = 0;
            WAVE_SYNC();
            if (kParse) rv = parse_to_area<kW>(in, p.src_len, table, rec, ws + page * ws_page, enc_rec_cap(in_cap), lane, lmap);
            else rv = encode_page(in, p.src_len, table, map, rec, seq, htab, wts, p.dst, p.dst_cap, logcap, lane);
        }
        if (lane == 0) {
            if (kParse) st[page] = rv;
            else b.results[first + page] = rv;
        }
        if (next >= count) break;
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

// ---- pass A1 on two pipelined waves per page (round 3, TYCHE_ZSTD_PARSE_PIPE=1; not the
// default: 1,205 vs 1,026 ms per 1M x 32 KiB pages for the one-wave kernel above).  lzp::parse_page_piped: the finder wave hashes block k+1 while
// the walker wave takes block k's repeat candidates and walk; the records (and so the frames)
// are the one-wave parse's except that the finder also inserts the blocks the walk skips.
// LDS: header, the table, the two-slot ring, the walker's records and the page (41.9 KiB at
// 32 KiB pages: 3 pages, 6 waves per CU).
struct ZPipeHdr {
    uint32_t next_lo, next_hi, next2_lo, next2_hi, flag, pad[11];
};
static_assert(sizeof(ZPipeHdr) == 64, "pipe header");
constexpr size_t kZPipeStage = sizeof(ZPipeHdr) + kTableSlots * sizeof(uint16_t) + 2 * sizeof(lzp::PipeSlot) + kWave * 8;
__global__ __launch_bounds__(128) void zstd_parse_pipe_kernel(tyche_batch_t b, size_t first, size_t count,
                                                              uint32_t in_cap, unsigned *ctr, uint8_t *ws,
                                                              size_t ws_page, int32_t *st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = rfl(tid >> 6);
    ZPipeHdr *hdr = (ZPipeHdr *)smem;
    uint16_t *table = (uint16_t *)(smem + sizeof(ZPipeHdr));
    lzp::PipeSlot *slots = (lzp::PipeSlot *)(smem + sizeof(ZPipeHdr) + kTableSlots * sizeof(uint16_t));
    uint2 *rec = (uint2 *)(slots + 2);
    uint8_t *stage = smem + kZPipeStage;
    const uint32_t rec_cap = enc_rec_cap(in_cap);

    size_t page = blockIdx.x;   // chunk-local
    if (page >= count) return;
    PageRef p = batch_page(b, first + page);
    uint32_t head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, tid, 2 * kWave);
    if (tid == 0) {
        const size_t nx = (size_t)atomicAdd(ctr, 1u) + gridDim.x;   // dynamic assignment (engine.h)
        hdr->next_lo = (uint32_t)nx;
        hdr->next_hi = (uint32_t)(nx >> 32);
    }
    for (;;) {
        for (uint32_t w = tid; w < kTableSlots / 8; w += 2 * kWave) ((u32x4 *)table)[w] = u32x4{0, 0, 0, 0};
        if (tid < kWave) stage[head + p.src_len + tid] = 0;
        __syncthreads();
        const size_t next = (size_t)rfl(hdr->next_lo) | ((size_t)rfl(hdr->next_hi) << 32);
        const uint8_t *in = stage + head;
        const uint32_t L = p.src_len;
        int32_t rv = kResultTooLarge;
        if (L <= in_cap) {   // uniform over the workgroup: both waves run the parse's barriers
            if (wave == 1) {
                rv = parse_to_area_with(in, L, ws + page * ws_page, rec_cap, lane, [&](auto &sink) {
                    return lzp::parse_page_piped(in, L, table, rec, slots, &hdr->flag, 1u, lane, sink);
                }, nullptr, nullptr);   // (the piped parse's records carry their extension)
            } else {
                auto none = [](const uint2 *, uint32_t, uint32_t) -> bool { return true; };
                (void)lzp::parse_page_piped(in, L, table, rec, slots, &hdr->flag, 0u, lane, none);
            }
        }
        if (tid == 0) {
            const size_t nx = (size_t)atomicAdd(ctr, 1u) + gridDim.x;
            hdr->next2_lo = (uint32_t)nx;
            hdr->next2_hi = (uint32_t)(nx >> 32);
        }
        if (wave == 1 && lane == 0) st[page] = rv;
        __syncthreads();   // the stage, the table and the header are free
        if (next >= count) break;
        page = next;
        p = batch_page(b, first + page);
        head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, tid, 2 * kWave);
        if (tid == 0) {
            hdr->next_lo = hdr->next2_lo;
            hdr->next_hi = hdr->next2_hi;
        }
    }
}

// ---- pass A1 on kNW waves per page (round 3, TYCHE_ZSTD_PARSE_WAVES 2 / 4; not the default:
// the parts' parses cost ratio, 4.947 -> 4.910 at 2 waves).
//
// The one-wave A1 holds page + hash table (40.8 KiB at 32 KiB pages: 4 waves per
// CU, one per SIMD) and was 737 of the encoder's 995 ms per 1M x 32 KiB pages --
// latency-bound.  Here kNW waves share the staged page as the LZ4 split encoder
// does (lz4_encode.hip): wave w parses part [b_w, b_{w+1}) (64-aligned) with its
// own table, seeded with the kZSeed positions before the part, matches of part w
// ending by b_{w+1}.  Each wave writes its sequences to its own slice of the
// area's code region (pass B's, unused until A2 runs); after a barrier every
// wave copies its slice to its place in the page's sequence list (the first
// sequence's literal length extended back to the previous part's last match end,
// whose catch-up it did not see -- any catch-up <= the one taken is valid), and
// wave 0 cuts the list into parse blocks of kZBlk sequences.  Repeat candidates
// restart at zstd's {1, 4} in each part; the repeat codes themselves are
// assigned by A2 over the whole list, as before.
#ifndef TYCHE_ZSTD_SEED
#define TYCHE_ZSTD_SEED 8192   // positions seeded before a part (multiple of 64)
#endif
constexpr uint32_t kZSeed = TYCHE_ZSTD_SEED;
constexpr uint32_t kZWarm = 256;   // bytes parsed (and dropped) before a part, for its repeat offsets
template <uint32_t kNW>
struct ZSplitHdr {
    uint32_t next_lo, next_hi, next2_lo, next2_hi;
    uint32_t n[kNW];        // sequences of part w
    uint32_t cursor[kNW];   // end of part w's last match (its start if none)
    uint32_t ok[kNW];       // part w's sequences fit its slice
    uint32_t lit[kNW];      // part w's literal bytes (before its first run's extension)
    uint32_t span[kNW];     // part w's page bytes (likewise)
    uint32_t xb[kNW];       // part w's extra bits at raw offsets (emit_block's bound; likewise)
    uint32_t ll0[kNW];      // part w's first literal length (likewise)
};
template <uint32_t kNW>
constexpr size_t zsplit_hdr_bytes() { return (sizeof(ZSplitHdr<kNW>) + 63) & ~(size_t)63; }
constexpr size_t kZWaveRegion = kTableSlots * sizeof(uint16_t) + kWave * 8 + kWave * 4;   // table, 64 records, copy map
template <uint32_t kNW>
constexpr size_t zsplit_stage_off() { return zsplit_hdr_bytes<kNW>() + kNW * kZWaveRegion; }

template <uint32_t kNW>
__global__ __launch_bounds__(kNW * 64) void zstd_parse_split_kernel(tyche_batch_t b, size_t first, size_t count,
                                                                    uint32_t in_cap, unsigned *ctr, uint8_t *ws,
                                                                    size_t ws_page, int32_t *st, uint32_t seed,
                                                                    uint32_t p0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr uint32_t kT = kNW * kWave;
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = rfl(tid >> 6);
    ZSplitHdr<kNW> *hdr = (ZSplitHdr<kNW> *)smem;
    uint8_t *region = smem + zsplit_hdr_bytes<kNW>() + wave * kZWaveRegion;
    uint16_t *table = (uint16_t *)region;
    uint2 *rec = (uint2 *)(region + kTableSlots * sizeof(uint16_t));
    uint32_t *cmap = (uint32_t *)(rec + kWave);   // copy_runs' map
    uint8_t *stage = smem + zsplit_stage_off<kNW>();
    const uint32_t rec_cap = enc_rec_cap(in_cap);
    const uint32_t slice = (2u * rec_cap) / kNW;   // the code region holds 2 rec_cap sequences of 8 bytes

    size_t page = blockIdx.x;   // chunk-local
    if (page >= count) return;
    PageRef p = batch_page(b, first + page);
    uint32_t head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, tid, kT);
    if (tid == 0) {
        const size_t nx = (size_t)atomicAdd(ctr, 1u) + gridDim.x;
        hdr->next_lo = (uint32_t)nx;
        hdr->next_hi = (uint32_t)(nx >> 32);
    }
    for (;;) {
        for (uint32_t w = lane; w < kTableSlots / 8; w += kWave) ((u32x4 *)table)[w] = u32x4{0, 0, 0, 0};
        if (tid < kWave) stage[head + p.src_len + tid] = 0;
        __syncthreads();
        const size_t next = (size_t)rfl(hdr->next_lo) | ((size_t)rfl(hdr->next_hi) << 32);
        const uint8_t *in = stage + head;
        const uint32_t L = p.src_len;
        const bool fits = L <= in_cap;
        uint8_t *area = ws + page * ws_page;
        uint2 *W = (uint2 *)area_rec(area) + (size_t)wave * slice;
        // part w starts at bnd(w): equal parts, or (p0 > 0) p0/64 of the page for part 0 -- the one part
        // without a seed and a warm-up -- and equal shares of the rest
        auto bnd = [&](uint32_t w) -> uint32_t {
            if (w == 0) return 0u;
            if (w == kNW) return L;
            if (!p0) return ((L * w) / kNW) & ~(kWave - 1u);
            const uint32_t h = (L * p0 / 64u) & ~(kWave - 1u);
            return (h + ((L - h) * (w - 1u)) / (kNW - 1u)) & ~(kWave - 1u);
        };
        const uint32_t b0 = bnd(wave);
        const uint32_t b1 = bnd(wave + 1);
        const uint32_t Lp = wave + 1 == kNW ? L : b1 + kLastLiterals;
        if (fits) {
            uint32_t rep[2] = {1u, 4u};
            if (wave > 0) {   // seed: the positions before the part, block order, as the parse inserts them
                const uint32_t ib = (uint32_t)(uintptr_t)in & 3u;
                uint32_t *T = (uint32_t *)table;
                const uint32_t wstart = b0 > kZWarm ? b0 - kZWarm : 0u;
                // four blocks' words and hashes at once (one LDS round trip for their windows, from
                // this lane's base address), then each block's bucket update in block order
                const uint32_t la = lzp::lds_addr(in - ib) + ((lane + ib) & ~3u), ls = (lane + ib) & 3u;
                auto hash_at = [&](uint32_t blk) {
                    const lzp::lds_u32_t *P = (const lzp::lds_u32_t *)(uintptr_t)(la + blk);
                    const uint32_t d0 = P[0], d1 = P[1], d2 = P[2];
                    return lzp::bucket_of<kZWays>(lzp::word_at(d0, d1, ls), lzp::word_at(d1, d2, ls), TYCHE_HASH_BYTES);
                };
                auto insert = [&](uint32_t h, uint32_t pos) {
                    const uint32_t bk = T[h];
                    __builtin_amdgcn_wave_barrier();
                    T[h] = pos | (bk << 16);
                    __builtin_amdgcn_wave_barrier();
                };
                uint32_t blk = wstart > seed ? wstart - seed : 0u;
                for (; blk + 4u * kWave <= wstart; blk += 4u * kWave) {
                    uint32_t h[4];
#pragma unroll
                    for (uint32_t u = 0; u < 4u; u++) h[u] = hash_at(blk + kWave * u);
#pragma unroll
                    for (uint32_t u = 0; u < 4u; u++) insert(h[u], blk + kWave * u + lane);
                }
                for (; blk < wstart; blk += kWave) insert(hash_at(blk), blk + lane);
                // warm-up: parse the kZWarm bytes before the part, sequences dropped, for the repeat
                // offsets the part's parse starts from (a cold {1, 4} cost the 4-wave split 1.7 % of
                // ratio; tools/parse_sim.c zsplit: 4.999 -> 5.069 of 5.100)
                auto drop = [&](const uint2 *, uint32_t, uint32_t) -> bool { return true; };
                (void)lzp::parse_page<true, false, kZWays>(in, b0 + kLastLiterals, table, rec, lane, drop, wstart, rep);
            }
            uint32_t nseq = 0, a_lit = 0, a_span = 0, a_xb = 0, ll0 = 0, lown = 0;
            uint8_t *lits = area_lit(area, rec_cap) + b0;   // the part's own literals, in order (round 6)
            auto sink = [&](const uint2 *r, uint32_t n, uint32_t anchor) -> bool {
                uint32_t ls, ll, ml, off;
                lzp::decode_record(r, n, anchor, lane, ls, ll, ml, off, TYCHE_SINK_BACK ? in : nullptr);
                if (nseq + n > slice) return false;
                lown += copy_runs(in, ls, ll, lits + lown, lane, cmap);
                if (lane < n) {
                    W[nseq + lane] = make_uint2(ll | (off << 16), ml);
                    const SeqCode c = seq_code(ll, ml, off + 3u);   // emit_block's bound: no repeat offsets
                    a_lit += ll;
                    a_span += ll + ml;
                    a_xb += c.llb + c.mlb + c.ofc;
                }
                if (nseq == 0) ll0 = rdlane(ll, 0);
                nseq += n;
                __builtin_amdgcn_wave_barrier();
                return true;
            };
            const uint32_t cur = lzp::parse_page<true, false, kZWays>(in, Lp, table, rec, lane, sink, b0, rep);
            a_lit = huf::wave_sum(a_lit);
            a_span = huf::wave_sum(a_span);
            a_xb = huf::wave_sum(a_xb);
            if (lane == 0) {
                hdr->lit[wave] = a_lit;
                hdr->span[wave] = a_span;
                hdr->xb[wave] = a_xb;
                hdr->ll0[wave] = ll0;
                hdr->ok[wave] = cur != 0xFFFFFFFFu ? 1u : 0u;
                hdr->n[wave] = nseq;
                hdr->cursor[wave] = nseq ? cur : b0;
                if (wave == 0) {
                    const size_t nx = (size_t)atomicAdd(ctr, 1u) + gridDim.x;
                    hdr->next2_lo = (uint32_t)nx;
                    hdr->next2_hi = (uint32_t)(nx >> 32);
                }
            }
        }
        __syncthreads();   // every part parsed
        bool ok = fits;
        // prev_end / pe: the end of the last part with a sequence before this one / of all
        uint32_t prev_end = 0, total = 0, pe = 0;
        for (uint32_t w = 0; w < kNW; w++) {
            const uint32_t nw = rfl(hdr->n[w]);
            ok = ok && rfl(hdr->ok[w]);
            if (w < wave && nw) prev_end = rfl(hdr->cursor[w]);
            total += nw;
            if (nw) pe = rfl(hdr->cursor[w]);
        }
        if (ok) {
            // the part's first literal run starts at the end of the last part before it with a
            // sequence: its first sequence is extended back in place (ll, the low 16 bits: cannot
            // carry out, < 2^16), and the bytes it now covers join the literal region at their
            // page positions, right below the part's own literals (copied by the sink)
            const uint32_t nw = rfl(hdr->n[wave]);
            if (lane == 0 && wave > 0 && nw) {
                uint2 q = W[0];
                q.x += b0 - prev_end;
                W[0] = q;   // (the store waits for the load it depends on)
            }
            uint8_t *lits = area_lit(area, rec_cap);
            if (wave > 0 && nw)
                for (uint32_t j = lane; prev_end + j < b0; j += kWave) lits[prev_end + j] = in[prev_end + j];
            if (wave == kNW - 1)   // the literals after the page's last match, at their page positions
                for (uint32_t j = lane; pe + j < L; j += kWave) lits[pe + j] = in[pe + j];
        }
        __syncthreads();   // every part's first sequence extended
        if (wave == 0) {
            if (!fits) {
                if (lane == 0) st[page] = kResultTooLarge;
            } else if (!ok || (total + kZBlk - 1) / kZBlk + 1 > kMaxBlk) {
                if (lane == 0) st[page] = 0;
            } else {
                // parse blocks of kZBlk sequences over the whole list (the parts' slices, in page
                // order: the sequence map): page spans from the sequences' sizes
                SeqMap m;
                m.slice = slice;
                m.c1 = rfl(hdr->n[0]);
                m.c2 = kNW > 1 ? m.c1 + rfl(hdr->n[min(1u, kNW - 1u)]) : 0xFFFFu;
                m.c3 = kNW > 2 ? m.c2 + rfl(hdr->n[min(2u, kNW - 1u)]) : 0xFFFFu;
                if (kNW < 4) m.c3 = 0xFFFFu;
                if (kNW < 3) m.c2 = 0xFFFFu;
                if (kNW < 2) m.c1 = 0xFFFFu;
                const uint2 *Wall = (const uint2 *)area_rec(area);
                // one block (almost every page up to 32 KiB): its sums are the parts' from the parse,
                // each part's first run extended back as in its first sequence (round 6: the list
                // is not read again)
                uint32_t one_lit = 0, one_span = 0, one_xb = 0, pe1 = 0;
                for (uint32_t w = 0; w < kNW; w++) {
                    const uint32_t nw = rfl(hdr->n[w]);
                    if (!nw) continue;
                    const uint32_t adj = w > 0 ? bnd(w) - pe1 : 0u, a = rfl(hdr->ll0[w]);
                    one_lit += rfl(hdr->lit[w]) + adj;
                    one_span += rfl(hdr->span[w]) + adj;
                    one_xb += rfl(hdr->xb[w]) + seq_code(a + adj, 3u, 4u).llb - seq_code(a, 3u, 4u).llb;
                    pe1 = rfl(hdr->cursor[w]);
                }
                uint32_t npb = 0, pos = 0, lpos = 0;
                for (uint32_t bs = 0; bs < total || npb == 0; bs += kZBlk) {
                    const uint32_t cnt = min(kZBlk, total - bs);
                    uint32_t span = 0, lit = 0, xb = 0;
                    for (uint32_t j = lane; total > kZBlk && j < cnt; j += kWave) {
                        const uint2 q = Wall[seq_slot(m, bs + j)];
                        const uint32_t ll = q.x & 0xFFFFu;
                        const SeqCode c = seq_code(ll, q.y, (q.x >> 16) + 3u);   // emit_block's bound
                        span += ll + q.y;
                        lit += ll;
                        xb += c.llb + c.mlb + c.ofc;
                    }
                    span = total > kZBlk ? huf::wave_sum(span) : one_span;
                    lit = total > kZBlk ? huf::wave_sum(lit) : one_lit;
                    xb = total > kZBlk ? huf::wave_sum(xb) : one_xb;
                    const bool last = bs + kZBlk >= total;
                    if (lane == 0) {
                        uint32_t *P = area_pblk(area, npb);
                        P[0] = pos;
                        P[1] = last ? L : pos + span;
                        P[2] = bs;
                        P[3] = cnt;
                        P[4] = lit;
                        P[5] = span;
                        P[6] = xb;
                        P[7] = lpos;
                    }
                    pos += span;
                    lpos += lit;
                    npb++;
                    if (last) break;
                }
                if (lane == 0) {
                    ((uint32_t *)area)[1] = npb;
                    put_seq_map(area, m.c1, m.c2, m.c3, m.slice);
                    // the literal map: each part with a sequence from the end of the last one before
                    // it (its extended first run, then its own literals), then the last literals
                    uint32_t lc = 0, pe2 = 0, ns = 0;
                    for (uint32_t w = 0; w < kNW; w++) {
                        const uint32_t nw = hdr->n[w];
                        if (!nw) continue;
                        ((uint32_t *)area)[4 + ns++] = lc | (pe2 << 16);
                        lc += bnd(w) - pe2 + hdr->lit[w];
                        pe2 = hdr->cursor[w];
                    }
                    ((uint32_t *)area)[4 + ns++] = lc | (pe2 << 16);
                    for (; ns < 5u; ns++) ((uint32_t *)area)[4 + ns] = 0xFFFFu;
                    st[page] = 1;
                }
            }
        }
        __syncthreads();   // the stage, the tables and the header are free
        if (next >= count) break;
        page = next;
        p = batch_page(b, first + page);
        head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, tid, kT);
        if (tid == 0) {
            hdr->next_lo = hdr->next2_lo;
            hdr->next_hi = hdr->next2_hi;
        }
    }
}

// ---- pass A2
constexpr uint32_t kA2Lds = kWave + kWave * 8u + kHtab * 4u + 256u;   // map, stage, htab, weights
__global__ __launch_bounds__(64) void zstd_block_kernel(tyche_batch_t b, size_t first, size_t count, uint32_t in_cap,
                                                        uint8_t *ws, size_t ws_page, int32_t *st, unsigned *ctr,
                                                        uint32_t logcap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint8_t *map = smem;
    uint2 *stage = (uint2 *)(smem + kWave);
    uint32_t *htab = (uint32_t *)(stage + kWave);
    uint8_t *wts = (uint8_t *)(htab + kHtab);
    for (size_t j = blockIdx.x; j < count; j = ctr ? claim_page(ctr, lane) : j + gridDim.x) {
        const int32_t s0 = st[j];
        if (s0 != 1) continue;   // 0: does not fit; kResultTooLarge passes through
        const PageRef p = batch_page(b, first + j);
        WAVE_SYNC();
        const int32_t rv = emit_page(p.src, p.src_len, ws + j * ws_page, enc_rec_cap(in_cap), map, stage, htab, wts,
                                     p.dst, p.dst_cap, logcap, lane);
        if (lane == 0) st[j] = rv;
    }
}

// ---- pass B: the FSE bitstreams, one page per lane

// Appends bytes to global memory in aligned 8-byte words (bytes only at the ends)
struct ByteSink {
    uintptr_t addr;   // next byte
    uint64_t w;       // pending bytes of the word holding addr
    uint32_t lo;      // first byte of that word that is ours
};
__device__ __forceinline__ void sink_word(uintptr_t a, uint64_t w, uint32_t lo, uint32_t hi) {
    if (lo == 0 && hi == 8) {
        *(uint64_t *)a = w;
    } else {
        for (uint32_t k = lo; k < hi; k++) ((uint8_t *)a)[k] = (uint8_t)(w >> (8u * k));
    }
}
__device__ __forceinline__ void sink_put(ByteSink &s, uint64_t v, uint32_t nb) {   // nb <= 7 low bytes of v
    if (nb == 0) return;
    v &= (1ull << (8u * nb)) - 1ull;
    const uint32_t k = (uint32_t)(s.addr & 7u);
    s.w |= v << (8u * k);
    if (k + nb >= 8u) {
        sink_word(s.addr - k, s.w, s.lo, 8u);
        s.w = v >> (8u * (8u - k));
        s.lo = 0;
    }
    s.addr += nb;
}
__device__ __forceinline__ void sink_end(ByteSink &s) {
    const uint32_t k = (uint32_t)(s.addr & 7u);
    if (k > s.lo) sink_word(s.addr - k, s.w, s.lo, k);
}

struct LaneBits {
    uint64_t c;
    uint32_t pos;
};
__device__ __forceinline__ void lb_add(LaneBits &b, uint32_t v, uint32_t nb) {
    b.c |= (uint64_t)(v & ((1u << nb) - 1u)) << b.pos;
    b.pos += nb;
}
__device__ __forceinline__ void lb_flush(LaneBits &b, ByteSink &s) {   // BIT_flushBits
    const uint32_t nbytes = b.pos >> 3;
    sink_put(s, b.c, nbytes);
    b.pos &= 7u;
    b.c = nbytes >= 8u ? 0ull : b.c >> (8u * nbytes);
}
// FSE_initCState2 / FSE_encodeSymbol over a packed table in LDS: S the symbol words, X the state bytes
__device__ __forceinline__ uint32_t lct_init2(const uint32_t *S, const uint8_t *X, uint32_t sym) {
    const uint32_t pk = S[sym], dnb = pk & 0x7FFFFu;
    const uint32_t nbo = (dnb + (1u << 15)) >> 16;
    const uint32_t v = (nbo << 16) - dnb;
    return X[(uint32_t)((int32_t)(v >> nbo) + (int32_t)(pk >> 19) - 128)];
}
__device__ __forceinline__ void lct_encode(LaneBits &b, uint32_t &st, const uint32_t *S, const uint8_t *X, uint32_t sym) {
    const uint32_t pk = S[sym];
    const uint32_t nbo = (st + (pk & 0x7FFFFu)) >> 16;
    lb_add(b, st, nbo);
    st = X[(uint32_t)((int32_t)(st >> nbo) + (int32_t)(pk >> 19) - 128)];
}

// Pass B's LDS slot per lane.  TYCHE_ZSTD_FSE_SLOT 1 (default): only what the alphabets use --
// 36 LL, 32 OF and 53 ML symbol words, each table's log after its words, then 128 / 64 / 128
// state bytes (OF log <= 6): 816 bytes, 3 workgroups per CU instead of 2 at the full 1,152.
#ifndef TYCHE_ZSTD_FSE_SLOT
#define TYCHE_ZSTD_FSE_SLOT 1
#endif
struct FseSlot {
    uint32_t sll, sof, sml, xll, xof, xml, lll, lof, lml, words;   // word offsets in the slot
};
constexpr FseSlot kFseSlot = TYCHE_ZSTD_FSE_SLOT ? FseSlot{0, 37, 70, 124, 156, 172, 36, 69, 123, 204}
                                                 : FseSlot{0, kCtWords, 2 * kCtWords, 64, kCtWords + 64,
                                                           2 * kCtWords + 64, 63, kCtWords + 63, 2 * kCtWords + 63,
                                                           3 * kCtWords};
static_assert(kFseSlot.words % 4u == 0, "slot of 16-byte pieces");

#ifndef TYCHE_ZSTD_FSE_PF
#define TYCHE_ZSTD_FSE_PF 8
#endif
constexpr uint32_t kFsePf = TYCHE_ZSTD_FSE_PF;   // sequence records in flight per lane (pass B)
// ZSTD_compressSequences' bitstream (zstd_compress.c:695-735) for n >= 1
// sequences; the same steps as emit_block's wave-uniform loop.  Returns its size.
__device__ uint32_t fse_lane(uint8_t *out, const uint2 *Rg, const SeqMap m, uint32_t first, uint32_t n, const uint32_t *T) {
    auto R = [&](uint32_t i) { return Rg[seq_slot(m, first + i)]; };   // record i of the block
    const uint32_t *tll = T + kFseSlot.sll, *tof = T + kFseSlot.sof, *tml = T + kFseSlot.sml;
    const uint8_t *xll = (const uint8_t *)(T + kFseSlot.xll), *xof = (const uint8_t *)(T + kFseSlot.xof),
                  *xml = (const uint8_t *)(T + kFseSlot.xml);
    ByteSink s;
    s.addr = (uintptr_t)out;
    s.w = 0;
    s.lo = (uint32_t)(s.addr & 7u);
    LaneBits b;
    b.c = 0;
    b.pos = 0;
    uint32_t sll = 0, sml = 0, sof = 0;
    // the records are loaded kFsePf steps ahead (a ring of registers, slot u of each pass of
    // kFsePf steps): at one wave per two SIMDs (the LDS slots) a load one step ahead left
    // every step waiting on HBM
    uint2 q[kFsePf];
#pragma unroll
    for (uint32_t u = 0; u < kFsePf; u++) q[u] = u < n ? R(n - 1u - u) : make_uint2(0, 0);
    for (uint32_t base = n; base > 0; base = base > kFsePf ? base - kFsePf : 0u) {
#pragma unroll
        for (uint32_t u = 0; u < kFsePf; u++) {
            const bool live = base > u;
            const uint32_t i = base - 1u - u;   // wraps when !live: every use below is gated
            const uint2 r = q[u];
            if (live && i >= kFsePf) q[u] = R(i - kFsePf);
            if (!live) continue;
            const SeqCode c = seq_record_codes(r);
            const uint32_t llc = c.llc, mlc = c.mlc, ofc = c.ofc;
            const uint32_t llb = c.llb, mlb = c.mlb;
            if (i == n - 1u) {
                sml = lct_init2(tml, xml, mlc);
                sof = lct_init2(tof, xof, ofc);
                sll = lct_init2(tll, xll, llc);
            } else {
                lct_encode(b, sof, tof, xof, ofc);
                lct_encode(b, sml, tml, xml, mlc);
                lct_encode(b, sll, tll, xll, llc);
                if (ofc + mlb + llb >= 64u - 7u - (9u + 9u + 8u)) lb_flush(b, s);
            }
            lb_add(b, c.llv, llb);
            lb_add(b, c.mlv, mlb);
            lb_add(b, c.ofv, ofc);
            lb_flush(b, s);
        }
    }
    lb_add(b, sml, T[kFseSlot.lml]);
    lb_flush(b, s);
    lb_add(b, sof, T[kFseSlot.lof]);
    lb_flush(b, s);
    lb_add(b, sll, T[kFseSlot.lll]);
    lb_flush(b, s);
    lb_add(b, 1u, 1u);
    lb_flush(b, s);
    if (b.pos > 0) sink_put(s, b.c, 1u);
    sink_end(s);
    return (uint32_t)(s.addr - (uintptr_t)out);
}

// Each lane copies its block's three tables into its own LDS slot (kFseSlot).
__global__ __launch_bounds__(64) void zstd_fse_kernel(tyche_batch_t b, size_t first, size_t count, uint8_t *ws,
                                                      size_t ws_page, const int32_t *st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const size_t j = (size_t)blockIdx.x * kWave + threadIdx.x;
    if (j >= count || st[j] <= 0) return;
    uint8_t *area = ws + j * ws_page;
    const uint32_t nblk = ((const uint32_t *)area)[0];
    uint8_t *dst = batch_page(b, first + j).dst;
    uint32_t *lt = (uint32_t *)smem + threadIdx.x * kFseSlot.words;
    for (uint32_t k = 0; k < nblk; k++) {
        uint32_t *B = area_blk(area, k);
        if (!(B[7] & 2u)) continue;
        const uint32_t *g = area_tab(area, B[6]);
        if (TYCHE_ZSTD_FSE_SLOT) {
            for (uint32_t w = 0; w < 36u; w++) lt[kFseSlot.sll + w] = g[w];
            for (uint32_t w = 0; w < 32u; w++) lt[kFseSlot.sof + w] = g[kCtWords + w];
            for (uint32_t w = 0; w < 53u; w++) lt[kFseSlot.sml + w] = g[2u * kCtWords + w];
            lt[kFseSlot.lll] = g[63];
            lt[kFseSlot.lof] = g[kCtWords + 63u];
            lt[kFseSlot.lml] = g[2u * kCtWords + 63u];
            for (uint32_t w = 0; w < 32u; w++) lt[kFseSlot.xll + w] = g[64u + w];
            for (uint32_t w = 0; w < 16u; w++) lt[kFseSlot.xof + w] = g[kCtWords + 64u + w];
            for (uint32_t w = 0; w < 32u; w++) lt[kFseSlot.xml + w] = g[2u * kCtWords + 64u + w];
        } else {
            for (uint32_t w = 0; w < 3u * kCtWords / 4u; w++) ((u32x4 *)lt)[w] = ((const u32x4 *)g)[w];
        }
        B[3] = fse_lane(dst + B[0] + 3u + B[2], (const uint2 *)area_rec(area), seq_map(area, false), B[5], B[4], lt);
    }
}

// ---- pass C: close the gaps, patch the compressed blocks' headers.  One page per lane
// (round 6; a wave per page before, 12 ms per 1M pages of mostly three-byte header patches):
// a page whose blocks all sit where the frame needs them (every 32 KiB page: one block) is
// patched by its lane; a page with a gap to close is left to the whole wave, one such page
// at a time, after the lane pass.
__device__ __forceinline__ int32_t pack_page_wave(uint8_t *dst, const uint8_t *area, uint32_t lane) {
    const uint32_t nblk = __builtin_amdgcn_readfirstlane(((const uint32_t *)area)[0]);
    uint32_t q = 0;
    for (uint32_t k = 0; k < nblk; k++) {
        const uint32_t *B = (const uint32_t *)(area + kAreaHdr) + k * kBlkWords;
        const uint32_t g = __builtin_amdgcn_readfirstlane(B[0]), glen = __builtin_amdgcn_readfirstlane(B[1]);
        const uint32_t pre = __builtin_amdgcn_readfirstlane(B[2]), fse = __builtin_amdgcn_readfirstlane(B[3]);
        const uint32_t fl = __builtin_amdgcn_readfirstlane(B[7]);
        if (k == 0) q = g;   // the frame header stays
        const bool comp = (fl & 2u) != 0;
        const uint32_t clen = comp ? 3u + pre + fse : glen;
        const uint32_t bh = (fl & 1u) | (2u << 1) | ((pre + fse) << 3);
        if (g == q) {
            if (comp && lane < 3) dst[q + lane] = (uint8_t)(bh >> (8u * lane));
        } else {
            // left move in 64-byte steps: a step's reads precede its writes
            for (uint32_t c0 = 0; c0 < clen; c0 += kWave) {
                const uint32_t i = c0 + lane;
                uint8_t v = i < clen ? dst[g + i] : 0;
                if (comp && i < 3u) v = (uint8_t)(bh >> (8u * i));
                __builtin_amdgcn_wave_barrier();
                if (i < clen) dst[q + i] = v;
                __builtin_amdgcn_wave_barrier();
            }
        }
        q += clen;
    }
    return (int32_t)q;
}
__global__ __launch_bounds__(64) void zstd_pack_kernel(tyche_batch_t b, size_t first, size_t count, uint8_t *ws,
                                                       size_t ws_page, const int32_t *st) {
    const uint32_t lane = threadIdx.x;
    const size_t j = (size_t)blockIdx.x * kWave + lane;
    int32_t rv = j < count ? st[j] : 0;
    bool wave_page = false;
    if (j < count && rv > 0) {
        const uint8_t *area = ws + j * ws_page;
        uint8_t *dst = batch_page(b, first + j).dst;
        const uint32_t nblk = ((const uint32_t *)area)[0];
        uint32_t q = 0;
        for (uint32_t k = 0; k < nblk; k++) {
            const uint32_t *B = (const uint32_t *)(area + kAreaHdr) + k * kBlkWords;
            const uint32_t g = B[0], glen = B[1], pre = B[2], fse = B[3], fl = B[7];
            if (k == 0) q = g;
            if (g != q) {   // a gap to close: the wave's
                wave_page = true;
                break;
            }
            const bool comp = (fl & 2u) != 0;
            if (comp) {
                const uint32_t bh = (fl & 1u) | (2u << 1) | ((pre + fse) << 3);
                dst[q] = (uint8_t)bh;
                dst[q + 1] = (uint8_t)(bh >> 8);
                dst[q + 2] = (uint8_t)(bh >> 16);
            }
            q += comp ? 3u + pre + fse : glen;
        }
        rv = (int32_t)q;
    }
    if (j < count && !wave_page) b.results[first + j] = rv;
    for (uint64_t m = __ballot(wave_page); m; m &= m - 1ull) {
        const uint32_t k = (uint32_t)__builtin_ctzll(m);
        const size_t jj = (size_t)blockIdx.x * kWave + k;
        const int32_t r = pack_page_wave(batch_page(b, first + jj).dst, ws + jj * ws_page, lane);
        if (lane == 0) b.results[first + jj] = r;
    }
}

}  // namespace

#ifdef TYCHE_PROFILE
extern "C" int tyche_debug_zstd_encode_profile(unsigned long long *host16, int reset) {
    if (reset) {
        unsigned long long z[16] = {0};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_seprof), z, sizeof(z)) == hipSuccess ? 0 : 1;
    }
    return hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_seprof), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : 1;
}
#endif

// TYCHE_ZSTD_ENC_SPLIT: 1 (default) four-pass encode for batches of at least
// TYCHE_ZSTD_SPLIT_MIN (4096) pages, 0 one kernel.
hipError_t launch_zstd_encode(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    if (in_cap > 65535u) return hipErrorInvalidValue;    // 16-bit positions in the parse and sequence records
    const size_t page_lds = (in_cap + 16u + kPad + 15u) & ~15u;
    const size_t lds = kTableSlots * sizeof(uint16_t) + kWave + kWave * 8 + kSeqCap * 8 + kHtab * 4 + 256 + page_lds;
    const size_t lds1 = kTableSlots * sizeof(uint16_t) + kWave + kWave * 8 + kWave * 4 + page_lds;   // pass A1 (+ copy map)
    const long mn = knob("ZSTD_SPLIT_MIN", 4096);   // small batches: one launch (latency)
    const size_t split_min = mn > 0 ? (size_t)mn : 4096;
    const bool split = knob("ZSTD_ENC_SPLIT", 1) != 0 && b.count >= split_min;
    // sequence-table accuracy: FSE_optimalTableLog capped at LL/ML 7, OF 6 (6: fixed 6 / 5 / 6, round 2's)
    const uint32_t logcap = knob("ZSTD_FSE_LOG", 7) <= 6 ? 6u : 7u;
    const size_t page_bytes = enc_area_bytes(in_cap);
    // scratch: at most 16 GiB or a quarter of the free memory, as the decoder's (round 6: 8 GiB or an
    // eighth before -- 28 instead of 14 chunks per 1M x 32 KiB pages, encode 553.7 vs 542.6 ms, the
    // FSE pass and every chunk's tail paid per launch; profiles/r06_zstd_ab/c3_pass_ms_litcopy.json)
    size_t budget = (size_t)16 << 30;
    size_t free_b = 0, total_b = 0;
    if (b.count * page_bytes > ((size_t)1 << 30) && hipMemGetInfo(&free_b, &total_b) == hipSuccess && ((free_b += scratch_idle_bytes()), true) &&
        free_b / 4 < budget)
        budget = free_b / 4;
    const long mb = knob("ZSTD_SCRATCH_MB", 0);
    if (mb > 0) budget = (size_t)mb << 20;
    const size_t chunk = split ? std::max<size_t>(1, std::min<size_t>(b.count, budget / page_bytes)) : b.count;
    const size_t st_bytes = (chunk * 4u + 255u) & ~(size_t)255u;
    ScratchLease lease(s, split ? st_bytes + chunk * page_bytes : 0);
    if (!split || !lease.get()) {
        const void *k = (const void *)zstd_encode_kernel<false>;
        const size_t ncu = prepare_launch(k);
        const size_t grid = std::min<size_t>(b.count, ncu * waves_per_cu(k, lds));
        WorkCounter ctr(s, grid < b.count);
        if (!ctr.get()) return hipErrorOutOfMemory;
        hipLaunchKernelGGL(zstd_encode_kernel<false>, dim3((unsigned)grid), dim3(kWave), lds, s, b, (size_t)0, b.count,
                           in_cap, ctr.get(), (uint8_t *)nullptr, (size_t)0, (int32_t *)nullptr, logcap);
        return hipGetLastError();
    }
    int32_t *st = (int32_t *)lease.get();
    uint8_t *ws = (uint8_t *)lease.get() + st_bytes;
    // pass A1's buckets: 4 ways for pages up to TYCHE_ZSTD_WAYS4_MAX bytes (default 16 KiB), 2 above --
    // the same LDS (round 3, 64K bench pages with the repeat slack: 16 KiB ratio 4.709 -> see DESIGN
    // §3.5; tools/parse_sim.c zstd: +0.4 % at 16 KiB, +0.55 % at 32 KiB for the two extra candidates)
    const bool four = kZWays == 2 && (long)in_cap <= knob("ZSTD_WAYS4_MAX", 16384);
    const void *k1 = four ? (const void *)zstd_encode_kernel<true, 4> : (const void *)zstd_encode_kernel<true>;
    const size_t ncu = prepare_launch(k1);
    (void)prepare_launch((const void *)zstd_block_kernel);
    (void)prepare_launch((const void *)zstd_fse_kernel);
    (void)prepare_launch((const void *)zstd_pack_kernel);
    const size_t cu1 = waves_per_cu(k1, lds1), cu2 = waves_per_cu((const void *)zstd_block_kernel, kA2Lds);
    // pass A1 on 1 to 4 waves per page (1: the one-wave parse, 4-way buckets, up to 16 KiB):
    // 4 by default above 16 KiB.  Round 3, 32 KiB bench pages with one block per page
    // (profiles/r03_zstd_parse_ab.log): 2 parts 793 ms per 1M pages at ratio 4.940; 3 parts 823
    // (2 workgroups per CU, the same 6 waves, twice the seeding); 4 parts, part 0 22/64 of the
    // page and 12,288 seed positions: 709 ms at 4.921 -- the reference's level 1 gives 4.915
    const long pw = knob("ZSTD_PARSE_WAVES", four ? 1 : 4);
    const bool psplit = pw >= 2 && pw <= 4;
    const void *kp = pw == 4 ? (const void *)zstd_parse_split_kernel<4>
                   : pw == 3 ? (const void *)zstd_parse_split_kernel<3> : (const void *)zstd_parse_split_kernel<2>;
    const size_t ldsp = (pw == 4 ? zsplit_stage_off<4>() : pw == 3 ? zsplit_stage_off<3>() : zsplit_stage_off<2>()) + page_lds;
    size_t cup = 1;
    if (psplit) {
        (void)prepare_launch(kp);
        int per = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kp, (int)(pw * kWave), ldsp) == hipSuccess && per > 0)
            cup = (size_t)per;
    }
    // pass A1 on two pipelined waves (TYCHE_ZSTD_PARSE_PIPE=1; default 0: one wave per page)
    const bool pipe = !psplit && knob("ZSTD_PARSE_PIPE", 0) != 0;
    const size_t ldsq = kZPipeStage + page_lds;
    size_t cuq = 1;
    if (pipe) {
        (void)prepare_launch((const void *)zstd_parse_pipe_kernel);
        int per = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)zstd_parse_pipe_kernel, 2 * (int)kWave, ldsq) ==
                hipSuccess && per > 0)
            cuq = (size_t)per;
    }
    for (size_t first = 0; first < b.count; first += chunk) {
        const size_t n = std::min(chunk, b.count - first);
        if (pipe) {
            const size_t g = std::min<size_t>(n, ncu * cuq);
            WorkCounter ctr(s, g < n);
            if (!ctr.get()) return hipErrorOutOfMemory;
            hipLaunchKernelGGL(zstd_parse_pipe_kernel, dim3((unsigned)g), dim3(2 * kWave), ldsq, s, b, first, n, in_cap,
                               ctr.get(), ws, page_bytes, st);
        } else if (psplit) {   // pass A1 on pw waves per page
            const size_t g = std::min<size_t>(n, ncu * cup);
            WorkCounter ctr(s, g < n);
            if (!ctr.get()) return hipErrorOutOfMemory;
            unsigned *cp = ctr.get();
            size_t fst = first, cnt = n, wpage = page_bytes;
            uint32_t icap = in_cap;
            // positions seeded before each part (4 parts: 8,192 -> 12,288 seeds 701 -> 709 ms, ratio
            // 4.910 -> 4.921; 16,384: 719 ms at 4.921)
            uint32_t seed = (uint32_t)std::max(0L, knob("ZSTD_PARSE_SEED", pw == 4 ? 12288L : (long)kZSeed)) &
                            ~(kWave - 1u);
            // part 0's share in 64ths (0: equal parts), between 1/pw and 2/pw of the page: every part's
            // sequences (<= a quarter of its bytes) fit its slice of 2 * rec_cap / pw entries
            // (two parts: 35/64, 843 vs 869 ms per 1M x 32 KiB pages, ratio 4.946 vs 4.951; 33 / 34:
            // 854 / 847 ms.  Four parts: 22/64, 700 ms at 4.910 vs 16 (equal) 723 at 4.908, 20 702 at
            // 4.910, 24 719 at 4.904, 27 772 at 4.893)
            uint32_t p0 = (uint32_t)std::max(0L, knob("ZSTD_PARSE_P0", pw == 2 ? 35L : pw == 4 ? 22L : 0L));
            if (p0)
                p0 = std::min<uint32_t>(std::max<uint32_t>(p0, (64u + (uint32_t)pw - 1u) / (uint32_t)pw),
                                        std::min<uint32_t>(48u, 128u / (uint32_t)pw));
            void *args[] = {(void *)&b, &fst, &cnt, &icap, &cp, &ws, &wpage, &st, &seed, &p0};
            (void)hipLaunchKernel(kp, dim3((unsigned)g), dim3((unsigned)(pw * kWave)), args, ldsp, s);
        } else {
            const size_t g = std::min<size_t>(n, ncu * cu1);
            WorkCounter ctr(s, g < n);
            if (!ctr.get()) return hipErrorOutOfMemory;
            unsigned *cp = ctr.get();
            uint8_t *wsp = ws;
            size_t fst = first, cnt = n, wpage = page_bytes;
            uint32_t icap = in_cap, lc = logcap;
            void *args[] = {(void *)&b, &fst, &cnt, &icap, &cp, &wsp, &wpage, &st, &lc};
            (void)hipLaunchKernel(k1, dim3((unsigned)g), dim3(kWave), args, lds1, s);
        }
        {
            const size_t g = std::min<size_t>(n, ncu * cu2);
            WorkCounter ctr(s, g < n);
            if (!ctr.get()) return hipErrorOutOfMemory;
            hipLaunchKernelGGL(zstd_block_kernel, dim3((unsigned)g), dim3(kWave), kA2Lds, s, b, first, n, in_cap, ws,
                               page_bytes, st, ctr.get(), logcap);
        }
        hipLaunchKernelGGL(zstd_fse_kernel, dim3((unsigned)((n + kWave - 1) / kWave)), dim3(kWave),
                           kWave * kFseSlot.words * 4u, s, b, first, n, ws, page_bytes, (const int32_t *)st);
        hipLaunchKernelGGL(zstd_pack_kernel, dim3((unsigned)((n + kWave - 1) / kWave)), dim3(kWave), 0, s, b, first, n, ws,
                           page_bytes, (const int32_t *)st);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace tyche
