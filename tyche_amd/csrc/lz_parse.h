// lz_parse.h -- the wave-parallel greedy LZ77 parse shared by the gfx950
// encoders (LZ4 blocks, zstd frames).
//
// One 64-lane wave parses one page held in LDS next to a table of 2^11 16-bit
// positions (the byU16 scheme of lz4.c:402-408, hash 2654435761 of 4 bytes; the
// reference's table has 2^13 slots -- 2^11 keeps the ratio within 0.5 % on the
// bench pages and raises residency from 6 to 7 waves per CU at 16 KiB pages;
// the LZ4 encoder takes 2^10 for 8 waves per CU, lz4_encode.hip).
// The page is scanned in blocks of 64 positions:
//   * every lane hashes its position, takes the candidate left by earlier
//     blocks, verifies 4 bytes, probes the match length up to 20 bytes and the
//     backward extension up to 4 bytes (lz4.c:549's catch-up);
//   * the greedy parse over the block runs on scalar registers only: first
//     match at or after the cursor (ballot mask), cursor = its end; a match
//     that reached the probe limit is extended by the whole wave (256 bytes per
//     step);
//   * selected matches are appended to LDS records in stream order and handed
//     to the codec's sink in batches of at most 64.
// Every match starts at or before L-MFLIMIT (12) and ends at or before
// L-LASTLITERALS (5) (lz4.c:266-267): required by the LZ4 block format,
// harmless for zstd.
#pragma once
#include <hip/hip_runtime.h>

#include "engine.h"
#include "lds_io.h"

namespace tyche {
namespace lzp {

constexpr uint32_t kWave = 64;
#ifndef TYCHE_HASH_LOG
#define TYCHE_HASH_LOG 11
#endif
constexpr uint32_t kHashLog = TYCHE_HASH_LOG;
constexpr uint32_t kHashSize = 1u << kHashLog;
#ifndef TYCHE_PROBE_WORDS
#define TYCHE_PROBE_WORDS 4
#endif
constexpr uint32_t kProbeWords = TYCHE_PROBE_WORDS;   // 4-byte words probed per lane beyond MINMATCH
constexpr uint32_t kProbe = 4 * kProbeWords;

// Timing-only ablation builds (-DTYCHE_EABLATE=mask; outputs are wrong):
//   1 skip the byte emission loop (sizes still computed), 2 no probes (every match 4 bytes),
//   4 no greedy parse (no sequences: the page becomes one literal run)
//   8 no whole-wave extension of probe-capped matches (valid output, shorter matches)
#ifndef TYCHE_EABLATE
#define TYCHE_EABLATE 0
#endif

// Profiling-only builds (-DTYCHE_PHASES, tools/phase_prof.py): per-phase wave
// cycles of the parse (s_memtime; each read waits for outstanding LDS ops),
// summed over pages into g_phase.  Only the LZ4 encoder's translation unit
// (TYCHE_PHASES_OWNER) is instrumented.
#if defined(TYCHE_PHASES) && defined(TYCHE_PHASES_OWNER)
__device__ unsigned long long g_phase[16];
__device__ __forceinline__ uint32_t phase_clock() { return (uint32_t)__builtin_amdgcn_s_memtime(); }
#define PHASE_INIT() uint32_t ph_t_ = phase_clock(), ph_[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}
#define PHASE(i) do { const uint32_t t_ = phase_clock(); ph_[i] += t_ - ph_t_; ph_t_ = t_; } while (0)
#define PHASE_COUNT(i) ph_[i]++
#define PHASE_FLUSH() do { if (lane == 0) for (int i_ = 0; i_ < 12; i_++) if (i_ != 7) atomicAdd(&g_phase[i_], (unsigned long long)ph_[i_]); \
                           if (lane == 0) atomicAdd(&g_phase[7], 1ull); } while (0)
#else
#define PHASE_INIT() do {} while (0)
#define PHASE(i) do {} while (0)
#define PHASE_COUNT(i) do {} while (0)
#define PHASE_FLUSH() do {} while (0)
#endif

__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

// The page is read as aligned dwords only: an LDS read off its natural
// alignment (a 4-byte read at an odd address, a b64/b128 off 8/16) is replayed
// at ~64 LDS cycles per wave instruction, which made the parse LDS-bound
// (SQ_LDS_UNALIGNED_STALL ~90 % of LDS-active cycles).  A is the page's base
// rounded down to 4 bytes and q a byte offset from it (position + (in & 3)).
__device__ __forceinline__ uint32_t word_at(uint32_t lo, uint32_t hi, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);   // bytes s..s+3 of hi:lo
}
__device__ __forceinline__ uint32_t lds_word(const uint32_t *A, uint32_t q) {
    return word_at(A[q >> 2], A[(q >> 2) + 1], q & 3u);
}

// A 28-byte window around byte offset q (q - 4 .. q + 23, within 7 aligned
// dwords): the word at q - 4 (backward probe), at q (MINMATCH verify) and the
// kProbeWords words after it (forward probe).
struct Window {
    uint32_t back, w0, fw[kProbeWords];
};
__device__ __forceinline__ Window lds_window(const uint32_t *A, uint32_t q) {
    static_assert(kProbeWords == 4, "the window holds four probe words");
    const uint32_t i = q >> 2, s = q & 3u;
    const uint32_t dm = A[max(i, 1u) - 1];   // q < 4 only at positions < 4, whose backward probe is unused
    uint32_t d[6];
#pragma unroll
    for (int j = 0; j < 6; j++) d[j] = A[i + j];
    Window r;
    r.back = word_at(dm, d[0], s);
    r.w0 = word_at(d[0], d[1], s);
#pragma unroll
    for (int k = 0; k < 4; k++) r.fw[k] = word_at(d[k + 1], d[k + 2], s);
    return r;
}

// LDS byte address of a pointer into LDS, and a dword pointer from one: the LZ4
// encoder addresses a lane's windows from a per-lane base fixed for the page
// (TYCHE_LANE_ADDR below), so a block's window costs one add and one min
// instead of the nine address instructions of lds_window's general form.
typedef const __attribute__((address_space(3))) uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)p;
}
// the window of lds_window from the LDS byte address a of the dword before the
// one holding q (q's byte shift s = q & 3)
__device__ __forceinline__ Window lds_window_at(uint32_t a, uint32_t s) {
    const lds_u32_t *P = (const lds_u32_t *)(uintptr_t)a;
    uint32_t d[7];
#pragma unroll
    for (int j = 0; j < 7; j++) d[j] = P[j];
    Window r;
    r.back = word_at(d[0], d[1], s);
    r.w0 = word_at(d[1], d[2], s);
#pragma unroll
    for (int k = 0; k < 4; k++) r.fw[k] = word_at(d[k + 2], d[k + 3], s);
    return r;
}

// LDS byte address of 16-bit table slot h: one v_lshl_add_u32 (the compiler's own form of
// base + 2 * (x >> 22) is a shift, a mask and an add)
typedef __attribute__((address_space(3))) uint16_t lds_u16_t;
__device__ __forceinline__ uint32_t slot_addr(uint32_t tbase, uint32_t h) {
    uint32_t a;
    asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(a) : "v"(h), "s"(tbase));
    return a;
}

// v_ffbl_b32: the lowest set bit, 0xFFFFFFFF for 0 (cttz without the zero select)
__device__ __forceinline__ uint32_t ffbl_raw(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
// v_ffbh_u32: the leading zeros, 0xFFFFFFFF for 0
__device__ __forceinline__ uint32_t ffbh_raw(uint32_t x) {
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
// MINMATCH + the equal leading bytes of the forward probe words a, b (4 + kProbe when all
// are equal): the first set bit of the 128-bit difference from one min over per-word bit
// positions (0xFFFFFFFF stays above every real one), 15 instructions instead of 24
__device__ __forceinline__ uint32_t probe_len(const uint32_t (&a)[kProbeWords], const uint32_t (&b)[kProbeWords]) {
    static_assert(kProbeWords == 4, "four probe words");
    const uint32_t t0 = ffbl_raw(a[0] ^ b[0]), t1 = ffbl_raw(a[1] ^ b[1]) | 32u, t2 = ffbl_raw(a[2] ^ b[2]) | 64u,
                   t3 = ffbl_raw(a[3] ^ b[3]) | 96u;
    return 4u + (min(min(t0, t1), min(min(t2, t3), 128u)) >> 3);
}

// equal bytes at a and b going forward, a stopping before `limit` (whole wave,
// 256 bytes per step); a, b, limit are positions, ib = (in & 3)
__device__ inline uint32_t wave_extend(const uint8_t *in, const uint32_t *A, uint32_t ib, uint32_t a, uint32_t b,
                                       uint32_t limit, uint32_t lane) {
    uint32_t n = 0;
    for (;;) {
        const uint32_t pa = a + n + 4 * lane;
        const bool full = pa + 4 <= limit;
        const uint32_t x = full ? (lds_word(A, pa + ib) ^ lds_word(A, b + n + 4 * lane + ib)) : 1u;
        const uint64_t bad = __ballot(x != 0);
        if (bad == 0) {
            n += 4 * kWave;
            continue;
        }
        const uint32_t first = (uint32_t)__builtin_ctzll(bad);
        const uint32_t pf = a + n + 4 * first;
        if (pf + 4 <= limit) return n + 4 * first + (__builtin_ctz(rdlane(x, first)) >> 3);
        uint32_t m = n + 4 * first;   // fewer than 4 bytes left before the limit
        while (a + m < limit && in[a + m] == in[b + m]) m++;
        return rfl(m);
    }
}

// Backward extension of the match at pos from cand (lz4.c:549's catch-up, up to 4 bytes): the
// equal bytes before both, 0 when cand < 4 (a match has cand < pos).  Parses whose records leave
// it to the sink (parse_page's kSinkBack) compute it there for the ~50 selected matches of a call
// instead of for every lane of every block.
__device__ __forceinline__ uint32_t back_at(const uint8_t *in, uint32_t pos, uint32_t cand) {
    const uint32_t ib = (uint32_t)(uintptr_t)in & 3u;
    const uint32_t *A = (const uint32_t *)(in - ib);
    const uint32_t a = lds_word(A, max(pos, 4u) - 4u + ib), b = lds_word(A, max(cand, 4u) - 4u + ib);
    const uint32_t x = min(ffbh_raw(a ^ b), 32u) >> 3;   // (v_ffbh_u32: 0xFFFFFFFF for equal words)
    return cand < 4u ? 0u : x;
}

// A record: x = pos | cand << 16, y = len | back << 16 (match at pos from cand,
// len bytes forward, up to `back` bytes of backward extension available; with
// `in` given, the back field is not used and the extension comes from the page).
// The literal run before a record starts at the previous record's end (or the
// anchor); the catch-up actually taken is min(back, pos - prev_end, cand).
__device__ __forceinline__ void decode_record(const uint2 *rec, uint32_t n, uint32_t anchor, uint32_t lane,
                                              uint32_t &lit_start, uint32_t &lit_len, uint32_t &match_len,
                                              uint32_t &offset, const uint8_t *in = nullptr) {
    const bool is_sel = lane < n;
    const uint2 r = rec[is_sel ? lane : 0];
    const uint2 rp = rec[lane > 0 && is_sel ? lane - 1 : 0];
    const uint32_t pos = r.x & 0xFFFFu, cand = r.x >> 16, len = r.y & 0xFFFFu;
    const uint32_t back = in ? back_at(in, pos, cand) : r.y >> 16;
    const uint32_t prev_end = lane == 0 ? anchor : (rp.x & 0xFFFFu) + (rp.y & 0xFFFFu);
    const uint32_t k = min(min(back, pos - prev_end), cand);
    lit_start = prev_end;
    lit_len = is_sel ? pos - k - prev_end : 0u;
    match_len = is_sel ? len + k : 0u;
    offset = pos - cand;
}

// Greedy parse of in[0, L) (LDS, 64 zero bytes after).  table: kHashSize 16-bit
// slots, zeroed by the caller.  rec: 64 uint2 records.  sink(rec, n, anchor)
// consumes n >= 1 records whose literal runs start at `anchor`, and returns
// false to abort.  Returns the anchor where the last literal run starts, or
// 0xFFFFFFFF if the sink aborted.
//
// kRepCand (zstd): every position also tries the repeat-offset candidates
// pos - R and pos - R2, (R, R2) = the first two repeat offsets after the
// matches selected before this block (zstd's fast parse checks repeat offset 1
// at ip+1 before the hash candidate at ip, zstd_compress.c:951-958, and
// repeat offset 2 right after each match, :985-994).  A repeat candidate is
// taken when it verifies and is at least as long as the hash candidate's
// match, and a position whose successor has a repeat match starts none of its
// own: a repeat offset costs a few bits instead of ~10 (zstd_encode.hip).
//
// kMin3 (deflate): matches from 3 bytes on (MIN_MATCH, deflate.h; deflate_fast
// takes any match >= MIN_MATCH): candidates verify on 3 bytes, and every
// position also tries distance 4 straight from its own window -- arrays of
// 4-byte items that differ in one byte (page line pointers) are level 1's most
// common 3-byte match (16 % of its matches on the bench pages).  A 3-byte
// table of its own was tried: +0.3 % ratio for +8 % encode time.
//
// start (a multiple of 64, default 0): parse [start, L) only, with the table
// holding earlier positions already (the split LZ4 encoder's second wave); the
// first literal run starts at `start`.
//
// kWays (deflate: 4): the table is 2 * kHashSize (TYCHE_WAYS_SCALE) 16-bit slots in buckets of
// kWays positions, most recent first (table_slots<kWays>()); every position
// verifies all of its bucket's candidates and keeps the longest match (the
// most recent of equally long ones) -- deflate_fast's hash chain cut at 4
// (max_chain 4 at level 1, deflate.c:134), with a bucket standing in for the
// chain.  Lanes of one block that share a bucket insert in unspecified order
// (one of them wins), as the single-slot table does.
#ifndef TYCHE_HASH3
#define TYCHE_HASH3 1   // kMin3 with buckets: hash 3 bytes (deflate's MIN_MATCH), not 4
#endif
#ifndef TYCHE_WAYS_SCALE
#define TYCHE_WAYS_SCALE 2   // bucketed tables hold TYCHE_WAYS_SCALE * kHashSize slots
#endif
// kRepCand (zstd) with 2 or 4 ways: 2 * TYCHE_ZSTD_BUCKETS slots in buckets of
// kWays, a bucket count that is not a power of two -- 3,712 slots (7,424 bytes)
// keep a 32 KiB page's parse at 40,848 bytes of LDS, 4 waves per CU
// (zstd_encode.hip); the bucket is the high product of the hash
#ifndef TYCHE_ZSTD_BUCKETS
#define TYCHE_ZSTD_BUCKETS 1856
#endif
template <int kWays, bool kRepCand = false>
__host__ __device__ constexpr uint32_t table_slots() {
    return kRepCand && (kWays == 2 || kWays == 4) ? 2u * TYCHE_ZSTD_BUCKETS
                                                  : kWays > 1 ? TYCHE_WAYS_SCALE * kHashSize : kHashSize;
}

template <int kWays>
__device__ __forceinline__ uint32_t bucket_of(uint32_t v, uint32_t v2 = 0, uint32_t nbytes = 4) {
    constexpr uint32_t nb = table_slots<kWays>() / kWays;
    constexpr uint32_t lg = nb >= 4096 ? 12 : nb >= 2048 ? 11 : nb >= 1024 ? 10 : nb >= 512 ? 9 : 8;
    static_assert((1u << lg) == nb, "bucket count is a power of two");
    if (nbytes > 4) {   // 5 or 6 bytes: zstd's fast parse hashes searchLength bytes (ZSTD_hashPtr)
        const uint64_t x = ((uint64_t)(v2 & (nbytes == 5 ? 0xFFu : 0xFFFFu)) << 32) | v;
        const uint64_t hx = x * 0xCF1BBCDCB7A56463ull;
        if (kWays == 2 || kWays == 4) return (uint32_t)(((hx >> 32) * (uint64_t)(2u * TYCHE_ZSTD_BUCKETS / kWays)) >> 32);
        return (uint32_t)(hx >> (64 - lg));
    }
    return (v * 2654435761u) >> (32 - lg);
}
#ifndef TYCHE_PW_PREFETCH
// 1: parse_page loads the next block's window ahead, with the current block's candidate
// windows.  Measured (round 3, 1M x 16 KiB LZ4 pages): 85.0 ms off, 85.9-86.1 on; zlib 645 /
// 650 -- the LDS latency it hides is not what bounds the parse, and its 6 VGPRs cost.  Off.
#define TYCHE_PW_PREFETCH 0
#endif
#ifndef TYCHE_LANE_ADDR
// 1: parse_page's windows from LDS addresses (lds_window_at): a lane's own window from a base
// fixed for the page, candidates' from the page's base.  Lanes past mflimit read mflimit's dword
// (the LZ4 encoder with their own shift: unused values, inserts that no lookup follows); a window
// below position 4 reads the dword before the page (unused: such positions and candidates take no
// backward extension), so every caller keeps LDS in front of the page.
#define TYCHE_LANE_ADDR 1
#endif
#ifndef TYCHE_SINK_BACK
#define TYCHE_SINK_BACK 1   // zstd: backward extension computed by the sinks (decode_record with `in`)
#endif
#ifndef TYCHE_HASH_BYTES
#define TYCHE_HASH_BYTES 5   // kRepCand (zstd): bytes hashed -- zstd level 1 hashes searchLength bytes
#endif

//
// rep (kRepCand, optional): the repeat offsets {R, R2} to start from, and where the final ones go -- a
// part of a split parse (zstd_encode.hip) warms them up by parsing the bytes before it.
template <bool kRepCand = false, bool kMin3 = false, int kWays = 1, typename Sink>
__device__ inline uint32_t parse_page(const uint8_t *in, uint32_t L, uint16_t *table, uint2 *rec, uint32_t lane,
                                      Sink &sink, uint32_t start = 0, uint32_t *rep = nullptr) {
    static_assert(kWays == 1 || kWays == 2 || kWays == 4 || kWays == 8, "1, 2, 4 or 8 ways");
    uint32_t anchor = start;
    if (L < (uint32_t)(kMfLimit + 1) || start > L - kMfLimit) return start;   // (rep unchanged)
    const uint32_t mflimit = L - kMfLimit;          // last position a match may start
    const uint32_t matchlimit = L - kLastLiterals;  // matches end at or before this
    const uint32_t ib = (uint32_t)(uintptr_t)in & 3u;               // in's offset from a dword boundary
    const uint32_t *A = (const uint32_t *)(in - ib);                // the page as aligned dwords
    uint32_t cursor = start; // matches may start here (end of the last match)
    uint32_t nacc = 0;       // records accumulated since the last hand-off
    uint32_t blk = start;    // current 64-position block
    uint32_t R = rep ? rep[0] : 1u, R2 = rep ? rep[1] : 4u;   // repeat offsets 1 and 2 (kRepCand): zstd's initial {1, 4}
    bool done = false;
    Window pwn{};                       // TYCHE_PW_PREFETCH: the next block's window, loaded ahead
    uint32_t pwn_blk = 0xFFFFFFFFu;     // the block it belongs to (none yet)
    constexpr bool kLaneAddr = TYCHE_LANE_ADDR && !TYCHE_PW_PREFETCH;
    const uint32_t abase = rfl(lds_addr(A));
    const uint32_t la = abase + ((lane + ib) & ~3u) - 4u;              // this lane's window at block 0
    const uint32_t la_max = abase + ((mflimit + ib) & ~3u) - 4u;       // mflimit's window
    const uint32_t lsh = (lane + ib) & 3u;                             // (blocks are 64-aligned)
    const uint32_t tbase = rfl(lds_addr(table));
    // lanes past mflimit read mflimit's window exactly (its shift too) where their table inserts
    // can be followed by lookups: a zstd part's warm-up parse shares its table with the part
    constexpr bool kExactDead = kWays > 1 || kRepCand || kMin3;
    const uint32_t msh = (mflimit + ib) & 3u;
    // a candidate's window (a position <= mflimit) from its LDS address
    auto win_at = [&](uint32_t x) { return lds_window_at(abase - 4u + ((x + ib) & ~3u), (x + ib) & 3u); };
    PHASE_INIT();
    for (; !done && blk <= mflimit; blk = max(blk + kWave, cursor & ~(kWave - 1))) {
        const uint32_t pos = blk + lane;
        const bool live = pos <= mflimit;
        // ---- this position's window (lanes past mflimit read mflimit's: their
        // values are unused), its hash and the candidate left by earlier blocks,
        // then insert this block's positions.  Every lane takes part, branch-free:
        // lanes past mflimit only exist in the last block, and no lookup follows
        // their inserts.
        const Window pw = kLaneAddr ? lds_window_at(min(la + blk, la_max), kExactDead && !live ? msh : lsh)
                          : (TYCHE_PW_PREFETCH && pwn_blk == blk) ? pwn : lds_window(A, (live ? pos : mflimit) + ib);
        const uint32_t v = pw.w0;
        constexpr uint32_t vm = kMin3 ? 0xFFFFFFu : 0xFFFFFFFFu;   // the bytes a candidate must match
        uint32_t cands[kWays];
        if (kWays == 1) {
            const uint32_t h = kRepCand && TYCHE_HASH_BYTES > 4
                                   ? (uint32_t)(((((uint64_t)(pw.fw[0] & (TYCHE_HASH_BYTES == 5 ? 0xFFu : 0xFFFFu)) << 32) | v) *
                                                 0xCF1BBCDCB7A56463ull) >> (64 - kHashLog))
                                   : hash4(v);
            if (kLaneAddr && !kRepCand) {
                lds_u16_t *slot = (lds_u16_t *)(uintptr_t)slot_addr(tbase, h);
                cands[0] = *slot;
                __builtin_amdgcn_wave_barrier();
                *slot = (uint16_t)pos;
            } else {
                cands[0] = table[h];
                __builtin_amdgcn_wave_barrier();
                table[h] = (uint16_t)pos;
            }
        } else if (kWays == 2) {
            uint32_t *T = (uint32_t *)table;
            const uint32_t h = kRepCand ? bucket_of<kWays>(v, pw.fw[0], TYCHE_HASH_BYTES)
                                        : bucket_of<kWays>(kMin3 && TYCHE_HASH3 ? v & 0xFFFFFFu : v);
            const uint32_t bk = T[h];
            cands[0] = bk & 0xFFFFu;
            cands[kWays > 1 ? 1 : 0] = bk >> 16;
            __builtin_amdgcn_wave_barrier();
            T[h] = pos | (bk << 16);
        } else if (kWays == 4) {
            uint2 *T = (uint2 *)table;
            const uint32_t h = kRepCand ? bucket_of<kWays>(v, pw.fw[0], TYCHE_HASH_BYTES)
                                        : bucket_of<kWays>(kMin3 && TYCHE_HASH3 ? v & 0xFFFFFFu : v);
            const uint2 bk = T[h];
            cands[0] = bk.x & 0xFFFFu;
            cands[kWays > 1 ? 1 : 0] = bk.x >> 16;
            cands[kWays > 2 ? 2 : 0] = bk.y & 0xFFFFu;
            cands[kWays > 3 ? 3 : 0] = bk.y >> 16;
            __builtin_amdgcn_wave_barrier();
            T[h] = make_uint2(pos | (bk.x << 16), (bk.x >> 16) | (bk.y << 16));
        } else {
            // 8 ways (deflate): a bucket is one aligned 16-byte LDS word of 8 positions, most
            // recent first -- deflate_fast's chain of 4 over a 2^15-head table keeps more
            // distinct candidates than 4 ways over 2^10 buckets (tools/parse_sim.c: 16 KiB
            // pages 4.29 -> 4.35 in the cost model, zlib level 1's own parse 4.34)
            uint4 *T = (uint4 *)table;
            const uint32_t h = bucket_of<kWays>(kMin3 && TYCHE_HASH3 ? v & 0xFFFFFFu : v);
            const uint4 bk = T[h];
            cands[0] = bk.x & 0xFFFFu;
            cands[kWays > 1 ? 1 : 0] = bk.x >> 16;
            cands[kWays > 2 ? 2 : 0] = bk.y & 0xFFFFu;
            cands[kWays > 3 ? 3 : 0] = bk.y >> 16;
            cands[kWays > 4 ? 4 : 0] = bk.z & 0xFFFFu;
            cands[kWays > 5 ? 5 : 0] = bk.z >> 16;
            cands[kWays > 6 ? 6 : 0] = bk.w & 0xFFFFu;
            cands[kWays > 7 ? 7 : 0] = bk.w >> 16;
            __builtin_amdgcn_wave_barrier();
            T[h] = make_uint4(pos | (bk.x << 16), (bk.x >> 16) | (bk.y << 16), (bk.y >> 16) | (bk.z << 16),
                              (bk.z >> 16) | (bk.w << 16));
        }
        // ---- the candidate's window: 4-byte verify, forward probe (MINMATCH + up
        // to kProbe bytes) and backward probe (up to 4 bytes).  A candidate is a
        // position <= mflimit, so the window stays inside the page's zero pad.
        uint32_t cand = cands[0];
        Window cw = kLaneAddr ? win_at(cand) : lds_window(A, cand + ib);
        // deflate (kMin3): a candidate beyond the 32 KiB window cannot be coded; rejecting it here
        // lets a nearer bucket entry win (pages over 32 KiB)
        bool ok = live & (cand < pos) & (!kMin3 || pos - cand <= 32768u) & (((cw.w0 ^ v) & vm) == 0u);
        // one hash candidate and nothing else (LZ4): the probe waits until a match is known to
        // start at or after the cursor (kLateProbe), otherwise the candidates compare lengths here
        constexpr bool kLateProbe = kWays == 1 && !kRepCand && !kMin3;
        // the LZ4 encoder and the zstd encoder (TYCHE_SINK_BACK) take the backward extension in
        // their sinks; not deflate, whose distance-4 candidate takes none by construction
        constexpr bool kSinkBack = kLateProbe || (TYCHE_SINK_BACK && kRepCand && !kMin3);
        uint32_t n = kLateProbe ? 0u : probe_len(pw.fw, cw.fw);
        if (kMin3 && cw.w0 != v) n = 3u;
#pragma unroll
        for (int w = 1; w < kWays; w++) {
            // older bucket entries: taken only when strictly longer
            const uint32_t cw2 = cands[w];
            const Window ww = kLaneAddr ? win_at(cw2) : lds_window(A, cw2 + ib);
            const bool okw = live & (cw2 < pos) & (!kMin3 || pos - cw2 <= 32768u) & (((ww.w0 ^ v) & vm) == 0u);
            uint32_t nw = probe_len(pw.fw, ww.fw);
            if (kMin3 && ww.w0 != v) nw = 3u;
            if (okw && (!ok || nw > n)) {
                cand = cw2;
                cw = ww;
                n = nw;
                ok = true;
            }
        }
        if (TYCHE_PW_PREFETCH) {
            // the next block's window goes out with this block's candidate windows: its LDS
            // latency overlaps this block's compares and walk instead of heading the next
            // block's chain (window -> hash -> table -> candidate window).  A walk that
            // jumps past the next block (a match running beyond it) reloads.
            const uint32_t np = blk + kWave + lane;
            pwn = lds_window(A, (np <= mflimit ? np : mflimit) + ib);
            pwn_blk = blk + kWave;
        }
        if (kMin3) {
            // distance 4 straight from this position's window (arrays of 4-byte
            // items differing in one byte), taken when at least as long
            const bool okd = live & (pos >= 4u) & (((pw.back ^ v) & vm) == 0u);
            uint32_t nd = 4u + kProbe;
#pragma unroll
            for (int k = (int)kProbeWords - 1; k >= 0; k--) {
                const uint32_t x = pw.fw[k] ^ (k ? pw.fw[k > 0 ? k - 1 : 0] : v);
                if (x) nd = 4u + 4u * (uint32_t)k + ((uint32_t)__builtin_ctz(x) >> 3);
            }
            if (pw.back != v) nd = 3u;
            if (okd && (!ok || nd >= n)) {
                cand = pos - 4u;
                cw.back = ~pw.back;   // no backward extension (the word before pos - 4 is not in the window)
                cw.w0 = pw.back;
                n = nd;
                ok = true;
            }
        }
        bool rok = false;
        if (kRepCand) {
            // the repeat-offset candidate (consecutive windows: cheap loads)
            const uint32_t rc = pos >= R ? pos - R : 0u;
            const Window rw = kLaneAddr ? win_at(min(rc, mflimit)) : lds_window(A, min(rc, mflimit) + ib);
            rok = live & (pos >= R) & (((rw.w0 ^ v) & vm) == 0u);
            uint32_t rn = probe_len(pw.fw, rw.fw);
            if (kMin3 && rw.w0 != v) rn = 3u;
#ifndef TYCHE_REP_SLACK
// a repeat candidate wins when at most this many bytes shorter than the hash candidate: a repeat
// offset costs a few bits instead of ~10-14 (round 3, 64K bench pages: slack 0 / 2 / 3 / 4 ratio
// 4.676 / 4.708 / 4.709 / 4.704 at 16 KiB, 4.947 / 4.988 / 4.989 / 4.981 at 32 KiB, encode time
// unchanged; tools/parse_sim.c zfse put 3 at level 1's ratio)
#define TYCHE_REP_SLACK 3
#endif
            // repeat offset 2 (the other offset of two alternating ones)
            const uint32_t rc2 = pos >= R2 ? pos - R2 : 0u;
            const Window rw2 = kLaneAddr ? win_at(min(rc2, mflimit)) : lds_window(A, min(rc2, mflimit) + ib);
#ifndef TYCHE_REP2
#define TYCHE_REP2 1
#endif
            const bool rok2 = TYCHE_REP2 && live & (pos >= R2) & (((rw2.w0 ^ v) & vm) == 0u) & (R2 != R);
            uint32_t rn2 = probe_len(pw.fw, rw2.fw);
            if (kMin3 && rw2.w0 != v) rn2 = 3u;
            if (rok && (!ok || rn + TYCHE_REP_SLACK >= n)) {
                cand = rc;
                cw = rw;
                n = rn;
                ok = true;
            }
            if (rok2 && (!ok || rn2 + TYCHE_REP_SLACK >= n) && !(rok && rn >= rn2)) {
                cand = rc2;
                cw = rw2;
                n = rn2;
                ok = true;
            }
            rok |= rok2;
        }
        // match length within the probe limit and matchlimit; capped: it reached the probe limit
        // before matchlimit (its end is not known yet).  n <= kMinMatch + kProbe, so
        // min(n, min(matchlimit, pos + 20) - pos) is min(n, matchlimit - pos) (for lanes past
        // matchlimit both wrap to n; their values are never used)
        uint32_t len = 0, back = 0;
        bool capped = false;
        auto lengths = [&]() {
            if (kLateProbe) n = probe_len(pw.fw, cw.fw);
            n = min(n, matchlimit - pos);
            len = (TYCHE_EABLATE & 2) ? 4u : n;
            capped = !(TYCHE_EABLATE & 2) && n == kMinMatch + kProbe &&
                     (int32_t)pos < (int32_t)matchlimit - (int32_t)(kMinMatch + kProbe);
            // backward extension: the equal bytes before both positions, up to 4 (a selected match
            // has cand < pos, so cand < 4 covers pos < 4); v_ffbh_u32 gives 0xFFFFFFFF for equal
            // words (the asm result computed unconditionally: inline asm is never speculated, so
            // inside the select it would become a branch)
            // (kSinkBack: the sink computes the extension for the selected matches only, from the
            // page -- back_at; the record carries 0)
            if (!kSinkBack) {
                const uint32_t bx = min(ffbh_raw(pw.back ^ cw.back), 32u) >> 3;
                back = (TYCHE_EABLATE & 2) || cand < 4 ? 0u : bx;
            }
        };
        if (!kLateProbe) lengths();
        // ---- greedy parse of this block.  Every lane first finds the next match
        // lane at or after its own match's end (64: none in this block; 128: the
        // match reached the probe limit, end not known yet), so the walk from the
        // parse position is one v_readlane per selected match.  The parse
        // position is always inside the block (blk >= cursor & ~63), and no mask
        // bit lies past mflimit, so a match ending there ends the walk.
        // (the single-candidate parse ballots its three conditions separately: each compare's lane
        // mask goes straight into the scalar AND, where a ballot of the combined bool is turned into
        // a 0/1 vector value and compared back)
        uint64_t mall = (TYCHE_EABLATE & 4) ? 0ull
                      : kLateProbe ? __builtin_amdgcn_ballot_w64(live) & __builtin_amdgcn_ballot_w64(cand < pos) &
                                         __builtin_amdgcn_ballot_w64(((cw.w0 ^ v) & vm) == 0u)
                                   : __ballot(ok);
#ifndef TYCHE_REP_NEXT
#define TYCHE_REP_NEXT 1
#endif
        if (kRepCand && TYCHE_REP_NEXT) {
            // zstd's fast parse tries the repeat offset at ip+1 before the hash
            // candidate at ip (zstd_compress.c:951-958): a position whose
            // successor has a repeat match starts no match of its own unless
            // it is a repeat match itself
            const uint64_t mrep = __ballot(rok);
            mall &= ~(mrep >> 1) | mrep;
        }
        PHASE(0);
        PHASE_COUNT(8);
        // (a signed max on the scalar unit: an unsigned saturating subtract goes to a vector ALU)
        const uint32_t at = (uint32_t)max((int32_t)(cursor - blk), 0);
        const uint64_t rem = mall & (~0ull << at);
        if (rem == 0) continue;                                // no match starts at or after it
        PHASE_COUNT(10);
        if (kLateProbe) lengths();
        const uint32_t rl = lane + len;                        // the match's end, from blk
        const uint64_t after = rl < kWave ? mall & (~0ull << rl) : 0ull;
        const uint32_t nxt = (capped && !(TYCHE_EABLATE & 8)) ? 2u * kWave
                           : after ? (uint32_t)__builtin_ctzll(after) : kWave;
        uint64_t sel = 0;
        uint32_t li = (uint32_t)__builtin_ctzll(rem);
        uint32_t end;
        for (;;) {
            // the hop loop proper: one v_readlane and one taken branch per match
            uint32_t at_li;
            do {
                at_li = li;
                sel |= 1ull << li;
                PHASE_COUNT(9);
                if (kRepCand) {
                    // repeat history of the selected matches (a new offset shifts it)
                    const uint32_t off = blk + li - rdlane(cand, li);
                    if (off != R) {
                        R2 = R;
                        R = off;
                    }
                }
                li = rdlane(nxt, li);
            } while (li < kWave);
            if (li == kWave) {
                end = blk + at_li + rdlane(len, at_li);
                break;
            }
            // reached the probe limit: extend with the whole wave, then look for
            // the next match after the extended end
            const uint32_t mp = blk + at_li, mc = rdlane(cand, at_li), ln0 = rdlane(len, at_li);
            PHASE(1);
            const uint32_t ln = ln0 + wave_extend(in, A, ib, mp + ln0, mc + ln0, matchlimit, lane);
            PHASE(5);
            PHASE_COUNT(6);
            if (lane == at_li) len = ln;
            end = mp + ln;
            const uint32_t rel = end - blk;
            const uint64_t r = rel < kWave ? mall & (~0ull << rel) : 0ull;
            if (r == 0) break;
            li = (uint32_t)__builtin_ctzll(r);
        }
        cursor = end;
        done = cursor > mflimit;
        PHASE(1);
        // ---- append this block's records (stream order)
        const bool is_sel = (sel >> lane) & 1ull;
        const uint32_t rank = nacc + __builtin_amdgcn_mbcnt_hi((uint32_t)(sel >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sel, 0u));
        if (is_sel) rec[rank] = make_uint2(pos | (cand << 16), len | (back << 16));
        nacc += (uint32_t)__popcll(sel);
        // a block adds at most 16 records (each covers >= 4 positions; 22 of >= 3)
        PHASE(2);
        if (nacc > kWave - (kMin3 ? 22u : 16u) || done) {
            __builtin_amdgcn_wave_barrier();
            if (!sink(rec, nacc, anchor)) return 0xFFFFFFFFu;
            anchor = cursor;
            nacc = 0;
            PHASE(3);
        }
    }
    PHASE(4);
    if (nacc) {
        __builtin_amdgcn_wave_barrier();
        if (!sink(rec, nacc, anchor)) return 0xFFFFFFFFu;
        anchor = cursor;
    }
    if (rep) {
        rep[0] = R;
        rep[1] = R2;
    }
    PHASE(3);
    PHASE_FLUSH();
    return anchor;
}

// ---- Two-wave pipelined parse (zstd: repeat candidates, 2 ways, 5-byte hash).
//
// parse_page's block chain is window -> hash -> table -> candidate windows ->
// compares -> repeat candidates -> walk, and at one wave per SIMD (the zstd
// parse's LDS holds a CU to 4 waves) that chain is latency-bound.  Here a
// workgroup of two waves shares the page: the finder (wave 0) runs block k+1's
// hash side -- window, bucket read and insert, both bucket candidates' windows
// and compares -- while the walker (wave 1) runs block k's repeat candidates, the
// walk and the records; they meet at one workgroup barrier per block, the finder
// handing over (candidate, length, ok, backward extension) per lane in a
// two-slot LDS ring.  The finder processes every block: it cannot know which ones
// the walk will skip, so positions inside long matches are inserted too
// (tools/parse_sim.c zallblk: ratio unchanged, 5.034 / 4.785 at 32 / 16 KiB).
// Everything else -- which candidates a position tries, the walk, the records
// -- is parse_page<true, false, 2>'s.  Measured (round 3, C3 pages): encode
// 1,205 vs 1,026 ms per 1M pages for the one-wave A1 at the same ratio -- 3 pages
// per CU instead of 4 (41.9 KiB of LDS) and a barrier per block do not pay for the
// overlap, as with round 2's LZ4 finder/parser pipeline.  Off by default
// (TYCHE_ZSTD_PARSE_PIPE=1 selects it).
struct PipeSlot {
    uint32_t a[kWave];   // cand | n << 16 (n <= 20) | ok << 24 | back << 25 (0..4)
};

__device__ __forceinline__ void pipe_find(const uint32_t *A, uint32_t ib, uint32_t blk, uint32_t mflimit,
                                          uint16_t *table, PipeSlot &sl, uint32_t lane) {
    const uint32_t pos = blk + lane;
    const bool live = pos <= mflimit;
    const Window pw = lds_window(A, (live ? pos : mflimit) + ib);
    const uint32_t v = pw.w0;
    uint32_t *T = (uint32_t *)table;
    const uint32_t h = bucket_of<2>(v, pw.fw[0], TYCHE_HASH_BYTES);
    const uint32_t bk = T[h];
    __builtin_amdgcn_wave_barrier();
    T[h] = pos | (bk << 16);
    uint32_t cand = bk & 0xFFFFu;
    Window cw = lds_window(A, cand + ib);
    const uint32_t cand2 = bk >> 16;
    const Window ww = lds_window(A, cand2 + ib);
    bool ok = live & (cand < pos) & (cw.w0 == v);
    uint32_t n = 4u + kProbe;
#pragma unroll
    for (int k = (int)kProbeWords - 1; k >= 0; k--) {
        const uint32_t x = pw.fw[k] ^ cw.fw[k];
        if (x) n = 4u + 4u * (uint32_t)k + ((uint32_t)__builtin_ctz(x) >> 3);
    }
    const bool okw = live & (cand2 < pos) & (ww.w0 == v);
    uint32_t nw = 4u + kProbe;
#pragma unroll
    for (int k = (int)kProbeWords - 1; k >= 0; k--) {
        const uint32_t x = pw.fw[k] ^ ww.fw[k];
        if (x) nw = 4u + 4u * (uint32_t)k + ((uint32_t)__builtin_ctz(x) >> 3);
    }
    if (okw && (!ok || nw > n)) {   // the older bucket entry: taken only when strictly longer
        cand = cand2;
        cw = ww;
        n = nw;
        ok = true;
    }
    const uint32_t xb = pw.back ^ cw.back;
    const uint32_t back = pos < 4 || cand < 4 ? 0u : xb ? (__builtin_clz(xb) >> 3) : 4u;
    sl.a[lane] = cand | (n << 16) | ((ok ? 1u : 0u) << 24) | (back << 25);
}

// Both waves of the workgroup call this (wave 0 the finder, wave 1 the walker)
// with the same in, L; the walker's sink gets the records.  Returns (walker) the
// anchor of the last literal run, or 0xFFFFFFFF if the sink aborted.  slots:
// two PipeSlot in LDS; flag: one LDS word.
template <typename Sink>
__device__ uint32_t parse_page_piped(const uint8_t *in, uint32_t L, uint16_t *table, uint2 *rec, PipeSlot *slots,
                                     uint32_t *flag, uint32_t wave, uint32_t lane, Sink &sink) {
    if (L < (uint32_t)(kMfLimit + 1)) return 0;
    const uint32_t mflimit = L - kMfLimit;
    const uint32_t matchlimit = L - kLastLiterals;
    const uint32_t ib = (uint32_t)(uintptr_t)in & 3u;
    const uint32_t *A = (const uint32_t *)(in - ib);
    const uint32_t nblk = mflimit / kWave + 1u;   // blocks 0, 64, ... <= mflimit
    uint32_t anchor = 0, cursor = 0, nacc = 0, next_blk = 0, R = 1u, R2 = 4u;
    bool done = false, aborted = false;
    if (wave == 1 && lane == 0) *flag = 0;
    __syncthreads();
    for (uint32_t t = 0; t <= nblk; t++) {
        if (wave == 0) {
            if (t < nblk) pipe_find(A, ib, t * kWave, mflimit, table, slots[t & 1u], lane);
        } else if (t >= 1 && !done && (t - 1u) * kWave == next_blk) {
            const uint32_t blk = next_blk;
            const PipeSlot &sl = slots[(t - 1u) & 1u];
            const uint32_t pos = blk + lane;
            const bool live = pos <= mflimit;
            const Window pw = lds_window(A, (live ? pos : mflimit) + ib);
            const uint32_t v = pw.w0;
            const uint32_t sa = sl.a[lane];
            uint32_t cand = sa & 0xFFFFu, n = (sa >> 16) & 0xFFu, back = sa >> 25;
            bool ok = ((sa >> 24) & 1u) != 0u;
            // ---- repeat candidates (parse_page's kRepCand block)
            const uint32_t rc = pos >= R ? pos - R : 0u;
            const Window rw = lds_window(A, min(rc, mflimit) + ib);
            bool rok = live & (pos >= R) & (rw.w0 == v);
            uint32_t rn = 4u + kProbe;
#pragma unroll
            for (int k = (int)kProbeWords - 1; k >= 0; k--) {
                const uint32_t x = pw.fw[k] ^ rw.fw[k];
                if (x) rn = 4u + 4u * (uint32_t)k + ((uint32_t)__builtin_ctz(x) >> 3);
            }
            const uint32_t rc2 = pos >= R2 ? pos - R2 : 0u;
            const Window rw2 = lds_window(A, min(rc2, mflimit) + ib);
            const bool rok2 = TYCHE_REP2 && live & (pos >= R2) & (rw2.w0 == v) & (R2 != R);
            uint32_t rn2 = 4u + kProbe;
#pragma unroll
            for (int k = (int)kProbeWords - 1; k >= 0; k--) {
                const uint32_t x = pw.fw[k] ^ rw2.fw[k];
                if (x) rn2 = 4u + 4u * (uint32_t)k + ((uint32_t)__builtin_ctz(x) >> 3);
            }
            auto back_of = [&](uint32_t c, uint32_t cb) {
                const uint32_t x = pw.back ^ cb;
                return pos < 4 || c < 4 ? 0u : x ? (__builtin_clz(x) >> 3) : 4u;
            };
            if (rok && (!ok || rn + TYCHE_REP_SLACK >= n)) {
                cand = rc;
                back = back_of(rc, rw.back);
                n = rn;
                ok = true;
            }
            if (rok2 && (!ok || rn2 + TYCHE_REP_SLACK >= n) && !(rok && rn >= rn2)) {
                cand = rc2;
                back = back_of(rc2, rw2.back);
                n = rn2;
                ok = true;
            }
            rok |= rok2;
            const uint32_t e = min(matchlimit, pos + kMinMatch + kProbe);
            n = min(n, e - pos);
            uint32_t len = n;
            const bool capped = pos + n == e && e < matchlimit;
            // ---- the walk (parse_page's)
            uint64_t mall = __ballot(ok);
            if (TYCHE_REP_NEXT) {
                const uint64_t mrep = __ballot(rok);
                mall &= ~(mrep >> 1) | mrep;
            }
            const uint32_t at = cursor > blk ? cursor - blk : 0u;
            const uint64_t rem = mall & (~0ull << at);
            if (rem != 0) {
                const uint32_t endp = pos + len;
                const uint32_t rl = endp - blk;
                const uint64_t after = rl < kWave ? mall & (~0ull << rl) : 0ull;
                const uint32_t nxt = capped ? 2u * kWave : after ? (uint32_t)__builtin_ctzll(after) : kWave;
                uint64_t sel = 0;
                uint32_t li = (uint32_t)__builtin_ctzll(rem);
                uint32_t end;
                for (;;) {
                    uint32_t at_li;
                    do {
                        at_li = li;
                        sel |= 1ull << li;
                        const uint32_t off = blk + li - rdlane(cand, li);
                        if (off != R) {
                            R2 = R;
                            R = off;
                        }
                        li = rdlane(nxt, li);
                    } while (li < kWave);
                    if (li == kWave) {
                        end = rdlane(endp, at_li);
                        break;
                    }
                    const uint32_t mp = blk + at_li, mc = rdlane(cand, at_li), ln0 = rdlane(endp, at_li) - mp;
                    const uint32_t ln = ln0 + wave_extend(in, A, ib, mp + ln0, mc + ln0, matchlimit, lane);
                    if (lane == at_li) len = ln;
                    end = mp + ln;
                    const uint32_t rel = end - blk;
                    const uint64_t r = rel < kWave ? mall & (~0ull << rel) : 0ull;
                    if (r == 0) break;
                    li = (uint32_t)__builtin_ctzll(r);
                }
                cursor = end;
                done = cursor > mflimit;
                const bool is_sel = (sel >> lane) & 1ull;
                const uint32_t rank = nacc + (uint32_t)__popcll(sel & ((1ull << lane) - 1ull));
                if (is_sel) rec[rank] = make_uint2(pos | (cand << 16), len | (back << 16));
                nacc += (uint32_t)__popcll(sel);
                if (nacc > kWave - 16u || done) {
                    __builtin_amdgcn_wave_barrier();
                    if (!sink(rec, nacc, anchor)) {
                        aborted = true;
                        done = true;
                    }
                    anchor = cursor;
                    nacc = 0;
                }
            }
            next_blk = max(blk + kWave, cursor & ~(kWave - 1u));
            if (next_blk > mflimit) done = true;
            if (done && lane == 0) *flag = 1;
        }
        __syncthreads();
        if (rfl(*flag)) break;   // the walk is over: the finder stops too
    }
    if (wave == 0) return 0;
    if (aborted) return 0xFFFFFFFFu;
    if (nacc) {
        __builtin_amdgcn_wave_barrier();
        if (!sink(rec, nacc, anchor)) return 0xFFFFFFFFu;
        anchor = cursor;
    }
    return anchor;
}

}  // namespace lzp
}  // namespace tyche
