// lz4_encode.hip -- batched LZ4 block encode for gfx950 (the sweep path).
//
// Replaces the per-victim LZ4_compress_default call of buffer__compress
// (reference src/buffer.c:178-188 -> src/lz4/lz4.c:697 -> LZ4_compress_generic
// lz4.c:459-656) with one kernel over a batch of pages.  The output is a
// standard LZ4 block that LZ4_decompress_safe (lz4.c:1251) -- the reference's
// own decoder -- restores bit-exactly; it is not required to be the bytes 1.7.5
// emits.  The decoder's parsing rules are kept: every match
// starts at or before iend-MFLIMIT (12) and ends at or before iend-LASTLITERALS
// (5) (lz4.c:266-267, 1147-1156, 1225); output never exceeds the caller's
// capacity (limitedOutput semantics: 0 when it would not fit).
//
// One 64-lane wave per page, looping over pages with the next page prefetched
// into registers.  The page is staged in LDS next to a table of 2^10 16-bit
// positions (the byU16 scheme of lz4.c:402-408, hash 2654435761 of 4 bytes).
// The page is scanned in blocks of 64 positions:
//   * every lane hashes its position, takes the candidate left by earlier
//     blocks, verifies 4 bytes, probes the match length up to 20 bytes and the
//     backward extension up to 4 bytes (lz4.c:549's catch-up);
//   * the greedy parse over the block runs on scalar registers only: first
//     match at or after the cursor (ballot mask), cursor = its end; a match
//     that reached the probe limit is extended by the whole wave (256 bytes per
//     step);
//   * the block's sequences are encoded together: each selected lane computes
//     its literal run (from the previous selected match's end), catch-up, token
//     and length bytes; a wave prefix sum places them, and output bytes are
//     written 64 per store instruction, contiguous.
#include <hip/hip_runtime.h>

#define TYCHE_PHASES_OWNER   // only used by -DTYCHE_PHASES profiling builds
// 2^10 hash slots (2 KB): the wave's LDS (page 16.4 KB + table + records) drops
// to 20 KB, one 512-byte granule under 160 KB / 8, so 8 waves per CU instead of
// 7: 127.7 -> 111.6 ms per 1M pages for ratio 2.635 -> 2.621 (reference 2.647)
#ifndef TYCHE_LZ4_HASH_LOG
#define TYCHE_LZ4_HASH_LOG 10
#endif
#ifndef TYCHE_HASH_LOG
#define TYCHE_HASH_LOG TYCHE_LZ4_HASH_LOG
#endif
#ifndef TYCHE_LANE_ADDR
#define TYCHE_LANE_ADDR 1   // lz_parse.h: block windows from per-lane LDS addresses (every page has LDS in front)
#endif

#include <algorithm>
#include <cstdlib>

#include "engine.h"
#include "lds_io.h"
#include "lz_parse.h"

namespace tyche {

namespace {

using lzp::kWave;
using lzp::kHashSize;
constexpr uint32_t kPad = 64;
constexpr uint32_t kPrefetchVec = 16;    // 16-byte vectors per lane prefetched for the next page (16 KiB; 8 or 4
                                          // take the one-wave kernel to 132 / 119 VGPRs: 70.6 / 70.9 ms per 1M x 8 KiB)

// a sequence's encoding: token, literal-length bytes, literals, offset, match-length bytes
struct SeqFields {
    uint32_t lit, lext, anchor, off, mc, token, total;
};

// byte `rel` of a sequence's encoding, branch-free (the literal is read
// unconditionally, from a clamped in-page position): the selects cost less than
// the divergent branches of 64 lanes in different fields (134 -> 128 ms per 1M pages)
__device__ __forceinline__ uint32_t seq_byte(const SeqFields &f, const uint8_t *in, uint32_t rel) {
    const uint32_t lb = 1 + f.lext, ob = lb + f.lit;
    const uint32_t li = f.anchor + min(rel - lb, f.lit - 1u);   // rel in [lb, ob) when used
    const uint32_t litb = in[rel >= lb && f.lit ? li : 0u];
    const uint32_t ext = rel == f.lext ? (f.lit - 15u) % 255u : 255u;
    const uint32_t mext = rel == f.total - 1u ? (f.mc - 15u) % 255u : 255u;
    uint32_t v = mext;
    v = rel == ob + 1u ? f.off >> 8 : v;
    v = rel == ob ? f.off & 0xFFu : v;
    v = rel < ob ? litb : v;
    v = rel <= f.lext ? ext : v;
    v = rel == 0u ? f.token : v;
    return v;
}


// Encodes n accumulated sequences (records in LDS, stream order) after the
// literal run that starts at `anchor`, writing their bytes to dst + op.  One
// record per lane: the previous record's end gives each sequence's literal run;
// a DPP prefix sum places the encodings.  Output goes out 256 bytes per step,
// four consecutive bytes per lane and one dword store: sequence starts are
// stamped into a 256-byte LDS map, each lane reads its four stamps as a dword,
// and the owner of every byte is the last start at or before it (a wave
// exclusive max-scan of the lanes' last stamps, then a running max over the
// four).  Each sequence's packed fields sit in LDS (fld, 16 bytes), read once
// per distinct owner.  Returns false if the output would exceed cap.
__device__ bool emit_records(const uint2 *rec, uint32_t n, uint32_t anchor, const uint8_t *in, uint8_t *dst,
                             uint32_t &op, uint32_t cap, uint8_t *map, uint4 *fld, uint32_t lane) {
    const bool is_sel = lane < n;
    const uint2 r = rec[is_sel ? lane : 0];
    const uint2 rp = rec[lane > 0 && is_sel ? lane - 1 : 0];
    const uint32_t pos = r.x & 0xFFFFu, cand = r.x >> 16, len = r.y & 0xFFFFu, back = lzp::back_at(in, pos, cand);
    const uint32_t prev_end = lane == 0 ? anchor : (rp.x & 0xFFFFu) + (rp.y & 0xFFFFu);
    SeqFields f{};
    uint32_t enc = 0;
    if (is_sel) {
        const uint32_t k = min(min(back, pos - prev_end), cand);   // catch-up (lz4.c:549)
        f.anchor = prev_end;
        f.lit = pos - k - prev_end;
        f.lext = f.lit >= 15 ? (f.lit - 15) / 255 + 1 : 0;
        f.off = pos - cand;
        f.mc = len + k - kMinMatch;
        const uint32_t mext = f.mc >= 15 ? (f.mc - 15) / 255 + 1 : 0;
        f.token = (min(f.lit, 15u) << 4) | min(f.mc, 15u);
        f.total = 1 + f.lext + f.lit + 2 + mext;
        enc = f.total;
    }
    const int32_t incl = wave_incl_sum((int32_t)enc);
    const uint32_t eo = (uint32_t)incl - enc;
    const uint32_t et = rdlane((uint32_t)incl, 63);
    if (op + et > cap) return false;
    if (is_sel) fld[lane] = make_uint4(f.lit | (f.lext << 16), f.anchor | (f.off << 16), f.mc | (f.total << 16),
                                       eo | (f.token << 16));
    uint32_t *map32 = (uint32_t *)map;
    for (uint32_t j0 = 0; j0 < ((TYCHE_EABLATE & 1) ? 0u : et); j0 += 4u * kWave) {
        // the last sequence starting before this step, then the starts inside it
        const uint64_t before = __ballot(is_sel && eo < j0);
        const int32_t owner0 = before ? 63 - (int32_t)__builtin_clzll(before) : 0;
        map32[lane] = 0xFFFFFFFFu;
        __builtin_amdgcn_wave_barrier();
        if (is_sel && eo >= j0 && eo < j0 + 4u * kWave) map[eo - j0] = (uint8_t)lane;
        __builtin_amdgcn_wave_barrier();
        const uint32_t m = map32[lane];
        int32_t last = -1;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint32_t st = (m >> (8 * t)) & 0xFFu;
            if (st != 0xFFu) last = (int32_t)st;
        }
        // owner entering this lane's first byte: the last stamp of the lanes below
        const int32_t incl_max = wave_incl_max(last);
        int32_t cur = (int32_t)__shfl(incl_max, (int)(lane ? lane - 1u : 0u));
        cur = max(lane ? cur : -1, owner0);
        const uint32_t jb = j0 + 4u * lane;
        uint32_t word = 0, prev_o = 0xFFFFFFFFu;
        uint4 g = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint32_t st = (m >> (8 * t)) & 0xFFu;
            if (st != 0xFFu) cur = (int32_t)st;
            if (jb + (uint32_t)t < et) {
                if ((uint32_t)cur != prev_o) {
                    g = fld[cur];
                    prev_o = (uint32_t)cur;
                }
                SeqFields q;
                q.lit = g.x & 0xFFFFu;
                q.lext = g.x >> 16;
                q.anchor = g.y & 0xFFFFu;
                q.off = g.y >> 16;
                q.mc = g.z & 0xFFFFu;
                q.total = g.z >> 16;
                q.token = g.w >> 16;
                word |= seq_byte(q, in, jb + (uint32_t)t - (g.w & 0xFFFFu)) << (8 * t);
            }
        }
        if (jb + 4u <= et) {
            store_u32_unaligned(dst + op + jb, word);
        } else {
#pragma unroll
            for (int t = 0; t < 4; t++)
                if (jb + (uint32_t)t < et) dst[op + jb + (uint32_t)t] = (uint8_t)(word >> (8 * t));
        }
        __builtin_amdgcn_wave_barrier();
    }
    op += et;
    return true;
}

// ---- output staging (the default emission).
//
// emit_records above resolves every output byte's owner and field (a map
// stamp, a max-scan, a select chain per byte): ~330 instructions per 256 output
// bytes, 27 % of the encoder's wave cycles (tools/phase_prof.py, r02).  Here each
// sequence's lane writes its own bytes -- token, literal-length bytes, literals,
// offset, match-length bytes -- into a 2 KiB LDS ring with byte stores, and the
// ring leaves for HBM in 512-byte steps, one 8-byte store per lane.  The ring
// reuses emit_records' field area, so the LDS budget (and 8 waves per CU) is
// unchanged; a sink too large for the ring (long literal runs: the ring is
// flushed first) still takes emit_records straight to HBM.
// Output ring size and flush width (round 3, 256K x 16 KiB pages, ms per 1M, three-wave encoder):
// 1 KiB ring, 256-byte dword flushes 79.3-79.4; 2 KiB, 512-byte 8-byte flushes 78.1; 2 KiB, 1 KiB
// 16-byte flushes 78.2; 1 KiB, 512-byte flushes 80.2 (more batches overflow the ring).  A wave-wide
// copy of all long literal runs at once (instead of one run after another) ran 80.5.
// Round 4: 512-byte rings with dword flushes -- a 3-wave page's LDS drops from 30.5 to 26 KiB (6 pages per
// CU instead of 5) and, with the 5-waves-per-SIMD register budget (TYCHE_ENC_WPE), encode 77.5 -> 72.2 ms
// (8-byte flushes with the 512-byte ring: 74.7; without the register budget: 79.0); a sink whose bytes
// would overflow the ring takes emit_records, whose fields then span the records and the ring.
#ifndef TYCHE_LZ4_RING
#define TYCHE_LZ4_RING 512
#endif
#ifndef TYCHE_LZ4_FLUSH_VEC
#define TYCHE_LZ4_FLUSH_VEC 1
#endif
constexpr uint32_t kOutRing = TYCHE_LZ4_RING;        // bytes; head is always a multiple of kFlushStep
constexpr uint32_t kFlushVec = TYCHE_LZ4_FLUSH_VEC;  // dwords per lane per flush step (1, 2 or 4)
constexpr uint32_t kFlushStep = 4u * kWave * kFlushVec;
static_assert(kOutRing >= 512 && kOutRing % kFlushStep == 0 && (kOutRing & (kOutRing - 1)) == 0, "ring");
static_assert(kOutRing + 64u * 8u >= 1024u, "emit_records' fields fit the records and the ring");
typedef uint32_t u32x2_ua __attribute__((ext_vector_type(2), aligned(1)));
typedef __attribute__((address_space(1))) u32x2_ua g_u32x2_ua;
typedef uint32_t u32x4_uaf __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) u32x4_uaf g_u32x4_uaf;
#ifndef TYCHE_LIT_LANE
#define TYCHE_LIT_LANE 8
#endif
constexpr uint32_t kLitLane = TYCHE_LIT_LANE;
#ifndef TYCHE_LIT_GATHER
#define TYCHE_LIT_GATHER 1
#endif   // literal bytes a sequence's lane copies itself (emit_staged)
struct OutRing {
    uint32_t head, pend;   // wave-uniform: ring position of the first unflushed byte, unflushed bytes
};

__device__ __forceinline__ void out_flush_steps(const uint8_t *ring, OutRing &r, uint8_t *dst, uint32_t &op,
                                                uint32_t lane) {
    while (r.pend >= kFlushStep) {
        const uint8_t *src = ring + ((r.head + 4u * kFlushVec * lane) & (kOutRing - 1));
        uint8_t *d = dst + op + 4u * kFlushVec * lane;
        if (kFlushVec == 4) {
            *(g_u32x4_uaf *)(uintptr_t)d = *(const u32x4 *)src;
        } else if (kFlushVec == 2) {
            const uint2 w = *(const uint2 *)src;
            u32x2_ua v;
            v.x = w.x;
            v.y = w.y;
            *(g_u32x2_ua *)(uintptr_t)d = v;
        } else {
            store_u32_unaligned(d, *(const uint32_t *)src);
        }
        op += kFlushStep;
        r.head = (r.head + kFlushStep) & (kOutRing - 1);
        r.pend -= kFlushStep;
    }
}

__device__ __forceinline__ void out_flush_all(const uint8_t *ring, OutRing &r, uint8_t *dst, uint32_t &op,
                                              uint32_t lane) {
    out_flush_steps(ring, r, dst, op, lane);
    for (uint32_t j = 4 * lane; j < r.pend; j += 4 * kWave) {   // the rest (< kFlushStep), a dword per lane
        const uint32_t w = *(const uint32_t *)(ring + ((r.head + j) & (kOutRing - 1)));
        if (j + 4 <= r.pend) {
            store_u32_unaligned(dst + op + j, w);
        } else {
            for (uint32_t t = 0; j + t < r.pend; t++) dst[op + j + t] = (uint8_t)(w >> (8 * t));
        }
    }
    op += r.pend;
    r.head = 0;
    r.pend = 0;
    __builtin_amdgcn_wave_barrier();
}

// The sink of the default emission: n records (stream order) after the literal
// run that starts at `anchor`; op counts the bytes already in dst.  Returns
// false if the output would exceed cap.
__device__ __forceinline__ bool emit_staged(const uint2 *rec, uint32_t n, uint32_t anchor, const uint8_t *in, uint8_t *dst,
                            uint32_t &op, uint32_t cap, uint8_t *ring, OutRing &r, uint8_t *map, uint32_t lane) {
#if defined(TYCHE_PHASES)
    // profiling builds: sink sub-phases of every 64th workgroup's calls into g_phase[11..15]
    const bool sp_rec = blockIdx.x % 64u == 0u && lane == 0u;
    uint32_t sp_t = (uint32_t)__builtin_amdgcn_s_memtime();
#define SINK_PHASE(i) do { const uint32_t t_ = (uint32_t)__builtin_amdgcn_s_memtime(); \
                           if (sp_rec) atomicAdd(&lzp::g_phase[i], (unsigned long long)(t_ - sp_t)); sp_t = t_; } while (0)
#else
#define SINK_PHASE(i) do {} while (0)
#endif
    const bool is_sel = lane < n;
    const uint2 rc = rec[is_sel ? lane : 0];
    const uint2 rp = rec[lane > 0 && is_sel ? lane - 1 : 0];
    const uint32_t pos = rc.x & 0xFFFFu, cand = rc.x >> 16, len = rc.y & 0xFFFFu, back = lzp::back_at(in, pos, cand);
    const uint32_t prev_end = lane == 0 ? anchor : (rp.x & 0xFFFFu) + (rp.y & 0xFFFFu);
    // branch-free: lanes past n compute values from record 0 that are never stored (enc 0; lit 0
    // keeps them out of the long-run loop); a branch around these costs more exec-mask work
    const uint32_t k = min(min(back, pos - prev_end), cand);   // catch-up (lz4.c:549)
    const uint32_t lstart = prev_end;
    const uint32_t lit = is_sel ? pos - k - prev_end : 0u;
    const uint32_t lext = lit >= 15 ? (lit - 15) / 255 + 1 : 0;
    const uint32_t off = pos - cand;
    const uint32_t mc = len + k - kMinMatch;
    const uint32_t mext = mc >= 15 ? (mc - 15) / 255 + 1 : 0;
    const uint32_t token = (min(lit, 15u) << 4) | min(mc, 15u);
    const uint32_t enc = is_sel ? 1 + lext + lit + 2 + mext : 0u;
    const int32_t incl = wave_incl_sum((int32_t)enc);
    const uint32_t eo = (uint32_t)incl - enc;
    const uint32_t et = rdlane((uint32_t)incl, 63);
    if (op + r.pend + et > cap) return false;
    if (r.pend + et > kOutRing) {
        out_flush_all(ring, r, dst, op, lane);
        // emit_records' 64 packed fields (1 KiB): the ring, or for a ring under 1 KiB the records
        // before it and the ring (every layout puts the 64 records right before the ring; they are
        // read into registers before the fields are written)
        uint4 *fld = (uint4 *)(kOutRing >= 1024 ? ring : ring + kOutRing - 1024u);
        return emit_records(rec, n, anchor, in, dst, op, cap, map, fld, lane);
    }
    SINK_PHASE(11);
    constexpr uint32_t m = kOutRing - 1;
    const uint32_t q_lit = r.head + r.pend + eo + 1 + lext;   // ring position of this sequence's literals
    if (is_sel) {
        uint32_t q = r.head + r.pend + eo;
        ring[q & m] = (uint8_t)token;
        q++;
        for (uint32_t t = 0; t < lext; t++) ring[(q + t) & m] = (uint8_t)(t + 1 == lext ? (lit - 15) % 255 : 255);
        // literal runs: the first kLitLane bytes by the sequence's own lane, the
        // rest of a long run by the whole wave below -- a byte loop as long as the
        // batch's longest run kept every other lane idle (the sink was 56 % of
        // the parse's cycles, tools/phase_prof.py)
        const uint32_t ls = min(lit, kLitLane);
#if TYCHE_LIT_GATHER
        // the run's first 8 bytes from three aligned dwords (the staged page has 64 zero bytes of
        // padding), then up to 8 byte stores that wait on nothing: the byte-at-a-time copy put one
        // LDS read latency per literal byte on the sink's critical path
        static_assert(kLitLane == 8, "two gathered dwords");
        const uint32_t ib = (uint32_t)(uintptr_t)in & 3u;
        const uint32_t *A = (const uint32_t *)(in - ib);
        const uint32_t q0 = lstart + ib, i0 = q0 >> 2, sh = q0 & 3u;
        const uint32_t d0 = A[i0], d1 = A[i0 + 1], d2 = A[i0 + 2];
        const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
        // byte t >= ls goes to a dummy byte (the owner map, unused here): selects instead of eight
        // exec-mask branches
#pragma unroll
        for (uint32_t t = 0; t < 8; t++) {
            uint8_t *bp = t < ls ? ring + ((q_lit + t) & m) : map;
            *bp = (uint8_t)((t < 4 ? w0 : w1) >> (8 * (t & 3u)));
        }
#else
        for (uint32_t t = 0; t < ls; t++) ring[(q_lit + t) & m] = in[lstart + t];
#endif
        q = q_lit + lit;
        ring[q & m] = (uint8_t)off;
        ring[(q + 1) & m] = (uint8_t)(off >> 8);
        q += 2;
        for (uint32_t t = 0; t < mext; t++) ring[(q + t) & m] = (uint8_t)(t + 1 == mext ? (mc - 15) % 255 : 255);
    }
    SINK_PHASE(12);
    uint64_t longm = __ballot(is_sel && lit > kLitLane);
    while (longm) {
        const uint32_t k = (uint32_t)__builtin_ctzll(longm);
        longm &= longm - 1;
        const uint32_t kl = rdlane(lit, k) - kLitLane, kq = rdlane(q_lit, k) + kLitLane, ks = rdlane(lstart, k) + kLitLane;
        for (uint32_t i = lane; i < kl; i += kWave) ring[(kq + i) & m] = in[ks + i];
    }
    __builtin_amdgcn_wave_barrier();
    SINK_PHASE(13);
    r.pend += et;
    out_flush_steps(ring, r, dst, op, lane);
    __builtin_amdgcn_wave_barrier();
    SINK_PHASE(14);
#if defined(TYCHE_PHASES)
    if (sp_rec) atomicAdd(&lzp::g_phase[15], 1ull);
#endif
    return true;
}
#undef SINK_PHASE

#ifndef TYCHE_LZ4_SINK_CALL
// the sink as a call instead of inlined into the parse: bit 0 for the one-wave kernel (encode_page),
// bit 1 for the N-wave split kernels.  One wave per page, ms per 1M pages: 8 KiB 70.7 inlined ->
// 44.7 called, 4 KiB 34.8 -> 21.3 (the inlined sink was round 3's 38 -> 70 ms regression at 8 KiB);
// the three-wave kernel the other way: 16 KiB 77.9 inlined vs 86.9 called, 8 KiB 41.4 vs 46.6
#define TYCHE_LZ4_SINK_CALL 1
#endif
// the sink as a call (as in round 2)
__device__ __noinline__ bool emit_staged_call(const uint2 *rec, uint32_t n, uint32_t anchor, const uint8_t *in, uint8_t *dst,
                                              uint32_t &op, uint32_t cap, uint8_t *ring, OutRing &r, uint8_t *map,
                                              uint32_t lane) {
    return emit_staged(rec, n, anchor, in, dst, op, cap, ring, r, map, lane);
}

__device__ __forceinline__ bool emit_sink_n(const uint2 *rec, uint32_t n, uint32_t anchor, const uint8_t *in, uint8_t *dst,
                                            uint32_t &op, uint32_t cap, uint8_t *ring, OutRing &r, uint8_t *map,
                                            uint32_t lane) {
    if (TYCHE_LZ4_SINK_CALL & 2) return emit_staged_call(rec, n, anchor, in, dst, op, cap, ring, r, map, lane);
    return emit_staged(rec, n, anchor, in, dst, op, cap, ring, r, map, lane);
}

// Encodes one page held in LDS into dst (global, capacity cap).  Returns the
// compressed size, or 0 if it does not fit in cap.
__device__ int32_t encode_page(const uint8_t *in, uint32_t L, uint16_t *table, uint8_t *map, uint2 *rec,
                               uint4 *fld, uint8_t *dst, uint32_t cap, uint32_t lane) {
    uint32_t op = 0;
#ifndef TYCHE_LZ4_STAGED
#define TYCHE_LZ4_STAGED 1
#endif
    OutRing r{0u, 0u};
    uint8_t *ring = (uint8_t *)fld;
    auto sink = [&](const uint2 *rr, uint32_t n, uint32_t anchor) -> bool {
        if ((TYCHE_LZ4_STAGED != 0) & ((TYCHE_LZ4_SINK_CALL & 1) != 0)) return emit_staged_call(rr, n, anchor, in, dst, op, cap, ring, r, map, lane);
        if (TYCHE_LZ4_STAGED) return emit_staged(rr, n, anchor, in, dst, op, cap, ring, r, map, lane);
        // emit_records' 1 KiB field area ends where the ring does (as in emit_staged's fallback):
        // with a ring under 1 KiB it starts in the record array, never past the ring into the page
        return emit_records(rr, n, anchor, in, dst, op, cap, map,
                            (uint4 *)(kOutRing >= 1024 ? ring : ring + kOutRing - 1024u), lane);
    };
    const uint32_t anchor = lzp::parse_page(in, L, table, rec, lane, sink);
    if (anchor == 0xFFFFFFFFu) return 0;
    if (TYCHE_LZ4_STAGED) out_flush_all(ring, r, dst, op, lane);
    // ---- last literals: in[anchor, L)
    const uint32_t lit = L - anchor;
    const uint32_t lext = lit >= 15 ? (lit - 15) / 255 + 1 : 0;
    const uint32_t total = 1 + lext + lit;
    if (op + total > cap) return 0;
    for (uint32_t j = lane; j < total; j += kWave) {
        uint32_t v;
        if (j == 0) v = min(lit, 15u) << 4;
        else if (j <= lext) v = j == lext ? (lit - 15) % 255 : 255;
        else v = in[anchor + j - 1 - lext];
        dst[op + j] = (uint8_t)v;
    }
    return (int32_t)(op + total);
}

// ---- two-wave split encoder (round 2's default for pages >= kSplitMin; TYCHE_LZ4_ENC_WAVES=2).
//
// The one-wave encoder is latency-bound: its page, hash table and sequence
// buffers take 20 KiB of LDS, so a CU holds 8 of them (2 waves per SIMD), and
// 8 KiB pages -- 13 waves per CU -- encode 25 % faster per byte.  Here two
// waves share one staged page: wave A parses [0, H) and wave B [H, L), with
// H = 9/16 L rounded down to 64 (B also seeds its table), each with its own
// table and buffers (24 KiB per page for both: 6 workgroups = 12 waves per
// CU).  The parts join exactly:
//   * A's matches end at or before H (its parse sees L' = H + LASTLITERALS) and
//     it emits no trailing literal run: its output is complete sequences;
//   * B first inserts every position of [0, H) into its table, so its matches
//     reach back into A's half as the one-wave parse's would, then parses
//     [H, L) (lz_parse.h start = H) into a per-workgroup scratch buffer,
//     holding back its first sequence;
//   * after a barrier A emits the joint sequence -- literals from its own
//     last match's end up to B's first match, then that match -- and the
//     workgroup copies B's scratch after it.  With no match in B's half the
//     joint is the page's last literal run.
// The LZ4 block rules hold on the joined stream (every match starts <= L-12 and
// ends <= L-5; the last sequence is literals only); output never exceeds cap.
// 16 KiB pages: 108.2 -> 93.3 ms per 1M pages (12 waves per CU instead of 8); 8 KiB pages stay on the
// one-wave kernel (13 waves per CU already: 45.0 vs 57.6 ms split)
constexpr uint32_t kSplitMin = 12288;
#ifndef TYCHE_SPLIT_AT
#define TYCHE_SPLIT_AT 36   // H = L * TYCHE_SPLIT_AT / 64, rounded down to 64 (ms per 1M x 16 KiB pages: 32: 98.7, 34: 94.3, 35: 93.2, 36: 93.3, 38: 95.4, 40: 99.1)
#endif
static_assert(TYCHE_SPLIT_AT >= 32 && TYCHE_SPLIT_AT < 64, "B's half must fit its scratch (sized for L / 2 + 64)");
constexpr uint32_t kSplitPrefetch = 8;   // 16-byte vectors per thread prefetched for the next page
struct SplitHdr {
    uint32_t next_lo, next_hi, next2_lo, next2_hi;
    uint32_t len_a;       // bytes of the page's output in dst (A's stream, then the joint)
    uint32_t len_b;       // B: bytes in its scratch
    uint32_t has_first;   // B: its first sequence was held back
    int32_t result;
    uint2 first;          // B's first record
    uint32_t pad[6];
};
static_assert(sizeof(SplitHdr) == 64, "split header");
// Inserts the positions of blocks [from, to) (multiples of 64) into the table in
// block order, as parse_page would have (later blocks overwrite earlier ones).
// Four blocks' words are read before their inserts, so one LDS round trip covers
// four blocks, and each lane addresses its words from a base fixed for the page.
__device__ __forceinline__ void seed_table(const uint8_t *in, uint16_t *table, uint32_t from, uint32_t to,
                                           uint32_t lane) {
    const uint32_t ib = (uint32_t)(uintptr_t)in & 3u;
    const uint32_t la = lzp::lds_addr(in - ib) + ((lane + ib) & ~3u), ls = (lane + ib) & 3u;
    const uint32_t tbase = rfl(lzp::lds_addr(table));
    auto slot = [&](uint32_t w) { return (lzp::lds_u16_t *)(uintptr_t)lzp::slot_addr(tbase, lzp::hash4(w)); };
    uint32_t blk = from;
    for (; blk + 4u * kWave <= to; blk += 4u * kWave) {
        const lzp::lds_u32_t *P = (const lzp::lds_u32_t *)(uintptr_t)(la + blk);
        uint32_t w[4];
#pragma unroll
        for (uint32_t u = 0; u < 4u; u++) w[u] = lzp::word_at(P[16u * u], P[16u * u + 1u], ls);
#pragma unroll
        for (uint32_t u = 0; u < 4u; u++) {
            *slot(w[u]) = (uint16_t)(blk + kWave * u + lane);
            __builtin_amdgcn_wave_barrier();
        }
    }
    for (; blk < to; blk += kWave) {
        const lzp::lds_u32_t *P = (const lzp::lds_u32_t *)(uintptr_t)(la + blk);
        *slot(lzp::word_at(P[0], P[1], ls)) = (uint16_t)(blk + lane);
        __builtin_amdgcn_wave_barrier();
    }
}

// per-wave region: table | map (256) | records (512) | fields / output ring (1 KiB)
constexpr size_t kWaveRegion = kHashSize * sizeof(uint16_t) + 4 * kWave + kWave * sizeof(uint2) + kOutRing;
constexpr size_t kSplitStage = sizeof(SplitHdr) + 2 * kWaveRegion;

// the last literal run in[anchor, L) at dst + op (encode_page's tail); false if it does not fit cap
__device__ bool write_last_literals(const uint8_t *in, uint32_t anchor, uint32_t L, uint8_t *dst, uint32_t &op,
                                    uint32_t cap, uint32_t lane) {
    const uint32_t lit = L - anchor;
    const uint32_t lext = lit >= 15 ? (lit - 15) / 255 + 1 : 0;
    const uint32_t total = 1 + lext + lit;
    if (op + total > cap) return false;
    for (uint32_t j = lane; j < total; j += kWave) {
        uint32_t v;
        if (j == 0) v = min(lit, 15u) << 4;
        else if (j <= lext) v = j == lext ? (lit - 15) % 255 : 255;
        else v = in[anchor + j - 1 - lext];
        dst[op + j] = (uint8_t)v;
    }
    op += total;
    return true;
}

typedef uint32_t u32x4_ua __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) u32x4_ua g_u32x4_ua;

__global__ __launch_bounds__(128, 3) void lz4_encode_split_kernel(tyche_batch_t b, uint32_t in_cap, unsigned *ctr,
                                                                   uint8_t *ws, uint32_t ws_stride) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = rfl(tid >> 6);   // wave-uniform: the two halves' branches stay scalar
    SplitHdr *hdr = (SplitHdr *)smem;
    uint8_t *region = smem + sizeof(SplitHdr) + wave * kWaveRegion;
    uint16_t *table = (uint16_t *)region;
    uint8_t *map = region + kHashSize * sizeof(uint16_t);
    uint2 *rec = (uint2 *)(map + 4 * kWave);
    uint4 *fld = (uint4 *)(rec + kWave);
    uint8_t *ring = (uint8_t *)fld;
    uint8_t *stage = smem + kSplitStage;
    uint8_t *scratch = ws + (size_t)blockIdx.x * ws_stride;

    size_t page = blockIdx.x;
    if (page >= b.count) return;
    PageRef p = batch_page(b, page);
    uint32_t head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, tid, 2 * kWave);
    if (tid == 0) {
        const size_t nx = (size_t)atomicAdd(ctr, 1u) + gridDim.x;   // dynamic assignment (engine.h)
        hdr->next_lo = (uint32_t)nx;
        hdr->next_hi = (uint32_t)(nx >> 32);
    }
    for (;;) {
        for (uint32_t w = lane; w < kHashSize / 8; w += kWave) ((u32x4 *)table)[w] = u32x4{0, 0, 0, 0};
        if (tid < kWave) stage[head + p.src_len + tid] = 0;
        __syncthreads();
        const size_t next = (size_t)rfl(hdr->next_lo) | ((size_t)rfl(hdr->next_hi) << 32);
        PageRef pn;
        u32x4 pf[kSplitPrefetch];
        uint32_t nhead = 0, nvec = 0;
        if (next < b.count) {
            pn = batch_page(b, next);
            if (pn.src_len <= in_cap && pn.src_len > 0) {
                const uintptr_t a = (uintptr_t)pn.src;
                nhead = (uint32_t)(a & 15u);
                nvec = (nhead + pn.src_len + 15u) >> 4;
                const u32x4 *g = (const u32x4 *)(a - nhead);
#pragma unroll
                for (uint32_t k = 0; k < kSplitPrefetch; k++) pf[k] = gload_nt(g + min(tid + k * 2 * kWave, nvec - 1u));
            }
        }
        const uint8_t *in = stage + head;
        const uint32_t L = p.src_len;
        const bool fits = L <= in_cap;
        const bool split = fits && L >= kSplitMin;
        const uint32_t H = (L * TYCHE_SPLIT_AT / 64u) & ~(kWave - 1u);   // A takes a little more than half: B also seeds
        uint32_t opA = 0, cursorA = 0;
        bool okA = true;
        OutRing rA{0u, 0u};
        int32_t rv = 0;
        if (wave == 0) {
            if (fits && !split) {
                rv = encode_page(in, L, table, map, rec, fld, p.dst, p.dst_cap, lane);
            } else if (split) {
                auto sink = [&](const uint2 *rr, uint32_t n, uint32_t anchor) -> bool {
                    return emit_staged(rr, n, anchor, in, p.dst, opA, p.dst_cap, ring, rA, map, lane);
                };
                cursorA = lzp::parse_page(in, H + kLastLiterals, table, rec, lane, sink);
                okA = cursorA != 0xFFFFFFFFu;
                if (okA) out_flush_all(ring, rA, p.dst, opA, lane);
            }
            if (lane == 0) {
                const size_t nx = (size_t)atomicAdd(ctr, 1u) + gridDim.x;
                hdr->next2_lo = (uint32_t)nx;
                hdr->next2_hi = (uint32_t)(nx >> 32);
            }
        } else if (split) {
            seed_table(in, table, 0u, H, lane);   // the positions of A's half
            uint32_t op = 0;
            OutRing r{0u, 0u};
            bool first = true;
            if (lane == 0) hdr->has_first = 0;
            auto sink = [&](const uint2 *rr, uint32_t n, uint32_t anchor) -> bool {
                if (first) {
                    first = false;
                    if (lane == 0) {
                        hdr->first = rr[0];
                        hdr->has_first = 1;
                    }
                    if (n == 1) return true;
                    const uint32_t a = (rr[0].x & 0xFFFFu) + (rr[0].y & 0xFFFFu);
                    return emit_staged(rr + 1, n - 1, a, in, scratch, op, 0xFFFFFFFFu, ring, r, map, lane);
                }
                return emit_staged(rr, n, anchor, in, scratch, op, 0xFFFFFFFFu, ring, r, map, lane);
            };
            const uint32_t anchor = lzp::parse_page(in, L, table, rec, lane, sink, H);
            out_flush_all(ring, r, scratch, op, lane);
            if (!first) (void)write_last_literals(in, anchor, L, scratch, op, 0xFFFFFFFFu, lane);
            if (lane == 0) hdr->len_b = first ? 0u : op;
        }
        __syncthreads();   // both halves parsed
        if (wave == 0) {
            if (!fits) {
                rv = kResultTooLarge;
            } else if (split) {
                rv = 0;
                if (okA) {
                    const uint32_t lb = rfl(hdr->len_b);
                    bool ok;
                    if (rfl(hdr->has_first)) {
                        if (lane == 0) rec[0] = hdr->first;
                        __builtin_amdgcn_wave_barrier();
                        ok = emit_staged(rec, 1, cursorA, in, p.dst, opA, p.dst_cap, ring, rA, map, lane);
                        if (ok) out_flush_all(ring, rA, p.dst, opA, lane);
                    } else {
                        ok = write_last_literals(in, cursorA, L, p.dst, opA, p.dst_cap, lane);
                    }
                    if (ok && (uint64_t)opA + lb <= p.dst_cap) rv = (int32_t)(opA + lb);
                }
                if (lane == 0) hdr->len_a = opA;
            }
            if (lane == 0) {
                hdr->result = rv;
                b.results[page] = rv;
            }
        }
        __syncthreads();
        if (split) {   // B's stream after A's and the joint
            const int32_t res = (int32_t)rfl((uint32_t)hdr->result);
            const uint32_t la = rfl(hdr->len_a), lb = rfl(hdr->len_b);
            if (res > 0 && lb) {
                uint8_t *d = p.dst + la;
                const uint32_t nv = lb >> 4;
                for (uint32_t v = tid; v < nv; v += 2 * kWave)
                    *(g_u32x4_ua *)(uintptr_t)(d + 16 * v) = gload_nt((const u32x4 *)(scratch + 16 * v));
                for (uint32_t j = (nv << 4) + tid; j < lb; j += 2 * kWave) d[j] = scratch[j];
            }
        }
        __syncthreads();   // the stage, the tables and the header are free
        if (next >= b.count) break;
        page = next;
        p = pn;
        head = nhead;
        if (p.src_len <= in_cap && p.src_len > 0) {
            u32x4 *l = (u32x4 *)stage;
#pragma unroll
            for (uint32_t k = 0; k < kSplitPrefetch; k++) {
                const uint32_t v = tid + k * 2 * kWave;
                if (v < nvec) l[v] = pf[k];
            }
            const u32x4 *g = (const u32x4 *)((uintptr_t)p.src - nhead);
            for (uint32_t v = tid + kSplitPrefetch * 2 * kWave; v < nvec; v += 2 * kWave) l[v] = gload_nt(g + v);
        }
        if (tid == 0) {
            hdr->next_lo = hdr->next2_lo;
            hdr->next_hi = hdr->next2_hi;
        }
    }
}

// ---- N-wave split encoder (round 3; 3 waves are the default for pages >= kSplitMin).
//
// The two-wave kernel above runs 12 waves per CU; its counters (r03 PMC) show
// the waves waiting ~42 % of their cycles with no unit saturated (VALU ~35 %,
// the CU's scalar unit ~42 %): latency-bound.  Here kNW waves share one staged
// page, wave w parsing part [b_w, b_{w+1}) with b_w = (w L / kNW) rounded down
// to 64; every wave but the first seeds its table with the kSeed positions
// before its part (block order, as the one-wave parse would have inserted
// them; the 2^10-slot table holds little older than that anyway) and holds back
// its first sequence.  Matches of part w end by b_{w+1} (its parse sees
// L' = b_{w+1} + LASTLITERALS).  After a barrier wave 0 lays out the page:
// part 0's stream (already in dst), then for each later part the joint
// sequence (literals from the previous part's last match end, then the part's
// held-back first match), then the part's stream from its scratch; a part with
// no match joins the literal run.  The waves then copy their streams into place.
// Per page LDS: header + kNW x (table, map, records, ring) + the stage: 31.5 KiB
// for 4 waves at 16 KiB pages, 5 pages (20 waves) per CU by LDS.
#ifndef TYCHE_LZ4_SEED
#define TYCHE_LZ4_SEED 4096   // positions seeded before a part (a multiple of 64)
#endif
constexpr uint32_t kSeed = TYCHE_LZ4_SEED;
template <uint32_t kNW>
struct SplitHdrN {
    uint32_t next_lo, next_hi, next2_lo, next2_hi;
    int32_t result;
    uint32_t pad0[3];
    uint32_t len[kNW];        // bytes of part w's stream (part 0: in dst, the rest in their scratch)
    uint32_t cursor[kNW];     // end of part w's last match (its parse's final anchor)
    uint32_t has_first[kNW];  // part w > 0: its first record was held back
    uint32_t ok[kNW];         // part 0: its emission fit the capacity
    uint32_t seg[kNW];        // part w > 0: its stream's offset in dst
    uint2 first[kNW];         // part w > 0: the held-back record
};
template <uint32_t kNW>
constexpr size_t split_hdr_bytes() { return (sizeof(SplitHdrN<kNW>) + 63) & ~(size_t)63; }
template <uint32_t kNW>
constexpr size_t split_stage_off() { return split_hdr_bytes<kNW>() + kNW * kWaveRegion; }
template <uint32_t kNW>
__host__ __device__ constexpr uint32_t part_scratch(uint32_t in_cap) {   // a part's worst-case stream, 256-aligned
    return (lz4_bound(in_cap / kNW + 2u * kWave) + 64u + 255u) & ~255u;
}
template <uint32_t kNW>
constexpr uint32_t split_prefetch() { return (16384u / 16u + kNW * kWave - 1u) / (kNW * kWave); }   // 16 KiB per page

template <uint32_t kNW>
#ifndef TYCHE_ENC_WPE
#define TYCHE_ENC_WPE 5   // amdgpu_waves_per_eu register budget of the split kernels (4 waves: 87 VGPRs, no spills; 0: none)
#endif
#if TYCHE_ENC_WPE > 0
#define TYCHE_ENC_WPE_ATTR __attribute__((amdgpu_waves_per_eu(TYCHE_ENC_WPE)))
#else
#define TYCHE_ENC_WPE_ATTR
#endif
__global__ __launch_bounds__(kNW * 64) TYCHE_ENC_WPE_ATTR void lz4_encode_splitn_kernel(tyche_batch_t b, uint32_t in_cap, unsigned *ctr,
                                                                     uint8_t *ws, uint32_t ws_stride, uint32_t seed,
                                                                     uint32_t p0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr uint32_t kT = kNW * kWave;                 // threads per page
    constexpr uint32_t kPf = split_prefetch<kNW>();       // 16-byte vectors per thread prefetched
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = rfl(tid >> 6);
    SplitHdrN<kNW> *hdr = (SplitHdrN<kNW> *)smem;
    uint8_t *region = smem + split_hdr_bytes<kNW>() + wave * kWaveRegion;
    uint16_t *table = (uint16_t *)region;
    uint8_t *map = region + kHashSize * sizeof(uint16_t);
    uint2 *rec = (uint2 *)(map + 4 * kWave);
    uint4 *fld = (uint4 *)(rec + kWave);
    uint8_t *ring = (uint8_t *)fld;
    uint8_t *stage = smem + split_stage_off<kNW>();
    const uint32_t part_ws = part_scratch<kNW>(in_cap);
    uint8_t *scratch = ws + (size_t)blockIdx.x * ws_stride + (size_t)(wave ? wave - 1u : 0u) * part_ws;

    size_t page = blockIdx.x;
    if (page >= b.count) return;
    PageRef p = batch_page(b, page);
    uint32_t head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, tid, kT);
    if (tid == 0) {
        const size_t nx = (size_t)atomicAdd(ctr, 1u) + gridDim.x;   // dynamic assignment (engine.h)
        hdr->next_lo = (uint32_t)nx;
        hdr->next_hi = (uint32_t)(nx >> 32);
    }
    for (;;) {
        for (uint32_t w = lane; w < kHashSize / 8; w += kWave) ((u32x4 *)table)[w] = u32x4{0, 0, 0, 0};
        if (tid < kWave) stage[head + p.src_len + tid] = 0;
        __syncthreads();
        const size_t next = (size_t)rfl(hdr->next_lo) | ((size_t)rfl(hdr->next_hi) << 32);
        PageRef pn;
        u32x4 pf[kPf];
        uint32_t nhead = 0, nvec = 0;
        if (next < b.count) {
            pn = batch_page(b, next);
            if (pn.src_len <= in_cap && pn.src_len > 0) {
                const uintptr_t a = (uintptr_t)pn.src;
                nhead = (uint32_t)(a & 15u);
                nvec = (nhead + pn.src_len + 15u) >> 4;
                const u32x4 *g = (const u32x4 *)(a - nhead);
#pragma unroll
                for (uint32_t k = 0; k < kPf; k++) pf[k] = gload_nt(g + min(tid + k * kT, nvec - 1u));
            }
        }
        const uint8_t *in = stage + head;
        const uint32_t L = p.src_len;
        const bool fits = L <= in_cap;
        // part w starts at bnd(w): equal parts, or (p0 > 0) p0/64 of the page for part 0 -- the one
        // part that seeds nothing -- and equal shares of the rest for the others
        auto bnd = [&](uint32_t w) -> uint32_t {
            if (w == 0) return 0u;
            if (w == kNW) return L;
            if (!p0) return ((L * w) / kNW) & ~(kWave - 1u);
            const uint32_t h = (L * p0 / 64u) & ~(kWave - 1u);
            return (h + ((L - h) * (w - 1u)) / (kNW - 1u)) & ~(kWave - 1u);
        };
        const uint32_t b0 = bnd(wave);
        const uint32_t b1 = bnd(wave + 1);
        const uint32_t Lp = wave + 1 == kNW ? L : b1 + kLastLiterals;   // part w's matches end by b1
        if (fits) {
            // one parse instance and one inlined sink for every wave (26 KiB of kernel code instead of
            // 51; 77.8 vs 78.0 ms per 1M x 16 KiB pages): part 0 writes to dst within its capacity,
            // later parts seed their table, hold back their first record and write to their scratch
            if (wave > 0) {
                seed_table(in, table, b0 > seed ? b0 - seed : 0u, b0, lane);   // the positions before the part
                if (lane == 0) hdr->has_first[wave] = 0;
            }
            uint8_t *odst = wave == 0 ? p.dst : scratch;
            const uint32_t ocap = wave == 0 ? p.dst_cap : 0xFFFFFFFFu;
            uint32_t op = 0;
            OutRing r{0u, 0u};
            bool first = wave > 0;
            auto sink = [&](const uint2 *rr, uint32_t n, uint32_t anchor) -> bool {
                const uint2 *r2 = rr;
                uint32_t n2 = n, a2 = anchor;
                if (first) {
                    first = false;
                    if (lane == 0) {
                        hdr->first[wave] = rr[0];
                        hdr->has_first[wave] = 1;
                    }
                    r2 = rr + 1;
                    n2 = n - 1;
                    a2 = (rr[0].x & 0xFFFFu) + (rr[0].y & 0xFFFFu);
                    if (n2 == 0) return true;
                }
                return emit_sink_n(r2, n2, a2, in, odst, op, ocap, ring, r, map, lane);
            };
            const uint32_t cur = lzp::parse_page(in, Lp, table, rec, lane, sink, b0);
            if (wave == 0) {
                const bool ok = cur != 0xFFFFFFFFu;
                if (ok) out_flush_all(ring, r, p.dst, op, lane);
                if (lane == 0) {
                    hdr->ok[0] = ok ? 1u : 0u;
                    hdr->len[0] = op;
                    hdr->cursor[0] = ok ? cur : 0u;
                    const size_t nx = (size_t)atomicAdd(ctr, 1u) + gridDim.x;
                    hdr->next2_lo = (uint32_t)nx;
                    hdr->next2_hi = (uint32_t)(nx >> 32);
                }
            } else {
                const bool had = !first;   // the sink held back a first record: the part has a match
                out_flush_all(ring, r, scratch, op, lane);
                if (had && wave + 1 == kNW) (void)write_last_literals(in, cur, L, scratch, op, 0xFFFFFFFFu, lane);
                if (lane == 0) {
                    hdr->len[wave] = had ? op : 0u;
                    hdr->cursor[wave] = cur;
                }
            }
        }
        __syncthreads();   // every part parsed
        if (wave == 0) {
            int32_t rv = 0;
            if (!fits) {
                rv = kResultTooLarge;
            } else if (rfl(hdr->ok[0])) {
                // layout: part 0's stream, then per later part the joint sequence and its stream
                uint32_t op = rfl(hdr->len[0]), cur = rfl(hdr->cursor[0]);
                bool ok = true, tail_done = false;
                OutRing r{0u, 0u};
                for (uint32_t w = 1; w < kNW && ok; w++) {
                    if (!rfl(hdr->has_first[w])) {
                        if (lane == 0) hdr->seg[w] = op;
                        continue;
                    }
                    if (lane == 0) rec[0] = hdr->first[w];
                    __builtin_amdgcn_wave_barrier();
                    ok = emit_sink_n(rec, 1, cur, in, p.dst, op, p.dst_cap, ring, r, map, lane);
                    if (ok) out_flush_all(ring, r, p.dst, op, lane);
                    if (lane == 0) hdr->seg[w] = op;
                    op += rfl(hdr->len[w]);
                    cur = rfl(hdr->cursor[w]);
                    tail_done = w + 1 == kNW;
                }
                if (ok && !tail_done) ok = write_last_literals(in, cur, L, p.dst, op, p.dst_cap, lane);
                if (ok && op <= p.dst_cap) rv = (int32_t)op;
            }
            if (lane == 0) {
                hdr->result = rv;
                b.results[page] = rv;
            }
        }
        __syncthreads();
        if (wave > 0 && fits) {   // part w's stream into place
            const int32_t res = (int32_t)rfl((uint32_t)hdr->result);
            const uint32_t lw = rfl(hdr->len[wave]);
            if (res > 0 && lw) {
                uint8_t *d = p.dst + rfl(hdr->seg[wave]);
                const uint32_t nv = lw >> 4;
                for (uint32_t v = lane; v < nv; v += kWave)
                    *(g_u32x4_ua *)(uintptr_t)(d + 16 * v) = gload_nt((const u32x4 *)(scratch + 16 * v));
                for (uint32_t j = (nv << 4) + lane; j < lw; j += kWave) d[j] = scratch[j];
            }
        }
        __syncthreads();   // the stage, the tables and the header are free
        if (next >= b.count) break;
        page = next;
        p = pn;
        head = nhead;
        if (p.src_len <= in_cap && p.src_len > 0) {
            u32x4 *l = (u32x4 *)stage;
#pragma unroll
            for (uint32_t k = 0; k < kPf; k++) {
                const uint32_t v = tid + k * kT;
                if (v < nvec) l[v] = pf[k];
            }
            const u32x4 *g = (const u32x4 *)((uintptr_t)p.src - nhead);
            for (uint32_t v = tid + kPf * kT; v < nvec; v += kT) l[v] = gload_nt(g + v);
        }
        if (tid == 0) {
            hdr->next_lo = hdr->next2_lo;
            hdr->next_hi = hdr->next2_hi;
        }
    }
}

__global__ __launch_bounds__(64) void lz4_encode_kernel(tyche_batch_t b, uint32_t in_cap, unsigned *ctr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint16_t *table = (uint16_t *)smem;
    uint8_t *map = smem + kHashSize * sizeof(uint16_t);                 // 256-byte owner map
    uint2 *rec = (uint2 *)(map + 4 * kWave);                           // 64 sequence records
    uint4 *fld = (uint4 *)(rec + kWave);                               // 64 packed sequence fields / output ring
    uint8_t *stage = (uint8_t *)fld + kOutRing;
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
            for (uint32_t w = lane; w < kHashSize / 8; w += kWave) ((u32x4 *)table)[w] = u32x4{0, 0, 0, 0};
            WAVE_SYNC();
            in[p.src_len + lane] = 0;
            WAVE_SYNC();
            rv = encode_page(in, p.src_len, table, map, rec, fld, p.dst, p.dst_cap, lane);
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

hipError_t launch_lz4_encode(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    if (in_cap > 65535u) return hipErrorInvalidValue;    // 16-bit positions (byU16 regime)
    // TYCHE_LZ4_ENC=1: the one-wave kernel for every batch (A/B timing)
    const bool one_wave = knob("LZ4_ENC", 0) == 1;
    // waves per page of the split encoders (2: the two-wave kernel; 3 in round 3: 79.4 vs 85.0 ms per
    // 1M x 16 KiB pages at ratio 2.6193 vs 2.6204, part 0 taking 27/64 of the page and the later parts
    // seeded with the 10,240 positions before them).  Round 4: 512-byte output rings and a 5-waves-
    // per-SIMD register budget (18-20 waves per CU instead of 15) -- three waves 72.2 ms at 2.6188,
    // four (default) 70.5 at 2.6184 with 9,216 seeds and part 0 22/64 (seeds 8,192-12,288 x shares
    // 18-24/64: 69.5-72.9 ms at 2.6158-2.6184, profiles/r04_lz4_encode_occupancy.log)
    const long nw = knob("LZ4_ENC_WAVES", 4);
    // TYCHE_LZ4_SPLIT_MIN: the smallest in_cap that takes a split kernel.  8 KiB pages split into
    // three parts too since round 3 (256K x 8 KiB pages, ms per 1M: one wave per page 70.6 -- it holds
    // 168 VGPRs, 12 waves per CU --, three waves 41.5 at ratio 2.525 vs 2.528, four 37.9 at 2.519);
    // the two-wave kernel keeps kSplitMin for its own per-page split
    const uint32_t split_min = (uint32_t)std::max(0L, knob("LZ4_SPLIT_MIN", nw == 3 || nw == 4 || nw == 8 ? 8192L
                                                                                                       : (long)kSplitMin));
    if (!one_wave && in_cap >= split_min && (nw == 3 || nw == 4 || nw == 8)) {
        const void *k = nw == 8   ? (const void *)lz4_encode_splitn_kernel<8>
                        : nw == 4 ? (const void *)lz4_encode_splitn_kernel<4>
                                  : (const void *)lz4_encode_splitn_kernel<3>;
        const uint32_t T = (uint32_t)nw * kWave;
        const size_t lds = (nw == 8 ? split_stage_off<8>() : nw == 4 ? split_stage_off<4>() : split_stage_off<3>()) +
                           ((in_cap + 16u + kPad + 15u) & ~15u);
        const size_t ncu = prepare_launch(k);
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, (int)T, lds) != hipSuccess || per_cu < 1) per_cu = 1;
        const long cap_cu = knob("LZ4_ENC_PAGES_PER_CU", 0);   // (occupancy A/B: resident pages per CU)
        if (cap_cu > 0) per_cu = std::min<int>(per_cu, (int)cap_cu);
        const size_t grid = std::min<size_t>(b.count, ncu * (size_t)per_cu);
        const uint32_t pws = nw == 8 ? part_scratch<8>(in_cap) : nw == 4 ? part_scratch<4>(in_cap) : part_scratch<3>(in_cap);
        uint32_t seed = (uint32_t)std::max(0L, knob("LZ4_ENC_SEED", nw == 3 ? 10240L : nw == 4 ? 8192L : (long)kSeed)) &
                        ~(kWave - 1u);   // positions seeded before a part
        // part 0's share of the page in 64ths (0: equal parts); at least 1/kNW, so the later parts fit
        // their scratch (part_scratch: a 1/kNW part)
        // Round 5, after the parse's instruction diet made seeding cheaper (profiles/r05_knob_enc*.log,
        // 256K pages): part 0 19/64 and 8,192 seeds 63.6 ms at ratio 2.6175 (22/64 and 9,216: 65.0 at 2.6189)
        uint32_t p0 = (uint32_t)std::max(0L, knob("LZ4_ENC_P0", nw == 3 ? 27L : nw == 4 ? 19L : 0L));
        if (p0) p0 = std::min<uint32_t>(std::max<uint32_t>(p0, (64u + (uint32_t)nw - 1u) / (uint32_t)nw), 48u);
        const uint32_t ws_stride = (uint32_t)(nw - 1) * pws;
        ScratchLease ws(s, grid * (size_t)ws_stride);
        if (ws.get()) {
            WorkCounter ctr(s, grid < b.count);
            if (!ctr.get()) return hipErrorOutOfMemory;
            unsigned *cp = ctr.get();
            uint8_t *wp = (uint8_t *)ws.get();
            void *args[] = {(void *)&b, &in_cap, &cp, &wp, (void *)&ws_stride, &seed, &p0};
            (void)hipLaunchKernel(k, dim3((unsigned)grid), dim3(T), args, lds, s);
            return hipGetLastError();
        }
    }
    if (!one_wave && in_cap >= split_min) {
        const size_t lds = kSplitStage + ((in_cap + 16u + kPad + 15u) & ~15u);
        const size_t ncu = prepare_launch((const void *)lz4_encode_split_kernel);
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)lz4_encode_split_kernel, 2 * kWave,
                                                         lds) != hipSuccess || per_cu < 1)
            per_cu = 1;
        const size_t grid = std::min<size_t>(b.count, ncu * (size_t)per_cu);
        // B's scratch: its half's worst case (LZ4_compressBound of L - H < in_cap / 2 + 64), 256-byte aligned
        const uint32_t ws_stride = (lz4_bound(in_cap / 2u + kWave) + 64u + 255u) & ~255u;
        ScratchLease ws(s, grid * (size_t)ws_stride);
        if (ws.get()) {   // else the one-wave kernel below, which needs no scratch
            WorkCounter ctr(s, grid < b.count);
            if (!ctr.get()) return hipErrorOutOfMemory;
            hipLaunchKernelGGL(lz4_encode_split_kernel, dim3((unsigned)grid), dim3(2 * kWave), lds, s, b, in_cap,
                               ctr.get(), (uint8_t *)ws.get(), ws_stride);
            return hipGetLastError();
        }
    }
    const size_t lds = kHashSize * sizeof(uint16_t) + 4 * kWave + kWave * 8 + kOutRing +
                       ((in_cap + 16u + kPad + 15u) & ~15u);
    const size_t ncu = prepare_launch((const void *)lz4_encode_kernel);
    const size_t per_cu = waves_per_cu((const void *)lz4_encode_kernel, lds);
    const size_t grid = std::min<size_t>(b.count, ncu * per_cu);
    WorkCounter ctr(s, grid < b.count);
    if (!ctr.get()) return hipErrorOutOfMemory;
    hipLaunchKernelGGL(lz4_encode_kernel, dim3((unsigned)grid), dim3(kWave), lds, s, b, in_cap, ctr.get());
    return hipGetLastError();
}

#ifdef TYCHE_PHASES
// profiling builds only: per-phase parse cycles summed since the last call (then cleared)
extern "C" int tyche_phase_read(unsigned long long *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lzp::g_phase), 16 * sizeof(unsigned long long)) != hipSuccess) return -1;
    static const unsigned long long zero[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(lzp::g_phase), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace tyche
