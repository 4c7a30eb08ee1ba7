// lz4_encode.hip -- batched LZ4 block encode for gfx950 (the sweep path).
//
// Replaces the per-victim LZ4_compress_default call of buffer__compress
// (reference src/buffer.c:178-188 -> src/lz4/lz4.c:697 -> LZ4_compress_generic
// lz4.c:459-656) with one kernel over a batch of pages.  The output is a
// standard LZ4 block that LZ4_decompress_safe (lz4.c:1251) -- the reference's
// own decoder -- restores bit-exactly; it is not required to be the same bytes
// 1.7.5 emits.  The parsing rules the decoder enforces are
// kept: every match starts at or before iend-MFLIMIT (12) and ends at or before
// iend-LASTLITERALS (5), lz4.c:266-267, 1147-1156, 1225.
//
// Layout: one 64-lane wave per page.  The page is staged into LDS; a position
// table of 2^kHashLog 16-bit offsets (the byU16 scheme of lz4.c:402-408) lives
// next to it.  Match finding is lane-parallel: for a 64-position block every
// lane hashes its 4 bytes, reads the candidate left by earlier blocks, checks
// it and measures the match length.  The greedy parse then walks the block
// with ballots (first position >= cursor that has a match), and each chosen
// sequence is emitted as one coalesced byte store per lane (token, length
// bytes, literals, offset).
#include <hip/hip_runtime.h>

#include "engine.h"
#include "lds_io.h"

namespace tyche {

namespace {

constexpr uint32_t kWave = 64;
constexpr uint32_t kHashLog = 12;
constexpr uint32_t kHashSize = 1u << kHashLog;
constexpr uint32_t kPad = 64;
constexpr uint32_t kLaneExtendCap = 128;   // per-lane length probe; the chosen match extends further

// 4 bytes at an arbitrary LDS byte offset (little endian), from two aligned dwords
__device__ __forceinline__ uint32_t ld32(const uint8_t *base, uint32_t off) {
    const uint32_t *w = (const uint32_t *)base;
    uint32_t lo = w[off >> 2], hi = w[(off >> 2) + 1];
    return __builtin_amdgcn_alignbyte(hi, lo, off & 3u);
}

__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

// number of equal bytes at a and b, a advancing up to (exclusive) limit;
// positions are offsets from the 16-byte-aligned staging base
__device__ __forceinline__ uint32_t match_extend(const uint8_t *in, uint32_t a, uint32_t b, uint32_t limit) {
    uint32_t n = 0;
    while (a + n + 4 <= limit) {
        uint32_t x = ld32(in, a + n) ^ ld32(in, b + n);
        if (x) return n + (__builtin_ctz(x) >> 3);
        n += 4;
    }
    while (a + n < limit && in[a + n] == in[b + n]) n++;
    return n;
}

// wave-cooperative extension from a (match) / b (candidate), 256 bytes per step
__device__ uint32_t wave_extend(const uint8_t *in, uint32_t a, uint32_t b, uint32_t limit, uint32_t lane) {
    uint32_t n = 0;
    for (;;) {
        uint32_t pa = a + n + 4 * lane;
        bool full = pa + 4 <= limit;
        uint32_t x = full ? (ld32(in, pa) ^ ld32(in, b + n + 4 * lane)) : 1u;
        uint64_t bad = __ballot(x != 0);
        if (bad == 0) { n += 4 * kWave; continue; }
        uint32_t first = (uint32_t)__builtin_ctzll(bad);
        uint32_t xf = rdlane(x, first);
        uint32_t pf = a + n + 4 * first;
        if (pf + 4 <= limit) return n + 4 * first + (__builtin_ctz(xf) >> 3);
        // tail shorter than 4 bytes
        uint32_t m = n + 4 * first;
        while (a + m < limit && rfl(in[a + m]) == rfl(in[b + m])) m++;
        return m;
    }
}

struct Emitter {
    uint8_t *dst;
    uint32_t cap;
    uint32_t op;
    bool overflow;
};

// Emits one sequence (literals in[anchor, anchor+lit), then, if has_match, a
// match of length ml at distance off) with one byte store per lane per 64 bytes.
__device__ void emit_sequence(Emitter &e, const uint8_t *in, uint32_t anchor, uint32_t lit, bool has_match,
                              uint32_t off, uint32_t ml, uint32_t lane) {
    uint32_t lit_ext = lit >= 15 ? (lit - 15) / 255 + 1 : 0;
    uint32_t mc = has_match ? ml - kMinMatch : 0;
    uint32_t ml_ext = (has_match && mc >= 15) ? (mc - 15) / 255 + 1 : 0;
    uint32_t total = 1 + lit_ext + lit + (has_match ? 2 : 0) + ml_ext;
    if (e.overflow || e.op + total > e.cap) {
        e.overflow = true;
        return;
    }
    uint32_t token = ((lit >= 15 ? 15u : lit) << 4) | (has_match ? (mc >= 15 ? 15u : mc) : 0u);
    const uint32_t lit_begin = 1 + lit_ext, off_begin = lit_begin + lit, ml_begin = off_begin + 2;
    for (uint32_t j = lane; j < total; j += kWave) {
        uint32_t v;
        if (j == 0) v = token;
        else if (j < lit_begin) v = (j == lit_begin - 1) ? (lit - 15) % 255 : 255;
        else if (j < off_begin) v = in[anchor + (j - lit_begin)];
        else if (j == off_begin) v = off & 0xFF;
        else if (j == off_begin + 1) v = off >> 8;
        else v = (j == total - 1) ? (mc - 15) % 255 : 255;
        e.dst[e.op + j] = (uint8_t)v;
    }
    e.op += total;
}

__global__ __launch_bounds__(64) void lz4_encode_wave_kernel(tyche_batch_t b, uint32_t in_cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    const size_t page = blockIdx.x;
    PageRef p = batch_page(b, page);
    if (p.src_len > in_cap) {
        if (lane == 0) b.results[page] = kResultTooLarge;
        return;
    }
    uint16_t *table = (uint16_t *)smem;                              // kHashSize entries
    uint8_t *stage = smem + kHashSize * sizeof(uint16_t);
    // stage the page so that it starts 16-byte aligned: copy at head then the
    // matcher addresses it through `in`
    uint32_t head = stage_in(p.src, p.src_len, stage, lane, kWave);
    uint8_t *in = stage + head;
    const uint32_t L = p.src_len;
    for (uint32_t h = lane; h < kHashSize / 2; h += kWave) ((uint32_t *)table)[h] = 0;
    __syncthreads();
    in[L + lane] = 0;
    __syncthreads();

    Emitter e{p.dst, p.dst_cap, 0, false};
    uint32_t anchor = 0;
    if (L >= (uint32_t)(kMfLimit + 1)) {
        const uint32_t mflimit = L - kMfLimit;          // last position a match may start
        const uint32_t matchlimit = L - kLastLiterals;  // matches end before this
        uint32_t cursor = 0;
        while (cursor <= mflimit && !e.overflow) {
            const uint32_t blk = cursor & ~(kWave - 1);
            const uint32_t pos = blk + lane;
            // ---- lane-parallel match finding for positions blk .. blk+63
            uint32_t cand = 0, len = 0;
            bool live = pos <= mflimit;
            uint32_t v = 0, h = 0;
            if (live) {
                v = ld32(stage, head + pos);
                h = hash4(v);
                cand = table[h];
            }
            __builtin_amdgcn_wave_barrier();
            if (live) table[h] = (uint16_t)pos;
            if (live && cand < pos && ld32(stage, head + cand) == v) {
                uint32_t lim = min(matchlimit, pos + kLaneExtendCap);
                len = kMinMatch + match_extend(stage, head + pos + kMinMatch, head + cand + kMinMatch, head + lim);
            }
            // ---- greedy parse over this block
            for (;;) {
                uint64_t m = __ballot(len != 0 && pos >= cursor);
                if (m == 0) {
                    cursor = blk + kWave;
                    break;
                }
                uint32_t ln = (uint32_t)__builtin_ctzll(m);
                uint32_t mpos = blk + ln;
                uint32_t mcand = rdlane(cand, ln);
                uint32_t mlen = rdlane(len, ln);
                if (mlen >= kLaneExtendCap && mpos + mlen < matchlimit) {
                    mlen = kMinMatch + wave_extend(stage, head + mpos + kMinMatch, head + mcand + kMinMatch,
                                                   head + matchlimit, lane);
                }
                // catch up backwards over pending literals (lz4.c:549)
                while (mpos > anchor && mcand > 0 && rfl(in[mpos - 1]) == rfl(in[mcand - 1])) {
                    mpos--;
                    mcand--;
                    mlen++;
                }
                emit_sequence(e, in, anchor, mpos - anchor, true, mpos - mcand, mlen, lane);
                anchor = mpos + mlen;
                cursor = anchor;
                if (cursor >= blk + kWave || cursor > mflimit || e.overflow) break;
            }
        }
    }
    // last literals
    emit_sequence(e, in, anchor, L - anchor, false, 0, 0, lane);
    if (lane == 0) b.results[page] = e.overflow ? 0 : (int32_t)e.op;
}

}  // namespace

hipError_t launch_lz4_encode(const tyche_batch_t &b, uint32_t in_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    if (in_cap > 65535u) return hipErrorInvalidValue;    // 16-bit positions (byU16 regime)
    size_t lds = kHashSize * sizeof(uint16_t) + ((in_cap + 16u + kPad + 15u) & ~15u);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)lz4_encode_wave_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(lz4_encode_wave_kernel, dim3((unsigned)b.count), dim3(kWave), lds, s, b, in_cap);
    return hipGetLastError();
}

}  // namespace tyche
