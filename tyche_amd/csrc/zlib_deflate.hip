// zlib_deflate.hip -- gfx950 encoder for zlib streams, the codec behind
// buffer__compress for ZLIB_COMPRESSOR_ID (src/buffer.c:190-200 -> compress2
// level 1, src/zlib/compress.c:22-60 -> deflate_fast, deflate.c:1628).  The
// output is a standard zlib stream that the reference's uncompress()
// (uncompr.c:22-59) restores bit-exactly with the exact length buffer.c:257-260
// requires; it is not required to be the bytes zlib 1.2.8 emits (SURVEY §8a
// A10).  Its ratio is below level 1's: matches are coded with the fixed Huffman
// codes of RFC 1951 3.2.6 (dynamic trees are the §8f rank-4 follow-up).
//
// Stream: header 78 01 (compress2 at level 1, deflate.c:781-800), one final
// fixed-Huffman block (BTYPE 01) holding the page's literals and
// length/distance pairs, end-of-block, and the adler32 of the page
// (big-endian).  A page whose fixed-code stream would not be smaller than the
// stored form is written as stored blocks (BTYPE 00) instead.
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
#include "lz_parse.h"

namespace tyche {
namespace {

using lzp::kHashSize;
using lzp::kWave;
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

// Codes a batch of runs (lane i < n: literals in[ls, ls+ll), then a match of ml
// bytes at distance off; ml may be 0).  Returns false when the stream reaches
// o.limit.
__device__ bool code_runs(Out &o, const uint8_t *in, uint32_t n, uint32_t ls, uint32_t ll, uint32_t ml, uint32_t off,
                          uint8_t *map, uint32_t lane) {
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
        uint32_t bits = 0, len = 0;
        if (j < total) {
            const uint32_t k = j - os0;
            if (k < oll) {
                fixed_ll(in[ols + k], bits, len);
            } else {
                match_bits(chunk_len(oml, k - oll), ooff, bits, len);
            }
        }
        const int32_t bi = wave_incl_sum((int32_t)len);
        const uint32_t b = o.nbits + (uint32_t)bi - len;
        if (len) {
            const uint32_t w = b >> 5, sh = b & 31u;
            atomicOr(&o.stage[w], bits << sh);
            if (sh + len > 32u) atomicOr(&o.stage[w + 1], bits >> (32u - sh));
        }
        __builtin_amdgcn_wave_barrier();
        o.nbits += rdlane((uint32_t)bi, kWave - 1);
        if (!drain(o, lane)) return false;
    }
    return true;
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

// Encodes in[0, L) (LDS, 64 zero bytes after).  Returns the stream size, or 0
// if even the stored form does not fit in cap.
__device__ int32_t encode_page(const uint8_t *in, uint32_t L, uint16_t *table, uint8_t *map, uint2 *rec,
                               uint32_t *stage, uint8_t *dst, uint32_t cap, uint32_t lane) {
    const uint32_t adler = lds_adler32(in, L, lane);
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
            lzp::decode_record(r, n, anc, lane, ls, ll, ml, off);
            if (off > 32768u) { ll += ml; ml = 0; }     // beyond the deflate window: literals
            return code_runs(o, in, n, ls, ll, ml, off, map, lane);
        };
        anchor = lzp::parse_page(in, L, table, rec, lane, sink);
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

__global__ __launch_bounds__(64) void zlib_deflate_kernel(tyche_batch_t b, uint32_t in_cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint16_t *table = (uint16_t *)smem;
    uint32_t *stage_bits = (uint32_t *)(smem + kHashSize * sizeof(uint16_t));
    uint8_t *map = (uint8_t *)(stage_bits + kStageWords);
    uint2 *rec = (uint2 *)(map + kWave);
    uint8_t *stage = (uint8_t *)(rec + kWave);
    const size_t stride = gridDim.x;

    size_t page = blockIdx.x;
    if (page >= b.count) return;
    PageRef p = batch_page(b, page);
    uint32_t head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, lane, kWave);
    for (;;) {
        const size_t next = page + stride;
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
            rv = encode_page(in, p.src_len, table, map, rec, stage_bits, p.dst, p.dst_cap, lane);
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
    const size_t lds = kHashSize * sizeof(uint16_t) + kStageWords * 4 + kWave + kWave * 8 +
                       ((in_cap + 16u + kPad + 15u) & ~15u);
    int dev = 0;
    (void)hipGetDevice(&dev);
    static int cus[64] = {0};
    if (dev < 64 && cus[dev] == 0) {
        (void)hipFuncSetAttribute((const void *)zlib_deflate_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        int n = 0;
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        cus[dev] = n > 0 ? n : 256;
    }
    const size_t per_cu = std::max<size_t>(1, std::min<size_t>(32, (160 * 1024) / lds));
    const size_t grid = std::min<size_t>(b.count, (size_t)(dev < 64 ? cus[dev] : 256) * per_cu);
    hipLaunchKernelGGL(zlib_deflate_kernel, dim3((unsigned)grid), dim3(kWave), lds, s, b, in_cap);
    return hipGetLastError();
}

}  // namespace tyche
