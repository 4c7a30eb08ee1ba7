// lz_exec.h -- byte-parallel execution of LZ77 sequences into an LDS window,
// shared by the gfx950 decoders (LZ4 blocks, zstd frames).
//
// A batch of up to 64 decoded sequences sits in lanes (lane j: output start o,
// literal length lit, literal source ls, match offset off, match length ml).
// Instead of copying sequence by sequence (the dependency order of the
// reference's forward byte copies, lz4.c:1209-1236 / zstd_decompress.c:975-1001),
// the batch's output range is built 256 bytes at a time, 4 bytes per lane:
//
//   1. owner: every sequence that starts inside the chunk stamps its lane into
//      a 256-byte LDS map; a per-lane max over its 4 map bytes and a DPP
//      prefix-max give every output byte the sequence it belongs to;
//   2. source: a literal byte comes from the literal buffer; a match byte at p
//      copies p - off, which for a self-overlapping match (off < ml) folds to
//      d - off + ((p - d) mod off) -- the byte the forward copy ultimately
//      repeats;
//   3. every byte whose source lies before the chunk (or in the literal buffer)
//      is read and written at once (4-byte LDS store when a lane's 4 bytes are
//      all final);
//   4. bytes whose source lies inside the chunk (a match reaching back less than
//      256 bytes into bytes made in the same step) are settled in rounds with a
//      per-chunk ready bitmap; the rounds follow cross-sequence chains, which
//      are short (folding removes the self-overlap chains).
//
// Every chunk reads all of its literal and window bytes before it writes any,
// so a literal buffer placed at the tail of the window (zstd's layout, whose
// literal k is stored at or after its output position) is never overwritten
// before it is read.
#pragma once
#include <hip/hip_runtime.h>

#include "lds_io.h"

namespace tyche {
namespace lzx {

constexpr uint32_t kWave = 64;
constexpr uint32_t kChunk = 256;

__device__ __forceinline__ uint32_t mod_small(uint32_t i, uint32_t m) {
    // i % m for i < 2^20, m >= 1 without an integer divide
    uint32_t q = (uint32_t)((float)i * __frcp_rn((float)m));
    int32_t r = (int32_t)i - (int32_t)(q * m);
    if (r < 0) r += (int32_t)m;
    if (r >= (int32_t)m) r -= (int32_t)m;
    return (uint32_t)r;
}

// exclusive prefix max over lanes (lane 0 gets -1)
__device__ __forceinline__ int32_t wave_excl_max(int32_t v) {
    const int32_t incl = wave_incl_max(v);
    const int32_t up = __shfl_up(incl, 1);
    return threadIdx.x == 0 ? -1 : up;
}

// Source of output byte p owned by a sequence (o, lit, ls, off, ml):
// returns the window position to copy (>= 0), or ~(literal position) for a literal.
__device__ __forceinline__ int32_t byte_source(int32_t p, int32_t o, int32_t lit, int32_t ls, int32_t off, int32_t ml) {
    const int32_t d = o + lit;
    if (p < d) return ~(ls + (p - o));
    // offset 0 (accepted by LZ4_decompress_safe, which then copies bytes it never
    // wrote; the output is unspecified) reads the byte before the match
    if (off <= 0) return d > 0 ? d - 1 : ~0;
    const int32_t q = p - d;
    if (off >= ml || q < off) return p - off;
    return d - off + (int32_t)mod_small((uint32_t)q, (uint32_t)off);
}

// Builds win[B0, B1) from the n sequences in lanes [0, n).  Zero-length
// sequences are allowed.  map: 256 bytes, rdy: 64 bytes of LDS scratch.
__device__ inline void exec_chunks(uint8_t *win, const uint8_t *lit_base, uint32_t n, int32_t o, int32_t lit,
                                   int32_t ls, int32_t off, int32_t ml, int32_t B0, int32_t B1, uint8_t *map,
                                   uint8_t *rdy, uint32_t lane) {
    const bool act = lane < n;
    const int32_t olen = act ? lit + ml : 0;
    const uint32_t pk_a = (uint32_t)o | ((uint32_t)lit << 16);
    const uint32_t pk_b = (uint32_t)ls | ((uint32_t)off << 16);
    for (int32_t c0 = B0; c0 < B1; c0 += (int32_t)kChunk) {
        const int32_t cend = min(c0 + (int32_t)kChunk, B1);
        // ---- 1. owners
        lds_st32(map + 4 * lane, 0xFFFFFFFFu);
        __builtin_amdgcn_wave_barrier();
        const bool stamp = act && olen > 0 && o >= c0 && o < cend;
        if (stamp) map[o - c0] = (uint8_t)lane;
        __builtin_amdgcn_wave_barrier();
        const uint64_t before = __ballot(act && olen > 0 && o < c0);
        const int32_t carry = before ? 63 - (int32_t)__builtin_clzll(before) : -1;
        const uint32_t m4 = lds_ld32(map + 4 * lane);
        int32_t own[4];
        int32_t run = -1;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t s = (m4 >> (8 * k)) & 0xFFu;
            run = max(run, s == 0xFFu ? -1 : (int32_t)s);
            own[k] = run;
        }
        const int32_t start = max(wave_excl_max(run), carry);
        // ---- 2. sources
        int32_t src[4];
        bool dep[4];
        uint32_t valid = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int32_t p = c0 + 4 * (int32_t)lane + k;
            const int32_t ow = max(own[k], start);
            const uint32_t a = __shfl(pk_a, ow & 63), b = __shfl(pk_b, ow & 63);
            const int32_t mlw = __shfl(ml, ow & 63);
            const bool v = p < cend;
            valid |= (v ? 1u : 0u) << k;
            src[k] = v ? byte_source(p, (int32_t)(a & 0xFFFFu), (int32_t)(a >> 16), (int32_t)(b & 0xFFFFu),
                                     (int32_t)(b >> 16), mlw)
                       : 0;
            dep[k] = v && src[k] >= c0;
        }
        // ---- 3. final bytes: read everything, then write
        uint32_t w = 0, ready = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if ((valid >> k) & 1u && !dep[k]) {
                const uint32_t x = src[k] < 0 ? lit_base[~src[k]] : win[src[k]];
                w |= x << (8 * k);
                ready |= 1u << k;
            }
        }
        __builtin_amdgcn_wave_barrier();
        const int32_t pb = c0 + 4 * (int32_t)lane;
        if (ready == 0xFu) {
            lds_st32(win + pb, w);
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++)
                if ((ready >> k) & 1u) win[pb + k] = (uint8_t)(w >> (8 * k));
        }
        // ---- 4. in-chunk dependencies
        uint32_t pend = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) pend |= (dep[k] ? 1u : 0u) << k;
        if (__ballot(pend != 0)) {
            rdy[lane] = (uint8_t)(ready | (~valid & 0xFu));
            __builtin_amdgcn_wave_barrier();
            // each round settles at least the lowest pending byte: <= 256 rounds
            for (int it = 0; it < (int)kChunk && __ballot(pend != 0); it++) {
                uint32_t got = 0, vals = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if ((pend >> k) & 1u) {
                        const int32_t rr = src[k] - c0;
                        if ((rdy[rr >> 2] >> (rr & 3)) & 1u) {
                            vals |= (uint32_t)win[src[k]] << (8 * k);
                            got |= 1u << k;
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if ((got >> k) & 1u) win[pb + k] = (uint8_t)(vals >> (8 * k));
                pend &= ~got;
                ready |= got;
                if (got) rdy[lane] = (uint8_t)(ready | (~valid & 0xFu));
                __builtin_amdgcn_wave_barrier();
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}


// ---------------------------------------------------------------------------
// Frontier-ordered match copies, 16 at a time.
//
// Matches (lane j: destination d, offset off, length ml) of a batch whose
// literals are already placed are copied in dependency order: the first pending
// match's destination F bounds every byte that is already final, so every
// pending match whose source ends at or before F is independent of the others
// still pending.  Each round hands up to 16 such matches (in stream order) to
// the 16 quads of the wave: a ds_permute sends each selected match to its quad
// leader, a DPP quad broadcast spreads it, and the quad copies 16 bytes per
// step as 4-byte LDS accesses (offsets >= 16 never overlap inside a step; a
// shorter period folds each byte to d - off + (i mod off), the byte the
// reference's forward copy repeats).  Matches above 64 bytes go to the whole
// wave, one at a time.
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false);   // quad_perm [0,0,0,0]
}

__device__ inline void exec_frontier(uint8_t *out, bool applied, int32_t d, int32_t off, int32_t ml, uint32_t lane) {
    const int32_t src_end = d - off + min(ml, off);
    uint64_t pending = __ballot(applied && ml > 0);
    const uint64_t longm = __ballot(applied && ml > 64);
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t grp = lane >> 2, ql = lane & 3u;
    const uint32_t pk1 = (uint32_t)d | ((uint32_t)off << 16);
    while (pending) {
        const uint32_t f = (uint32_t)__builtin_ctzll(pending);
        if ((longm >> f) & 1ull) {
            const int32_t F = (int32_t)rdlane((uint32_t)d, f);
            const int32_t fo = (int32_t)rdlane((uint32_t)off, f), fm = (int32_t)rdlane((uint32_t)ml, f);
            const int32_t fs = F - fo;
            if (fo >= (int32_t)kWave || fo <= 0) {
                for (int32_t i = (int32_t)lane; i < fm; i += (int32_t)kWave) out[F + i] = out[fs + i];
            } else {
                for (int32_t i = (int32_t)lane; i < fm; i += (int32_t)kWave)
                    out[F + i] = out[fs + (int32_t)mod_small((uint32_t)i, (uint32_t)fo)];
            }
            pending &= ~(1ull << f);
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        const int32_t F = (int32_t)rdlane((uint32_t)d, f);
        // ready: pending short matches whose source is final (f itself always is)
        const uint64_t ready = pending & ~longm & __ballot(src_end <= F);
        const uint32_t rank = (uint32_t)__builtin_popcountll(ready & below);
        const bool sel = ((ready >> lane) & 1ull) && rank < 16u;
        const uint64_t taken = __ballot(sel);
        const uint32_t ntaken = (uint32_t)__builtin_popcountll(taken);
        pending &= ~taken;
        // selected lane -> leader lane 4*rank; everyone else writes an odd lane (never read)
        const int32_t dst = sel ? (int32_t)(16u * rank) : (int32_t)(4u * (lane | 1u));
        const uint32_t x1 = quad_bcast((uint32_t)__builtin_amdgcn_ds_permute(dst, (int)pk1));
        const uint32_t x2 = quad_bcast((uint32_t)__builtin_amdgcn_ds_permute(dst, ml));
        const bool gact = grp < ntaken;
        const int32_t gd = (int32_t)(x1 & 0xFFFFu), go = (int32_t)(x1 >> 16), gm = gact ? (int32_t)x2 : 0;
        const int32_t gs = gd - go;
        const bool fold = gact && go < 16 && go < gm;
        for (int32_t i = 4 * (int32_t)ql; i < gm; i += 16) {
            const int32_t nb = min(4, gm - i);
            uint32_t w;
            if (!fold) {
                w = lds_ld32(out + gs + i);
            } else {
                w = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int32_t si = gs + (int32_t)mod_small((uint32_t)(i + k), (uint32_t)max(go, 1));
                    w |= (uint32_t)out[si] << (8 * k);
                }
            }
            if (nb == 4) {
                lds_st32(out + gd + i, w);
            } else {
                for (int k = 0; k < nb; k++) out[gd + i + k] = (uint8_t)(w >> (8 * k));
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace lzx
}  // namespace tyche
