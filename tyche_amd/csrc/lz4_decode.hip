// lz4_decode.hip -- batched LZ4 block decode for gfx950 (the restore path).
//
// Replaces the per-hit LZ4_decompress_safe call of buffer__decompress
// (reference src/buffer.c:248-253 -> src/lz4/lz4.c:1251, generic decoder
// lz4.c:1089-1248) with one kernel over a batch of pages.  Results are
// LZ4_decompress_safe's: decoded size, or -(input bytes consumed)-1 at the same
// consumption point for a malformed stream; decoded bytes are bit-identical.
//
// One 64-lane wave per page; compressed stream and rebuilt page both live in
// LDS, so HBM sees comp_len bytes read and page_len bytes written (16-byte
// accesses).  The serial parts of LZ4 decoding are split apart:
//
//  1. token chain (parse): the stream is cut into 64 segments; every lane walks
//     the token chain speculatively from its segment start, marking visited
//     positions.  A walk from the true entry point (the previous segment's exit)
//     usually lands on a marked position after a few steps and then agrees with
//     the speculative walk, so a short fix-up walk per lane, repeated until no
//     entry changes, yields the exact chain.  The token positions are then
//     compacted into an ordered list.
//  2. per 64 sequences, one per lane: literal length, offset and match length
//     are decoded in parallel, output positions come from a wave prefix sum, and
//     the reference's acceptance checks are evaluated per sequence; the first
//     failing sequence in stream order gives the return value.
//  3. literals are placed in parallel (they depend on nothing).
//  4. matches are copied in dependency order: the first pending match fixes a
//     frontier F (every byte before it is final); all pending matches whose
//     source ends at or before F are independent and are copied together, up to
//     four per instruction (16 lanes each), with modulo addressing for
//     self-overlapping matches (offset < length).  This is exactly the forward
//     byte-copy semantics of lz4.c:1209-1236.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "lds_io.h"

#include <algorithm>
#include <cstdlib>

#ifndef TYCHE_BRIDGE_STEPS
#define TYCHE_BRIDGE_STEPS 4   // token-chain bridge steps per hand-off round (A/B builds)
#endif

namespace tyche {

namespace {

constexpr uint32_t kWave = 64;
constexpr uint32_t kPad = 64;        // zeroed tail after the staged stream
constexpr uint32_t kEnd = 0xFFFFFFFFu;

// Timing-only ablation builds (-DTYCHE_ABLATE=mask; outputs are wrong):
//   1 skip literal placement, 2 skip match copies, 4 skip stage-out,
//   (bit 8 unused)
#ifndef TYCHE_ABLATE
#define TYCHE_ABLATE 0
#endif

// Optional phase profile (diagnostic build only: -DTYCHE_PROFILE).  Shares of
// shader cycles per phase, summed over pages by lane 0.
#ifdef TYCHE_PROFILE
__device__ unsigned long long g_prof[16];
#define PROF_DECL unsigned long long _pt = clock64();
#define PROF_MARK(slot)                                                        \
    do {                                                                       \
        unsigned long long _n = clock64();                                     \
        if (lane == 0) atomicAdd(&g_prof[slot], _n - _pt);                     \
        _pt = _n;                                                              \
    } while (0)
#define PROF_ADD(slot, v) do { if (lane == 0) atomicAdd(&g_prof[slot], (unsigned long long)(v)); } while (0)
#else
#define PROF_DECL
#define PROF_MARK(slot) do { } while (0)
#define PROF_ADD(slot, v) do { } while (0)
#endif



struct SeqIn {
    int32_t lit, ls, off, ml, q2;
    bool in_term, ml_err;
    bool lit_win;     // lit <= 16 and its bytes are in lb[]
    uint32_t lb[4];   // literal bytes 0..15 (lit_win)
};
// Input side of the sequence whose token is at p (the reads of lz4.c:1134-1143,
// 1165, 1172-1182).  One round trip of 6 aligned dwords covers the token, up to
// 14 literals and the offset (stream positions p .. p+19), so the common
// sequence costs one LDS latency; length-extension bytes are read one by one.
// (Byte-addressed reads cost a dependent LDS trip each, and an unaligned dword
// read a replay.)
__device__ __forceinline__ SeqIn decode_seq_in(const uint8_t *in, int32_t L, int32_t p) {
    SeqIn s;
    const uint32_t ib = (uint32_t)(uintptr_t)in & 3u;
    const uint32_t *A = (const uint32_t *)(in - ib);
    const uint32_t qa = (uint32_t)p + ib, sh = qa & 3u;
    uint32_t w[6];
#pragma unroll
    for (int j = 0; j < 6; j++) w[j] = A[(qa >> 2) + j];
    uint32_t x[5];   // bytes p .. p+19
#pragma unroll
    for (int j = 0; j < 5; j++) x[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
    const uint32_t t = x[0] & 0xFFu;
    int32_t q = p + 1;
    s.lit = (int32_t)(t >> 4);
    s.lit_win = s.lit < kRunMask;
#pragma unroll
    for (int j = 0; j < 4; j++) s.lb[j] = __builtin_amdgcn_alignbyte(x[j + 1], x[j], 1u);
    if (s.lit == kRunMask) {
        uint32_t b;
        do {
            b = in[q];
            q++;
            s.lit += (int32_t)b;
        } while (q < L - kRunMask && b == 255);
    }
    s.ls = q;
    s.in_term = q + s.lit > L - 8;
    s.off = 0;
    s.ml = 0;
    s.q2 = 0;
    s.ml_err = false;
    if (!s.in_term) {
        if (s.lit_win) {
            // offset = bytes 1+lit, 2+lit of the window (lit <= 14)
            const uint32_t k = 1u + (uint32_t)s.lit, kd = k >> 2;
            const uint32_t lo = kd == 0 ? x[0] : kd == 1 ? x[1] : kd == 2 ? x[2] : x[3];
            const uint32_t hi = kd == 0 ? x[1] : kd == 1 ? x[2] : kd == 2 ? x[3] : x[4];
            s.off = (int32_t)(__builtin_amdgcn_alignbyte(hi, lo, k & 3u) & 0xFFFFu);
        } else {
            s.off = (int32_t)lds_ld16(in + q + s.lit);
        }
        int32_t q2 = q + s.lit + 2;
        int32_t ml = (int32_t)(t & 15);
        if (ml == 15) {
            uint32_t b;
            do {
                b = in[q2];
                q2++;
                if (q2 > L - kLastLiterals) { s.ml_err = true; break; }
                ml += (int32_t)b;
            } while (b == 255);
        }
        s.ml = ml + kMinMatch;
        s.q2 = q2;
    }
    return s;
}
// Position of the token after the sequence whose token is at p, or kEnd when
// that sequence ends the chain on the input side (terminal literal run, or an
// overrun while reading match-length bytes): the input-side reads of
// lz4.c:1134-1143, 1147, 1165, 1172-1182.
__device__ __forceinline__ uint32_t next_token_w(const uint8_t *in, int32_t L, uint32_t p) {
    const SeqIn s = decode_seq_in(in, L, (int32_t)p);
    return s.in_term || s.ml_err ? kEnd : (uint32_t)s.q2;
}

// Parallel token-chain parse.  Writes the ordered token positions to the top
// of the page window (seqpos = the last `total` u16 slots below win_end) and
// returns their number.  owner: L bytes of scratch at the window's start
// (unused until the copy phases; no stamp is read once positions are written).
//
//  1. lane k walks the chain from its segment start k*S to the segment end,
//     stamping owner[p] = k+1 on every position it visits;
//  2. from its exit it keeps walking ("bridge") until it reaches a position
//     stamped by a later lane, or the end of the chain;
//  3. the true chain starts with lane 0's walk; wherever an on-chain lane's
//     bridge meets lane j's stamp, the chain continues along lane j's walk from
//     that position.  Following these hand-offs (at most 64, uniform scalar
//     code) gives every on-chain lane its entry point;
//  4. each on-chain lane re-walks entry -> hand-off position to count and then
//     write its positions.
// Steps 1-3 of parse_chain: this lane's part of the true chain is [entry, y)
// (entry = kEnd: the lane holds none of it).
__device__ __forceinline__ void chain_entries(const uint8_t *in, int32_t L, uint8_t *owner, uint32_t lane,
                                              uint32_t &entry_out, uint32_t &y_out) {
    PROF_DECL
    const uint32_t S = ((uint32_t)L + kWave - 1) / kWave;
    const uint32_t seg0 = lane * S;
    const uint32_t seg1 = min(seg0 + S, (uint32_t)L);
    for (uint32_t w = lane; w < ((uint32_t)L + 3) / 4; w += kWave) ((uint32_t *)owner)[w] = 0;
    WAVE_SYNC();
    uint32_t p = seg0;
    while (p < seg1) {
        owner[p] = (uint8_t)(lane + 1);
        p = next_token_w(in, L, p);
    }
    WAVE_SYNC();
    PROF_MARK(2);
    // Bridges in rounds of kBridgeSteps tokens, each followed by the hand-off
    // walk as far as the finished bridges reach: only the lanes still ahead on
    // the true chain keep walking.  (A lane whose speculative walk never meets
    // a later lane's stamps can bridge for hundreds of tokens; one bridge loop
    // for all lanes waited for the longest of them.)
    constexpr uint32_t kBridgeSteps = TYCHE_BRIDGE_STEPS;
    uint32_t y = p, o = 0;
    bool done = seg0 >= seg1 || y >= (uint32_t)L;
    uint32_t entry = kEnd, cur = 0, e = 0;
    for (bool fin = false; !fin;) {
        for (uint32_t it = 0; it < kBridgeSteps; it++) {
            if (!done) {
                const uint32_t ow = owner[y];
                if (ow > lane + 1) {
                    o = ow;
                    done = true;
                } else {
                    y = next_token_w(in, L, y);
                    done = y >= (uint32_t)L;
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
        if (lane < cur) done = true;                    // behind the resolved part of the chain
    }
    PROF_MARK(3);
    entry_out = entry;
    y_out = y;
}

__device__ uint32_t parse_chain(const uint8_t *in, int32_t L, uint8_t *owner, uint16_t *win_end, uint16_t *&seqpos,
                                uint32_t lane) {
    PROF_DECL
    uint32_t entry, y;
    chain_entries(in, L, owner, lane, entry, y);
    uint32_t cnt = 0;
    for (uint32_t q = entry; q < (uint32_t)L && q != y; q = next_token_w(in, L, q)) cnt++;
    const int32_t incl = wave_incl_sum((int32_t)cnt);
    uint32_t base = (uint32_t)incl - cnt;
    const uint32_t total = rdlane((uint32_t)incl, kWave - 1);
    seqpos = win_end - total;
    for (uint32_t q = entry; q < (uint32_t)L && q != y; q = next_token_w(in, L, q)) seqpos[base++] = (uint16_t)q;
    WAVE_SYNC();
    PROF_MARK(5);
    PROF_ADD(11, total);
    return total;
}


// Decodes one page held in LDS.  in: stream of L bytes (kPad zero bytes after),
// out: LDS window of W >= C + 16 bytes whose top holds the token positions.
// Returns LZ4_decompress_safe's value.
//
// The positions of batches not yet read sit above the output: every sequence
// but the last writes >= 4 bytes and takes 2 bytes of positions, so a valid
// stream's output never reaches them.  A malformed one could (its sequences
// need not fit in C), so each batch checks its write extent first and hands
// the page to the sequential decoder, which gives the same result, when it
// would overlap.
__device__ int32_t decode_page_serial(const uint8_t *in, int32_t L, uint8_t *out, int32_t C, uint32_t lane);
__device__ int32_t decode_page(const uint8_t *in, int32_t L, uint8_t *out, int32_t C, uint32_t W, uint32_t lane) {
    if (C == 0) return (L == 1 && in[0] == 0) ? 0 : -1;
    if (L <= 0) return -1;
    uint16_t *seqpos;
    const uint32_t nseq = parse_chain(in, L, out, (uint16_t *)(out + W), seqpos, lane);
    PROF_DECL
    const uint32_t grp = lane >> 4, gl = lane & 15;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    int32_t op_base = 0;
    for (uint32_t b0 = 0; b0 < nseq; b0 += kWave) {
        const uint32_t j = b0 + lane;
        const bool active = j < nseq;
        PROF_ADD(10, 1);
        // ---- decode this lane's sequence (input side)
        int32_t lit = 0, ls = 0, off = 0, ml = 0, q2 = 0;
        bool in_term = false, ml_err = false;
        if (active) {
            int32_t p = seqpos[j];
            uint32_t t = in[p];
            int32_t q = p + 1;
            lit = (int32_t)(t >> 4);
            if (lit == kRunMask) {
                uint32_t s;
                do {
                    s = in[q];
                    q++;
                    lit += (int32_t)s;
                } while (q < L - kRunMask && s == 255);
            }
            ls = q;
            in_term = q + lit > L - 8;
            if (!in_term) {
                off = (int32_t)lds_ld16(in + q + lit);
                q2 = q + lit + 2;
                ml = (int32_t)(t & 15);
                if (ml == 15) {
                    uint32_t s;
                    do {
                        s = in[q2];
                        q2++;
                        if (q2 > L - kLastLiterals) { ml_err = true; break; }
                        ml += (int32_t)s;
                    } while (s == 255);
                }
                ml += kMinMatch;
            }
        }
        // ---- output positions
        const int32_t olen = active ? (in_term ? lit : lit + ml) : 0;
        const int32_t incl = wave_incl_sum(olen);
        const int32_t o = op_base + incl - olen;   // output position of this sequence
        const int32_t d = o + lit;                 // match destination
        // ---- acceptance checks in the reference's order (lz4.c:1147-1168, 1176, 1225)
        // status: 0 ok, 1 terminal success, 2 error (rv carried)
        int32_t status = 0, rv = 0;
        if (active) {
            if (o + lit > C - kMfLimit || in_term) {
                if (ls + lit != L || o + lit > C) { status = 2; rv = -ls - 1; }
                else { status = 1; rv = o + lit; }
            } else if (off > d) {
                status = 2; rv = -(ls + lit + 2) - 1;
            } else if (ml_err) {
                status = 2; rv = -q2 - 1;
            } else if (d + ml > C - kLastLiterals) {
                status = 2; rv = -q2 - 1;
            }
        }
        const uint64_t stop = __ballot(status != 0);
        const uint32_t n_ok = stop ? (uint32_t)__builtin_ctzll(stop) : kWave;   // sequences fully applied
        int32_t final_rv = 0;
        const bool finished = stop != 0;
        if (finished) {
            final_rv = (int32_t)rdlane((uint32_t)rv, n_ok);
            if (final_rv < 0) return final_rv;                 // output is discarded on error
        }
        const bool term_lane = finished && lane == n_ok;       // terminal literal run
        if (b0 + kWave < nseq) {
            // writes reach op_base + (this batch's output) + 3 (dword literal overrun)
            const int64_t wend = (int64_t)op_base + (int64_t)rdlane((uint32_t)incl, kWave - 1) + 3;
            if (wend > (int64_t)W - 2 * (int64_t)(nseq - b0 - kWave)) return decode_page_serial(in, L, out, C, lane);
        }
        PROF_MARK(6);
        // ---- literals: short ones per lane (4 bytes per step), long ones by the whole wave
        const bool do_lit = (lane < n_ok && active) || term_lane;
        const bool short_lit = do_lit && lit <= 32 && !(TYCHE_ABLATE & 1);
        if (short_lit) {
            // whole unaligned dwords; the up-to-3-byte overrun lands in this
            // sequence's own match area (rewritten by the match phase) or past the
            // page end (slack in the window)
            for (int32_t i = 0; i < lit; i += 4) lds_st32(out + o + i, lds_ld32(in + ls + i));
        }
        uint64_t longl = __ballot(do_lit && !short_lit && !(TYCHE_ABLATE & 1));
        while (longl) {
            const uint32_t k = (uint32_t)__builtin_ctzll(longl);
            longl &= longl - 1;
            const int32_t kl = (int32_t)rdlane((uint32_t)lit, k), ko = (int32_t)rdlane((uint32_t)o, k);
            const int32_t ks = (int32_t)rdlane((uint32_t)ls, k);
            for (int32_t i = (int32_t)lane; i < kl; i += kWave) out[ko + i] = in[ks + i];
        }
        PROF_MARK(7);
        // ---- matches: frontier groups.  The first pending match's destination F
        // bounds every byte that is already final; all pending matches whose source
        // ends at or before F are independent of each other.
        const int32_t src = d - off;
        const int32_t src_end = src + min(ml, off);
        const bool applied = lane < n_ok && active;
        uint64_t pending = (TYCHE_ABLATE & 2) ? 0ull : __ballot(applied);
        const uint64_t shortm = __ballot(applied && ml <= 64);
        const uint32_t dpk = (uint32_t)d | ((uint32_t)off << 16);
        while (pending) {
            const uint32_t f = (uint32_t)__builtin_ctzll(pending);
            const int32_t F = (int32_t)rdlane((uint32_t)d, f);
            PROF_ADD(9, 1);
            if (!((shortm >> f) & 1ull)) {
                // a long match (> 64 bytes) is copied by the whole wave, on its own
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
            // up to four ready short matches, in stream order, go to the four 16-lane
            // groups; their fields are fetched with v_readlane (scalar picks, no LDS trip)
            uint64_t ready = pending & shortm & __ballot(src_end <= F);
            PROF_ADD(14, __builtin_popcountll(ready));
            uint32_t gpk = 0, gml = 0;          // this group's packed (d | off << 16) and length
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
            {
                const int32_t md = (int32_t)(gpk & 0xFFFFu), mo = (int32_t)(gpk >> 16), mm = (int32_t)gml;
                const int32_t ms = md - mo;
                for (int32_t i = (int32_t)gl; i < mm; i += 16) {
                    const int32_t si = (mo >= 16 || mo >= mm) ? i : (int32_t)mod_small((uint32_t)i, (uint32_t)mo);
                    out[md + i] = out[ms + si];
                }
            }
        }
        PROF_MARK(8);
        if (finished) return final_rv;
        op_base += (int32_t)rdlane((uint32_t)incl, kWave - 1);
    }
    return -1;   // unreachable: the chain always ends in a terminal or failing sequence
}

struct Window {
    uint32_t base;   // stream position of lane 0
    uint32_t v;      // byte base+lane (zero past the end)
};

__device__ __forceinline__ uint32_t window_byte(const Window &w, const uint8_t *in, uint32_t pos) {
    uint32_t d = pos - w.base;
    if (d < kWave) return rdlane(w.v, d);
    return rfl(in[pos]);
}

// Sequential decoder for pages too large for the parallel kernel's LDS layout
// (no parse scratch): one sequence at a time, wave-uniform parse from a 64-byte
// window, 64-byte copies.  in: stream (len L, kPad zero bytes after), out: LDS
// window of C bytes.  Returns LZ4_decompress_safe's value.
__device__ int32_t decode_page_serial(const uint8_t *in, int32_t L, uint8_t *out, int32_t C, uint32_t lane) {
    if (C == 0) return (L == 1 && rfl(in[0]) == 0) ? 0 : -1;
    if (L <= 0) return -1;
    int32_t ip = 0, op = 0;
    for (;;) {
        Window w;
        w.base = (uint32_t)ip;
        w.v = in[ip + lane];
        uint32_t token = rdlane(w.v, 0);
        int32_t lit = (int32_t)(token >> 4);
        ip++;
        if (lit == kRunMask) {
            uint32_t s;
            do {
                s = window_byte(w, in, (uint32_t)ip);
                ip++;
                lit += (int32_t)s;
            } while (ip < L - kRunMask && s == 255);
        }
        // terminal literal run, or error (lz4.c:1147-1163)
        if (op + lit > C - kMfLimit || ip + lit > L - 8) {
            if (ip + lit != L || op + lit > C) return -ip - 1;
            for (int32_t j = (int32_t)lane; j < lit; j += kWave) out[op + j] = in[ip + j];
            return op + lit;
        }
        {
            // literal bytes: straight from the window when they are all in it
            uint32_t k = (uint32_t)ip - w.base;
            if (k + (uint32_t)lit <= kWave) {
                if (lane >= k && lane < k + (uint32_t)lit) out[op + (int32_t)(lane - k)] = (uint8_t)w.v;
            } else {
                for (int32_t j = (int32_t)lane; j < lit; j += kWave) out[op + j] = in[ip + j];
            }
        }
        ip += lit;
        op += lit;
        int32_t off = (int32_t)(window_byte(w, in, (uint32_t)ip) | (window_byte(w, in, (uint32_t)ip + 1) << 8));
        ip += 2;
        if (off > op) return -ip - 1;                          // lz4.c:1168
        int32_t ml = (int32_t)(token & 15);
        if (ml == 15) {
            uint32_t s;
            do {
                s = window_byte(w, in, (uint32_t)ip);
                ip++;
                if (ip > L - kLastLiterals) return -ip - 1;    // lz4.c:1176
                ml += (int32_t)s;
            } while (s == 255);
        }
        ml += kMinMatch;
        if (op + ml > C - kLastLiterals) return -ip - 1;       // lz4.c:1225
        const int32_t src = op - off;
        if (off >= ml || off >= (int32_t)kWave) {
            // every source byte of a 64-byte step is final before the step
            for (int32_t j = (int32_t)lane; j < ml; j += kWave) out[op + j] = out[src + j];
        } else {
            // self-overlapping: byte j repeats the period-`off` pattern at src
            for (int32_t j = (int32_t)lane; j < ml; j += kWave) out[op + j] = out[src + (j % off)];
        }
        op += ml;
    }
}


__global__ __launch_bounds__(64) void lz4_decode_serial_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    const size_t page = blockIdx.x;
    PageRef p = batch_page(b, page);
    if (p.src_len > in_cap || p.dst_cap > out_cap) {
        if (lane == 0) b.results[page] = kResultTooLarge;
        return;
    }
    uint8_t *out = smem;
    uint8_t *stage = smem + ((out_cap + 15u) & ~15u);
    uint32_t head = stage_in(p.src, p.src_len, stage, lane, kWave);
    uint8_t *in = stage + head;
    WAVE_SYNC();
    in[p.src_len + lane] = 0;
    WAVE_SYNC();
    int32_t rv = decode_page_serial(in, (int32_t)p.src_len, out, (int32_t)p.dst_cap, lane);
    WAVE_SYNC();
    if (rv > 0) stage_out(p.dst, out, (uint32_t)rv, lane, kWave);
    if (lane == 0) b.results[page] = rv;
}

constexpr uint32_t kPrefetchVec = 8;   // 16-byte vectors per lane prefetched for the next page (8 KiB)

// Dynamic assignment in chunks of K <= 64 pages: chunk c is pages [c*K, c*K+K),
// the first chunk of a wave is blockIdx.x, later ones are claimed (engine.h).
// A chunk's pages whose stream length is in [lo, hi] are taken one by one
// (mask); the others belong to the other size class.
struct Claims {
    size_t base;
    uint64_t mask;
};
__device__ __forceinline__ void load_chunk(const tyche_batch_t &b, size_t c, uint32_t K, uint32_t lo, uint32_t hi,
                                           uint32_t lane, Claims &cl) {
    cl.base = c * K;
    const size_t i = cl.base + lane;
    bool take = lane < K && i < b.count;
    if (take && b.src_lengths) {
        const uint32_t l = ld_meta(b.src_lengths, i);
        take = l >= lo && l <= hi;
    }
    cl.mask = __ballot(take);
}
__device__ __forceinline__ size_t next_chunked(const tyche_batch_t &b, unsigned *ctr, uint32_t K, uint32_t lo,
                                               uint32_t hi, uint32_t lane, Claims &cl) {
    while (cl.mask == 0) {
        if (cl.base >= b.count) return b.count;
        load_chunk(b, claim_page(ctr, lane), K, lo, hi, lane, cl);
    }
    const uint32_t j = (uint32_t)__builtin_ctzll(cl.mask);
    cl.mask &= cl.mask - 1ull;
    return cl.base + j;
}

// First page at or after i (step stride) whose stream length is in [lo, hi].
__device__ __forceinline__ size_t next_in_class(const tyche_batch_t &b, size_t i, size_t stride, uint32_t lo,
                                                uint32_t hi) {
    if (!b.src_lengths) return i;
    for (; i < b.count; i += stride) {
        const uint32_t l = ld_meta(b.src_lengths, i);
        if (l >= lo && l <= hi) break;
    }
    return i;
}

// One wave per page, looping over pages; the next page's stream is prefetched
// into registers while the current one is decoded.  Only pages whose stream
// length lies in [cls_lo, cls_hi] are taken (launch_lz4_decode's size classes).
__global__ __launch_bounds__(64) void lz4_decode_wave_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap,
                                                             uint32_t off_in, uint32_t cls_lo, uint32_t cls_hi,
                                                             unsigned *ctr, uint32_t chunk) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint8_t *out = smem;                 // page window [0, off_in): output, parse stamps, token positions
    uint8_t *stage = smem + off_in;
    const size_t stride = gridDim.x;

    size_t page;
    Claims cl;
    if (ctr) {
        load_chunk(b, blockIdx.x, chunk, cls_lo, cls_hi, lane, cl);
        page = next_chunked(b, ctr, chunk, cls_lo, cls_hi, lane, cl);
    } else {
        page = next_in_class(b, blockIdx.x, stride, cls_lo, cls_hi);
    }
    if (page >= b.count) return;
    PageRef p = batch_page(b, page);
    uint32_t head = stage_in(p.src, p.src_len <= in_cap ? p.src_len : 0, stage, lane, kWave);
    for (;;) {
        PROF_DECL
        // dynamic assignment (engine.h): single pages for a launch that takes
        // (nearly) every page, chunks for the long-stream class
        const size_t next = ctr ? next_chunked(b, ctr, chunk, cls_lo, cls_hi, lane, cl)
                                : next_in_class(b, page + stride, stride, cls_lo, cls_hi);
        // ---- prefetch the next page's stream (first 8 KiB) into registers
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
        // ---- current page
        int32_t rv;
        if (p.src_len > in_cap || p.dst_cap > out_cap) {
            rv = kResultTooLarge;
        } else {
            uint8_t *in = stage + head;
            WAVE_SYNC();
            in[p.src_len + lane] = 0;                           // kPad zero bytes past the end
            WAVE_SYNC();
            PROF_MARK(1);
            PROF_ADD(0, 1);
            rv = decode_page(in, (int32_t)p.src_len, out, (int32_t)p.dst_cap, off_in, lane);
            WAVE_SYNC();
            PROF_MARK(13);
            if (rv > 0 && !(TYCHE_ABLATE & 4)) stage_out(p.dst, out, (uint32_t)rv, lane, kWave);
        }
        if (lane == 0) b.results[page] = rv;
        if (next >= b.count) break;
        // ---- install the prefetched stream (and load any remainder past 8 KiB)
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
        PROF_MARK(12);
    }
}

// ---------------------------------------------------------------------------
// Small-batch decoder (restore latency): one workgroup of kJumpThreads per page,
// matches resolved by pointer jumping instead of dependency rounds.
//
// The page is rebuilt as 16-bit cells in LDS, one per output byte: a literal
// byte is final (0x8000 | byte); a match byte holds the position it copies
// (d - off + j, or d - off + j mod off for a self-overlapping match, so a cell
// always points below its own match).  Every pointer leads down a chain that
// ends at a literal, so "cell = cells[cell]" over all unresolved cells, repeated
// until none is left, yields the forward byte-copy result of lz4.c:1209-1236 in
// log2(chain depth) rounds (8 on the bench pages) -- the wave decoder needs ~294
// dependent frontier rounds per 16 KiB page for the same copies.  Cells are
// independent of fill order, so all runs are written in parallel.
//
// Wave 0 parses the token chain (chain_entries, as parse_chain) and walks its
// lane's part of it once, recording every sequence as an item (token position,
// output offset within the lane's part; jump_walk).  Then every thread takes
// sequences of its own: decodes it again, runs the reference's acceptance
// checks (lz4.c:1147-1168, 1176, 1225) at its absolute position and
// atomicMin's the number of a failing one; the first failing sequence in
// stream order gives the exact -(consumed)-1 return, and the sequences before
// it write their literals and match start markers (a marker run is filled by
// jump_scan; runs longer than kJumpLong go to a list the whole workgroup
// fills).  Then all waves jump, pack cells to bytes and store.  Pages whose
// lane parts overflow the items take jump_front: the same checks and fills as
// a second per-lane walk.
// 512 threads per page, 1,024 when the batch has no more pages than the device has CUs
// (one page per CU: the parallel phases take half the time; 512 fits two pages per CU)
constexpr int32_t kJumpLong = 16;

constexpr uint32_t kLitFlag = 0x8000u;
// LDS bytes before the cells: the workgroup's shared words (8) and jump_scan's
// chunk keys (one per 64 cells, pages <= 32 KiB)
constexpr uint32_t kJumpHdr = 32 + 4 * 512 + 4 * 3 * 64;   // + JumpLanes

// cells [o + i0, o + n) step `step` of a literal run read from in[ls..]
__device__ __forceinline__ void fill_lit(uint16_t *cells, const uint8_t *in, int32_t o, int32_t ls, int32_t n,
                                         int32_t i0, int32_t step) {
    for (int32_t i = i0; i < n; i += step) cells[o + i] = (uint16_t)(kLitFlag | in[ls + i]);
}
// cells of a match of ml bytes at d from offset off
__device__ __forceinline__ void fill_match(uint16_t *cells, int32_t d, int32_t off, int32_t ml, int32_t i0,
                                           int32_t step) {
    const int32_t src = d - off;
    if (off == 0) {
        // the reference copies bytes it never wrote: only its return value is a parity target
        for (int32_t i = i0; i < ml; i += step) cells[d + i] = (uint16_t)kLitFlag;
    } else if (off >= ml) {
        for (int32_t i = i0; i < ml; i += step) cells[d + i] = (uint16_t)(src + i);
    } else {
        for (int32_t i = i0; i < ml; i += step) cells[d + i] = (uint16_t)(src + (int32_t)mod_small((uint32_t)i, (uint32_t)off));
    }
}
// a long run for the workgroup: x = dst | len << 16, y = ls | 1 << 31 (literals) or off (match)
__device__ __forceinline__ void fill_item(uint16_t *cells, const uint8_t *in, uint2 it, int32_t i0, int32_t step) {
    const int32_t dst = (int32_t)(it.x & 0xFFFFu), n = (int32_t)(it.x >> 16);
    if (it.y >> 31) fill_lit(cells, in, dst, (int32_t)(it.y & 0x7FFFFFFFu), n, i0, step);
    else fill_match(cells, dst, (int32_t)it.y, n, i0, step);
}

// Wave 0 alone: parse, checks and fills of one page (in: L bytes + kPad zeros,
// cells: >= max(C, (L + 4) / 2) cells) -- jump_walk's fallback for pages whose
// lane parts do not fit its items.  Returns LZ4_decompress_safe's value.
__device__ int32_t jump_front(const uint8_t *in, int32_t L, uint16_t *cells, int32_t C, uint32_t lane, uint2 *list,
                              uint32_t list_cap, uint32_t *nlist, uint2 *lits, uint32_t lits_cap, uint32_t *nseq) {
    if (C == 0) return (L == 1 && in[0] == 0) ? 0 : -1;
    if (L <= 0) return -1;
    uint32_t entry, y;
    chain_entries(in, L, (uint8_t *)cells, lane, entry, y);   // owner stamps in the cells (dead after this)
    PROF_DECL
    {
        // empty cells (0) are match bytes after their run's start marker (jump_scan)
        const uint32_t nv = (((uint32_t)C + 63u) & ~63u) / 8u;
        u32x4 *c4 = (u32x4 *)cells;
        const u32x4 z = {0u, 0u, 0u, 0u};
        for (uint32_t v = lane; v < nv; v += kWave) c4[v] = z;
    }
    // pass 1: output bytes of this lane's part of the chain
    int32_t olen = 0, cnt = 0;
    for (uint32_t q = entry; q < (uint32_t)L && q != y;) {
        const SeqIn s = decode_seq_in(in, L, (int32_t)q);
        cnt++;
        if (s.in_term) { olen += s.lit; break; }
        if (s.ml_err) break;
        olen += s.lit + s.ml;
        q = (uint32_t)s.q2;
    }
    WAVE_SYNC();
    PROF_MARK(4);
    const int32_t incl = wave_incl_sum(olen);
    int32_t o = incl - olen;
    const int32_t cincl = wave_incl_sum(cnt);
    uint32_t k = (uint32_t)(cincl - cnt);   // this lane's first sequence number
    if (nseq && lane == kWave - 1) *nseq = (uint32_t)cincl;
    // pass 2: checks in the reference's order, then the fills
    int32_t status = 0, rv = 0;   // 1 terminal success, 2 error
    for (uint32_t q = entry; q < (uint32_t)L && q != y;) {
        const SeqIn s = decode_seq_in(in, L, (int32_t)q);
        const int32_t d = o + s.lit;
        if (o + s.lit > C - kMfLimit || s.in_term) {
            if (s.ls + s.lit != L || o + s.lit > C) { status = 2; rv = -s.ls - 1; }
            else { status = 1; rv = o + s.lit; }
        } else if (s.off > d) {
            status = 2; rv = -(s.ls + s.lit + 2) - 1;
        } else if (s.ml_err) {
            status = 2; rv = -s.q2 - 1;
        } else if (d + s.ml > C - kLastLiterals) {
            status = 2; rv = -s.q2 - 1;
        }
        if (status == 2) break;
        // literal runs: short ones as this sequence's item for the workgroup (lits[k]), long
        // ones on the run list; per lane only when lits[] is full
        const bool short_lit = s.lit <= kJumpLong;
        if (lits && k < lits_cap)
            lits[k] = short_lit ? make_uint2((uint32_t)o | ((uint32_t)s.lit << 16), (uint32_t)s.ls) : make_uint2(0u, 0u);
        if (!short_lit) {
            const uint32_t kl = atomicAdd(nlist, 1u);
            const uint2 it = make_uint2((uint32_t)o | ((uint32_t)s.lit << 16), (uint32_t)s.ls | 0x80000000u);
            if (kl < list_cap) list[kl] = it;
            else fill_item(cells, in, it, 0, 1);
        } else if (s.lit > 0 && k >= lits_cap) {
            // literal bytes straight from the decode window (or, for 15-16 of them, aligned dwords)
            uint32_t w[4];
            if (s.lit_win) {
#pragma unroll
                for (int32_t j = 0; j < 4; j++) w[j] = s.lb[j];
            } else {
                const uint32_t ib = (uint32_t)(uintptr_t)in & 3u, qa = (uint32_t)s.ls + ib;
                const uint32_t *A = (const uint32_t *)(in - ib);
                uint32_t a[5];
#pragma unroll
                for (int32_t j = 0; j < 5; j++) a[j] = A[(qa >> 2) + j];
#pragma unroll
                for (int32_t j = 0; j < 4; j++) w[j] = __builtin_amdgcn_alignbyte(a[j + 1], a[j], qa & 3u);
            }
#pragma unroll
            for (int32_t i = 0; i < 16; i++)
                if (i < s.lit) cells[o + i] = (uint16_t)(kLitFlag | ((w[i >> 2] >> (8 * (i & 3))) & 0xFFu));
        }
        if (status == 1) break;
        if (s.off != 0) {
            cells[d] = (uint16_t)s.off;   // the run's start marker (off <= d < 2^15); jump_scan fills the rest
        } else if (s.ml > kJumpLong) {
            const uint32_t k = atomicAdd(nlist, 1u);
            const uint2 it = make_uint2((uint32_t)d | ((uint32_t)s.ml << 16), 0u);
            if (k < list_cap) list[k] = it;
            else fill_item(cells, in, it, 0, 1);
        } else {
            fill_match(cells, d, 0, s.ml, 0, 1);
        }
        o = d + s.ml;
        q = (uint32_t)s.q2;
        k++;
    }
    WAVE_SYNC();
    PROF_MARK(5);
    const uint64_t stop = __ballot(status != 0);
    if (stop == 0) return -1;   // unreachable: the chain always ends in a terminal or failing sequence
    return (int32_t)rdlane((uint32_t)rv, (uint32_t)__builtin_ctzll(stop));
}

// Literal run of sequence s at output o: short ones from the decode window (or
// aligned dwords), long ones onto the workgroup's run list.
__device__ __forceinline__ void put_literals(uint16_t *cells, const uint8_t *in, const SeqIn &s, int32_t o, uint2 *list,
                                             uint32_t list_cap, uint32_t *nlist) {
    if (s.lit > kJumpLong) {
        const uint32_t kl = atomicAdd(nlist, 1u);
        const uint2 it = make_uint2((uint32_t)o | ((uint32_t)s.lit << 16), (uint32_t)s.ls | 0x80000000u);
        if (kl < list_cap) list[kl] = it;
        else fill_item(cells, in, it, 0, 1);
        return;
    }
    if (s.lit <= 0) return;
    uint32_t w[4];
    if (s.lit_win) {
#pragma unroll
        for (int32_t j = 0; j < 4; j++) w[j] = s.lb[j];
    } else {
        const uint32_t ib = (uint32_t)(uintptr_t)in & 3u, qa = (uint32_t)s.ls + ib;
        const uint32_t *A = (const uint32_t *)(in - ib);
        uint32_t a[5];
#pragma unroll
        for (int32_t j = 0; j < 5; j++) a[j] = A[(qa >> 2) + j];
#pragma unroll
        for (int32_t j = 0; j < 4; j++) w[j] = __builtin_amdgcn_alignbyte(a[j + 1], a[j], qa & 3u);
    }
#pragma unroll
    for (int32_t i = 0; i < 16; i++)
        if (i < s.lit) cells[o + i] = (uint16_t)(kLitFlag | ((w[i >> 2] >> (8 * (i & 3))) & 0xFFu));
}

// The workgroup's view of wave 0's walk: items[i * 64 + l] = token position of
// lane l's i-th sequence | its output offset within the lane's part << 16, and
// per lane the sequence count, the output base and the first sequence number.
struct JumpLanes {
    uint32_t cnt[kWave], base_o[kWave], base_k[kWave];   // column items, output base, first sequence number
};
constexpr int32_t kJumpPending = INT32_MIN + 2;   // rv decided by the workgroup's checks
constexpr uint32_t kJumpOvf = 512;                // overflow items (sequences past a lane's rows)

// Wave 0: chain entries, zeroed cells, one walk per lane recording its
// sequences (items, rows per lane), the lanes' prefix sums.  Returns
// kJumpPending, or the final value when no check is left to run (empty page),
// or jump_front's value when a lane's part does not fit the items (> rows
// sequences or > 64 KiB of output): the two-walk path below.
__device__ int32_t jump_walk(const uint8_t *in, int32_t L, uint16_t *cells, int32_t C, uint32_t lane, uint32_t *items,
                             uint32_t rows, uint2 *ovf, uint32_t ovf_cap, uint32_t *novf, JumpLanes *lanes, uint2 *list,
                             uint32_t list_cap, uint32_t *nlist) {
    if (C == 0) return (L == 1 && in[0] == 0) ? 0 : -1;
    if (L <= 0) return -1;
    // chain_entries' speculative walks and bridges, recording every token a lane
    // visits as an item (position | output bytes before it in the lane's walk,
    // mod 2^16): the true chain enters a lane's walk at a position that lane
    // stamped, so its part of the chain is a suffix of its items -- no second walk
    uint8_t *owner = (uint8_t *)cells;
    const uint32_t S = ((uint32_t)L + kWave - 1) / kWave;
    const uint32_t seg0 = lane * S;
    const uint32_t seg1 = min(seg0 + S, (uint32_t)L);
    for (uint32_t w = lane; w < ((uint32_t)L + 3) / 4; w += kWave) ((uint32_t *)owner)[w] = 0;
    WAVE_SYNC();
    uint32_t cum = 0, cnt = 0, q_over = 0, c_over = 0;
    auto record = [&](uint32_t q, const SeqIn &sq) {
        if (cnt < rows) items[cnt * kWave + lane] = q | (cum << 16);
        if (cnt == rows) {
            q_over = q;
            c_over = cum;
        }
        cnt++;
        cum += (uint32_t)(sq.in_term ? sq.lit : sq.lit + sq.ml);
    };
    uint32_t p = seg0;
    while (p < seg1) {
        owner[p] = (uint8_t)(lane + 1);
        const SeqIn sq = decode_seq_in(in, L, (int32_t)p);
        record(p, sq);
        p = sq.in_term || sq.ml_err ? kEnd : (uint32_t)sq.q2;
    }
    WAVE_SYNC();
    PROF_DECL
    constexpr uint32_t kBridgeSteps = TYCHE_BRIDGE_STEPS;
    uint32_t y = p, o = 0;
    bool done = seg0 >= seg1 || y >= (uint32_t)L;
    uint32_t entry = kEnd, cur = 0, e = 0;
    for (bool fin = false; !fin;) {
        for (uint32_t it = 0; it < kBridgeSteps; it++) {
            if (!done) {
                const uint32_t ow = owner[y];
                if (ow > lane + 1) {
                    o = ow;
                    done = true;
                } else {
                    const SeqIn sq = decode_seq_in(in, L, (int32_t)y);
                    record(y, sq);
                    y = sq.in_term || sq.ml_err ? kEnd : (uint32_t)sq.q2;
                    done = y >= (uint32_t)L;
                }
            }
        }
        for (;;) {
            if (lane == cur) entry = e;
            if (!rdlane((uint32_t)done, cur)) break;
            e = rdlane(y, cur);
            const uint32_t nx = rdlane(o, cur);
            if (nx == 0) { fin = true; break; }
            cur = nx - 1;
        }
        if (lane < cur) done = true;
    }
    WAVE_SYNC();
    PROF_MARK(3);
    {
        const uint32_t nv = (((uint32_t)C + 63u) & ~63u) / 8u;
        u32x4 *c4 = (u32x4 *)cells;
        const u32x4 z = {0u, 0u, 0u, 0u};
        for (uint32_t v = lane; v < nv; v += kWave) c4[v] = z;
    }
    // this lane's part: items [first, cnt), found by binary search (positions grow)
    const bool on = entry != kEnd;
    const uint32_t nrec = min(cnt, rows);
    uint32_t first = 0;
    bool bad = false;
    if (on) {
        uint32_t lo = 0, hi = nrec;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((items[mid * kWave + lane] & 0xFFFFu) < entry) lo = mid + 1;
            else hi = mid;
        }
        first = lo;
        bad = first >= nrec || (items[first * kWave + lane] & 0xFFFFu) != entry || cum >= 0x10000u;
    }
    uint32_t cum_entry = 0;
    if (on && !bad) cum_entry = items[first * kWave + lane] >> 16;
    const uint32_t extra = on && cnt > rows ? cnt - rows : 0u;
    const uint32_t xi = (uint32_t)wave_incl_sum((int32_t)extra);
    const uint32_t nx = rdlane(xi, kWave - 1);
    if (__ballot(bad) || nx > ovf_cap)
        return jump_front(in, L, cells, C, lane, list, list_cap, nlist, nullptr, 0u, nullptr);
    const uint32_t ncol = on ? nrec - first : 0u;
    for (uint32_t k = 0; k < ncol; k++) {
        const uint32_t it = items[(first + k) * kWave + lane];
        items[k * kWave + lane] = (it & 0xFFFFu) | (((it >> 16) - cum_entry) << 16);
    }
    if (lane == 0) *novf = nx;
    if (extra) {
        uint32_t at = xi - extra, q = q_over, oc = c_over;
        for (uint32_t i = rows - first; i < cnt - first; i++) {
            const SeqIn sq = decode_seq_in(in, L, (int32_t)q);
            ovf[at++] = make_uint2(q | ((oc - cum_entry) << 16), lane | (i << 8));
            oc += (uint32_t)(sq.in_term ? sq.lit : sq.lit + sq.ml);
            q = (uint32_t)sq.q2;
        }
    }
    const uint32_t part = on ? cnt - first : 0u, olen = on ? cum - cum_entry : 0u;
    const int32_t oi = wave_incl_sum((int32_t)olen), ci = wave_incl_sum((int32_t)part);
    lanes->cnt[lane] = ncol;
    lanes->base_o[lane] = (uint32_t)oi - olen;
    lanes->base_k[lane] = (uint32_t)ci - part;
    PROF_MARK(4);
    return kJumpPending;
}

// Item j of the workgroup's loops: lane l's i-th sequence (column items first, then the overflow)
__device__ __forceinline__ bool jump_item(const uint32_t *items, const uint2 *ovf, uint32_t rows, uint32_t j,
                                          const JumpLanes *lanes, uint32_t &l, uint32_t &i, uint32_t &it) {
    if (j < rows * kWave) {
        l = j & (kWave - 1);
        i = j / kWave;
        if (i >= lanes->cnt[l]) return false;   // cnt: the lane's column items
        it = items[j];
        return true;
    }
    const uint2 x = ovf[j - rows * kWave];
    l = x.y & 0xFFu;
    i = x.y >> 8;
    it = x.x;
    return true;
}

// The reference's acceptance checks for one sequence at output position o
// (lz4.c:1147-1168, 1176, 1225): 0 ok, 1 terminal success, 2 error; rv the value.
__device__ __forceinline__ int32_t seq_check(const SeqIn &s, int32_t o, int32_t L, int32_t C, int32_t &rv) {
    const int32_t d = o + s.lit;
    if (o + s.lit > C - kMfLimit || s.in_term) {
        if (s.ls + s.lit != L || o + s.lit > C) { rv = -s.ls - 1; return 2; }
        rv = o + s.lit;
        return 1;
    }
    if (s.off > d) { rv = -(s.ls + s.lit + 2) - 1; return 2; }
    if (s.ml_err) { rv = -s.q2 - 1; return 2; }
    if (d + s.ml > C - kLastLiterals) { rv = -s.q2 - 1; return 2; }
    return 0;
}

// Match cells from their start markers: a cell is a literal (0x8000 | byte), a
// run start (its offset, 1..0x7FFF) or empty (0: a later byte of the run that
// started at the nearest marker to its left).  Chunks of 64 cells: (A) each
// chunk's last marker as key = position << 16 | offset, (B) an inclusive
// max-scan of the keys (positions grow, so the max is the nearest marker to the
// left), (C) each chunk rewrites its cells with the carried-in run: byte d + j of
// a run with offset off points at d - off + (j mod off).
template <uint32_t kT>
__device__ __forceinline__ void jump_scan(uint16_t *cells, uint32_t n64, uint32_t *keys, uint32_t tid) {
    u32x4 *c4 = (u32x4 *)cells;
    const uint32_t nch = n64 / 64u;
    for (uint32_t c = tid; c < nch; c += kT) {
        uint32_t key = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const u32x4 v = c4[8u * c + j];
#pragma unroll
            for (uint32_t h = 0; h < 8; h++) {
                const uint32_t x = (v[h >> 1] >> (16u * (h & 1u))) & 0xFFFFu;
                if (x != 0 && !(x & kLitFlag)) key = ((64u * c + 8u * j + h) << 16) | x;
            }
        }
        keys[c] = key;
    }
    __syncthreads();
    if (tid < kWave) {
        int32_t carry = 0;
        for (uint32_t base = 0; base < nch; base += kWave) {
            const uint32_t c = base + tid;
            int32_t m = wave_incl_max(c < nch ? (int32_t)keys[c] : 0);
            m = max(m, carry);
            if (c < nch) keys[c] = (uint32_t)m;
            carry = (int32_t)rdlane((uint32_t)m, kWave - 1);
        }
    }
    __syncthreads();
    for (uint32_t c = tid; c < nch; c += kT) {
        const uint32_t key = c ? keys[c - 1] : 0u;
        uint32_t d = key >> 16, off = key & 0xFFFFu;
        uint32_t k = off ? mod_small(64u * c - d, off) : 0u;
        for (uint32_t j = 0; j < 8; j++) {
            u32x4 v = c4[8u * c + j];
#pragma unroll
            for (uint32_t h = 0; h < 8; h++) {
                const uint32_t b = 64u * c + 8u * j + h;
                const uint32_t sh = 16u * (h & 1u);
                const uint32_t x = (v[h >> 1] >> sh) & 0xFFFFu;
                const bool lit = (x & kLitFlag) != 0, start = !lit && x != 0;
                if (start) {
                    d = b;
                    off = x;
                    k = 0;
                }
                const uint32_t y = lit ? x : d - off + k;
                if (!lit) {
                    k++;
                    if (k == off) k = 0;
                }
                v[h >> 1] = (v[h >> 1] & ~(0xFFFFu << sh)) | (y << sh);
            }
            c4[8u * c + j] = v;
        }
    }
}

// one round's update of 2 cells packed in a dword; `open` gathers the cells still unresolved afterwards.
// kRacy: the barrier-free rounds of the single-page decoder, where other threads rewrite the cells
// being read -- volatile loads, so that no compiler may cache, merge or move them (the hardware
// returns the old or the new value, and the algorithm accepts either: ADVICE r05)
template <bool kRacy = false>
__device__ __forceinline__ uint32_t jump_pair(const uint16_t *cells, uint32_t w, uint32_t &open) {
    uint32_t lo = w & 0xFFFFu, hi = w >> 16;
    if constexpr (kRacy) {
        const volatile uint16_t *vc = cells;
        if (!(lo & kLitFlag)) lo = vc[lo];
        if (!(hi & kLitFlag)) hi = vc[hi];
    } else {
        if (!(lo & kLitFlag)) lo = cells[lo];
        if (!(hi & kLitFlag)) hi = cells[hi];
    }
    open |= ~(lo & hi) & kLitFlag;
    return lo | (hi << 16);
}

template <uint32_t kJumpThreads>
__global__ __launch_bounds__(kJumpThreads) void lz4_decode_jump_kernel(tyche_batch_t b, uint32_t in_cap,
                                                                       uint32_t out_cap, uint32_t cells_bytes,
                                                                       uint32_t list_cap, uint32_t rows,
                                                                       unsigned *ctr) {
    // no static __shared__: prepare_launch raises the dynamic limit to the whole 160 KiB
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
    uint32_t *shared_words = (uint32_t *)smem;   // [0] rv, [1] long-run count, [2] claimed page, [3..5] round flags, [6] overflow items, [7] first failing sequence, [8..519] chunk keys, then JumpLanes
    int32_t &s_rv = *(int32_t *)&shared_words[0];
    uint32_t &s_nlist = shared_words[1];
    uint32_t &s_page = shared_words[2];
    uint16_t *cells = (uint16_t *)(smem + kJumpHdr);
    uint2 *list = (uint2 *)(smem + kJumpHdr + cells_bytes);
    uint32_t *items = (uint32_t *)(list + list_cap);
    uint2 *ovf = (uint2 *)(items + kWave * rows);
    uint8_t *stage = smem + kJumpHdr + cells_bytes + 8u * list_cap + 4u * kWave * rows + 8u * kJumpOvf;
    JumpLanes *lanes = (JumpLanes *)(shared_words + 8 + 512);
    size_t page = blockIdx.x;
    while (page < b.count) {
        PROF_DECL
        PROF_ADD(0, 1);
        const PageRef p = batch_page(b, page);
        const bool fits = p.src_len <= in_cap && p.dst_cap <= out_cap;
        const uint32_t head = stage_in(p.src, fits ? p.src_len : 0u, stage, tid, kJumpThreads);
        if (tid == 0) {
            s_nlist = 0;
            shared_words[3] = 0;   // round 0's flag
        }
        __syncthreads();
        uint8_t *in = stage + head;
        if (fits && tid < kPad) in[p.src_len + tid] = 0;   // kPad zero bytes past the end
        __syncthreads();
        PROF_MARK(1);
        const int32_t L = (int32_t)p.src_len, C = (int32_t)p.dst_cap;
        if (wave == 0) {
            const int32_t r = fits ? jump_walk(in, L, cells, C, lane, items, rows, ovf, kJumpOvf, &shared_words[6], lanes,
                                               list, list_cap, &s_nlist)
                                   : kResultTooLarge;
            if (lane == 0) {
                s_rv = r;
                shared_words[7] = 0xFFFFFFFFu;   // first failing sequence
            }
        }
        __syncthreads();
        PROF_MARK(5);
        if (s_rv == kJumpPending) {
            // every sequence checked at once; the first failing one in stream order decides
            const uint32_t nitems = rows * kWave + shared_words[6];
            for (uint32_t j = tid; j < nitems; j += kJumpThreads) {
                uint32_t l, i, it;
                if (!jump_item(items, ovf, rows, j, lanes, l, i, it)) continue;
                const SeqIn sq = decode_seq_in(in, L, (int32_t)(it & 0xFFFFu));
                int32_t r;
                if (seq_check(sq, (int32_t)(lanes->base_o[l] + (it >> 16)), L, C, r))
                    atomicMin(&shared_words[7], lanes->base_k[l] + i);
            }
            __syncthreads();
            const uint32_t first = shared_words[7];
            if (first == 0xFFFFFFFFu && tid == 0) s_rv = -1;   // unreachable: the chain ends in a stop
            // fills of every sequence up to it (and its verdict)
            for (uint32_t j = tid; j < nitems; j += kJumpThreads) {
                uint32_t l, i, it;
                if (!jump_item(items, ovf, rows, j, lanes, l, i, it) || lanes->base_k[l] + i > first) continue;
                const SeqIn sq = decode_seq_in(in, L, (int32_t)(it & 0xFFFFu));
                const int32_t o = (int32_t)(lanes->base_o[l] + (it >> 16));
                int32_t r;
                const int32_t st = seq_check(sq, o, L, C, r);
                if (lanes->base_k[l] + i == first) s_rv = r;
                if (st == 2) continue;
                put_literals(cells, in, sq, o, list, list_cap, &s_nlist);
                if (st == 1) continue;
                const int32_t d = o + sq.lit;
                if (sq.off != 0) {
                    cells[d] = (uint16_t)sq.off;   // the run's start marker; jump_scan fills the rest
                } else if (sq.ml > kJumpLong) {
                    const uint32_t kl = atomicAdd(&s_nlist, 1u);
                    const uint2 li = make_uint2((uint32_t)d | ((uint32_t)sq.ml << 16), 0u);
                    if (kl < list_cap) list[kl] = li;
                    else fill_item(cells, in, li, 0, 1);
                } else {
                    fill_match(cells, d, 0, sq.ml, 0, 1);
                }
            }
            __syncthreads();
        }
        const int32_t rv = s_rv;
        if (rv > 0) {
            // long runs, then the tail of the last 64-cell chunk marked final
            const uint32_t nl = min(s_nlist, list_cap);
            for (uint32_t k = 0; k < nl; k++) fill_item(cells, in, list[k], (int32_t)tid, (int32_t)kJumpThreads);
            const uint32_t n64 = ((uint32_t)rv + 63u) & ~63u;
            if (tid < n64 - (uint32_t)rv) cells[(uint32_t)rv + tid] = (uint16_t)kLitFlag;
            __syncthreads();
            PROF_ADD(10, nl);
            PROF_MARK(6);
            jump_scan<kJumpThreads>(cells, n64, shared_words + 8, tid);
            __syncthreads();
            PROF_MARK(7);
            // pointer jumping, 8 cells per group
            u32x4 *c4 = (u32x4 *)cells;
            const uint32_t ng = n64 / 8u;
            // round r's verdict: OR of every thread's open cells in flag[r % 3], which thread 0
            // clears one round ahead (its last readers passed a barrier since)
            uint32_t *flag = shared_words + 3;
            for (uint32_t r = 0;; r++) {
                if (tid == 0) flag[(r + 1) % 3] = 0;
                uint32_t open = 0;
                // two groups per step: 16 independent gathers in flight
                for (uint32_t g = tid; g < ng; g += 2 * kJumpThreads) {
                    const uint32_t g2 = g + kJumpThreads;
                    const u32x4 fin = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
                    u32x4 v = c4[g], u = g2 < ng ? c4[g2] : fin;
                    const bool dv = ((v.x & v.y & v.z & v.w) & 0x80008000u) != 0x80008000u;
                    const bool du = ((u.x & u.y & u.z & u.w) & 0x80008000u) != 0x80008000u;
                    if (dv) {
                        v.x = jump_pair(cells, v.x, open);
                        v.y = jump_pair(cells, v.y, open);
                        v.z = jump_pair(cells, v.z, open);
                        v.w = jump_pair(cells, v.w, open);
                    }
                    if (du) {
                        u.x = jump_pair(cells, u.x, open);
                        u.y = jump_pair(cells, u.y, open);
                        u.z = jump_pair(cells, u.z, open);
                        u.w = jump_pair(cells, u.w, open);
                    }
                    if (dv) c4[g] = v;
                    if (du) c4[g2] = u;
                }
                if (open) atomicOr(&flag[r % 3], 1u);
                __syncthreads();
                PROF_ADD(9, 1);
                if (flag[r % 3] == 0) break;
            }
            PROF_MARK(8);
            // cells -> bytes, 16 per thread
            uint8_t *dst = p.dst;
            const bool al = ((uintptr_t)dst & 15u) == 0;
            for (uint32_t g = tid; g < n64 / 16u; g += kJumpThreads) {
                const u32x4 a = c4[2 * g], c = c4[2 * g + 1];
                u32x4 o;
                o.x = __builtin_amdgcn_perm(a.y, a.x, 0x06040200u);
                o.y = __builtin_amdgcn_perm(a.w, a.z, 0x06040200u);
                o.z = __builtin_amdgcn_perm(c.y, c.x, 0x06040200u);
                o.w = __builtin_amdgcn_perm(c.w, c.z, 0x06040200u);
                const uint32_t base = 16u * g;
                if (al && base + 16u <= (uint32_t)rv) {
                    __builtin_nontemporal_store(o, (u32x4 *)(dst + base));
                } else {
                    const uint32_t n = min(16u, (uint32_t)rv - base);
                    for (uint32_t j = 0; j < n; j++) dst[base + j] = (uint8_t)(o[j >> 2] >> (8u * (j & 3u)));
                }
            }
        }
        PROF_MARK(12);
        if (tid == 0) b.results[page] = rv;
        if (ctr) {
            if (tid == 0) s_page = atomicAdd(ctr, 1u) + gridDim.x;
            __syncthreads();
            page = s_page;
        } else {
            page += gridDim.x;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Round 5: the single-page decoder (the restore path's latency).  One 1,024-thread
// workgroup per page; the jump kernel's cells and pointer jumping, with its two
// slowest phases replaced (one 16 KiB page alone on a CU: token chain walked by one
// wave while the others wait, then a run-start scan):
//
//  1. token chain by pointer doubling over stream positions.  Every position q
//     gets J(q) = where the token after a token at q would start (next_token_w;
//     a terminal or malformed token and the stream's end map to the sink L).
//     Position 0 is marked; in each round every marked q marks J(q), then
//     J <- J o J, so after k rounds every position at chain distance < 2^k from 0
//     is marked; the rounds stop when J(0) is the sink.  Marks only grow and only
//     land on chain positions, so a round needs no order among its threads.  The
//     marked positions in position order are the token list (a block prefix sum
//     of per-thread counts places them).  Every position costs the same: no walk
//     can start out of phase (segment walks with stamps, tried first, stay out of
//     phase through runs of 3-byte sequences and their bridges ran 100+ tokens);
//  2. one block scan of (marked positions, their output lengths -- kept with J) per
//     thread gives each token its number and output offset; each thread decodes its
//     own tokens once (solo_seq), runs the reference's checks at those offsets
//     (seq_check; atomicMin of the first failing token gives the exact
//     -(consumed)-1) and writes a record per token (output offset, literal count,
//     literal start, match offset) and, at slot ceil(o / 4), its number into the
//     covering table, whose running maximum then names the token that holds the
//     first cell of every 4-cell group;
//  3. cells, a 4-cell group per lane and step: literals final (0x8000 | byte),
//     match bytes pointing at the byte they copy (d - off + ((c - d) mod off));
//  4. pointer jumping without barriers, each thread's 16 cells in registers until
//     they are all final (lock-step rounds for a thread that runs async_rounds of
//     them), then packed to bytes and stored.

constexpr uint32_t kSoloNpt = 8;      // positions per thread chunk
constexpr uint32_t kSoloChunks = 3;   // chunks per thread: streams up to 3 * 8 * 1,024 - 1 bytes
constexpr uint32_t kSoloGroups = 4;   // 8-cell groups per thread in the jump rounds: pages up to 32 KiB
constexpr long kSoloAsyncRounds = 64;   // barrier-free jump rounds per thread before lock-step ones
// next_token_w for the token at p = base + u, and the token's output length (lit + ml, or lit for a
// terminal literal run): the reads of lz4.c:1134-1143, 1165, 1172-1182 without the offset and the
// literals.  x holds bytes base .. base+11: the token and its first literal-length byte (compile-time
// indices -- a run-time index into x sends it to scratch memory); other length bytes come from LDS.
__device__ __forceinline__ uint32_t solo_next(const uint8_t *in, int32_t L, int32_t p, uint32_t u,
                                              const uint32_t (&x)[3], uint32_t &olen) {
    const uint32_t t = (x[u >> 2] >> (8u * (u & 3u))) & 0xFFu;
    int32_t q = p + 1, lit = (int32_t)(t >> 4);
    if (lit == kRunMask) {
        uint32_t b = (x[(u + 1u) >> 2] >> (8u * ((u + 1u) & 3u))) & 0xFFu;
        q++;
        lit += (int32_t)b;
        while (q < L - kRunMask && b == 255) {
            b = in[q];
            q++;
            lit += (int32_t)b;
        }
    }
    if (q + lit > L - 8) {   // terminal literal run
        olen = (uint32_t)lit;
        return kEnd;
    }
    int32_t q2 = q + lit + 2, ml = (int32_t)(t & 15u);
    if (ml == 15) {
        uint32_t b;
        do {
            b = in[q2];
            q2++;
            if (q2 > L - kLastLiterals) {   // overrun in the match length
                olen = 0;
                return kEnd;
            }
            ml += (int32_t)b;
        } while (b == 255);
    }
    olen = (uint32_t)(lit + ml + kMinMatch);
    return (uint32_t)q2;
}

// decode_seq_in without the literal window (the single-page decoder reads literal bytes per cell):
// token, length-extension bytes and the offset, the reads of lz4.c:1134-1143, 1165, 1172-1182
__device__ __forceinline__ SeqIn solo_seq(const uint8_t *in, int32_t L, int32_t p) {
    SeqIn s;
    const uint32_t t = in[p];
    int32_t q = p + 1;
    s.lit = (int32_t)(t >> 4);
    s.lit_win = false;
    if (s.lit == kRunMask) {
        uint32_t b;
        do {
            b = in[q];
            q++;
            s.lit += (int32_t)b;
        } while (q < L - kRunMask && b == 255);
    }
    s.ls = q;
    s.in_term = q + s.lit > L - 8;
    s.off = 0;
    s.ml = 0;
    s.q2 = 0;
    s.ml_err = false;
    if (!s.in_term) {
        s.off = (int32_t)lds_ld16(in + q + s.lit);
        int32_t q2 = q + s.lit + 2;
        int32_t ml = (int32_t)(t & 15u);
        if (ml == 15) {
            uint32_t b;
            do {
                b = in[q2];
                q2++;
                if (q2 > L - kLastLiterals) { s.ml_err = true; break; }
                ml += (int32_t)b;
            } while (b == 255);
        }
        s.ml = ml + kMinMatch;
        s.q2 = q2;
    }
    return s;
}

// LDS layout of the single-page decoder (host and device agree through this)
struct SoloLay {
    uint32_t stage, scr;   // byte offsets in LDS
    uint32_t jb, mark;     // byte offsets in scr: the second J buffer, the marks (token chain)
    uint32_t rec, slot;    // byte offsets in scr: token records (after the cells), 4-cell group covering table
    uint32_t nslots, total;
};
__host__ __device__ inline uint32_t solo_up16(uint32_t x) { return (x + 15u) & ~15u; }
__host__ __device__ inline SoloLay solo_layout(uint32_t in_cap, uint32_t out_cap) {
    SoloLay l;
    l.stage = 256u;   // 64 header words
    l.scr = l.stage + solo_up16(in_cap + 16u + kPad);
    const uint32_t max_tok = in_cap / 3u + 2u;   // a chain token consumes >= 3 bytes, but the last
    const uint32_t nodes = solo_up16(2u * (in_cap + 1u));   // u16 per position, + the sink
    l.jb = nodes;
    l.mark = 2u * nodes;
    const uint32_t chain_bytes = 2u * nodes + solo_up16(in_cap + 8u);   // (marks read as 8-byte words)
    const uint32_t cells_bytes = 2u * ((out_cap + 63u) & ~63u);
    l.rec = cells_bytes;
    // the covering table is zeroed while J is built: it overlaps neither J nor the marks
    l.slot = std::max(chain_bytes, l.rec + 8u * (max_tok + 1u));
    l.nslots = ((out_cap + 63u) & ~63u) / 4u;
    l.total = l.scr + l.slot + solo_up16(2u * l.nslots);
    return l;
}

// exclusive prefix sum over the workgroup (every thread calls it; wsum: kT / 64 words)
template <uint32_t kT>
__device__ __forceinline__ uint32_t solo_excl_sum(uint32_t v, uint32_t *wsum, uint32_t tid, uint32_t &total) {
    const uint32_t w = tid >> 6;
    const uint32_t incl = (uint32_t)wave_incl_sum((int32_t)v);
    if ((tid & 63u) == 63u) wsum[w] = incl;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < kT / 64u; k++) {
        const uint32_t x = wsum[k];
        base += k < w ? x : 0u;
        tot += x;
    }
    total = tot;
    __syncthreads();   // wsum may be reused
    return base + incl - v;
}

// the same over two values at once (wsum: 2 kT / 64 words)
template <uint32_t kT>
__device__ __forceinline__ uint2 solo_excl_sum2(uint32_t a, uint32_t b, uint32_t *wsum, uint32_t tid, uint32_t &ta,
                                                uint32_t &tb) {
    constexpr uint32_t kW = kT / 64u;
    const uint32_t w = tid >> 6;
    const uint32_t ia = (uint32_t)wave_incl_sum((int32_t)a), ibb = (uint32_t)wave_incl_sum((int32_t)b);
    if ((tid & 63u) == 63u) {
        wsum[w] = ia;
        wsum[kW + w] = ibb;
    }
    __syncthreads();
    uint32_t ba = 0, bb = 0, sa = 0, sb = 0;
#pragma unroll
    for (uint32_t k = 0; k < kW; k++) {
        const uint32_t x = wsum[k], y = wsum[kW + k];
        ba += k < w ? x : 0u;
        bb += k < w ? y : 0u;
        sa += x;
        sb += y;
    }
    ta = sa;
    tb = sb;
    __syncthreads();   // wsum may be reused
    return make_uint2(ba + ia - a, bb + ibb - b);
}

template <uint32_t kT>
__global__ __launch_bounds__(kT) void lz4_decode_solo_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap,
                                                             SoloLay lay, unsigned *ctr, uint32_t async_rounds) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1);
    // words: [0] rv, [2] first failing (or the terminal) token, [5] claimed page, [6..8] jump round flags,
    // [10] barrier-free jump rounds gave up, [16..47] block-sum scratch
    uint32_t *hw = (uint32_t *)smem;
    int32_t &s_rv = *(int32_t *)&hw[0];
    uint32_t *wsum = hw + 16;
    uint8_t *stage = smem + lay.stage;
    uint8_t *scr = smem + lay.scr;
    uint16_t *ja0 = (uint16_t *)scr, *jb0 = (uint16_t *)(scr + lay.jb);   // J, double-buffered
    uint8_t *mark = scr + lay.mark;
    uint16_t *cells = (uint16_t *)scr;   // the same bytes once the token list is out
    uint2 *rec = (uint2 *)(scr + lay.rec);
    uint16_t *slot = (uint16_t *)(scr + lay.slot);
    size_t page = blockIdx.x;
    while (page < b.count) {
        PROF_DECL
        const PageRef p = batch_page(b, page);
        const bool fits = p.src_len <= in_cap && p.dst_cap <= out_cap;
        const uint32_t head = stage_in(p.src, fits ? p.src_len : 0u, stage, tid, kT);
        const int32_t L = (int32_t)p.src_len, C = (int32_t)p.dst_cap;
        if (tid == 0) {
            hw[2] = 0xFFFFFFFFu;
            hw[6] = 0;    // round 0's flag
            hw[10] = 0;   // barrier-free jump rounds gave up
        }
        uint8_t *in = stage + head;
        const bool go = fits && C > 0 && L > 0;
        __syncthreads();
        if (fits && tid < kPad) in[L + tid] = 0;   // kPad zero bytes past the end
        if (tid == 0)
            s_rv = !fits ? kResultTooLarge : C == 0 ? ((L == 1 && in[0] == 0) ? 0 : -1) : L == 0 ? -1 : kJumpPending;
        __syncthreads();
        PROF_MARK(1);
        if (go) {
            // ---- 1. J(q) for every position, position 0 marked.  Thread t owns positions
            // [8 (t nch + c), +8) for its nch chunks c and keeps their J values in registers (two per
            // word), so a round reads only its marks (one 8-byte word) and the 8 J(J(q)) from LDS and
            // writes one 16-byte word of J (and the marks it sets).  The output length of the token
            // each position would start is kept too (the chain's offsets need no second parse).
            const uint32_t n = (uint32_t)L + 1u;   // positions + the sink
            const uint32_t nch = (n + kSoloNpt * kT - 1u) / (kSoloNpt * kT);
            uint32_t jr[kSoloChunks][4], ol[kSoloChunks][4];
            {
                const uint32_t ib = (uint32_t)(uintptr_t)in & 3u;
                const uint32_t *A = (const uint32_t *)(in - ib);
#pragma unroll
                for (uint32_t c = 0; c < kSoloChunks; c++) {
                    const uint32_t base = (tid * nch + c) * kSoloNpt;
#pragma unroll
                    for (uint32_t k = 0; k < 4u; k++) jr[c][k] = ol[c][k] = 0;
                    if (c < nch && base < n) {
                        // bytes base .. base+11: the 8 tokens and their first literal-length bytes
                        const uint32_t qa = base + ib;
                        uint32_t w[4], x[3];
#pragma unroll
                        for (uint32_t k = 0; k < 4u; k++) w[k] = A[(qa >> 2) + k];
#pragma unroll
                        for (uint32_t k = 0; k < 3u; k++) x[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], qa & 3u);
                        uint32_t nx[8], no[8];
#pragma unroll
                        for (uint32_t u = 0; u < 8u; u++) {
                            const uint32_t q = base + u;
                            no[u] = 0;
                            nx[u] = q < (uint32_t)L ? min(solo_next(in, L, (int32_t)q, u, x, no[u]), (uint32_t)L) : (uint32_t)L;
                        }
#pragma unroll
                        for (uint32_t k = 0; k < 4u; k++) {
                            jr[c][k] = nx[2 * k] | nx[2 * k + 1] << 16;
                            ol[c][k] = min(no[2 * k], 0xFFFFu) | min(no[2 * k + 1], 0xFFFFu) << 16;
                        }
                        *(uint4 *)(ja0 + base) = make_uint4(jr[c][0], jr[c][1], jr[c][2], jr[c][3]);
                        *(uint2 *)(mark + base) = make_uint2(base == 0 ? 1u : 0u, 0u);
                    }
                }
                for (uint32_t w = tid; w < lay.nslots; w += kT) slot[w] = 0;   // (its own bytes)
            }
            __syncthreads();
            PROF_MARK(2);
            // doubling rounds (at most 16: J^(2^16)(0) is the sink for any u16 position chain)
            uint16_t *Ja = ja0, *Jb = jb0;
            uint32_t lev = 0;
            for (; lev < 17u && Ja[0] != (uint16_t)L; lev++) {
#pragma unroll
                for (uint32_t c = 0; c < kSoloChunks; c++) {
                    const uint32_t base = (tid * nch + c) * kSoloNpt;
                    if (c < nch && base < n) {
                        const uint2 mw = *(const uint2 *)(mark + base);
                        uint32_t jj[8];
#pragma unroll
                        for (uint32_t u = 0; u < 8u; u++) {
                            const uint32_t j = (jr[c][u >> 1] >> (16u * (u & 1u))) & 0xFFFFu;
                            jj[u] = j == (uint32_t)L ? j : (uint32_t)Ja[j];   // (the sink maps to itself)
                        }
#pragma unroll
                        for (uint32_t u = 0; u < 8u; u++)
                            if ((((u < 4u ? mw.x : mw.y) >> (8u * (u & 3u))) & 1u) != 0u)
                                mark[(jr[c][u >> 1] >> (16u * (u & 1u))) & 0xFFFFu] = 1;
#pragma unroll
                        for (uint32_t k = 0; k < 4u; k++) jr[c][k] = jj[2 * k] | jj[2 * k + 1] << 16;
                        *(uint4 *)(Jb + base) = make_uint4(jr[c][0], jr[c][1], jr[c][2], jr[c][3]);
                    }
                }
                __syncthreads();
                uint16_t *x = Ja;
                Ja = Jb;
                Jb = x;
            }
            PROF_MARK(3);
            PROF_ADD(11, lev);
            // ---- the tokens: each thread's marked positions below L, in position (= chain) order; one
            // scan of (tokens, output bytes) per thread gives its first token number and output offset
            uint32_t cnt = 0, osum = 0;
            uint64_t mk[kSoloChunks];
#pragma unroll
            for (uint32_t c = 0; c < kSoloChunks; c++) {
                const uint32_t base = (tid * nch + c) * kSoloNpt;
                mk[c] = 0;
                if (c < nch && base < (uint32_t)L) {
                    const uint64_t keep = (uint32_t)L - base >= 8u ? ~0ull : (1ull << (8u * ((uint32_t)L - base))) - 1ull;
                    mk[c] = *(const uint64_t *)(mark + base) & keep & 0x0101010101010101ull;
                    cnt += (uint32_t)__builtin_popcountll(mk[c]);
#pragma unroll
                    for (uint32_t u = 0; u < 8u; u++)
                        if ((mk[c] >> (8u * u)) & 1u) osum += (ol[c][u >> 1] >> (16u * (u & 1u))) & 0xFFFFu;
                }
            }
            uint32_t ntok = 0, otot = 0;
            const uint2 ex = solo_excl_sum2<kT>(cnt, osum, wsum, tid, ntok, otot);   // (marks read: J's bytes are free)
            PROF_MARK(4);
            // ---- 2. per token: decode, the reference's checks at its output offset, a record (output
            // offset, literal count, literal start, match offset); the covering table gets, at slot
            // ceil(o / 4), the token whose output holds the first cell of 4-cell group (o + 3) / 4
            uint32_t my_first = 0xFFFFFFFFu;
            int32_t my_rv = -1;
            {
                uint32_t i = ex.x;
                int32_t ob = (int32_t)ex.y;
                bool stop = false;
                auto chunk = [&](uint64_t m, uint32_t base) {
                    while (m && !stop) {
                        const uint32_t u = (uint32_t)__builtin_ctzll(m) >> 3;
                        m &= m - 1ull;
                        const SeqIn sq = solo_seq(in, L, (int32_t)(base + u));
                        int32_t r;
                        const int32_t st = seq_check(sq, ob, L, C, r);
                        if (st) {
                            my_first = i;
                            my_rv = r;
                            atomicMin(&hw[2], i);
                            stop = true;
                        }
                        if (st != 2) {   // (a token that passes its own checks lies inside [0, C))
                            const int32_t e = ob + sq.lit + (st == 1 ? 0 : sq.ml);
                            rec[i] = make_uint2((uint32_t)ob | ((uint32_t)sq.lit << 16), (uint32_t)sq.ls | ((uint32_t)sq.off << 16));
                            const uint32_t s0 = ((uint32_t)ob + 3u) >> 2;
                            if (s0 < (((uint32_t)e + 3u) >> 2)) slot[s0] = (uint16_t)i;
                            ob = e;
                        }
                        i++;
                    }
                };
                chunk(mk[0], tid * nch * kSoloNpt);
                if (nch > 1u) chunk(mk[1], (tid * nch + 1u) * kSoloNpt);
                if (nch > 2u) chunk(mk[2], (tid * nch + 2u) * kSoloNpt);
            }
            __syncthreads();
            if (my_first != 0xFFFFFFFFu && my_first == hw[2]) s_rv = my_rv;
            if (hw[2] == 0xFFFFFFFFu && tid == 0) s_rv = -1;   // unreachable: the chain ends in a stop
            __syncthreads();
            PROF_MARK(5);
        }
        PROF_ADD(9, 1);
        const int32_t rv = s_rv;
        if (rv > 0) {
            // ---- 3. cells, one per lane (consecutive lanes, consecutive cells): the token holding cell
            // c is the covering token of its 4-cell group (the running maximum of the slots) or the next
            // one (a token other than the last spans >= 4 cells); literal cells final (0x8000 | byte),
            // match cells pointing at the byte they copy (d - off + ((c - d) mod off): the match's own
            // earlier bytes when it overlaps itself), cells past rv final
            const uint32_t n64 = ((uint32_t)rv + 63u) & ~63u;
            const uint32_t ng4 = n64 / 4u, gpt = (ng4 + kT - 1u) / kT;   // groups per thread: <= 8
            const uint32_t last = hw[2];   // the terminal token
            {
                uint32_t m = 0;
                for (uint32_t u = 0; u < gpt; u++) {
                    const uint32_t g = tid * gpt + u;
                    if (g < ng4) m = max(m, (uint32_t)slot[g]);
                }
                const uint32_t w = tid >> 6;
                const uint32_t incl = (uint32_t)wave_incl_max((int32_t)m);
                if ((tid & 63u) == 63u) wsum[w] = incl;
                uint32_t before = (uint32_t)__shfl_up((int32_t)incl, 1);
                if ((tid & 63u) == 0u) before = 0;
                __syncthreads();
                for (uint32_t k = 0; k < w; k++) before = max(before, wsum[k]);
                for (uint32_t u = 0; u < gpt; u++) {
                    const uint32_t g = tid * gpt + u;
                    if (g < ng4) {
                        before = max(before, (uint32_t)slot[g]);
                        slot[g] = (uint16_t)before;
                    }
                }
                __syncthreads();
            }
            PROF_MARK(10);
            // (each lane takes 4-cell groups tid + i kT: one covering-table read and two record reads per
            // group, its 4 cells written as one 8-byte word)
            for (uint32_t g0 = tid; g0 < ng4; g0 += 4u * kT) {
                uint32_t gk[4];
                uint2 r0[4], r1[4];
#pragma unroll
                for (uint32_t u = 0; u < 4u; u++) {
                    const uint32_t g = g0 + u * kT;
                    gk[u] = g < ng4 && 4u * g < (uint32_t)rv ? (uint32_t)slot[g] : 0u;
                }
#pragma unroll
                for (uint32_t u = 0; u < 4u; u++) {
                    r0[u] = rec[gk[u]];
                    r1[u] = rec[gk[u] < last ? gk[u] + 1u : gk[u]];
                }
                uint32_t lb[4][4];
#pragma unroll
                for (uint32_t u = 0; u < 4u; u++) {
                    const uint32_t o1 = gk[u] < last ? (r1[u].x & 0xFFFFu) : 0xFFFFFFFFu;
#pragma unroll
                    for (uint32_t j = 0; j < 4u; j++) {
                        const uint32_t c = 4u * (g0 + u * kT) + j;
                        const uint2 r = c >= o1 ? r1[u] : r0[u];
                        const uint32_t o = r.x & 0xFFFFu, d = o + (r.x >> 16);
                        lb[u][j] = c < (uint32_t)rv && c < d ? (uint32_t)in[(r.y & 0xFFFFu) + c - o] : 0u;
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < 4u; u++) {
                    const uint32_t g = g0 + u * kT;
                    if (g >= ng4) continue;
                    const uint32_t o1 = gk[u] < last ? (r1[u].x & 0xFFFFu) : 0xFFFFFFFFu;
                    uint32_t v[4];
#pragma unroll
                    for (uint32_t j = 0; j < 4u; j++) {
                        const uint32_t c = 4u * g + j;
                        const uint2 r = c >= o1 ? r1[u] : r0[u];
                        const uint32_t o = r.x & 0xFFFFu, d = o + (r.x >> 16), off = r.y >> 16;
                        uint32_t jm = c - d;   // (wraps below d: a literal cell)
                        if (c >= d && jm >= off && off != 0u) jm = mod_small(jm, off);   // overlapping match
                        v[j] = c >= (uint32_t)rv ? kLitFlag : c < d ? kLitFlag | lb[u][j] : off == 0u ? kLitFlag : d - off + jm;
                    }
                    *(uint2 *)(cells + 4u * g) = make_uint2(v[0] | v[1] << 16, v[2] | v[3] << 16);
                }
            }
            __syncthreads();
            PROF_MARK(6);
            // pointer jumping, 8 cells per group; each thread keeps its groups (tid + i kT) in registers
            // across the rounds, so a round reads LDS only for its unresolved cells' targets and writes
            // back only the groups that changed, and the last round's registers are packed and stored
            u32x4 *c4 = (u32x4 *)cells;
            const uint32_t ng = n64 / 8u;
            uint32_t *flag = hw + 6;
            const u32x4 fin = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
            u32x4 cv[kSoloGroups];
#pragma unroll
            for (uint32_t i = 0; i < kSoloGroups; i++) {
                const uint32_t g = tid + i * kT;
                cv[i] = g < ng ? c4[g] : fin;
            }
            // Rounds without barriers: a thread jumps its own cells until they are all final.  Reading a
            // cell another thread is rewriting returns its old or its new value, both pointers further
            // back along the same copy chain (or the final byte), and a pointer only ever moves back: each
            // round strictly advances every open cell, so the loop ends; the others' jumps make it
            // ~log2(depth) rounds as in lock-step.  A thread that runs async_rounds rounds (kSoloAsyncRounds;
            // TYCHE_LZ4_SOLO_ASYNC, a test hook) leaves the rest to lock-step rounds.
            uint32_t ar = 0;
            for (;; ar++) {
                uint32_t open = 0;
#pragma unroll
                for (uint32_t i = 0; i < kSoloGroups; i++) {
                    u32x4 v = cv[i];
                    if (((v.x & v.y & v.z & v.w) & 0x80008000u) != 0x80008000u) {
                        v.x = jump_pair<true>(cells, v.x, open);
                        v.y = jump_pair<true>(cells, v.y, open);
                        v.z = jump_pair<true>(cells, v.z, open);
                        v.w = jump_pair<true>(cells, v.w, open);
                        c4[tid + i * kT] = v;
                        cv[i] = v;
                    }
                }
                if (!open) break;
                if (ar + 1 >= async_rounds) {
                    atomicOr(&hw[10], 1u);
                    break;
                }
            }
            PROF_ADD(12, ar + 1);
            __syncthreads();
            if (hw[10]) {
                for (uint32_t r = 0;; r++) {
                    if (tid == 0) flag[(r + 1) % 3] = 0;
                    uint32_t open = 0;
#pragma unroll
                    for (uint32_t i = 0; i < kSoloGroups; i++) {
                        u32x4 v = cv[i];
                        if (((v.x & v.y & v.z & v.w) & 0x80008000u) != 0x80008000u) {
                            v.x = jump_pair(cells, v.x, open);
                            v.y = jump_pair(cells, v.y, open);
                            v.z = jump_pair(cells, v.z, open);
                            v.w = jump_pair(cells, v.w, open);
                            c4[tid + i * kT] = v;
                            cv[i] = v;
                        }
                    }
                    if (open) atomicOr(&flag[r % 3], 1u);
                    __syncthreads();
                    if (flag[r % 3] == 0) break;
                }
            }
            PROF_MARK(7);
            // cells -> bytes, 8 per group
            uint8_t *dst = p.dst;
            const bool al = ((uintptr_t)dst & 7u) == 0;
#pragma unroll
            for (uint32_t i = 0; i < kSoloGroups; i++) {
                const uint32_t g = tid + i * kT;
                if (g >= ng) continue;
                const u32x4 a = cv[i];
                const uint32_t lo = __builtin_amdgcn_perm(a.y, a.x, 0x06040200u);
                const uint32_t hi = __builtin_amdgcn_perm(a.w, a.z, 0x06040200u);
                const uint32_t base = 8u * g;
                if (al && base + 8u <= (uint32_t)rv) {
                    __builtin_nontemporal_store(u32x2{lo, hi}, (u32x2 *)(dst + base));
                } else if (base < (uint32_t)rv) {
                    const uint32_t nb8 = min(8u, (uint32_t)rv - base);
                    for (uint32_t j = 0; j < nb8; j++) dst[base + j] = (uint8_t)((j < 4u ? lo : hi) >> (8u * (j & 3u)));
                }
            }
        }
        PROF_MARK(8);
        if (tid == 0) b.results[page] = rv;
        if (ctr) {
            if (tid == 0) hw[5] = atomicAdd(ctr, 1u) + gridDim.x;
            __syncthreads();
            page = hw[5];
        } else {
            page += gridDim.x;
        }
        __syncthreads();
    }
}

}  // namespace

// Batches below this many pages (TYCHE_LZ4_JUMP_MAX) take the jump decoder when
// the page fits its layout (16-bit cells: pages <= 32 KiB).
constexpr long kJumpMax = 16384;
static hipError_t launch_lz4_decode_jump(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s,
                                         bool &launched) {
    launched = false;
    const long jmax = knob("LZ4_JUMP_MAX", kJumpMax);
    if ((long)b.count >= jmax || out_cap > 32768u) return hipSuccess;
    const uint32_t cells_bytes = std::max(2u * ((out_cap + 63u) & ~63u), (in_cap + 4u + 15u) & ~15u);
    const uint32_t list_cap = out_cap / (uint32_t)(kJumpLong + 1) + 2u;
    // items: rows sequences per lane (the bench pages' segments hold <= 44 tokens at 16 KiB,
    // <= 85 at 32 KiB), the rest of a longer lane part in kJumpOvf overflow items; a page
    // with more takes jump_front's two walks
    const uint32_t rows = std::min(std::max(out_cap / 512u, 24u), 64u);
    const size_t lds = kJumpHdr + (size_t)cells_bytes + 8u * list_cap + 4u * 64u * rows + 8u * kJumpOvf +
                       ((in_cap + 16u + kPad + 15u) & ~15u);
    if (lds > 150 * 1024) return hipSuccess;
    const long wide_env = knob("LZ4_JUMP_WIDE", 1);
    const void *k512 = (const void *)lz4_decode_jump_kernel<512>, *k1024 = (const void *)lz4_decode_jump_kernel<1024>;
    const size_t ncu = prepare_launch(k512);
    const bool wide = wide_env && b.count <= ncu;
    const void *k = wide ? k1024 : k512;
    const uint32_t threads = wide ? 1024u : 512u;
    if (wide) (void)prepare_launch(k1024);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, (int)threads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const size_t grid = std::min<size_t>(b.count, ncu * (size_t)per_cu);
    WorkCounter ctr(s, grid < b.count);
    if (grid < b.count && !ctr.get()) return hipErrorOutOfMemory;
    unsigned *cp = grid < b.count ? ctr.get() : nullptr;
    void *args[] = {(void *)&b, &in_cap, &out_cap, (void *)&cells_bytes, (void *)&list_cap, (void *)&rows, &cp};
    (void)hipLaunchKernel(k, dim3((unsigned)grid), dim3(threads), args, lds, s);
    launched = true;
    return hipGetLastError();
}

// Batches of at most this many pages (TYCHE_LZ4_SOLO_MAX; 0 turns it off) take the single-page
// decoder when its LDS layout fits (pages <= 16 KiB and streams up to their bound; larger pages
// take the jump decoder)
constexpr long kSoloMax = 4096;
static hipError_t launch_lz4_decode_solo(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s,
                                         bool &launched) {
    launched = false;
    const long smax = knob("LZ4_SOLO_MAX", kSoloMax);
    if ((long)b.count > smax || out_cap > 32768u || in_cap >= kSoloChunks * kSoloNpt * 1024u) return hipSuccess;
    constexpr uint32_t kT = 1024;
    const SoloLay lay = solo_layout(in_cap, out_cap);
    if (lay.total > 160u * 1024u) return hipSuccess;
    const void *k = (const void *)lz4_decode_solo_kernel<kT>;
    const size_t ncu = prepare_launch(k);
    int per_cu = 1;   // (batches up to one page per CU -- the restore path's -- skip the occupancy query)
    if (b.count > ncu &&
        (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, (int)kT, lay.total) != hipSuccess || per_cu < 1))
        per_cu = 1;
    const size_t grid = std::min<size_t>(b.count, ncu * (size_t)per_cu);
    WorkCounter ctr(s, grid < b.count);
    if (grid < b.count && !ctr.get()) return hipErrorOutOfMemory;
    unsigned *cp = grid < b.count ? ctr.get() : nullptr;
    uint32_t async_rounds = (uint32_t)std::max(1L, knob("LZ4_SOLO_ASYNC", kSoloAsyncRounds));
    void *args[] = {(void *)&b, &in_cap, &out_cap, (void *)&lay, &cp, &async_rounds};
    (void)hipLaunchKernel(k, dim3((unsigned)grid), dim3(kT), args, lay.total, s);
    launched = true;
    return hipGetLastError();
}

hipError_t launch_lz4_decode(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s,
                             bool allow_lane) {
    if (b.count == 0) return hipSuccess;
    // large batches: one page per lane (lz4_decode_lane.hip); never into host memory (allow_lane
    // false): that decoder reads its flushed output back
    if (allow_lane && lz4_lane_decode_wanted(b.count, in_cap, out_cap)) return launch_lz4_decode_lane(b, in_cap, out_cap, s);
    // small batches: workgroup per page, pointer-jumping match resolution -- the single-page decoder
    // (round 5) when its layout fits, else the jump decoder
    {
        bool launched = false;
        const hipError_t es = launch_lz4_decode_solo(b, in_cap, out_cap, s, launched);
        if (launched || es != hipSuccess) return es;
    }
    {
        bool launched = false;
        const hipError_t e = launch_lz4_decode_jump(b, in_cap, out_cap, s, launched);
        if (launched || e != hipSuccess) return e;
    }
    // page window (output; the parse's owner stamps, so at least in_cap bytes;
    // the token positions at its top, <= in_cap / 3 + 1 of them, which always
    // fit: W >= in_cap + 20), then the staged stream
    const uint32_t off_in = (std::max(out_cap, in_cap + 4u) + 16u + 15u) & ~15u;
#ifndef TYCHE_LDS_EXTRA
#define TYCHE_LDS_EXTRA 0
#endif
    const size_t lds = off_in + ((in_cap + 16u + kPad + 15u) & ~15u) + TYCHE_LDS_EXTRA;   // EXTRA: occupancy experiments
    if (lds > 160 * 1024) {
        // large pages: sequential decoder, LDS = page window + stream only
        const size_t lds2 = ((out_cap + 15u) & ~15u) + ((in_cap + 16u + kPad + 15u) & ~15u);
        if (lds2 > 160 * 1024) return hipErrorInvalidValue;
        (void)prepare_launch((const void *)lz4_decode_serial_kernel);
        hipLaunchKernelGGL(lz4_decode_serial_kernel, dim3((unsigned)b.count), dim3(kWave), lds2, s, b, in_cap,
                           out_cap);
        return hipGetLastError();
    }
    const size_t ncu = prepare_launch((const void *)lz4_decode_wave_kernel);
    // LDS is granted in 512-byte granules per workgroup
    auto lds_for = [&](uint32_t cap) -> size_t {
        return ((std::max(out_cap, cap + 4u) + 16u + 15u) & ~15u) + ((cap + 16u + kPad + 15u) & ~15u) + TYCHE_LDS_EXTRA;
    };
    auto granted = [](size_t l) -> size_t { return (l + 511u) & ~(size_t)511u; };
    auto launch = [&](uint32_t cap, uint32_t lo, uint32_t hi, uint32_t chunk) -> hipError_t {
        const size_t l = lds_for(cap);
        const uint32_t win = (std::max(out_cap, cap + 4u) + 16u + 15u) & ~15u;
        const size_t per_cu = waves_per_cu((const void *)lz4_decode_wave_kernel, l);
        const size_t grid = std::min<size_t>(b.count, ncu * per_cu);
        WorkCounter ctr(s, grid < b.count);
        if (chunk && !ctr.get()) return hipErrorOutOfMemory;
        hipLaunchKernelGGL(lz4_decode_wave_kernel, dim3((unsigned)grid), dim3(kWave), l, s, b, cap, out_cap, win, lo, hi,
                           chunk ? ctr.get() : nullptr, chunk);
        return hipGetLastError();
    };
    // Size classes: the decoder is latency-bound and its residency is set by
    // the LDS per wave, i.e. by the longest stream of the batch.  When streams
    // up to some T < in_cap fit one more wave per CU, those pages go in a
    // first launch sized for T and the rest in a second one sized for in_cap
    // (1M bench pages: mean 6.2 KB, max 8.1 KB: streams <= 6.5 KB run 7 waves per CU
    // instead of 6, 129.6 -> 121.8 ms per 1M pages).
    // Each wave skips the pages of the other class.  TYCHE_DECODE_CLASSES=0
    // turns the split off (A/B timing).
#ifndef TYCHE_CLASS_CHUNK
#define TYCHE_CLASS_CHUNK 1
#endif
    // chunk of the long-stream class (1M bench pages, ms: static 118.9, chunks of
    // 64: 117.4, 8: 111.1, 2: 110.2, 1: 109.9 -- skipped claims are cheap)
    constexpr uint32_t kClassChunk = TYCHE_CLASS_CHUNK;   // static striding when 0
    const long split_env = knob("DECODE_CLASSES", 1);
    const size_t waves = split_env && b.src_lengths && b.count >= 8192
                             ? waves_per_cu((const void *)lz4_decode_wave_kernel, lds) : 32;
    if (waves < 16) {
        const size_t target = (160 * 1024) / (waves + 1);
        uint32_t T = in_cap;
        while (T > 16u && granted(lds_for(T)) > target) T -= 16u;
        if (granted(lds_for(T)) <= target && T >= in_cap / 2u && T < in_cap &&
            waves_per_cu((const void *)lz4_decode_wave_kernel, lds_for(T)) > waves) {
            hipError_t e = launch(T, 0u, T, 1u);
            if (e != hipSuccess) return e;
            return launch(in_cap, T + 1u, 0xFFFFFFFFu, kClassChunk);
        }
    }
    return launch(in_cap, 0u, 0xFFFFFFFFu, 1u);
}

#ifdef TYCHE_PROFILE
extern "C" int tyche_debug_decode_profile(unsigned long long *host16, int reset) {
    if (reset) {
        unsigned long long z[16] = {0};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) == hipSuccess ? 0 : 1;
    }
    return hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : 1;
}
#endif

}  // namespace tyche
