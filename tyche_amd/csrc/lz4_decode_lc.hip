// lz4_decode_lc.hip -- LZ4 block decode for large batches, round 4: one page
// per LANE, decoded in chunks of kLC records (reference: buffer__decompress,
// src/buffer.c:248-253 -> LZ4_decompress_safe, src/lz4/lz4.c:1251; generic
// decoder lz4.c:1089-1248).
//
// The round-3 lane decoder (lz4_decode_lane.hip) runs the reference loop per
// lane and issues, inside that loop, the far-match loads (sources further back
// than its LDS ring), the stream line loads and the 64-byte line flushes.  Loads
// and stores share one in-order counter (vmcnt), so almost every iteration
// waits a full memory round trip -- the wave is busy 33-42 % of its cycles.
// This kernel keeps the one-lane-per-page parse (64 pages per wave
// instruction: the fewest instructions per page of every design we tried, see
// DESIGN 3.1e for the quad-per-page one) but moves all HBM traffic out of the
// sequence loop:
//
//  * stage 1 parses up to kLC records per lane from a 64-byte LDS window of its
//    stream into registers (one 32-bit record per unrolled slot: window
//    position, literal and match part lengths <= 16, offset), the reference's
//    checks in the reference's order on the way.  A sequence larger than a
//    record is cut into parts (long literal runs, long matches); the parse is a
//    state machine that resumes inside a literal run or a match in the next
//    chunk.  A far match part (offset > R - 24: its source has left the ring)
//    issues its 16-byte load right away, into that slot's registers;
//  * the next chunk's window is loaded behind them; stage 3 then copies the
//    records window/ring/registers -> ring with aligned LDS qwords only
//    (byte-unaligned LDS accesses replay per lane, tools/probes/lds_wide.hip):
//    a run is written as the three qwords from d & ~7, the lane's "tail"
//    register supplying the bytes below d;
//  * stage 4 writes the finished 16-byte pieces of all 64 pages cooperatively,
//    one piece per lane and store instruction, a page's pieces on neighbouring
//    lanes (a lane storing only its own page's pieces would touch 64 lines per
//    instruction).  Flushing 16-byte pieces rather than 64-byte lines keeps the
//    unflushed tail under 16 bytes, which lets a 128-byte ring carry 88-byte
//    chunks (lz4_lc_core.h, lc_budget): LDS per wave 14 KiB, 11 waves per CU.
//
// Results are LZ4_decompress_safe's: the decoded size, or -(input bytes
// consumed)-1 for a malformed stream (stream bytes past its end read as zero,
// as in the other decoders); on error the page's output is partial.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "lane_ring.h"
#include "lds_io.h"
#include "lds_qword.h"

namespace tyche {

// Timing-only ablation builds (-DTYCHE_ABLATE=mask: _build.build(ablate=mask), tools/time_variant.py;
// their outputs are wrong, the product build has mask 0 and none of these branches):
//   1024 no far loads | 2048 no flush stores | 4096 no copy stage | 8192 four extra window loads per chunk
#if defined(TYCHE_ABLATE) && TYCHE_ABLATE
#define LC_ABLATE(bit) ((TYCHE_ABLATE & (bit)) != 0)
#else
#define LC_ABLATE(bit) false
#endif

// Optional stage profile (diagnostic build only: -DTYCHE_PROFILE, tools/lc_profile.py):
// shader cycles per stage and event counts, summed per wave in scalar registers and added to
// g_lcprof once when the wave ends (an atomic per stamp would itself sit in vmcnt and be
// waited for by the stage that follows).
#ifdef TYCHE_PROFILE
__device__ unsigned long long g_lcprof[16];
#define LPROF_DECL                                  \
    unsigned long long _pt = clock64(), _acc[16]; \
    for (int _k = 0; _k < 16; _k++) _acc[_k] = 0;
#define LPROF_MARK(k)                  \
    do {                               \
        unsigned long long _n = clock64(); \
        _acc[k] += _n - _pt;           \
        _pt = _n;                      \
    } while (0)
#define LPROF_ADD(k, v) do { _acc[k] += (unsigned long long)(v); } while (0)
#define LPROF_END                                                              \
    do {                                                                       \
        if (lane == 0)                                                         \
            for (int _k = 0; _k < 16; _k++) atomicAdd(&g_lcprof[_k], _acc[_k]); \
    } while (0)
#else
#define LPROF_DECL
#define LPROF_MARK(k) do { } while (0)
#define LPROF_ADD(k, v) do { } while (0)
#define LPROF_END do { } while (0)
#endif

namespace {

// the match-copy table entry of class c (lz4_lc_core.h): 9 u32 of a 48-byte LDS entry
__device__ __forceinline__ void lc_lut_load(const uint32_t *lut, int32_t c, uint32_t *ent) {
    const uint8_t *p = (const uint8_t *)lut + 48 * c;
    const uint64_t a = lq(p), b = lq(p + 8), x = lq(p + 16), y = lq(p + 24);
    ent[0] = (uint32_t)a;
    ent[1] = (uint32_t)(a >> 32);
    ent[2] = (uint32_t)b;
    ent[3] = (uint32_t)(b >> 32);
    ent[4] = (uint32_t)x;
    ent[5] = (uint32_t)(x >> 32);
    ent[6] = (uint32_t)y;
    ent[7] = (uint32_t)(y >> 32);
    ent[8] = ld32(p + 32);
}

#include "lz4_lc_core.h"

// LDS of one wave: the 64 windows first (8 rows of 64 interleaved qwords; a parse
// read may run up to 4 rows past them, into the rings), the 64 rings (R / 8 rows),
// the flush tables.
template <int32_t R>
struct LCL {
    static_assert(lc_ring_ok<R>(), "ring too small for the flush granule (lc_budget)");
    static constexpr uint32_t win = 0;
    static constexpr uint32_t ring = 64u * kLWS;
    static constexpr uint32_t tab_out = ring + 64u * (uint32_t)R;         // 64 x u64: page output pointers
    static constexpr uint32_t tab_fl = tab_out + 64u * 8u;                // 64 x u32: first pending piece
    static constexpr int32_t max_pieces = (lc_budget<R>() + kLcLine - 1) / 16 + 1;   // 16-byte pieces per lane per chunk
    static constexpr uint32_t own = tab_fl + 64u * 4u;                    // 64 x max_pieces x u16
    static constexpr uint32_t lut = own + ((64u * (uint32_t)max_pieces * 2u + 15u) & ~15u);   // match-copy table
    static constexpr uint32_t total = lut + (uint32_t)kLutBytes;
};

// page `idx` of the batch (its metadata; src may be read for the C == 0 case)
struct LMeta {
    const uint8_t *in;
    uint8_t *out;
    uint32_t L, C;
};
__device__ __forceinline__ LMeta lmeta(const tyche_batch_t &b, size_t idx) {
    const PageRef r = batch_page(b, idx);
    return LMeta{r.src, r.dst, r.src_len, r.dst_cap};
}

// the window [ns, ns + 64) of the stream (ns >= 0), zero from L on.  The loads
// are issued unconditionally from clamped addresses and their results used only
// in wstore, after the chunk's other work: a shift applied where a load is made
// would wait for it (and for every load issued before it) right there.
struct LWin {
    u128 c0, c1, c2, c3;
    uint32_t sh;   // per piece (8 bits each): bytes to drop from the clamped load; >= 16: zero
};
__device__ __forceinline__ LWin wload(const uint8_t *__restrict__ in, int32_t ns, int32_t L) {
    LWin w;
    if (L >= 16) {
        const int32_t top = L - 16;
        const int32_t a0 = min(ns, top), a1 = min(ns + 16, top), a2 = min(ns + 32, top), a3 = min(ns + 48, top);
        w.c0 = ld16(in + a0);
        w.c1 = ld16(in + a1);
        w.c2 = ld16(in + a2);
        w.c3 = ld16(in + a3);
        w.sh = (uint32_t)min(ns - a0, 16) | ((uint32_t)min(ns + 16 - a1, 16) << 8) |
               ((uint32_t)min(ns + 32 - a2, 16) << 16) | ((uint32_t)min(ns + 48 - a3, 16) << 24);
    } else {   // a stream shorter than one piece (rare): bytes, zero-padded
        w.c0 = chunk16z(in, ns, L);
        w.c1 = chunk16z(in, ns + 16, L);
        w.c2 = chunk16z(in, ns + 32, L);
        w.c3 = chunk16z(in, ns + 48, L);
        w.sh = 0;
    }
    return w;
}
__device__ __forceinline__ u128 wshift(u128 v, uint32_t k) {
    k &= 0xFFu;
    return k >= 16u ? (u128)0 : (k == 0u ? v : v >> (8u * k));
}
// 16-byte piece j of a lane's window / a ring piece at qword k (even), in the interleaved layout
__device__ __forceinline__ void lc_put_piece(uint8_t *base, int32_t k, u128 v) {
    lq(LC_Q(base, k), (uint64_t)v);
    lq(LC_Q(base, k + 1), (uint64_t)(v >> 64));
}
__device__ __forceinline__ u128 lc_get_piece(const uint8_t *base, int32_t k) {
    return (u128)lq(LC_Q(base, k)) | ((u128)lq(LC_Q(base, k + 1)) << 64);
}
__device__ __forceinline__ void wstore(uint8_t *w16, const LWin &w) {
    if (w.sh == 0) {
        lc_put_piece(w16, 0, w.c0);
        lc_put_piece(w16, 2, w.c1);
        lc_put_piece(w16, 4, w.c2);
        lc_put_piece(w16, 6, w.c3);
    } else {
        lc_put_piece(w16, 0, wshift(w.c0, w.sh));
        lc_put_piece(w16, 2, wshift(w.c1, w.sh >> 8));
        lc_put_piece(w16, 4, wshift(w.c2, w.sh >> 16));
        lc_put_piece(w16, 6, wshift(w.c3, w.sh >> 24));
    }
}

// s_waitcnt vmcnt(0) (expcnt, lgkmcnt not waited), as a builtin so the compiler's own wait
// placement knows of it
constexpr int kVmDrain = 0x0F70;

// starts the lane on page idx or a later one of its stride (pages with an
// immediate result -- empty capacity, empty stream, over the launch's sizing --
// are answered here); false when the lane has no page left.  The window of the
// page's first 64 bytes is loaded synchronously.
__device__ bool lpage_start(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, size_t idx, size_t G,
                            LPage &P, uint8_t *w16) {
    for (; idx < b.count; idx += G) {
        const LMeta m = lmeta(b, idx);
        int32_t rv;
        if (m.L > in_cap || m.C > out_cap) {
            rv = kResultTooLarge;
        } else if (m.C == 0) {
            rv = (m.L == 1 && ld1(m.in) == 0) ? 0 : -1;
        } else if (m.L == 0) {
            rv = -1;
        } else {
            P.in = m.in;
            P.out = m.out;
            P.L = (int32_t)m.L;
            P.C = (int32_t)m.C;
            P.idx = idx;
            P.ip = P.op = P.fl = P.wb = 0;
            P.tail = 0;
            P.lp = P.lrem = P.moff = P.mrem = P.mtok = P.hdr = P.term = 0;
            wstore(w16, wload(P.in, 0, P.L));
            // every metadata load done here, where this path waits anyway: a load still in flight
            // at the loop's back edge would make the compiler drain all stores at the loop's top
            __builtin_amdgcn_s_waitcnt(kVmDrain);
            return true;
        }
        b.results[idx] = rv;
    }
    return false;
}

// 64 bytes of zeros: the window source of a lane with no page (its loads are issued anyway, so that
// exactly four window loads follow the far loads: lc_far_wait)
__device__ __attribute__((aligned(64))) uint8_t g_lc_pad[64];

// A record slot's far source: [src, src + 16) and, for a part over 16 bytes, [src + 16, src + 32)
// of the page's output, loaded by the lanes that have one only.  The return path of the CU's
// vector memory (TD) is this kernel's busiest unit (r04 PMC: busy 94 % of the cycles), and a
// load costs it per active lane.  The loads are inline asm with the destination tied to its
// zero-initialised register, so the branch joins without a copy (a compiler-visible load in a
// branch is joined by a copy that waits for it right there, in the next slot); the compiler
// does not see them, and lc_far_wait waits for them before stage 3.
template <int32_t N>
__device__ __forceinline__ void far_load(const LPage &P, bool far, int32_t src, uint32_t rec, u32x4 (&fv)[N], int32_t t) {
    if (LC_ABLATE(1024)) far = false;
    if (far) {
        const uint8_t *a = P.out + src;
        asm volatile("global_load_dwordx4 %0, %1, off" : "+v"(fv[kFarPer * t]) : "v"(a) : "memory");
        if (kFarPer == 2 && ((rec >> 10) & 63u) > 16u)
            asm volatile("global_load_dwordx4 %0, %1, off offset:16" : "+v"(fv[kFarPer * t + (kFarPer - 1)]) : "v"(a) : "memory");
    }
}
// every far load done: all but the four window loads issued after them (vmcnt is in order); the
// empty asm statements tie the registers to this point, so no use moves above the wait
template <int32_t N>
__device__ __forceinline__ void lc_far_wait(u32x4 (&fv)[N]) {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
#pragma unroll
    for (int32_t i = 0; i < N; i++) asm volatile("" : "+v"(fv[i]));
}

#ifndef LC_WPE
#define LC_WPE 2   // register budget: waves per SIMD
#endif
template <int32_t R>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LC_WPE))) void lz4_decode_lc_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap) {
    typedef LCL<R> Lay;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint8_t *ring = smem + Lay::ring + lane * 8u;   // qword-interleaved (LC_Q)
    uint8_t *w16 = smem + Lay::win + lane * 8u;     // window byte 0, interleaved likewise
    uint64_t *tab_out = (uint64_t *)(smem + Lay::tab_out);
    uint32_t *tab_fl = (uint32_t *)(smem + Lay::tab_fl);
    uint16_t *own = (uint16_t *)(smem + Lay::own);
    const uint32_t *lut = (const uint32_t *)(smem + Lay::lut);
    const size_t G = (size_t)gridDim.x * 64u;
    if (lane <= 16) {   // the match-copy table, one entry per lane (the wave's later LDS reads see it)
        uint32_t ent[kLutStride];
        lc_lut_entry((int32_t)lane, ent);
        for (int32_t j = 0; j < kLutStride; j++) ld32(smem + Lay::lut + 48u * lane + 4u * (uint32_t)j, ent[j]);
    }

    LPage P;
    bool live = lpage_start(b, in_cap, out_cap, (size_t)blockIdx.x * 64u + lane, G, P, w16);
    LPROF_DECL
    while (__builtin_amdgcn_ballot_w64(live) != 0) {
        LPROF_ADD(0, 1);
        LPROF_MARK(9);   // loop back edge and top
        // ---- stage 1: records into registers; far sources loaded as they are found
        const int32_t op0 = P.op;
        int32_t st = live ? kLParse : kLCut, rv = 0, nrec = 0;
        uint32_t rec[kLC + 1];
        u32x4 fv[kFarPer * (kLC + 1)];   // far sources (far_load)
#pragma unroll
        for (int32_t i = 0; i < kFarPer * (kLC + 1); i++) fv[i] = u32x4{0u, 0u, 0u, 0u};
        bool go = live, gen = false;
        int32_t need_gen = 0;
        uint64_t wq[4];   // the next slot's window qwords (parse_fast)
        lc_wread(w16, lc_x0(P), wq);
        bool far0 = false, far1 = false;
        int32_t src0 = 0, src1 = 0;
#pragma unroll
        for (int32_t t = 0; t < kLC; t++) {
            rec[t] = 0;
            bool far = false;
            int32_t src = 0;
            if (go) {
                const int32_t k = parse_fast<R>(P, w16, op0, rec[t], far, src, wq);
                if (k == 1) {
                    nrec = t + 1;
                } else {
                    go = false;
                    need_gen = (k == 2 || t == 0) ? 1 : 0;   // the chunk's first record always makes progress
                    if (k == 0 && t != 0) st = kLCut;
                }
            }
            // The far sources lie below fl: stage 4 of an earlier chunk stored them, on other
            // lanes -- the last chunk's stores must have completed before the first one is read.
            // They drain during the parse of slots 0 and 1; then the loads go out, outside any
            // branch, so their registers are only waited for in stage 3.
            if (t == 0) {
                far0 = far;
                src0 = src;
            } else if (t == 1) {
                far1 = far;
                src1 = src;
                LPROF_MARK(1);   // slots 0, 1
                __builtin_amdgcn_s_waitcnt(kVmDrain);
                LPROF_MARK(2);   // the store drain
                asm volatile("" ::: "memory");
                far_load(P, far0, src0, rec[0], fv, 0);
                far_load(P, far1, src1, rec[1], fv, 1);
            } else {
                far_load(P, far, src, rec[t], fv, t);
            }
        }
        LPROF_MARK(3);   // slots 2.. and their far loads
        // one record of the general path (parse_slot) for the lanes that stopped on it; a lane
        // whose chunk made no progress (a length field longer than the window) takes it again
        // reading the stream straight from HBM, in its own rarely taken branch (window bytes and
        // HBM bytes in one code path would make every LDS byte read wait for the far loads)
        rec[kLC] = 0;
        {
            bool far = false;
            int32_t src = 0;
            if (__builtin_amdgcn_ballot_w64(need_gen != 0) != 0 && need_gen)
                gen = parse_slot<R>(P, w16, op0, false, st, rv, rec[kLC], far, src);
            const bool deep = need_gen && !gen && nrec == 0 && st == kLCut;
            if (__builtin_amdgcn_ballot_w64(deep) != 0 && deep) {
                st = kLParse;
                gen = parse_slot<R>(P, w16, op0, true, st, rv, rec[kLC], far, src);
            }
            far_load(P, far && gen, src, rec[kLC], fv, kLC);
        }
        LPROF_MARK(4);   // the general slot
        LPROF_ADD(12, __builtin_amdgcn_ballot_w64(need_gen != 0) != 0);
        // ---- the next window (the lane's next chunk), loaded behind the far sources
        const bool ended = live && st == kLEnd;
        const int32_t nwb = (P.lrem > 0 ? P.lp : P.ip) & ~15;   // the next stream byte the parse needs
        const bool wlive = live && !ended;   // (lanes without a next window load the pad)
        const LWin nw = wload(wlive ? P.in : g_lc_pad, wlive ? nwb : 0, wlive ? P.L : 64);
        if (ended && rv < 0) {   // a malformed page: its output is not defined
            nrec = 0;
            gen = false;
        }

        LPROF_MARK(5);   // window issue
        // ---- stage 3: copy the records into the ring (aligned qwords only)
        lc_far_wait(fv);
        if (LC_ABLATE(8192)) {
            const LWin xw = wload(wlive ? P.in : g_lc_pad, wlive ? min(nwb + 64, max(P.L - 64, 0)) : 0, wlive ? P.L : 64);
            __builtin_amdgcn_s_waitcnt(kVmDrain);
            if (xw.c0 == (u128)0x123457 && xw.c3 == (u128)1) P.tail ^= 1;
        }
        if (live && !LC_ABLATE(4096)) {
            u128 farv[kFarPer * (kLC + 1)];
#pragma unroll
            for (int32_t i = 0; i < kFarPer * (kLC + 1); i++) farv[i] = __builtin_bit_cast(u128, fv[i]);
            uint64_t tail = P.tail;
            copy_records<R>(ring, w16, op0, tail, rec, farv, nrec, gen, lut);
            P.tail = tail;
        }
        LPROF_MARK(6);   // copy (far-load wait included)

        // the next window into LDS now, before stage 4 issues its stores: this wait covers
        // loads only, and the stores drain during the next chunk's parse
        if (live && !ended) {
            P.wb = nwb;
            wstore(w16, nw);   // (the compiler waits for the window loads here)
        }
        LPROF_MARK(7);   // window wait and store
        // ---- stage 4: the finished 16-byte pieces of all 64 pages, one per lane and store
        // instruction (a page's pieces on neighbouring lanes: whole lines per few lanes)
        const int32_t lend = !live ? 0 : (ended && rv < 0) ? P.fl : (P.op & ~(kLcLine - 1));
        const int32_t nl = live ? (lend - P.fl) >> 4 : 0;
        const int32_t incl = wave_incl_sum(nl);
        const int32_t total = (int32_t)rdlane((uint32_t)incl, 63);
        if (total > 0) {
            // piece g of the wave (g = lane + 64 * it) belongs to the lane own[g] names; the
            // iterations' LDS reads are issued phase by phase (table entry, page, ring piece) so
            // the whole flush waits three LDS round trips, not three per iteration
            constexpr int32_t MP = Lay::max_pieces;
            tab_out[lane] = (uint64_t)(uintptr_t)P.out;
            tab_fl[lane] = (uint32_t)P.fl;
#pragma unroll
            for (int32_t k = 0; k < MP; k++)
                if (k < nl) own[incl - nl + k] = (uint16_t)(lane | ((uint32_t)k << 6));
            asm volatile("" ::: "memory");
            const int32_t iters = (total + 63) >> 6;   // wave-uniform
            uint32_t e[MP];
#pragma unroll
            for (int32_t it = 0; it < MP; it++) e[it] = it < iters ? (uint32_t)own[lane + 64 * it] : 0u;
            uint64_t o[MP];
            int32_t f[MP];
#pragma unroll
            for (int32_t it = 0; it < MP; it++) {
                o[it] = 0;
                f[it] = 0;
                if (it < iters) {
                    const uint32_t L2 = e[it] & 63u;
                    o[it] = tab_out[L2];
                    f[it] = (int32_t)tab_fl[L2] + 16 * (int32_t)(e[it] >> 6);
                }
            }
            u128 v[MP];
#pragma unroll
            for (int32_t it = 0; it < MP; it++)
                v[it] = it < iters ? lc_get_piece(smem + Lay::ring + (e[it] & 63u) * 8u, lc_row<R>(f[it] >> 3))
                                   : (u128)0;
#pragma unroll
            for (int32_t it = 0; it < MP; it++) {
                if ((int32_t)lane + 64 * it < total) {
                    uint8_t *dst = (uint8_t *)(uintptr_t)o[it] + f[it];
                    if (!LC_ABLATE(2048)) st16f(dst, v[it]);
                    else if (v[it] == (u128)0x1234567) dst[0] = 1;   // (keeps the LDS read)
                }
            }
            asm volatile("" ::: "memory");
        }
        if (live) P.fl = lend > P.fl ? lend : P.fl;
        LPROF_MARK(8);   // flush
        LPROF_ADD(13, total);
        LPROF_ADD(14, __builtin_popcountll(__builtin_amdgcn_ballot_w64(ended)));

        // ---- stage 5: the page's last bytes; the next page
        if (ended) {
            if (rv >= 0) {
                // bytes [fl, op): whole 16-byte pieces, then single bytes
                for (int32_t a = P.fl; a < P.op; a += 16) {
                    const u128 v = lc_get_piece(ring, lc_row<R>(a >> 3));
                    if (a + 16 <= P.op) {
                        st16(P.out + a, v);
                    } else {
                        for (int32_t x = a; x < P.op; x++) st1(P.out + x, (uint32_t)(v >> (8 * (x - a))) & 0xFFu);
                    }
                }
            }
            b.results[P.idx] = rv;
            live = lpage_start(b, in_cap, out_cap, P.idx + G, G, P, w16);
        }
        LPROF_MARK(10);   // stage 5: tails, page switch (uniform position: the stamps stay scalar)
        asm volatile("" ::: "memory");
    }
    LPROF_END;
}

}  // namespace

#ifdef TYCHE_PROFILE
extern "C" int tyche_debug_lc_profile(unsigned long long *host16, int reset) {
    if (reset) {
        unsigned long long z[16] = {0};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_lcprof), z, sizeof(z)) == hipSuccess ? 0 : 1;
    }
    return hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_lcprof), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : 1;
}
#endif

hipError_t launch_lz4_decode_lc(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    // R = 192 (24 qword rows, 18.9 KiB of LDS per wave, 8 waves per CU).  Round 6, ms per 1M x 16 KiB pages
    // with / without LC_FAR16: at 256K pages per launch R = 160 24.07 / 24.37, 192 24.22 / 24.46, 128
    // 28.9 / 25.1 (11 waves per CU with LC_FAR16: more waves in flight made it slower; 256: 28.6 in round
    // 4) -- r06_ring_ab.log, r06_far16.log; at the bench's 1M pages 160 and 192 tie (23.8-24.1 either
    // way, r06_1m_ab.log), while 192 reads less (57 vs 60 KB per page) and decodes the C4 shard's 8 KiB
    // pages faster (12.0 vs 13.0 ms per 1M)
    const long r = knob("LZ4_LC_RING", 192);
#if LC_LINE == 16
    const void *k = r == 256   ? (const void *)lz4_decode_lc_kernel<256>
                    : r == 192 ? (const void *)lz4_decode_lc_kernel<192>
                    : r == 160 ? (const void *)lz4_decode_lc_kernel<160>
                               : (const void *)lz4_decode_lc_kernel<128>;
    const size_t lds = r == 256   ? LCL<256>::total
                       : r == 192 ? LCL<192>::total
                       : r == 160 ? LCL<160>::total
                                  : LCL<128>::total;
#else   // 64-byte lines need R >= 192 (lc_ring_ok)
    const void *k = r == 256 ? (const void *)lz4_decode_lc_kernel<256> : (const void *)lz4_decode_lc_kernel<192>;
    const size_t lds = r == 256 ? LCL<256>::total : LCL<192>::total;
#endif
    const size_t ncu = prepare_launch(k);
    size_t waves = waves_per_cu(k, lds);
    const long env_waves = knob("LZ4_LC_WAVES", 8);   // (LC_FAR16's 154 VGPRs would allow more at R = 128 / 160: slower)
    if (env_waves > 0) waves = std::min<size_t>(waves, (size_t)env_waves);
    const size_t grid = std::min<size_t>((b.count + 63) / 64, ncu * waves);
    void *args[] = {(void *)&b, &in_cap, &out_cap};
    (void)hipLaunchKernel(k, dim3((unsigned)grid), dim3(64), args, lds, s);
    return hipGetLastError();
}

}  // namespace tyche
