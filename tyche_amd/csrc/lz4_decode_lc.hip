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
//    chunk.  A far match part (offset > R - 32: its source has left the ring)
//    issues its 16-byte load right away, into that slot's registers;
//  * the next chunk's window is loaded behind them; stage 3 then copies the
//    records window/ring/registers -> ring with aligned LDS qwords only
//    (byte-unaligned LDS accesses replay per lane, tools/probes/lds_wide.hip):
//    a run is written as the three qwords from d & ~7, the lane's "tail"
//    register supplying the bytes below d;
//  * stage 4 writes the finished 64-byte lines of all 64 pages cooperatively:
//    four lanes per line, 16 lines per store instruction, so every line leaves
//    in one instruction (a lane writing its own lines as four 16-byte stores
//    leaves them partially written for the L2 to merge).
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

// Optional stage profile (diagnostic build only: -DTYCHE_PROFILE, tools/lc_profile.py):
// shader cycles per stage summed over waves by lane 0, and event counts.
#ifdef TYCHE_PROFILE
__device__ unsigned long long g_lcprof[16];
#define LPROF_DECL unsigned long long _pt = clock64();
#define LPROF_MARK(k)                                                          \
    do {                                                                       \
        unsigned long long _n = clock64();                                     \
        if (lane == 0) atomicAdd(&g_lcprof[k], _n - _pt);                      \
        _pt = _n;                                                              \
    } while (0)
#define LPROF_ADD(k, v) do { if (lane == 0) atomicAdd(&g_lcprof[k], (unsigned long long)(v)); } while (0)
#else
#define LPROF_DECL
#define LPROF_MARK(k) do { } while (0)
#define LPROF_ADD(k, v) do { } while (0)
#endif

namespace {

#include "lz4_lc_core.h"

template <int32_t R>
struct LCL {
    static constexpr int32_t rs = R + 16;                                 // ring stride (16-aligned, bank spread)
    static constexpr uint32_t ring = 0;
    static constexpr uint32_t win = 64u * rs;
    static constexpr uint32_t tab_out = win + 64u * kLWS;                 // 64 x u64: page output pointers
    static constexpr uint32_t tab_fl = tab_out + 64u * 8u;                // 64 x u32: first pending line
    static constexpr int32_t max_lines = (R - 127 + 63) / 64 + 2;         // whole lines per lane per chunk
    static constexpr uint32_t own = tab_fl + 64u * 4u;                    // 64 x max_lines x u32
    static constexpr uint32_t total = own + 64u * (uint32_t)max_lines * 4u;
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

// the window [ns, ns + 64) of the stream, zero outside [0, L)
struct LWin {
    u128 c0, c1, c2, c3;
};
__device__ __forceinline__ LWin wload(const uint8_t *__restrict__ in, int32_t ns, int32_t L) {
    LWin w;
    w.c0 = chunk16z(in, ns, L);
    w.c1 = chunk16z(in, ns + 16, L);
    w.c2 = chunk16z(in, ns + 32, L);
    w.c3 = chunk16z(in, ns + 48, L);
    return w;
}
__device__ __forceinline__ void wstore(uint8_t *w16, const LWin &w) {
    lds16(w16, w.c0);
    lds16(w16 + 16, w.c1);
    lds16(w16 + 32, w.c2);
    lds16(w16 + 48, w.c3);
}

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
            return true;
        }
        b.results[idx] = rv;
    }
    return false;
}

template <int32_t R>
__global__ __launch_bounds__(64) void lz4_decode_lc_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap) {
    typedef LCL<R> Lay;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint8_t *ring = smem + Lay::ring + lane * (uint32_t)Lay::rs;
    uint8_t *w16 = smem + Lay::win + lane * (uint32_t)kLWS + 16;   // window byte 0
    uint64_t *tab_out = (uint64_t *)(smem + Lay::tab_out);
    uint32_t *tab_fl = (uint32_t *)(smem + Lay::tab_fl);
    uint32_t *own = (uint32_t *)(smem + Lay::own);
    const size_t G = (size_t)gridDim.x * 64u;

    LPage P;
    bool live = lpage_start(b, in_cap, out_cap, (size_t)blockIdx.x * 64u + lane, G, P, w16);
    LPROF_DECL
    while (__builtin_amdgcn_ballot_w64(live) != 0) {
        LPROF_ADD(0, 1);
        LPROF_MARK(7);
        // ---- stage 1: records into registers; far sources loaded as they are found
        const int32_t op0 = P.op;
        int32_t st = live ? kLParse : kLCut, rv = 0, nrec = 0;
        uint32_t rec[kLC + 1];
        u128 farv[2 * kLC + 2];
        bool go = live, gen = false;
        int32_t need_gen = 0;
#pragma unroll
        for (int32_t t = 0; t < kLC; t++) {
            rec[t] = 0;
            farv[2 * t] = farv[2 * t + 1] = 0;
            if (go) {
                bool far = false;
                int32_t src = 0;
                const int32_t k = parse_fast<R>(P, w16, op0, rec[t], far, src);
                if (k == 1) {
                    nrec = t + 1;
                    // the source lies below fl (stage 4 of an earlier chunk wrote it): lc_budget
                    if (far) {
                        farv[2 * t] = ld16(P.out + src);
                        farv[2 * t + 1] = ld16(P.out + src + 16);
                    }
                } else {
                    go = false;
                    need_gen = (k == 2 || t == 0) ? 1 : 0;   // the chunk's first record always makes progress
                    if (k == 0 && t != 0) st = kLCut;
                }
            }
        }
        // one record of the general path (parse_slot) for the lanes that stopped on it
        rec[kLC] = 0;
        farv[2 * kLC] = farv[2 * kLC + 1] = 0;
        if (__builtin_amdgcn_ballot_w64(need_gen != 0) != 0 && need_gen) {
            bool far = false;
            int32_t src = 0;
            if (parse_slot<R>(P, w16, op0, nrec == 0, st, rv, rec[kLC], far, src)) {
                gen = true;
                if (far) {
                    farv[2 * kLC] = ld16(P.out + src);
                    farv[2 * kLC + 1] = ld16(P.out + src + 16);
                }
            }
        }
        LPROF_MARK(1);
        LPROF_ADD(8, __builtin_amdgcn_ballot_w64(need_gen != 0) != 0);
        // ---- the next window (the lane's next chunk), loaded behind the far sources
        const bool ended = live && st == kLEnd;
        const int32_t nwb = (P.lrem > 0 ? P.lp : P.ip) & ~15;   // the next stream byte the parse needs
        LWin nw;
        nw.c0 = nw.c1 = nw.c2 = nw.c3 = 0;
        if (live && !ended) nw = wload(P.in, nwb, P.L);
        if (ended && rv < 0) {   // a malformed page: its output is not defined
            nrec = 0;
            gen = false;
        }

        LPROF_MARK(2);
        // ---- stage 3: copy the records into the ring (aligned qwords only)
        if (live) {
            uint64_t tail = P.tail;
            copy_records<R>(ring, w16, op0, tail, rec, farv, nrec, gen);
            P.tail = tail;
        }

        LPROF_MARK(3);
        // ---- stage 4: the finished lines of all 64 pages, four lanes per line
        const int32_t lend = !live ? 0 : (ended && rv < 0) ? P.fl : (P.op & ~63);
        const int32_t nl = live ? (lend - P.fl) >> 6 : 0;
        const int32_t incl = wave_incl_sum(nl);
        const int32_t total = (int32_t)rdlane((uint32_t)incl, 63);
        if (total > 0) {
            tab_out[lane] = (uint64_t)(uintptr_t)P.out;
            tab_fl[lane] = (uint32_t)P.fl;
            for (int32_t k = 0; k < nl; k++) own[incl - nl + k] = lane | ((uint32_t)k << 8);
            asm volatile("" ::: "memory");
            const uint32_t j = lane & 3u, q = lane >> 2;
            for (int32_t g0 = 0; g0 < total; g0 += 16) {
                const int32_t g = g0 + (int32_t)q;
                if (g < total) {
                    const uint32_t e = own[g];
                    const uint32_t L2 = e & 63u, k = e >> 8;
                    uint8_t *o = (uint8_t *)(uintptr_t)tab_out[L2];
                    const int32_t f = (int32_t)tab_fl[L2] + 64 * (int32_t)k + 16 * (int32_t)j;
                    const u128 v = lds16(smem + Lay::ring + L2 * (uint32_t)Lay::rs + (f & (R - 1)));
                    st16f(o + f, v);
                }
            }
            asm volatile("" ::: "memory");
        }
        if (live) P.fl = lend > P.fl ? lend : P.fl;
        LPROF_MARK(4);
        LPROF_ADD(9, total);
        LPROF_ADD(10, __builtin_popcountll(__builtin_amdgcn_ballot_w64(ended)));

        // ---- stage 5: the page's last bytes; the next page; the next window
        if (ended) {
            if (rv >= 0) {
                // bytes [fl, op): whole 16-byte pieces, then single bytes
                for (int32_t a = P.fl; a < P.op; a += 16) {
                    const u128 v = lds16(ring + (a & (R - 1)));
                    if (a + 16 <= P.op) {
                        st16(P.out + a, v);
                    } else {
                        for (int32_t x = a; x < P.op; x++) st1(P.out + x, (uint32_t)(v >> (8 * (x - a))) & 0xFFu);
                    }
                }
            }
            b.results[P.idx] = rv;
            live = lpage_start(b, in_cap, out_cap, P.idx + G, G, P, w16);
            LPROF_MARK(5);
        } else if (live) {
            P.wb = nwb;
            wstore(w16, nw);
        }
        asm volatile("" ::: "memory");
    }
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
    const long r = knob("LZ4_LC_RING", 256);
    const void *k = r == 512 ? (const void *)lz4_decode_lc_kernel<512> : (const void *)lz4_decode_lc_kernel<256>;
    const size_t lds = r == 512 ? LCL<512>::total : LCL<256>::total;
    const size_t ncu = prepare_launch(k);
    size_t waves = waves_per_cu(k, lds);
    const long env_waves = knob("LZ4_LC_WAVES", 0);
    if (env_waves > 0) waves = std::min<size_t>(waves, (size_t)env_waves);
    const size_t grid = std::min<size_t>((b.count + 63) / 64, ncu * waves);
    void *args[] = {(void *)&b, &in_cap, &out_cap};
    (void)hipLaunchKernel(k, dim3((unsigned)grid), dim3(64), args, lds, s);
    return hipGetLastError();
}

}  // namespace tyche
