// lz4_decode_quad.hip -- LZ4 block decode for large batches, round 4: one page
// per QUAD (4 lanes, 16 pages per wave), decoded in chunks of up to kQN
// sequences (reference: buffer__decompress, src/buffer.c:248-253 ->
// LZ4_decompress_safe, src/lz4/lz4.c:1251; generic decoder lz4.c:1089-1248).
//
// Why not one page per lane (lz4_decode_lane.hip).  That kernel spends most of
// its time waiting: every sequence that reaches further back than its 128-byte
// per-lane ring reads the page's flushed bytes from HBM, and because loads and
// stores share one in-order counter (vmcnt), each such wait also drains the
// line flushes issued before it -- a full memory round trip on most wave
// iterations (timing ablations).  Here the three costs are taken
// apart:
//
//  * history: a quad's page keeps its last H output bytes (H = 512 / 1024,
//    against 128) in an LDS ring, so 69-75 % of the bench pages' sequences copy
//    on chip (oracle parses: 31 % reach further than 512 B, 25 % further
//    than 1 KiB);
//  * chunks: stage 1 parses up to kQN sequences of every page of the wave from
//    a 256-byte LDS window of its stream into 4-byte records (the reference's
//    checks, in its order, on the way); stage 2 issues every far source of the
//    chunk (kQF of them per page, 64 bytes each, straight into LDS with
//    global_load_lds_dwordx4) together with the next chunk's stream window and
//    waits ONCE; stage 3 copies the records LDS to LDS with no global access;
//    stage 4 writes the finished 64-byte lines, one line per quad and store
//    instruction, and no load waits behind those stores until the next chunk's
//    stage 2;
//  * alignment: LDS reads and writes at byte-unaligned addresses replay per
//    lane (~64 cycles per wave instruction, tools/probes/lds_wide.hip, against
//    11-17 aligned), so every LDS access here is a naturally aligned qword:
//    unaligned 8-byte windows are two aligned reads and a funnel shift
//    (v_alignbyte), and a quad writes a run as whole aligned qwords -- lane j
//    takes the j-th qword from the END of a <= 32-byte step, so lane 0 always
//    holds the run's partial last qword (the "tail"), which a quad_perm DPP
//    broadcast hands to the lane that merges it into the next step's first
//    qword.
//
// Sequences the chunk machinery does not take (literal runs that leave the
// stream window, a far match longer than its 64-byte entry, a single sequence
// larger than the chunk's output budget, lengths past the record fields) stop
// the chunk; at the start of a chunk such a sequence goes to a slow path that
// decodes exactly that one sequence straight between HBM buffers (after a full
// flush), then reloads the ring from the page's output.  Results are
// LZ4_decompress_safe's: the decoded size, or -(input bytes consumed)-1 for a
// malformed stream (stream bytes past its end read as zero, as in the other
// decoders); on error the page's destination holds partial output.
#include <hip/hip_runtime.h>

#include "../engine.h"
#include "../lane_ring.h"
#include "../lds_io.h"
#include "../lds_qword.h"

namespace tyche {

// Optional stage profile (diagnostic build only: -DTYCHE_PROFILE, tools/quad_profile.py):
// shader cycles per stage and event counts, summed over waves by lane 0.
#ifdef TYCHE_PROFILE
__device__ unsigned long long g_qprof[16];
#define QPROF_DECL unsigned long long _pt = clock64();
#define QPROF_MARK(k)                                                          \
    do {                                                                       \
        unsigned long long _n = clock64();                                     \
        if (lane == 0) atomicAdd(&g_qprof[k], _n - _pt);                       \
        _pt = _n;                                                              \
    } while (0)
#define QPROF_ADD(k, v) do { if (lane == 0) atomicAdd(&g_qprof[k], (unsigned long long)(v)); } while (0)
#else
#define QPROF_DECL
#define QPROF_MARK(k) do { } while (0)
#define QPROF_ADD(k, v) do { } while (0)
#endif

namespace {

constexpr int32_t kQN = 32;                    // records per chunk and page
constexpr int32_t kSB = 256;                   // stream window bytes
constexpr int32_t kSBStride = kSB + 32;        // + 16 B slack either side
constexpr int32_t kFarEnt = 64;                // bytes per far entry (one quad, 16 B per lane)
constexpr int32_t kFarMaxMl = 42;              // longest far match an entry serves (see stage 3)

// LDS per wave: 16 page slots
template <int32_t H, int32_t F>
struct QL {
    static constexpr uint32_t ring = 0;                                  // 16 x H
    static constexpr uint32_t sbuf = 16u * H;                            // 16 x kSBStride
    static constexpr uint32_t rec = sbuf + 16u * kSBStride;              // 16 x kQN x 4
    static constexpr uint32_t fsrc = rec + 16u * kQN * 4u;               // 16 x F x 4
    static constexpr uint32_t far = fsrc + 16u * (uint32_t)F * 4u;       // F x (16 x 64): one glds per entry index
    static constexpr uint32_t total = far + (uint32_t)F * 16u * kFarEnt;
};

// quad_perm [0,0,0,0]: lane 0 of every quad to its four lanes
__device__ __forceinline__ uint32_t qb0(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t qb0(uint64_t v) {
    return (uint64_t)qb0((uint32_t)v) | ((uint64_t)qb0((uint32_t)(v >> 32)) << 32);
}

// 8 bytes at byte offset p (any alignment, p >= -8) of an 8-aligned LDS buffer
__device__ __forceinline__ uint64_t rd8(const uint8_t *base, int32_t p) {
    const int32_t a = p & ~7;
    return funnel8(lq(base + a), lq(base + a + 8), (uint32_t)p & 7u);
}
// 8 bytes at page position p of a ring of H bytes (p may be negative: wraps)
template <int32_t H>
__device__ __forceinline__ uint64_t ring8(const uint8_t *ring, int32_t p) {
    const int32_t a = p & ~7;
    return funnel8(lq(ring + (a & (H - 1))), lq(ring + ((a + 8) & (H - 1))), (uint32_t)p & 7u);
}
// ---- slow path: one sequence at (ip, op) straight between HBM buffers
// (decode_lane's loop body, lz4_decode_lane.hip), every byte of out below op
// already in HBM.  Lane j of the quad copies the j-th 16 bytes of every 64.
// Returns 0 to continue (ip, op advanced), 1 when the page ended (rv set).
__device__ int32_t slow_sequence(const uint8_t *__restrict__ in, int32_t L, uint8_t *__restrict__ out, int32_t C,
                                 int32_t &ip, int32_t &op, int32_t &rv, uint32_t j) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the quad's flush stores retire before any load of them
    const uint32_t token = sbyte(in, ip, L);
    int32_t lit = (int32_t)(token >> 4);
    int32_t pos = 1;
    if (lit == kRunMask) {
        uint32_t s;
        do {
            s = sbyte(in, ip + pos, L);
            pos++;
            lit += (int32_t)s;
        } while (ip + pos < L - kRunMask && s == 255);
    }
    const bool term = op + lit > C - kMfLimit || ip + pos + lit > L - 8;   // lz4.c:1147-1163
    if (term && (ip + pos + lit != L || op + lit > C)) {
        rv = -(ip + pos) - 1;
        return 1;
    }
    // literals (terminal or not): in + ip + pos -> out + op; all of them inside [0, L) and [0, C)
    {
        const uint8_t *src = in + ip + pos;
        uint8_t *dst = out + op;
        for (int32_t k = 16 * (int32_t)j; k < lit; k += 64) {
            if (k + 16 <= lit) {
                st16(dst + k, ld16(src + k));
            } else {
                for (int32_t x = k; x < lit; x++) st1(dst + x, ld1(src + x));
            }
        }
    }
    if (term) {
        rv = op + lit;
        return 1;
    }
    pos += lit;
    const int32_t off = (int32_t)(sbyte(in, ip + pos, L) | (sbyte(in, ip + pos + 1, L) << 8));
    pos += 2;
    op += lit;
    if (off > op) {   // lz4.c:1168
        rv = -(ip + pos) - 1;
        return 1;
    }
    int32_t ml = (int32_t)(token & 15u);
    if (ml == 15) {
        uint32_t s;
        do {
            s = sbyte(in, ip + pos, L);
            pos++;
            if (ip + pos > L - kLastLiterals) {   // lz4.c:1176
                rv = -(ip + pos) - 1;
                return 1;
            }
            ml += (int32_t)s;
        } while (s == 255);
    }
    ml += kMinMatch;
    if (op + ml > C - kLastLiterals) {   // lz4.c:1225
        rv = -(ip + pos) - 1;
        return 1;
    }
    ip += pos;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the literal's stores (all four lanes) retire first
    // the match: forward byte-copy semantics (lz4.c:1209-1236), lane 0 of the quad
    // (its own stores precede its loads of the same bytes: one wave's vector memory
    // operations are performed in order)
    if (j == 0) {
        uint8_t *dst = out + op;
        const uint8_t *src = dst - off;
        if (off >= 16) {
            int32_t k = 0;
            for (; k + 16 <= ml && op + k + 16 <= C; k += 16) st16(dst + k, ld16(src + k));
            for (; k < ml; k++) st1(dst + k, ld1(src + k));
        } else {
            // period-`off` pattern (offset 0: undefined bytes, zeros here)
            const u128 m = off >= 9 ? ld16(src) : (u128)ld8(src);   // off <= 8: src + 8 <= op + 8 - off
            u128 p = 0;
            int32_t step = 16;
            if (off > 0) p = period_pattern(m, off, step);
            int32_t k = 0;
            for (; k < ml && op + k + 16 <= C; k += step) st16(dst + k, p);
            for (int32_t x = k; x < ml; x++) st1(dst + x, (uint32_t)(p >> (8 * (x - k))) & 0xFFu);
        }
    }
    op += ml;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // before the ring is reloaded from these bytes
    return 0;
}

// bytes [fl, end) of the page from the ring to HBM: whole 16-byte pieces, then
// single bytes; lane j takes pieces j, j + 4, ...  (fl a multiple of 16)
template <int32_t H>
__device__ __forceinline__ void flush_exact(const uint8_t *ring, uint8_t *__restrict__ out, int32_t fl, int32_t end,
                                            uint32_t j) {
    for (int32_t a = fl + 16 * (int32_t)j; a < end; a += 64) {
        const u128 v = lds16(ring + (a & (H - 1)));
        if (a + 16 <= end) {
            st16(out + a, v);
        } else {
            for (int32_t x = a; x < end; x++) st1(out + x, (uint32_t)(v >> (8 * (x - a))) & 0xFFu);
        }
    }
}

// the ring's H bytes below op (and the qword holding op) from the page's output in
// HBM, after the slow path wrote them there; returns the tail qword (bytes
// [op & ~7, op))
template <int32_t H>
__device__ __forceinline__ uint64_t ring_reload(uint8_t *ring, const uint8_t *__restrict__ out, int32_t op, int32_t C,
                                                uint32_t j) {
    const int32_t top = (op + 15) & ~15;
    for (int32_t a = top - H + 16 * (int32_t)j; a < top; a += 64) {
        if (a < 0) continue;
        u128 v;
        if (a + 16 <= C) {
            v = ld16(out + a);
        } else {
            v = 0;
            for (int32_t k = 15; k >= 0; k--) v = (v << 8) | (a + k < op ? ld1(out + a + k) : 0u);
        }
        lds16(ring + (a & (H - 1)), v);
    }
    WAVE_SYNC();
    return lq(ring + ((op & ~7) & (H - 1)));
}

// Per-slot page state (quad-uniform)
struct Page {
    const uint8_t *in;
    uint8_t *out;
    int32_t L, C;
    size_t idx;       // page index in the batch
    int32_t ip, op, fl, sbase;
    uint64_t tail;    // ring qword holding op (bytes below op valid)
};

// the stream window [ns, ns + kSB) into the slot's buffer (synchronous)
__device__ __forceinline__ void window_load(uint8_t *sb, const uint8_t *__restrict__ in, int32_t ns, int32_t L,
                                            uint32_t j) {
#pragma unroll
    for (int32_t c = 0; c < 4; c++) {
        const int32_t k = 16 * ((int32_t)j + 4 * c);
        lds16(sb + 16 + k, chunk16z(in, ns + k, L));
    }
}

// starts the slot on its page `idx` or a later one of its stride: pages with an
// immediate result (empty capacity, empty stream, over the launch's sizing) are
// answered here.  Returns false when the slot has no page left.
__device__ bool page_start(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, size_t idx, size_t G, Page &P,
                           uint8_t *sb, uint32_t j) {
    for (; idx < b.count; idx += G) {
        const PageRef r = batch_page(b, idx);
        int32_t rv;
        if (r.src_len > in_cap || r.dst_cap > out_cap) {
            rv = kResultTooLarge;
        } else if (r.dst_cap == 0) {
            rv = (r.src_len == 1 && ld1(r.src) == 0) ? 0 : -1;
        } else if (r.src_len == 0) {
            rv = -1;
        } else {
            P.in = r.src;
            P.out = r.dst;
            P.L = (int32_t)r.src_len;
            P.C = (int32_t)r.dst_cap;
            P.idx = idx;
            P.ip = P.op = P.fl = P.sbase = 0;
            P.tail = 0;
            window_load(sb, P.in, 0, P.L, j);
            return true;
        }
        if (j == 0) b.results[idx] = rv;
    }
    return false;
}

enum : int32_t { kParse = 0, kCut = 1, kBreak = 2, kEnd = 3, kIdle = 4 };

template <int32_t H, int32_t F>
__global__ __launch_bounds__(64) void lz4_decode_quad_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap) {
    typedef QL<H, F> Lay;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x, slot = lane >> 2, j = lane & 3u;
    uint8_t *ring = smem + Lay::ring + slot * (uint32_t)H;
    uint8_t *sb = smem + Lay::sbuf + slot * (uint32_t)kSBStride;   // stream byte p at sb + 16 + (p - sbase)
    uint8_t *rec = smem + Lay::rec + slot * (uint32_t)kQN * 4u;
    uint8_t *fsrc = smem + Lay::fsrc + slot * (uint32_t)F * 4u;
    const size_t G = (size_t)gridDim.x * 16u;
    constexpr int32_t kBudget = H - 192;   // output bytes per chunk (ring room: see stage 3)
    constexpr int32_t kFarOff = H - 32;    // matches reaching further back read far entries

    Page P;
    bool live = page_start(b, in_cap, out_cap, (size_t)blockIdx.x * 16u + slot, G, P, sb, j);
    WAVE_SYNC();
    QPROF_DECL
    while (__builtin_amdgcn_ballot_w64(live) != 0) {
        QPROF_ADD(0, 1);
        QPROF_MARK(7);
        // ---- stage 1: parse up to kQN sequences from the stream window into records
        int32_t st = live ? kParse : kIdle;
        int32_t nrec = 0, nfar = 0, rv = 0;
        const int32_t ip0 = P.ip, op0 = P.op;
        const int32_t lim = P.sbase + kSB;
        const int32_t sofs = 16 - P.sbase;        // stream byte p at sb + sofs + p (inside the window)
        while (__builtin_amdgcn_ballot_w64(st == kParse) != 0) {
            QPROF_ADD(8, 1);
            if (st != kParse) continue;
            const int32_t ip = P.ip, op = P.op;
            if (nrec == kQN || ip + 16 > lim) {
                st = nrec == 0 ? kBreak : kCut;
                continue;
            }
            const int32_t a0 = ip & ~7;
            const uint64_t wl = lq(sb + (sofs + a0)), wh = lq(sb + (sofs + a0 + 8));
            const uint32_t w0 = (uint32_t)wl, w1 = (uint32_t)(wl >> 32), w2 = (uint32_t)wh, w3 = (uint32_t)(wh >> 32);
            const uint32_t r0 = (uint32_t)(ip - a0);
            const uint32_t token = (sel4(w0, w1, w2, w3, r0 >> 2) >> (8u * (r0 & 3u))) & 0xFFu;
            int32_t lit = (int32_t)(token >> 4);
            int32_t pos = 1;
            bool over = false;
            if (lit == kRunMask) {
                uint32_t s;
                do {
                    if (ip + pos >= lim) {
                        over = true;
                        break;
                    }
                    s = lb(sb + (sofs + ip + pos));
                    pos++;
                    lit += (int32_t)s;
                } while (ip + pos < P.L - kRunMask && s == 255);
            }
            if (over) {
                st = nrec == 0 ? kBreak : kCut;
                continue;
            }
            if (op + lit > P.C - kMfLimit || ip + pos + lit > P.L - 8) {   // lz4.c:1147-1163
                const int32_t ip2 = ip + pos;
                if (ip2 + lit != P.L || op + lit > P.C) {
                    rv = -ip2 - 1;
                    st = kEnd;
                } else if (ip2 + lit > lim - 8 || lit > 255 || op + lit - op0 > kBudget) {
                    st = nrec == 0 ? kBreak : kCut;
                } else {
                    // terminal literal run: the off field holds its window position
                    ld32(rec + 4 * nrec, (uint32_t)(ip2 - P.sbase) | ((uint32_t)lit << 16) | (255u << 24));
                    nrec++;
                    P.op = op + lit;
                    P.ip = ip2 + lit;
                    rv = op + lit;
                    st = kEnd;
                }
                continue;
            }
            if (ip + pos + lit + 2 > lim - 8 || lit > 255) {
                st = nrec == 0 ? kBreak : kCut;
                continue;
            }
            const int32_t ro = ip + pos + lit - a0;   // the offset's bytes: from the window when they lie in it
            uint32_t off;
            if (ro <= 14) {
                const uint32_t q = (uint32_t)ro >> 2;
                const uint32_t lo = sel4(w0, w1, w2, w3, q), hi = q >= 3u ? 0u : sel4(w1, w2, w3, 0u, q);
                off = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)ro & 3u) & 0xFFFFu;
            } else {
                off = lb(sb + (sofs + ip + pos + lit)) | (lb(sb + (sofs + ip + pos + lit + 1)) << 8);
            }
            pos += lit + 2;
            if ((int32_t)off > op + lit) {   // lz4.c:1168
                rv = -(ip + pos) - 1;
                st = kEnd;
                continue;
            }
            int32_t ml = (int32_t)(token & 15u);
            if (ml == 15) {
                uint32_t s;
                bool bad = false;
                do {
                    if (ip + pos >= lim) {
                        over = true;
                        break;
                    }
                    s = lb(sb + (sofs + ip + pos));
                    pos++;
                    if (ip + pos > P.L - kLastLiterals) {   // lz4.c:1176
                        bad = true;
                        break;
                    }
                    ml += (int32_t)s;
                } while (s == 255);
                if (over) {
                    st = nrec == 0 ? kBreak : kCut;
                    continue;
                }
                if (bad) {
                    rv = -(ip + pos) - 1;
                    st = kEnd;
                    continue;
                }
            }
            ml += kMinMatch;
            if (op + lit + ml > P.C - kLastLiterals) {   // lz4.c:1225
                rv = -(ip + pos) - 1;
                st = kEnd;
                continue;
            }
            const bool far = (int32_t)off > kFarOff;
            if (ml > 258 || op + lit + ml - op0 > kBudget || (far && (ml > kFarMaxMl || nfar == F))) {
                st = nrec == 0 ? kBreak : kCut;
                continue;
            }
            if (far) {
                ld32(fsrc + 4 * nfar, (uint32_t)(op + lit - (int32_t)off));
                nfar++;
            }
            ld32(rec + 4 * nrec, off | ((uint32_t)lit << 16) | ((uint32_t)(ml - kMinMatch) << 24));
            nrec++;
            P.op = op + lit + ml;
            P.ip = ip + pos;
        }
        WAVE_SYNC();
        QPROF_MARK(1);

        // ---- stage 2: far sources (flushed lines of the page's output, straight
        // into LDS) and the next chunk's stream window, one wait for all of them
        const bool cont = st == kCut;   // the page goes on with the next chunk from P.ip
        if (st == kEnd && rv < 0) nrec = 0;   // a malformed page: its output is not defined, skip the copies
        const int32_t ns = P.ip & ~7;
        // far sources are lines the quad's lanes stored in earlier chunks: those stores retire first
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u128 pre0 = 0, pre1 = 0, pre2 = 0, pre3 = 0;
        if (cont) {
            pre0 = chunk16z(P.in, ns + 16 * (int32_t)j, P.L);
            pre1 = chunk16z(P.in, ns + 16 * ((int32_t)j + 4), P.L);
            pre2 = chunk16z(P.in, ns + 16 * ((int32_t)j + 8), P.L);
            pre3 = chunk16z(P.in, ns + 16 * ((int32_t)j + 12), P.L);
        }
#pragma unroll
        for (int32_t f = 0; f < F; f++) {
            if (f < nfar) {
                const int32_t src = (int32_t)ld32(fsrc + 4 * f) & ~7;
                const uint8_t *g = P.out + src + 16 * (int32_t)j;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(uintptr_t)g,
                                                 (__attribute__((address_space(3))) void *)(l_u8 *)(smem + Lay::far + (uint32_t)f * 1024u),
                                                 16, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        WAVE_SYNC();
        QPROF_MARK(2);
#ifdef TYCHE_PROFILE
        if (j == 0 && live) {
            atomicAdd(&g_qprof[12], (unsigned long long)nrec);
            atomicAdd(&g_qprof[13], (unsigned long long)nfar);
        }
#endif

        // ---- stage 3: copy the records, LDS to LDS.  A step writes up to 32 bytes
        // [d, d + n) as the aligned qwords ql - j (ql = the last one); a qword that
        // starts below d keeps the tail's bytes there.
        if (live) {
            int32_t d = op0, ipt = ip0, fo = 0;
            uint64_t tail = P.tail;
            const uint8_t *fbase = smem + Lay::far + slot * (uint32_t)kFarEnt;
            for (int32_t t = 0; t < nrec; t++) {
                const uint32_t r = ld32(rec + 4 * t);
                const int32_t off = (int32_t)(r & 0xFFFFu), lit = (int32_t)((r >> 16) & 0xFFu), mc = (int32_t)(r >> 24);
                int32_t lp, ml;
                if (mc == 255) {
                    lp = P.sbase + off;
                    ml = 0;
                } else {
                    lp = ipt + 1 + (lit >= 15 ? 1 : 0);
                    ml = mc + kMinMatch;
                    ipt = lp + lit + 2 + (mc >= 15 ? 1 : 0);
                }
                // literals from the stream window
                {
                    const int32_t sdelta = lp - d;   // stream position - output position
                    for (int32_t rem = lit; rem > 0;) {
                        const int32_t n = min(rem, 32 - (d & 7));
                        const int32_t qf = d >> 3, ql = (d + n - 1) >> 3, q = ql - (int32_t)j;
                        uint64_t v = 0;
                        if (q >= qf) {
                            v = rd8(sb, sofs + 8 * q + sdelta);
                            if (q == qf) v = keep_low(tail, v, (uint32_t)d & 7u);
                            lq(ring + ((8 * q) & (H - 1)), v);
                        }
                        tail = qb0(v);
                        d += n;
                        rem -= n;
                        asm volatile("" ::: "memory");
                    }
                }
                if (ml == 0) continue;
                const bool far = off > kFarOff;
                const bool pat = !far && off < 32 && off < ml;
                const int32_t dm = d;
                const uint8_t *fe = fbase + (uint32_t)fo * 1024u;
                const int32_t e0 = (dm - off) & ~7;
                if (far) fo++;
                u128 p16 = 0;   // pattern, off < 8: the off bytes below dm repeated over 16 bytes
                if (pat && off > 0 && off < 8) {
                    u128 p = (u128)(ring8<H>(ring, dm - off) & ((1ull << (8 * off)) - 1ull));
                    for (int32_t len = off; len < 16; len <<= 1) p |= p << (8 * len);
                    p16 = p;
                }
                for (int32_t rem = ml; rem > 0;) {
                    const int32_t n = min(rem, 32 - (d & 7));
                    const int32_t qf = d >> 3, ql = (d + n - 1) >> 3, q = ql - (int32_t)j;
                    uint64_t v = 0;
                    if (q >= qf) {
                        const int32_t x0 = 8 * q;
                        if (far) {
                            v = rd8(fe, x0 - off - e0);
                        } else if (!pat) {
                            v = ring8<H>(ring, x0 - off);
                        } else {
                            // period-off pattern of the bytes [dm - off, dm): byte x = P[(x - dm) mod off]
                            // (offset 0, a malformed stream the reference accepts: undefined bytes, zeros here)
                            const uint32_t ph = off > 0 ? mod_small((uint32_t)(x0 - dm + 8 * off), (uint32_t)off) : 0u;
                            if (off == 0) {
                                v = 0;
                            } else if (off >= 8) {
                                const uint64_t A = ring8<H>(ring, dm - off + (int32_t)ph);
                                const uint32_t k = (uint32_t)off - ph;   // bytes of A before the period wraps
                                if (k >= 8) {
                                    v = A;
                                } else {
                                    const uint64_t B = ring8<H>(ring, dm - off);
                                    v = keep_low(A, B << (8 * k), k);
                                }
                            } else {
                                v = (uint64_t)(p16 >> (8 * ph));   // ph < off < 8: inside the 16 bytes
                            }
                        }
                        if (q == qf) v = keep_low(tail, v, (uint32_t)d & 7u);
                        lq(ring + ((8 * q) & (H - 1)), v);
                    }
                    tail = qb0(v);
                    d += n;
                    rem -= n;
                    asm volatile("" ::: "memory");
                }
            }
            P.tail = tail;
        }
        WAVE_SYNC();
        QPROF_MARK(3);

        // ---- stage 4: whole lines to HBM; a page that ended: every byte up to its end
        if (live) {
            const int32_t end = st == kEnd ? (rv >= 0 ? P.op : P.fl) : (P.op & ~63);
            int32_t fl = P.fl;
            for (; fl + 64 <= end; fl += 64) {
                const u128 v = lds16(ring + ((fl + 16 * (int32_t)j) & (H - 1)));
                st16f(P.out + fl + 16 * (int32_t)j, v);
            }
            if (st == kEnd && rv >= 0) {
                flush_exact<H>(ring, P.out, fl, end, j);
                fl = end;
            } else if (st == kBreak) {
                // the slow path works from HBM: every byte below op goes out now
                flush_exact<H>(ring, P.out, fl, P.op, j);
            }
            P.fl = fl;
        }
        QPROF_MARK(4);
        QPROF_ADD(10, __builtin_popcountll(__builtin_amdgcn_ballot_w64(j == 0 && live && st == kBreak)));
        QPROF_ADD(11, __builtin_popcountll(__builtin_amdgcn_ballot_w64(j == 0 && live && st == kEnd)));

        // ---- stage 5: the next chunk's window; a sequence the chunks do not take; the next page
        if (live && st == kBreak) {
            int32_t ip = P.ip, op = P.op, r2 = 0;
            const int32_t done = slow_sequence(P.in, P.L, P.out, P.C, ip, op, r2, j);
            if (done) {
                st = kEnd;
                rv = r2;
            } else {
                P.ip = ip;
                P.op = op;
                P.fl = op & ~63;
                P.tail = ring_reload<H>(ring, P.out, op, P.C, j);
                P.sbase = ip & ~7;
                window_load(sb, P.in, P.sbase, P.L, j);
            }
        }
        QPROF_MARK(5);
        if (live && st == kEnd) {
            if (j == 0) b.results[P.idx] = rv;
            live = page_start(b, in_cap, out_cap, P.idx + G, G, P, sb, j);
            QPROF_MARK(6);
        } else if (cont) {
            P.sbase = ns;
            lds16(sb + 16 + 16 * (int32_t)j, pre0);
            lds16(sb + 16 + 16 * ((int32_t)j + 4), pre1);
            lds16(sb + 16 + 16 * ((int32_t)j + 8), pre2);
            lds16(sb + 16 + 16 * ((int32_t)j + 12), pre3);
        }
        WAVE_SYNC();
    }
}

}  // namespace

#ifdef TYCHE_PROFILE
extern "C" int tyche_debug_quad_profile(unsigned long long *host16, int reset) {
    if (reset) {
        unsigned long long z[16] = {0};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_qprof), z, sizeof(z)) == hipSuccess ? 0 : 1;
    }
    return hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_qprof), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : 1;
}
#endif

// 1M x 16 KiB bench pages: H / F / waves per CU chosen by A/B
hipError_t launch_lz4_decode_quad(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    const long h = knob("LZ4_QUAD_RING", 1024);
    const long f = knob("LZ4_QUAD_FAR", 8);
    const void *k;
    size_t lds;
    if (h == 512 && f == 6) {
        k = (const void *)lz4_decode_quad_kernel<512, 6>;
        lds = QL<512, 6>::total;
    } else if (h == 512) {
        k = (const void *)lz4_decode_quad_kernel<512, 8>;
        lds = QL<512, 8>::total;
    } else if (h == 2048) {
        k = (const void *)lz4_decode_quad_kernel<2048, 8>;
        lds = QL<2048, 8>::total;
    } else if (f == 6) {
        k = (const void *)lz4_decode_quad_kernel<1024, 6>;
        lds = QL<1024, 6>::total;
    } else {
        k = (const void *)lz4_decode_quad_kernel<1024, 8>;
        lds = QL<1024, 8>::total;
    }
    const size_t ncu = prepare_launch(k);
    size_t waves = waves_per_cu(k, lds);
    const long env_waves = knob("LZ4_QUAD_WAVES", 0);
    if (env_waves > 0) waves = std::min<size_t>(waves, (size_t)env_waves);
    const size_t grid = std::min<size_t>((b.count + 15) / 16, ncu * waves);
    void *args[] = {(void *)&b, &in_cap, &out_cap};
    (void)hipLaunchKernel(k, dim3((unsigned)grid), dim3(64), args, lds, s);
    return hipGetLastError();
}

}  // namespace tyche
