// legacy/lz4_decode_lane_legacy.hip -- the superseded large-batch LZ4 decoders of rounds 2-3
// (lane per page straight from HBM; LDS ring; line-buffered ring), kept for A/B timing only.
// Built into libtyche_codec_legacy_decoders.so (_build.build(legacy=True)); the product
// library does not compile this file (tests/test_legacy_decoders.py runs it).
//
// page per LANE (64 pages per wave), read straight from the compressed stream
// in HBM (reference path: buffer__decompress, src/buffer.c:248-253 ->
// LZ4_decompress_safe, src/lz4/lz4.c:1251, generic decoder lz4.c:1089-1248).
//
// The wave-per-page decoder (lz4_decode.hip) spends ~40 k wave instructions per
// 16 KiB page reconstructing LZ4's two serial chains (token chain, match
// dependencies) in parallel.  A lane that simply runs the reference's
// sequential loop (restated in decode_page_serial) issues ~50 instructions per
// sequence, and with 64 pages per wave that is ~1/20th of the instruction
// stream; the cost moves to memory latency, which a batch of >= 32K pages
// hides (launch_lz4_decode switches at kLaneMin).
//
// Two kernels:
//  * lz4_decode_ring_kernel (default): the page is assembled in a per-lane LDS
//    ring of its last kRing output bytes and leaves for HBM in aligned whole
//    64-byte lines; near matches read the ring, far ones the page's flushed
//    lines in HBM.  One 16-byte stream window per sequence, loaded before the
//    current sequence's copies.
//  * lz4_decode_lane_kernel (TYCHE_LZ4_LANE_RING=0, the A/B baseline): copies
//    16 bytes per access straight between HBM buffers, "wild" past a
//    sequence's end as lz4.c's LZ4_wildCopy but never past the capacity C.  A
//    lane's store followed by its own load of the same address returns the
//    stored value (one wave's vector memory operations are performed in order),
//    which overlapping forward copies rely on.
// Both expand self-overlapping matches with offset < 16 (offset 1 = a run) in
// registers to a 16-byte pattern of period `offset`, stored with a stride that
// is a multiple of the offset.
//
// Results are LZ4_decompress_safe's, checks in the reference's order: the
// decoded size, or -(input bytes consumed)-1 for a malformed stream (the
// stream is read as if padded with zero bytes, like the staged stream of the
// wave decoder; the reference reads the same positions).  On error the page's
#include <hip/hip_runtime.h>

#include "../engine.h"
#include "../lane_ring.h"
#include "../lds_io.h"

#include <algorithm>
#include <cstdlib>

#ifndef TYCHE_ABLATE
#define TYCHE_ABLATE 0   // timing-only bits: 64 far matches read the ring, 256 parse only (wrong output)
#endif

namespace tyche {

namespace {

// 32-byte stream window at ip, zero past L (windowN<16> below is the default
// 16-byte one).  The parse of a sequence reads its token, length bytes, short
// literals and offset from the window; the next sequence's window is loaded
// before the current one's copies, so one load latency per sequence sits on
// the serial chain.
struct Win {
    u128 lo, hi;
};
__device__ __forceinline__ Win shr256(Win w, int32_t n) {   // by n bytes, 0 <= n < 32
    Win r;
    if (n >= 16) {
        r.lo = w.hi >> (8 * (n - 16));
        r.hi = 0;
    } else if (n > 0) {
        r.lo = (w.lo >> (8 * n)) | (w.hi << (128 - 8 * n));
        r.hi = w.hi >> (8 * n);
    } else {
        r = w;
    }
    return r;
}
__device__ __forceinline__ Win window(const uint8_t *__restrict__ in, int32_t ip, int32_t L) {
    Win w;
    if (ip + 32 <= L) {
        w.lo = ld16(in + ip);
        w.hi = ld16(in + ip + 16);
        return w;
    }
    if (L >= 32) {
        w.lo = ld16(in + L - 32);
        w.hi = ld16(in + L - 16);
        return shr256(w, ip - (L - 32));
    }
    w.lo = 0;
    w.hi = 0;
    for (int32_t j = L - 1; j >= ip; j--) {
        w.hi = (w.hi << 8) | (w.lo >> 120);
        w.lo = (w.lo << 8) | ld1(in + j);
    }
    return w;
}
__device__ __forceinline__ uint32_t byte_at(const uint8_t *__restrict__ in, int32_t ip, int32_t L) {
    return ip < L ? ld1(in + ip) : 0u;
}
// byte ip + rel of the stream (zero past L): from the window when rel < 32
__device__ __forceinline__ uint32_t getb(const Win &w, const uint8_t *__restrict__ in, int32_t ip, int32_t rel,
                                         int32_t L) {
    if (rel < 16) return (uint32_t)(w.lo >> (8 * rel)) & 0xFFu;
    if (rel < 32) return (uint32_t)(w.hi >> (8 * (rel - 16))) & 0xFFu;
    return byte_at(in, ip + rel, L);
}

// n bytes from src to dst; room: bytes writable at dst, avail: readable at src
__device__ __forceinline__ void copy_run(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, int32_t n,
                                         int32_t room, int32_t avail) {
    int32_t k = 0;
    for (; k < n; k += 16) {
        if (k + 16 > room || k + 16 > avail) break;
        st16(dst + k, ld16(src + k));
    }
    for (; k < n; k++) st1(dst + k, ld1(src + k));
}

// Decode one page: LZ4_decompress_safe(in, out, L, C), as decode_page_serial.
__device__ int32_t decode_lane(const uint8_t *__restrict__ in, int32_t L, uint8_t *__restrict__ out, int32_t C) {
    if (C == 0) return (L == 1 && ld1(in) == 0) ? 0 : -1;
    if (L <= 0) return -1;
    int32_t ip = 0, op = 0;
    Win w = window(in, 0, L);
    for (;;) {
        const uint32_t token = (uint32_t)w.lo & 0xFFu;
        int32_t lit = (int32_t)(token >> 4);
        int32_t pos = 1;   // stream position relative to ip
        if (lit == kRunMask) {
            uint32_t s;
            do {
                s = getb(w, in, ip, pos, L);
                pos++;
                lit += (int32_t)s;
            } while (ip + pos < L - kRunMask && s == 255);
        }
        // terminal literal run, or error (lz4.c:1147-1163)
        if (op + lit > C - kMfLimit || ip + pos + lit > L - 8) {
            ip += pos;
            if (ip + lit != L || op + lit > C) return -ip - 1;
            copy_run(out + op, in + ip, lit, C - op, L - ip);
            return op + lit;
        }
        // literals: from the window when short (pos <= 2 then), else from HBM
        if (lit <= 16 && op + 16 <= C) {
            st16(out + op, shr256(w, pos).lo);
        } else {
            copy_run(out + op, in + ip + pos, lit, C - op, L - ip - pos);
        }
        pos += lit;
        const int32_t off = (int32_t)(getb(w, in, ip, pos, L) | (getb(w, in, ip, pos + 1, L) << 8));
        pos += 2;
        op += lit;
        if (off > op) return -(ip + pos) - 1;                   // lz4.c:1168
        int32_t ml = (int32_t)(token & 15u);
        if (ml == 15) {
            uint32_t s;
            do {
                s = getb(w, in, ip, pos, L);
                pos++;
                if (ip + pos > L - kLastLiterals) return -(ip + pos) - 1;   // lz4.c:1176
                ml += (int32_t)s;
            } while (s == 255);
        }
        ml += kMinMatch;
        if (op + ml > C - kLastLiterals) return -(ip + pos) - 1;   // lz4.c:1225
        uint8_t *dst = out + op;
        const uint8_t *src = dst - off;
        // first source chunk (after the literal store: it may overlap it), then
        // the next window, then the copy
        u128 m = off <= 8 ? (u128)ld8(src) : ld16(src);   // off >= 9: src + 16 <= op + 7 <= C; else src + 8 <= op + 8 - off
        ip += pos;
        w = window(in, ip, L);
        if (off >= 16) {
            // every 16-byte source chunk ends at or before its destination
            int32_t k = 0;
            if (op + 16 <= C) {
                st16(dst, m);
                for (k = 16; k < ml; k += 16) {
                    if (op + k + 16 > C) break;
                    st16(dst + k, ld16(src + k));
                }
            }
            for (; k < ml; k++) st1(dst + k, ld1(src + k));
        } else {
            // period-`off` pattern of the off final bytes before dst, doubled
            // (offset 0 passes the reference's checks and copies dst onto
            // itself -- undefined bytes; zeros here, and no endless doubling)
            u128 p = 0;
            int32_t step = 16;
            if (off > 0) {
                p = m & ((((u128)1) << (8 * off)) - 1);
                for (int32_t len = off; len < 16; len <<= 1) p |= p << (8 * len);
                step = 16 - (int32_t)mod_small(16u, (uint32_t)off);   // largest multiple of off <= 16
            }
            int32_t k = 0;
            for (; k < ml; k += step) {
                if (op + k + 16 > C) break;
                st16(dst + k, p);
            }
            for (int32_t j = k; j < ml; j++) st1(dst + j, (uint32_t)(p >> (8 * (j - k))) & 0xFFu);
        }
        op += ml;
    }
}

// ---- ring variant: the page's output is assembled in a per-lane LDS ring of
// the last kRing bytes and leaves for HBM only in whole 64-byte lines.
//
// Writing the page straight to HBM 16 bytes at a time (decode_lane) leaves
// every line partially written for ~10 sequences; with 256 pages in flight per
// CU the L2 evicts most of them half-full (PMC: 79 KiB written and ~1,000 L2
// misses per 16 KiB page).  Here the stores to HBM are aligned full lines
// written once, and matches whose source lies in the ring (70 % of them on the
// bench pages: offset <= kRing - 32) never touch HBM; the others read the
// page's already-flushed bytes back from HBM.
// kRing: ring bytes per lane (a multiple of 16); stride adds 16 B front slack and
// 32 B tail slack; offsets up to kRing - 32 read the ring (lane_ring.h)
__device__ __forceinline__ u128 stream16(const uint8_t *__restrict__ in, int32_t a, int32_t L) {
    return a + 16 <= L ? ld16(in + a) : window(in, a, L).lo;
}

// LZ4_decompress_safe(in, out, L, C) through the ring rb (as decode_lane)
// kWin = 16: one 16-byte load per sequence (covers the token, literals and
// offset of all but ~1 % of sequences; the rest read single bytes)
template <int32_t kWin>
__device__ __forceinline__ Win windowN(const uint8_t *__restrict__ in, int32_t ip, int32_t L) {
    if (kWin == 32) return window(in, ip, L);
    Win w;
    w.hi = 0;
    if (ip + 16 <= L) {
        w.lo = ld16s(in + ip);
    } else if (L >= 16) {
        w.lo = ld16s(in + L - 16) >> (8 * (ip - (L - 16)));
    } else {
        w.lo = 0;
        for (int32_t j = L - 1; j >= ip; j--) w.lo = (w.lo << 8) | ld1(in + j);
    }
    return w;
}
template <int32_t kWin>
__device__ __forceinline__ uint32_t getbN(const Win &w, const uint8_t *__restrict__ in, int32_t ip, int32_t rel,
                                          int32_t L) {
    if (kWin == 32) return getb(w, in, ip, rel, L);
    if (rel < 16) return (uint32_t)(w.lo >> (8 * rel)) & 0xFFu;
    return byte_at(in, ip + rel, L);
}

template <int32_t kRing, int32_t kWin>
__device__ int32_t decode_ring(const uint8_t *__restrict__ in, int32_t L, uint8_t *__restrict__ out, int32_t C,
                               uint8_t *rb) {
    if (C == 0) return (L == 1 && ld1(in) == 0) ? 0 : -1;
    if (L <= 0) return -1;
    int32_t ip = 0, op = 0, fl = 0;   // fl: bytes of the page already in HBM
    Win w = windowN<kWin>(in, 0, L);
    for (;;) {
        const uint32_t token = (uint32_t)w.lo & 0xFFu;
        int32_t lit = (int32_t)(token >> 4);
        int32_t pos = 1;
        if (lit == kRunMask) {
            uint32_t s;
            do {
                s = getbN<kWin>(w, in, ip, pos, L);
                pos++;
                lit += (int32_t)s;
            } while (ip + pos < L - kRunMask && s == 255);
        }
        if (op + lit > C - kMfLimit || ip + pos + lit > L - 8) {   // lz4.c:1147-1163
            ip += pos;
            if (ip + lit != L || op + lit > C) return -ip - 1;
            ring_flush_all<kRing>(rb, out, fl, op);
            copy_run(out + op, in + ip, lit, C - op, L - ip);
            return op + lit;
        }
        if (kWin == 32 ? lit <= 16 : pos + lit <= 16) {
            ring_wr<kRing>(rb, op, shr256(w, pos).lo);
        } else {
            for (int32_t k = 0; k < lit; k += 16) {
                ring_wr<kRing>(rb, op + k, stream16(in, ip + pos + k, L));
                ring_flush<kRing>(rb, out, fl, op + min(k + 16, lit));
            }
        }
        pos += lit;
        const int32_t off = (int32_t)(getbN<kWin>(w, in, ip, pos, L) | (getbN<kWin>(w, in, ip, pos + 1, L) << 8));
        pos += 2;
        op += lit;
        if (off > op) return -(ip + pos) - 1;                   // lz4.c:1168
        int32_t ml = (int32_t)(token & 15u);
        if (ml == 15) {
            uint32_t s;
            do {
                s = getbN<kWin>(w, in, ip, pos, L);
                pos++;
                if (ip + pos > L - kLastLiterals) return -(ip + pos) - 1;   // lz4.c:1176
                ml += (int32_t)s;
            } while (s == 255);
        }
        ml += kMinMatch;
        if (op + ml > C - kLastLiterals) return -(ip + pos) - 1;   // lz4.c:1225
        // the unflushed tail is < kLine + 16 bytes here and the ring holds every
        // position above op + 16 - kRing, so a source at offset > kRing - 32
        // (>= 96) is already in HBM and a nearer one is in the ring
        const bool far = (TYCHE_ABLATE & (64 | 256)) ? false : off > kRing - 32;   // 64: timing only (far matches read the ring: wrong output)
        u128 m = far ? ld16(out + op - off) : (TYCHE_ABLATE & 256) ? (u128)0 : ring_rd<kRing>(rb, op - off);
        ip += pos;
        w = windowN<kWin>(in, ip, L);
        if (off >= 16) {
            ring_wr<kRing>(rb, op, m);
            for (int32_t k = 16; k < ml; k += 16) {
                ring_flush<kRing>(rb, out, fl, op + k);
                m = far ? ld16(out + op + k - off) : (TYCHE_ABLATE & 256) ? (u128)0 : ring_rd<kRing>(rb, op + k - off);
                ring_wr<kRing>(rb, op + k, m);
            }
        } else {
            // period-`off` pattern (offset 0: undefined bytes, zeros here)
            u128 p = 0;
            int32_t step = 16;
            if (off > 0) {
                p = m & ((((u128)1) << (8 * off)) - 1);
                for (int32_t len = off; len < 16; len <<= 1) p |= p << (8 * len);
                step = 16 - (int32_t)mod_small(16u, (uint32_t)off);
            }
            for (int32_t k = 0; k < ml; k += step) {
                ring_flush<kRing>(rb, out, fl, op + k);
                ring_wr<kRing>(rb, op + k, p);
            }
        }
        op += ml;
        ring_flush<kRing>(rb, out, fl, op);
    }
}

// ---- round 3: the stream through a per-lane line buffer.
//
// decode_ring reads one unaligned 16-byte window straight from HBM per
// sequence: with 512 lanes per CU each walking its own stream, a lane's line
// is evicted between its windows (the calibration probe's "seq16" pattern
// fetches every line 2.3x) and every sequence waits on a global load.  Here
// the stream is fetched in whole aligned 64-byte lines (four 16-byte loads
// issued together: one L2 miss per line) one line ahead of the parse, and
// stored into a per-lane LDS window sb of 80 bytes = stream bytes
// [lb - 16, lb + 64) (zero outside [0, L)); a sequence's window is one LDS
// read.  Only far matches (and long literal runs / length bytes past the
// window) still read HBM on the serial chain.

// bytes [a, a + 16) of the stream, zero outside [0, L); never reads outside it
__device__ __forceinline__ u128 chunk16z(const uint8_t *__restrict__ in, int32_t a, int32_t L) {
    if (a >= L || a + 16 <= 0) return 0;
    if (a >= 0 && a + 16 <= L) return ld16(in + a);
    if (L >= 16) {
        if (a < 0) return ld16(in) << (8 * (-a));                   // a + 16 < 16 <= L
        return ld16(in + L - 16) >> (8 * (a - (L - 16)));          // 0 < a - (L - 16) < 16
    }
    u128 v = 0;
    for (int32_t j = 15; j >= 0; j--) {
        const int32_t x = a + j;
        v = (v << 8) | ((x >= 0 && x < L) ? ld1(in + x) : 0u);
    }
    return v;
}
struct Line {
    u128 c[4];
};
__device__ __forceinline__ Line line_load(const uint8_t *__restrict__ in, int32_t a, int32_t L) {
    Line l;
    if (a >= 0 && a + 64 <= L) {
#pragma unroll
        for (int32_t j = 0; j < 4; j++) l.c[j] = ld16(in + a + 16 * j);
    } else {
#pragma unroll
        for (int32_t j = 0; j < 4; j++) l.c[j] = chunk16z(in, a + 16 * j, L);
    }
    return l;
}
struct LineBuf {
    uint8_t *sb;    // 80 LDS bytes: stream [lb - 16, lb + 64)
    int32_t lb;     // stream position of the buffered line (in + lb is 64-byte aligned)
    int32_t ofs;    // (uintptr_t)in & 63
    u128 tail;      // stream [lb + 48, lb + 64): the next window's front slack
    Line pre;       // stream [lb + 64, lb + 128), in flight
};
__device__ __forceinline__ void lb_store(const LineBuf &s, u128 front, const Line &l) {
    lds16(s.sb, front);
#pragma unroll
    for (int32_t j = 0; j < 4; j++) lds16(s.sb + 16 + 16 * j, l.c[j]);
}
__device__ __forceinline__ void lb_init(LineBuf &s, const uint8_t *__restrict__ in, int32_t L, uint8_t *sb) {
    s.sb = sb;
    s.ofs = (int32_t)((uintptr_t)in & 63u);
    s.lb = -s.ofs;
    const Line l = line_load(in, s.lb, L);
    lb_store(s, 0, l);
    s.tail = l.c[3];
    s.pre = line_load(in, s.lb + 64, L);
}
// make [ip, ip + 16) readable from sb (ip >= lb - 16 holds: ip never decreases)
__device__ __forceinline__ void lb_reach(LineBuf &s, const uint8_t *__restrict__ in, int32_t ip, int32_t L) {
    if (ip <= s.lb + 48) return;
    if (ip <= s.lb + 112) {   // the next line, already in flight
        lb_store(s, s.tail, s.pre);
        s.tail = s.pre.c[3];
        s.lb += 64;
        s.pre = line_load(in, s.lb + 64, L);
        return;
    }
    // a long literal run jumped past it: reload around ip
    int32_t nl = ((ip + s.ofs) & ~63) - s.ofs;
    if (ip > nl + 48) nl += 64;
    const u128 front = chunk16z(in, nl - 16, L);
    const Line l = line_load(in, nl, L);
    lb_store(s, front, l);
    s.tail = l.c[3];
    s.lb = nl;
    s.pre = line_load(in, nl + 64, L);
}
__device__ __forceinline__ u128 lb_window(const LineBuf &s, int32_t ip) { return lds16(s.sb + (ip - s.lb + 16)); }

template <int32_t kRing>
__device__ __forceinline__ int32_t decode_ring_lb(const uint8_t *__restrict__ in, int32_t L, uint8_t *__restrict__ out, int32_t C,
                                  uint8_t *rb, uint8_t *sb) {
    if (C == 0) return (L == 1 && ld1(in) == 0) ? 0 : -1;
    if (L <= 0) return -1;
    int32_t ip = 0, op = 0, fl = 0;   // fl: bytes of the page already in HBM
    LineBuf s;
    lb_init(s, in, L, sb);
    lb_reach(s, in, 0, L);   // a page starting late in its 64-byte line
    Win w;
    w.hi = 0;
    w.lo = lb_window(s, 0);
    for (;;) {
        const uint32_t token = (uint32_t)w.lo & 0xFFu;
        int32_t lit = (int32_t)(token >> 4);
        int32_t pos = 1;
        if (lit == kRunMask) {
            uint32_t b;
            do {
                b = getbN<16>(w, in, ip, pos, L);
                pos++;
                lit += (int32_t)b;
            } while (ip + pos < L - kRunMask && b == 255);
        }
        if (op + lit > C - kMfLimit || ip + pos + lit > L - 8) {   // lz4.c:1147-1163
            ip += pos;
            if (ip + lit != L || op + lit > C) return -ip - 1;
            ring_flush_all<kRing>(rb, out, fl, op);
            copy_run(out + op, in + ip, lit, C - op, L - ip);
            return op + lit;
        }
        if (pos + lit <= 16) {
            ring_wr<kRing>(rb, op, w.lo >> (8 * pos));
        } else if (ip + pos + ((lit - 1) & ~15) <= s.lb + 48) {
            // a longer run that the line buffer still holds (every 16-byte read inside it): LDS reads,
            // no HBM round trip per 16 bytes
            for (int32_t k = 0; k < lit; k += 16) {
                ring_wr<kRing>(rb, op + k, lb_window(s, ip + pos + k));
                ring_flush<kRing>(rb, out, fl, op + min(k + 16, lit));
            }
        } else {
            for (int32_t k = 0; k < lit; k += 16) {
                ring_wr<kRing>(rb, op + k, stream16(in, ip + pos + k, L));
                ring_flush<kRing>(rb, out, fl, op + min(k + 16, lit));
            }
        }
        pos += lit;
        const int32_t off = (int32_t)(getbN<16>(w, in, ip, pos, L) | (getbN<16>(w, in, ip, pos + 1, L) << 8));
        pos += 2;
        op += lit;
        if (off > op) return -(ip + pos) - 1;                   // lz4.c:1168
        int32_t ml = (int32_t)(token & 15u);
        if (ml == 15) {
            uint32_t b;
            do {
                b = getbN<16>(w, in, ip, pos, L);
                pos++;
                if (ip + pos > L - kLastLiterals) return -(ip + pos) - 1;   // lz4.c:1176
                ml += (int32_t)b;
            } while (b == 255);
        }
        ml += kMinMatch;
        if (op + ml > C - kLastLiterals) return -(ip + pos) - 1;   // lz4.c:1225
        // as decode_ring: far sources are already in HBM (64: timing-only ablation, far reads from the ring).
        // (Round 3 tried fetching a far match's first 64 bytes together instead of one 16-byte load per
        // step: 36.7 vs 33.5 ms per 1M pages -- the loads' count, not their latency, is what costs.)
        const bool far = (TYCHE_ABLATE & (64 | 256)) ? false : off > kRing - 32;
        u128 m = far ? ld16(out + op - off) : (TYCHE_ABLATE & 256) ? (u128)0 : ring_rd<kRing>(rb, op - off);
        ip += pos;
        lb_reach(s, in, ip, L);
        w.lo = lb_window(s, ip);
        if (off >= 16) {
            ring_wr<kRing>(rb, op, m);
            for (int32_t k = 16; k < ml; k += 16) {
                ring_flush<kRing>(rb, out, fl, op + k);
                m = far ? ld16(out + op + k - off) : (TYCHE_ABLATE & 256) ? (u128)0 : ring_rd<kRing>(rb, op + k - off);
                ring_wr<kRing>(rb, op + k, m);
            }
        } else {
            u128 p = 0;
            int32_t step = 16;
            if (off > 0) {
                p = m & ((((u128)1) << (8 * off)) - 1);
                for (int32_t len = off; len < 16; len <<= 1) p |= p << (8 * len);
                step = 16 - (int32_t)mod_small(16u, (uint32_t)off);
            }
            for (int32_t k = 0; k < ml; k += step) {
                ring_flush<kRing>(rb, out, fl, op + k);
                ring_wr<kRing>(rb, op + k, p);
            }
        }
        op += ml;
        ring_flush<kRing>(rb, out, fl, op);
    }
}

template <int32_t kRing>
__global__ __launch_bounds__(64) void lz4_decode_ringlb_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap,
                                                               unsigned *ctr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *rb = smem + threadIdx.x * (kRing + 48) + 16;
    uint8_t *sb = smem + 64 * (kRing + 48) + threadIdx.x * 80;
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    size_t page = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    while (page < b.count) {
        const uint64_t so = b.src_offsets ? b.src_offsets[page] : (uint64_t)page * b.src_stride;
        const uint64_t dof = b.dst_offsets ? b.dst_offsets[page] : (uint64_t)page * b.dst_stride;
        const uint32_t L = b.src_lengths ? b.src_lengths[page] : b.src_length;
        const uint32_t C = b.dst_capacities ? b.dst_capacities[page] : b.dst_capacity;
        int32_t rv;
        if (L > in_cap || C > out_cap) {
            rv = kResultTooLarge;
        } else {
            rv = decode_ring_lb<kRing>((const uint8_t *)b.src + so, (int32_t)L, (uint8_t *)b.dst + dof, (int32_t)C, rb,
                                       sb);
        }
        b.results[page] = rv;
        page = (size_t)atomicAdd(ctr, 1u) + nthreads;
    }
}

template <int32_t kRing, int32_t kWin>
__global__ __launch_bounds__(64) void lz4_decode_ring_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap,
                                                             unsigned *ctr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *rb = smem + threadIdx.x * (kRing + 48) + 16;
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    size_t page = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    while (page < b.count) {
        const uint64_t so = b.src_offsets ? b.src_offsets[page] : (uint64_t)page * b.src_stride;
        const uint64_t dof = b.dst_offsets ? b.dst_offsets[page] : (uint64_t)page * b.dst_stride;
        const uint32_t L = b.src_lengths ? b.src_lengths[page] : b.src_length;
        const uint32_t C = b.dst_capacities ? b.dst_capacities[page] : b.dst_capacity;
        int32_t rv;
        if (L > in_cap || C > out_cap) {
            rv = kResultTooLarge;
        } else {
            rv = decode_ring<kRing, kWin>((const uint8_t *)b.src + so, (int32_t)L, (uint8_t *)b.dst + dof, (int32_t)C, rb);
        }
        b.results[page] = rv;
        page = (size_t)atomicAdd(ctr, 1u) + nthreads;
    }
}

// Pages are claimed per lane: lane g starts at page g, then takes the next
// unclaimed one from the launch's counter (engine.h: WorkCounter).
__global__ __launch_bounds__(64) void lz4_decode_lane_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap,
                                                              unsigned *ctr) {
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    size_t page = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    while (page < b.count) {
        const uint64_t so = b.src_offsets ? b.src_offsets[page] : (uint64_t)page * b.src_stride;
        const uint64_t dof = b.dst_offsets ? b.dst_offsets[page] : (uint64_t)page * b.dst_stride;
        const uint32_t L = b.src_lengths ? b.src_lengths[page] : b.src_length;
        const uint32_t C = b.dst_capacities ? b.dst_capacities[page] : b.dst_capacity;
        int32_t rv;
        if (L > in_cap || C > out_cap) {
            rv = kResultTooLarge;
        } else {
            rv = decode_lane((const uint8_t *)b.src + so, (int32_t)L, (uint8_t *)b.dst + dof, (int32_t)C);
        }
        b.results[page] = rv;
        page = (size_t)atomicAdd(ctr, 1u) + nthreads;
    }
}

}  // namespace

// ring-less kernel: resident waves per CU (1M x 16 KiB pages, ms: 4 waves 80.8, 8: 92.1, 2: 97.7)
constexpr size_t kLaneWaves = 4;
// ring bytes per lane (0: the ring-less kernel; a 208-byte ring, 10 waves per
// CU, ran 34.7 ms per 1M pages vs 34.5 at 256 bytes and 8 waves)
constexpr int kDefaultRing = 256;
// stream window bytes per sequence (16 or 32; 1M x 16 KiB pages at 256-byte rings: 34.2 / 37.8 ms)
constexpr int kDefaultWin = 16;

hipError_t launch_lz4_decode_lane_legacy(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    if (knob("LZ4_QUAD", 0) != 0) return launch_lz4_decode_quad(b, in_cap, out_cap, s);
    // round 4 default: the chunked lane decoder (lz4_decode_lc.hip; 24.1 ms per 1M x 16 KiB pages
    // vs 32.7 for the line-buffered ring kernel below, which TYCHE_LZ4_LC=0 selects)
    if (knob("LZ4_LC", 1) != 0) return launch_lz4_decode_lc(b, in_cap, out_cap, s);
    const long env_waves = knob("LZ4_LANE_WAVES", 0);
    // line-buffered stream (round 3, default): 128-byte rings, 10 waves per CU -- 32.7 vs 34.3 ms per
    // 1M x 16 KiB pages for the ring kernel's 256-byte rings (r03 lane timing; 160 / 192-byte rings
    // 33.5 / 33.6)
    const long lbuf = knob("LZ4_LANE_LB", 1);
    const long ring = knob("LZ4_LANE_RING", lbuf ? 128 : kDefaultRing);
    if (ring && lbuf) {
        const void *k = ring == 128   ? (const void *)lz4_decode_ringlb_kernel<128>
                        : ring == 160 ? (const void *)lz4_decode_ringlb_kernel<160>
                        : ring == 192 ? (const void *)lz4_decode_ringlb_kernel<192>
                        : ring == 224 ? (const void *)lz4_decode_ringlb_kernel<224>
                                      : (const void *)lz4_decode_ringlb_kernel<256>;
        const int32_t rbytes = ring == 128 ? 128 : ring == 160 ? 160 : ring == 192 ? 192 : ring == 224 ? 224 : 256;
        const size_t lds = 64 * (size_t)(rbytes + 48 + 80);
        const size_t ncu = prepare_launch(k);
        size_t waves = waves_per_cu(k, lds);
        if (env_waves > 0) waves = std::min<size_t>(waves, (size_t)env_waves);
        const size_t grid = std::min<size_t>((b.count + 63) / 64, ncu * waves);
        WorkCounter ctr(s, grid * 64 < b.count);
        unsigned *cp = ctr.get();
        if (!cp) return hipErrorOutOfMemory;
        void *args[] = {(void *)&b, &in_cap, &out_cap, &cp};
        (void)hipLaunchKernel(k, dim3((unsigned)grid), dim3(64), args, lds, s);
        return hipGetLastError();
    }
    if (ring) {
        const long win = knob("LZ4_LANE_WIN", kDefaultWin);
        const void *k = win == 16 ? (ring == 128   ? (const void *)lz4_decode_ring_kernel<128, 16>
                                     : ring == 256 ? (const void *)lz4_decode_ring_kernel<256, 16>
                                                   : (const void *)lz4_decode_ring_kernel<512, 16>)
                                  : (ring == 128   ? (const void *)lz4_decode_ring_kernel<128, 32>
                                     : ring == 256 ? (const void *)lz4_decode_ring_kernel<256, 32>
                                                   : (const void *)lz4_decode_ring_kernel<512, 32>);
        const int32_t rbytes = ring == 128 ? 128 : ring == 256 ? 256 : 512;
        const size_t lds = 64 * (size_t)(rbytes + 48);
        const size_t ncu = prepare_launch(k);
        size_t waves = waves_per_cu(k, lds);
        if (env_waves > 0) waves = std::min<size_t>(waves, (size_t)env_waves);
        const size_t grid = std::min<size_t>((b.count + 63) / 64, ncu * waves);
        WorkCounter ctr(s, grid * 64 < b.count);
        unsigned *cp = ctr.get();
        if (!cp) return hipErrorOutOfMemory;
        void *args[] = {(void *)&b, &in_cap, &out_cap, &cp};
        (void)hipLaunchKernel(k, dim3((unsigned)grid), dim3(64), args, lds, s);
        return hipGetLastError();
    }
    const size_t ncu = prepare_launch((const void *)lz4_decode_lane_kernel);
    size_t waves = waves_per_cu((const void *)lz4_decode_lane_kernel, 0);
    waves = std::min<size_t>(waves, env_waves > 0 ? (size_t)env_waves : kLaneWaves);
    const size_t grid = std::min<size_t>((b.count + 63) / 64, ncu * waves);
    WorkCounter ctr(s, grid * 64 < b.count);
    if (!ctr.get()) return hipErrorOutOfMemory;
    hipLaunchKernelGGL(lz4_decode_lane_kernel, dim3((unsigned)grid), dim3(64), 0, s, b, in_cap, out_cap, ctr.get());
    return hipGetLastError();
}

}  // namespace tyche
