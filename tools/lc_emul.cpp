// tools/lc_emul.cpp -- host emulator of the chunked lane-per-page LZ4 decoder
// (tyche_amd/csrc/lz4_decode_lc.hip) for one page at a time: the kernel's own
// per-lane code (lz4_lc_core.h: record parse, record copies, ring and window
// handling) driven by the same chunk loop as the kernel, with the cooperative
// line flush replaced by plain copies of the same lines.  TEST INFRASTRUCTURE:
// tests/test_lc_emul.py runs it against the oracle on the fixtures and seeded
// corruptions, on the CPU, so the algorithm is checked before (and apart from)
// the GPU parity tests.
//
//   g++ -O2 -shared -fPIC -o tools/bin/liblcemul.so tools/lc_emul.cpp
//   int lc_emul_decode(const uint8_t *in, int L, uint8_t *out, int C, int R);
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned __int128 u128;
using std::min;

#define BF_FN static inline
#define BF_ALIGNBYTE(a, b, c) ((uint32_t)(((((uint64_t)(a)) << 32) | (uint64_t)(b)) >> (8u * ((c) & 3u))))
#define LC_FN static inline
#define LC_Q(base, k) ((base) + ((uint32_t)(k) << 3))   // plain arrays (the kernel interleaves lanes)
#define LC_RCP(x) (1.0f / (x))
#define LC_UMUL24(a, b) ((uint32_t)(a) * (uint32_t)(b))
#define LC_MUL24(a, b) ((int32_t)(a) * (int32_t)(b))
static inline uint32_t lc_perm_host(uint32_t hi, uint32_t lo, uint32_t sel) {   // v_perm_b32
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t d = 0;
    for (int t = 0; t < 4; t++) {
        const uint32_t x = (sel >> (8 * t)) & 0xFFu;
        const uint32_t b = x < 8 ? (uint32_t)((v >> (8 * x)) & 0xFFu) : (x == 12 ? 0u : 0xFFu);
        d |= b << (8 * t);
    }
    return d;
}
#define LC_PERM(hi, lo, sel) lc_perm_host((hi), (lo), (sel))
static inline void lc_lut_load(const uint32_t *lut, int32_t c, uint32_t *ent) { memcpy(ent, lut + 12 * c, 48); }
#define LC_BARRIER() \
    do {             \
    } while (0)

constexpr int32_t kMinMatch = 4, kLastLiterals = 5, kMfLimit = 12, kRunMask = 15;

static inline uint64_t lq(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
static inline void lq(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static inline uint32_t lb(const uint8_t *p) { return *p; }
static inline uint32_t ld1(const uint8_t *p) { return *p; }
static inline u128 ld16(const uint8_t *p) {
    u128 v;
    memcpy(&v, p, 16);
    return v;
}
static inline uint32_t sbyte(const uint8_t *in, int32_t p, int32_t L) { return p >= 0 && p < L ? in[p] : 0u; }
static inline u128 chunk16z(const uint8_t *in, int32_t a, int32_t L) {
    u128 v = 0;
    for (int32_t k = 15; k >= 0; k--) v = (v << 8) | sbyte(in, a + k, L);
    return v;
}

#include "../tyche_amd/csrc/byte_funnel.h"
#include "../tyche_amd/csrc/lz4_lc_core.h"

// the window at nwb (the kernel's wload / wstore)
static void wfill(uint8_t *w16, const uint8_t *in, int32_t L, int32_t nwb) {
    for (int32_t k = 0; k < kLW; k += 16) {
        const u128 v = chunk16z(in, nwb + k, L);
        memcpy(w16 + k, &v, 16);
    }
}

// a far match part's source: its n2 used bytes must be in HBM already (lc_budget); the
// kernel's loads may run past them (bytes it does not use), the emulator's stop there
static void fetch_far(const LPage &P, uint32_t rec, int32_t src, u128 *f) {
    const int32_t n2 = (int32_t)((rec >> 10) & 63u);
    if (src < 0 || src + n2 > P.fl) {
        fprintf(stderr, "lc_emul: far source [%d, %d) not flushed (fl %d)\n", src, src + n2, P.fl);
        abort();
    }
    uint8_t b[32] = {0};
    memcpy(b, P.out + src, (size_t)n2);
    f[0] = ld16(b);
    if (kFarPer == 2) f[1] = n2 > 16 ? ld16(b + 16) : 0;
}

static uint32_t g_lut[17 * kLutStride];
static bool g_lut_ready = [] {
    for (int32_t c = 0; c <= 16; c++) lc_lut_entry(c, g_lut + kLutStride * c);
    return true;
}();

template <int32_t R>
static int lc_decode(const uint8_t *in, int32_t L, uint8_t *out, int32_t C) {
    if (C == 0) return (L == 1 && in[0] == 0) ? 0 : -1;
    if (L <= 0) return -1;
    alignas(16) uint8_t ring[R];
    alignas(16) uint8_t win[kLWS + 64];   // reads run up to 32 bytes past the window's (mirror) rows
    uint8_t *w16 = win + 16;
    memset(ring, 0xA5, sizeof(ring));
    memset(win, 0x5A, sizeof(win));
    LPage P;
    memset(&P, 0, sizeof(P));
    P.in = in;
    P.out = out;
    P.L = L;
    P.C = C;
    wfill(w16, in, L, 0);
    for (long chunk = 0; chunk < 100000000; chunk++) {
        const int32_t op0 = P.op;
        int32_t st = kLParse, rv = 0, nrec = 0;
        uint32_t rec[kLC + 1];
        u128 farv[2 * kLC + 2];   // (kFarPer per slot are used)
        bool go = true, gen = false;
        uint64_t wq[4];
        lc_wread(w16, lc_x0(P), wq);
        int32_t need_gen = 0;
        for (int32_t t = 0; t < kLC; t++) {
            rec[t] = 0;
            farv[kFarPer * t] = farv[kFarPer * t + kFarPer - 1] = 0;
            if (go) {
                bool far = false;
                int32_t src = 0;
                const int32_t k = getenv("LC_SLOW") ? 2 : parse_fast<R>(P, w16, op0, rec[t], far, src, wq);
                if (k == 1) {
                    nrec = t + 1;
                    if (far) fetch_far(P, rec[t], src, farv + kFarPer * t);
                } else {
                    go = false;
                    need_gen = (k == 2 || t == 0) ? 1 : 0;
                    if (k == 0 && t != 0) st = kLCut;
                }
            }
        }
        rec[kLC] = 0;
        farv[kFarPer * kLC] = farv[kFarPer * kLC + kFarPer - 1] = 0;
        if (need_gen) {
            bool far = false;
            int32_t src = 0;
            gen = parse_slot<R>(P, w16, op0, false, st, rv, rec[kLC], far, src);
            if (!gen && nrec == 0 && st == kLCut) {   // no progress: the deep retry, as the kernel
                st = kLParse;
                gen = parse_slot<R>(P, w16, op0, true, st, rv, rec[kLC], far, src);
            }
            if (gen && far) fetch_far(P, rec[kLC], src, farv + kFarPer * kLC);
        }
        const bool ended = st == kLEnd;
        const int32_t nwb = (P.lrem > 0 ? P.lp : P.ip) & ~15;
        if (ended && rv < 0) {
            nrec = 0;
            gen = false;
        }
        if (getenv("LC_TRACE")) {
            const int32_t lo = atoi(getenv("LC_TRACE"));
            int32_t d = op0;
            for (int32_t t = 0; t <= kLC; t++) {
                if (!(t < kLC ? t < nrec : gen)) continue;
                const uint32_t r = rec[t];
                const int32_t lpr = (int32_t)(r & 63u), n1 = (int32_t)((r >> 6) & 15u), n2 = (int32_t)((r >> 10) & 63u),
                              off = (int32_t)(r >> 16);
                if (d + n1 + n2 >= lo && d <= lo + 64)
                    fprintf(stderr, "chunk %ld t %d d %d wb %d lpr %d n1 %d n2 %d off %d far %d\n", chunk, t, d, P.wb, lpr,
                            n1, n2, off, off > lc_near<R>());
                d += n1 + n2;
            }
        }
        uint64_t tail = P.tail;
        copy_records<R>(ring, w16, op0, tail, rec, farv, nrec, gen, g_lut);
        P.tail = tail;
        const int32_t lend = (ended && rv < 0) ? P.fl : (P.op & ~(kLcLine - 1));
        for (int32_t f = P.fl; f + 16 <= lend; f += 16) memcpy(out + f, ring + 8 * lc_row<R>(f >> 3), 16);
        P.fl = lend > P.fl ? lend : P.fl;
        if (ended) {
            if (rv >= 0)
                for (int32_t a = P.fl; a < P.op; a++) out[a] = ring[8 * lc_row<R>(a >> 3) + (a & 7)];
            return rv;
        }
        wfill(w16, in, L, nwb);
        P.wb = nwb;
    }
    fprintf(stderr, "lc_emul: no end\n");
    abort();
}

extern "C" int lc_emul_decode(const uint8_t *in, int L, uint8_t *out, int C, int R) {
#if LC_LINE == 64
    if (R == 128) R = 192;   // (64-byte lines need R >= 192)
#endif
    return R == 256   ? lc_decode<256>(in, L, out, C)
           : R == 192 ? lc_decode<192>(in, L, out, C)
           : R == 160 ? lc_decode<160>(in, L, out, C)
                      : lc_decode<128>(in, L, out, C);
}
