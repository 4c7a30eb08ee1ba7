// byte_funnel.h -- byte shifts across qwords with v_alignbyte (funnel8) and
// byte merges (keep_low): the register side of the aligned-qword LDS access of
// lds_qword.h.  Host code (tools/lc_emul.cpp) includes it with BF_FN and
// BF_ALIGNBYTE defined to plain C++.
#pragma once

#ifndef BF_FN
#define BF_FN __device__ __forceinline__
#endif
#ifndef BF_ALIGNBYTE
#define BF_ALIGNBYTE(a, b, c) __builtin_amdgcn_alignbyte((a), (b), (c))
#endif

// bytes [s, s + 8) of the 16 bytes a (low) : b (high), 0 <= s < 8
BF_FN uint64_t funnel8(uint64_t a, uint64_t b, uint32_t s) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const bool h = (s & 4u) != 0;
    const uint32_t x0 = h ? a1 : a0, x1 = h ? b0 : a1, x2 = h ? b1 : b0;
    const uint32_t r = s & 3u;
    return (uint64_t)BF_ALIGNBYTE(x1, x0, r) | ((uint64_t)BF_ALIGNBYTE(x2, x1, r) << 32);
}
// bytes [0, m) of t, bytes [m, 8) of v (0 <= m <= 8)
BF_FN uint64_t keep_low(uint64_t t, uint64_t v, uint32_t m) {
    const uint32_t mlo = m >= 4u ? 0xFFFFFFFFu : ((1u << (8u * m)) - 1u);
    const uint32_t mhi = m <= 4u ? 0u : (m >= 8u ? 0xFFFFFFFFu : ((1u << (8u * (m - 4u))) - 1u));
    const uint32_t lo = (mlo & (uint32_t)t) | (~mlo & (uint32_t)v);
    const uint32_t hi = (mhi & (uint32_t)(t >> 32)) | (~mhi & (uint32_t)(v >> 32));
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
