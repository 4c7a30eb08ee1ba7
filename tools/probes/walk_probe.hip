// Diagnostic: cycles per token of a one-wave serial LZ4 token walk (the single-page decoder's
// chain, next_token_w / solo_next semantics, lz4.c:1134-1182) with the stream staged in LDS and a
// 256-byte window of it held in one VGPR (4 bytes per lane), read with v_readlane into scalar
// registers.  Writes the chain (position | output offset << 16, 64 entries per vector store) and
// the cycle count.  Built and driven by tools/probes/walk_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int32_t kRunMask = 15, kLastLiterals = 5;

struct Walk {
    const uint8_t *A;   // 4-aligned LDS base: stream position p is A[p + ib]
    int32_t ib, wa;     // stream offset in A, window base (A offset, 4-aligned)
    uint32_t v;         // this lane's 4 bytes of A[wa, wa + 256)
    uint32_t lane;
    __device__ __forceinline__ void load(int32_t a) {
        wa = a & ~3;
        v = *(const uint32_t *)(A + wa + 4 * lane);
    }
    // 8 bytes from stream position p (5 valid at least)
    __device__ __forceinline__ uint64_t get8(int32_t p) {
        const int32_t a = p + ib;
        if (a - wa > 248) load(a);
        const int32_t r = a - wa;
        const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)v, r >> 2);
        const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)v, (r >> 2) + 1);
        return ((((uint64_t)w1) << 32) | w0) >> (8 * (r & 3));
    }
    __device__ __forceinline__ uint32_t byte(int32_t p) { return (uint32_t)get8(p) & 0xFFu; }
};

__global__ __launch_bounds__(64) void walk_kernel(const uint8_t *src, int32_t L, uint32_t *list, uint32_t *count,
                                                  unsigned long long *cycles) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[32768 + 512];
    const uint32_t lane = threadIdx.x;
    for (int32_t i = (int32_t)lane; i < L + 512; i += 64) stage[i] = i < L ? src[i] : 0;
    __syncthreads();
    Walk w;
    w.A = stage;
    w.ib = 0;
    w.lane = lane;
    w.load(0);
    const unsigned long long t0 = clock64();
    int32_t p = 0;
    uint32_t d = 0, cnt = 0, rec = 0;
    while (p < L) {
        const uint64_t x = w.get8(p);
        const uint32_t t = (uint32_t)x & 0xFFu;
        int32_t lit = (int32_t)(t >> 4), q = p + 1;
        if (lit == kRunMask) {
            uint32_t b = (uint32_t)(x >> 8) & 0xFFu;
            q++;
            lit += (int32_t)b;
            while (q < L - kRunMask && b == 255) {
                b = w.byte(q);
                q++;
                lit += (int32_t)b;
            }
        }
        uint32_t olen;
        int32_t nxt;
        if (q + lit > L - 8) {
            olen = (uint32_t)lit;
            nxt = L;
        } else {
            int32_t q2 = q + lit + 2, ml = (int32_t)(t & 15u);
            nxt = q2;
            if (ml == 15) {
                uint32_t b;
                do {
                    b = w.byte(q2);
                    q2++;
                    if (q2 > L - kLastLiterals) {
                        ml = -4;
                        q2 = L;
                        break;
                    }
                    ml += (int32_t)b;
                } while (b == 255);
                nxt = q2;
            }
            olen = ml < 0 ? 0u : (uint32_t)(lit + ml + 4);
        }
        rec = lane == (cnt & 63u) ? ((uint32_t)p | (d << 16)) : rec;
        d += olen;
        cnt++;
        if ((cnt & 63u) == 0) list[cnt - 64 + lane] = rec;
        p = nxt;
    }
    if ((cnt & 63u) != 0 && lane < (cnt & 63u)) list[(cnt & ~63u) + lane] = rec;
    const unsigned long long t1 = clock64();
    if (lane == 0) {
        count[0] = cnt;
        cycles[0] = t1 - t0;
    }
}

}  // namespace

extern "C" int walk_probe(const uint8_t *src, int32_t L, uint32_t *list, uint32_t *count, unsigned long long *cycles) {
    hipLaunchKernelGGL(walk_kernel, dim3(1), dim3(64), 0, 0, src, L, list, count, cycles);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
