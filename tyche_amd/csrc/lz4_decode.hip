// lz4_decode.hip -- batched LZ4 block decode for gfx950 (the restore path).
//
// Replaces the per-hit LZ4_decompress_safe call of buffer__decompress
// (reference src/buffer.c:248-253 -> src/lz4/lz4.c:1251, generic decoder
// lz4.c:1089-1248) with one kernel over a batch of pages.  Results are
// LZ4_decompress_safe's: decoded size, or -(input bytes consumed)-1 at the
// same consumption point for a malformed stream; the decoded bytes are
// bit-identical.
//
// Layout: one 64-lane wave per page.  The compressed page is staged into LDS
// with 16-byte loads; the page is rebuilt in an LDS window and written back to
// HBM with 16-byte stores, so HBM sees exactly comp_len bytes read and page_len
// bytes written.  The token chain is parsed with wave-uniform scalar control
// from a 64-byte window of the stream held one byte per lane (one LDS read per
// sequence, fields picked out with v_readlane); literal and match bytes are
// copied 64 per instruction, with modulo addressing for self-overlapping
// matches (offset < length), which reproduces the forward byte-copy semantics of
// lz4.c:1209-1236.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "lds_io.h"

namespace tyche {

namespace {

constexpr uint32_t kWave = 64;
constexpr uint32_t kPad = 64;   // zeroed tail after the staged stream

struct Window {
    uint32_t base;   // stream position of lane 0
    uint32_t v;      // byte base+lane (zero past the end)
};

__device__ __forceinline__ uint32_t window_byte(const Window &w, const uint8_t *in, uint32_t pos) {
    uint32_t d = pos - w.base;
    if (d < kWave) return rdlane(w.v, d);
    return rfl(in[pos]);
}

// Decodes one page held in LDS.  in: stream (len L, kPad zero bytes after),
// out: LDS window of C bytes.  Returns LZ4_decompress_safe's value.
__device__ int32_t decode_page(const uint8_t *in, int32_t L, uint8_t *out, int32_t C, uint32_t lane) {
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

__global__ __launch_bounds__(64) void lz4_decode_wave_kernel(tyche_batch_t b, uint32_t in_cap, uint32_t out_cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    const size_t page = blockIdx.x;
    PageRef p = batch_page(b, page);
    if (p.src_len > in_cap || p.dst_cap > out_cap) {
        if (lane == 0) b.results[page] = kResultTooLarge;
        return;
    }
    uint8_t *out = smem;                                        // out_cap bytes (rounded to 16)
    uint8_t *stage = smem + ((out_cap + 15u) & ~15u);           // in_cap + 16 + kPad bytes
    uint32_t head = stage_in(p.src, p.src_len, stage, lane, kWave);
    uint8_t *in = stage + head;
    in[p.src_len + lane] = 0;                                   // kPad zero bytes past the end
    __syncthreads();
    int32_t rv = decode_page(in, (int32_t)p.src_len, out, (int32_t)p.dst_cap, lane);
    __syncthreads();
    if (rv > 0) stage_out(p.dst, out, (uint32_t)rv, lane, kWave);
    if (lane == 0) b.results[page] = rv;
}

}  // namespace

hipError_t launch_lz4_decode(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
    size_t lds = ((out_cap + 15u) & ~15u) + ((in_cap + 16u + kPad + 15u) & ~15u);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)lz4_decode_wave_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(lz4_decode_wave_kernel, dim3((unsigned)b.count), dim3(kWave), lds, s, b, in_cap, out_cap);
    return hipGetLastError();
}

}  // namespace tyche
