// lz4_decode_lane.hip -- the large-batch LZ4 decode dispatch: batches of at
// least kLaneMin pages decode one page per LANE (64 pages per wave), which
// needs ~512 pages per CU in flight to hide its memory latency (reference path:
// buffer__decompress, src/buffer.c:248-253 -> LZ4_decompress_safe,
// src/lz4/lz4.c:1251, generic decoder lz4.c:1089-1248).
//
// The product library runs the chunked lane decoder (lz4_decode_lc.hip).  The
// superseded round-2/3 lane kernels and the round-4 quad kernel live in
// legacy/ and are compiled only into the A/B library
// (-DTYCHE_LEGACY_DECODERS: _build.build(legacy=True), tests/test_legacy_decoders.py).
#include <hip/hip_runtime.h>

#include "engine.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>

namespace tyche {

// Threshold (env TYCHE_LZ4_LANE_MIN, for A/B timing): pages per batch that switch
// the batch to the lane decoders.  Crossover (16 KiB pages, ms per 1M pages,
// wave / lane kernel, round 2): 16K pages 130.6 / 170.2, 32K 114.4 / 91.6, 64K
// 108.0 / 52.9, 128K 104.2 / 41.2.
constexpr long kLaneMin = 32768;
// The lane kernels sum literal and match lengths in int32 without the
// reference's pointer-overflow guards (lz4.c:1142, 1181: op+length < op): a run
// of 0xFF length bytes adds 255 per byte, so streams are bounded to
// kLaneMaxStream bytes (255 * 4 MiB < 2^31); larger ones take the wave/serial
// decoders, whose LDS sizing rejects them.
constexpr uint32_t kLaneMaxStream = 4u << 20;
bool lz4_lane_decode_wanted(size_t count, uint32_t in_cap, uint32_t out_cap) {
    const long min_pages = knob("LZ4_LANE_MIN", kLaneMin);
    return min_pages >= 0 && count >= (size_t)min_pages && in_cap <= kLaneMaxStream && out_cap <= kLaneMaxStream;
}

#ifdef TYCHE_LEGACY_DECODERS
hipError_t launch_lz4_decode_lane_legacy(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s);
#else
// The legacy kernels' selection knobs mean nothing in the product library: say so once
// instead of timing the product decoder under a legacy label.
static void warn_legacy_knobs() {
    static std::atomic<bool> done{false};
    if (done.exchange(true)) return;
    static const char *const names[] = {"TYCHE_LZ4_QUAD", "TYCHE_LZ4_LC", "TYCHE_LZ4_LANE_WAVES", "TYCHE_LZ4_LANE_LB",
                                        "TYCHE_LZ4_LANE_RING", "TYCHE_LZ4_LANE_WIN"};
    for (const char *n : names)
        if (getenv(n))
            fprintf(stderr, "tyche: %s selects a legacy LZ4 decoder that only libtyche_codec_legacy_decoders.so "
                            "contains; ignored (the chunked lane decoder runs)\n", n);
}
#endif

hipError_t launch_lz4_decode_lane(const tyche_batch_t &b, uint32_t in_cap, uint32_t out_cap, hipStream_t s) {
    if (b.count == 0) return hipSuccess;
#ifdef TYCHE_LEGACY_DECODERS
    return launch_lz4_decode_lane_legacy(b, in_cap, out_cap, s);
#else
    warn_legacy_knobs();
    return launch_lz4_decode_lc(b, in_cap, out_cap, s);
#endif
}

}  // namespace tyche
