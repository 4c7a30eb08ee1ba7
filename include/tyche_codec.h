/*
 * include/tyche_codec.h -- C ABI of the MI355X page-codec engine (libtyche_codec.so).
 *
 * Drop-in replacement for tyche's codec boundary (reference src/buffer.h:67-68,
 * src/buffer.c:159-281): the same `Buffer` struct, the same buffer__* symbols
 * and signatures, the same compressor IDs (src/globals.h:16-19) and error codes
 * (src/globals.h:35-58), and the same ownership rules (compress returns a
 * free()-able *compressed_data; decompress swaps buf->data in place).  The
 * codec work runs as HIP kernels on gfx950; nothing here falls back to a CPU
 * codec.  Additional entry points expose the batch engine that the sweep
 * (list.c:824-838, 1039-1063) and restore (list.c:563-589) paths call with many
 * pages at once, and the device-resident batch API measured by bench.py.
 *
 * Plain C types only; no torch, no HIP types (streams are passed as void*).
 */
#ifndef TYCHE_CODEC_H_
#define TYCHE_CODEC_H_

#include <pthread.h>
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- compressor IDs: src/globals.h:16-19 -------------------------------- */
#define TYCHE_NO_COMPRESSOR_ID   0
#define TYCHE_LZ4_COMPRESSOR_ID  1
#define TYCHE_ZLIB_COMPRESSOR_ID 2
#define TYCHE_ZSTD_COMPRESSOR_ID 3

/* ---- error codes: src/globals.h:35-58 ----------------------------------- */
#define TYCHE_E_OK                          0
#define TYCHE_E_GENERIC                     1
#define TYCHE_E_BUFFER_NOT_FOUND          120
#define TYCHE_E_BUFFER_MISSING_DATA       123
#define TYCHE_E_BUFFER_ALREADY_COMPRESSED 124
#define TYCHE_E_BUFFER_ALREADY_DECOMPRESSED 125
#define TYCHE_E_BUFFER_COMPRESSION_PROBLEM 126
#define TYCHE_E_NO_MEMORY                 150
#define TYCHE_E_BAD_ARGS                  190
/* engine-specific (outside the reference's range): the HIP engine itself failed
 * (no device, launch failure, codec not built for the device) */
#define TYCHE_E_DEVICE                    199

/* ---- Buffer: identical layout to src/buffer.h:23-58 --------------------- */
typedef enum buffer_flags {
    dirty = 1 << 0,
    pending_sweep = 1 << 1,
    updating = 1 << 2,
    removing = 1 << 3,
    removed = 1 << 4,
    compressing = 1 << 5,
    compressed = 1 << 6,
} buffer_flags;

typedef uint32_t bufferid_t;
typedef uint8_t popularity_t;
typedef struct buffer Buffer;
struct buffer {
    Buffer *next;
    bufferid_t id;
    uint16_t ref_count;
    buffer_flags flags;
    popularity_t popularity;
    pthread_mutex_t lock;
    uint32_t comp_cost;     /* ns spent in compress+decompress (wraps like the reference's uint32) */
    uint16_t comp_hits;     /* restores */
    uint32_t data_length;   /* uncompressed page length */
    uint32_t comp_length;   /* bytes in data when compressed, else 0 */
    void *data;             /* free()-compatible host heap */
};

/* ---- drop-in symbols: src/buffer.h:62-69 --------------------------------- */
int buffer__initialize(Buffer **buf, bufferid_t id, uint32_t size, void *data, char *page_filespec);
void buffer__destroy(Buffer *buf, const bool destroy_data);
void buffer__lock(Buffer *buf);
void buffer__unlock(Buffer *buf);
void buffer__release_pin(Buffer *buf);
/* replaces src/buffer.c:159-219: LZ4/zlib/zstd by compressor_id, on the GPU.
 * On a codec or device failure (126 / TYCHE_E_DEVICE) *compressed_data is set
 * to NULL (the reference leaves it at a leaked, unfilled block). */
int buffer__compress(Buffer *buf, void **compressed_data, int compressor_id, int compressor_level);
/* replaces src/buffer.c:227-281 */
int buffer__decompress(Buffer *buf, int compressor_id);
void buffer__copy(Buffer *src, Buffer *dst, bool copy_data);

/* ---- batch extension over Buffers (sweep / restore callers) -------------- */
/* Compress n buffers in one GPU batch.  Per buffer, status[i] and side effects
 * are exactly what buffer__compress would produce for it (compressed[i] is a
 * malloc'd block the caller owns when status[i]==0).  Returns 0, or
 * TYCHE_E_DEVICE / TYCHE_E_NO_MEMORY if the batch could not run at all.
 * Replaces the per-victim loop of list__compressor_start (src/list.c:1039-1063). */
int tyche_buffers_compress(Buffer **bufs, void **compressed, int *status, size_t n, int compressor_id,
                           int compressor_level);
/* Restore n compressed buffers in one GPU batch (the list__search restore of
 * src/list.c:563-589, coalesced); status[i] as buffer__decompress. */
int tyche_buffers_decompress(Buffer **bufs, int *status, size_t n, int compressor_id);

/* ---- restore queue: coalesced per-hit restores (src/list.c:563-589) ------- */
/* Starts the dispatcher threads (per codec, TYCHE_RESTORE_DISPATCHERS each,
 * default one per active device; they inherit the calling thread's device
 * choice) that batch concurrent tyche_buffer_restore calls: once a request
 * arrives a dispatcher of its codec waits up to max_wait_us for up to max_batch
 * requests of that codec, then runs one GPU decompress batch while the next
 * dispatcher collects.  Idempotent. */
int tyche_restore_queue_start(int max_batch, int max_wait_us);
/* Drains and stops the dispatcher. */
void tyche_restore_queue_stop(void);
/* Drop-in for buffer__decompress at the list__search restore site
 * (src/list.c:572): same status and side effects, but concurrent callers share
 * GPU launches.  Without a running queue it is buffer__decompress. */
int tyche_buffer_restore(Buffer *buf, int compressor_id);
/* Launches and buffers served so far. */
void tyche_restore_queue_stats(uint64_t *batches, uint64_t *buffers);
/* Launches so far by batch size: counts[k] = launches of 2^k .. 2^(k+1)-1
 * buffers (the last bucket takes every larger one); fills min(n, 11) buckets
 * and returns that count. */
int tyche_restore_queue_hist(uint64_t *counts, int n);

/* ---- device-resident batch API ------------------------------------------- */
/* Page i of the batch reads src + src_offsets[i] (or i*src_stride when
 * src_offsets is NULL) for src_lengths[i] (or src_length) bytes and writes at
 * most dst_capacities[i] (or dst_capacity) bytes to dst + dst_offsets[i] (or
 * i*dst_stride).  All pointers are device pointers on the current device.
 * results[i] (device int32):
 *   compress   -- compressed size, or 0 when the output does not fit
 *                 (LZ4_compress_default semantics, lz4.c:697, for every codec)
 *   decompress -- the codec's own verdict:
 *                 LZ4  LZ4_decompress_safe (lz4.c:1251): decoded size, or
 *                      -(input bytes consumed)-1 for a malformed stream;
 *                 zlib uncompress (uncompr.c:22): decoded length, or -3
 *                      (Z_DATA_ERROR) / -5 (Z_BUF_ERROR);
 *                 zstd ZSTD_decompress (zstd_decompress.c:1459): decoded size,
 *                      or a negative value wherever ZSTD_isError holds.
 *   INT32_MIN marks a page larger than the launch's declared maximum.
 * max_src_length (0 = unknown) bounds src lengths for LDS sizing.
 * `stream` is a hipStream_t (NULL = default stream); the call is asynchronous. */
typedef struct tyche_batch {
    size_t count;
    const void *src;
    const uint64_t *src_offsets;
    const uint32_t *src_lengths;
    uint64_t src_stride;
    uint32_t src_length;
    uint32_t max_src_length;
    void *dst;
    const uint64_t *dst_offsets;
    const uint32_t *dst_capacities;
    uint64_t dst_stride;
    uint32_t dst_capacity;
    int32_t *results;
} tyche_batch_t;

int tyche_compress_batch(int compressor_id, int compressor_level, const tyche_batch_t *batch, void *stream);
int tyche_decompress_batch(int compressor_id, const tyche_batch_t *batch, void *stream);
/* worst-case compressed size for n input bytes: LZ4_compressBound (lz4.h:148),
 * compressBound (zlib compress.c:74-78) or ZSTD_compressBound (zstd_compress.c:37) */
uint32_t tyche_compress_bound(int compressor_id, uint32_t n);

/* ---- host batch API (pinned staging + H2D -> kernels -> D2H) ------------- */
/* Same per-page semantics as the device batch, with host pointers.  Used by
 * the Buffer entry points and by the PCIe-inclusive measurement. */
int tyche_compress_host(int compressor_id, int compressor_level, size_t n, const void *const *src,
                        const uint32_t *src_lengths, void *const *dst, const uint32_t *dst_capacities,
                        int32_t *results);
int tyche_decompress_host(int compressor_id, size_t n, const void *const *src, const uint32_t *src_lengths,
                          void *const *dst, const uint32_t *dst_capacities, int32_t *results);

/* ---- runtime ------------------------------------------------------------- */
/* The reference is one process whose compressor pool (src/list.c:142-168,
 * opts.cpu_count threads, src/manager.c:85) and workers call the codec
 * concurrently; it has no notion of devices.  By default the host entry points
 * (Buffer API, host batches, restore queue) therefore use every visible gfx950
 * device (the first TYCHE_DEVICES of them when that is set): a host batch of at
 * least two parts' worth of input is cut into contiguous page ranges of about
 * equal input bytes, one per device, run concurrently (tyche_plan_split); a
 * smaller one goes whole to the device with the fewest batches in flight, so
 * concurrent per-page callers spread over all devices.  tyche_set_device(d)
 * pins the calling thread to device d instead; TYCHE_ALL_DEVICES undoes that.
 * The device-resident batch API always runs on the caller's current device. */
#define TYCHE_ALL_DEVICES (-1)
int tyche_device_count(void);
/* pins the calling thread's host-path work to `device`, or TYCHE_ALL_DEVICES (default) */
int tyche_set_device(int device);
/* devices the calling thread's host-path work is spread over (1 when pinned) */
int tyche_active_devices(void);
/* The fan-out plan of a host batch (exported so it can be checked without a
 * GPU): splits n pages into at most ndev contiguous ranges of about equal input
 * bytes, each holding at least min_part_bytes of input (0 = no minimum).
 * Writes cuts[0..k] (cuts[0] = 0, cuts[k] = n; cuts needs ndev + 1 entries)
 * and returns the number of ranges k >= 1.  The engine uses
 * min_part_bytes = TYCHE_FANOUT_MIN_BYTES (default 64 MiB, one staging chunk). */
size_t tyche_plan_split(size_t n, const uint32_t *src_lengths, int ndev, uint64_t min_part_bytes, size_t *cuts);
/* Kernel-path switches and tunables (names without the TYCHE_ prefix, e.g.
 * "LZ4_LANE_MIN", "ZLIB_PAR"): the library reads TYCHE_<name> from the
 * environment once and checks for an override on every launch.  Set / drop an
 * in-process override; for tests and A/B timing.  No knob changes a decode
 * result; encoder-shape knobs (LZ4_ENC_WAVES, ZSTD_PARSE_WAVES, ZSTD_FSE_LOG)
 * change the compressed bytes and ratio, never whether they decode to the page.
 * Two are test hooks: FAIL_COMPRESS_EVERY=N fails every Nth compress launch
 * (TYCHE_E_DEVICE, the device-failure test) and LOG_ERRORS=1 prints engine
 * errors to stderr. */
int tyche_set_knob(const char *name, long value);
int tyche_clear_knob(const char *name);
/* Diagnostics: host-path stage clocks since the last call, then reset -- out[0..6] = ns waiting for
 * streams, ns scattering, ns gathering, ns enqueuing, bytes gathered, bytes scattered, chunks.
 * Returns the number of values written (at most n). */
int tyche_host_profile(uint64_t *out, int n);
/* message for the last TYCHE_E_DEVICE on this thread */
const char *tyche_last_error(void);
/* 1 if the library's gfx950 code object is usable on the calling thread's
 * (first) device */
int tyche_device_ready(void);

/* ---- synthetic input (bench/tests; same generator as the host copy) ------ */
/* fills `count` pages of page_len bytes at dst + i*stride on the device */
int tyche_pagegen(void *dst, uint64_t stride, uint32_t page_len, uint64_t seed, uint64_t first, size_t count,
                  uint32_t dist, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* TYCHE_CODEC_H_ */
