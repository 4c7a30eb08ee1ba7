// engine.hip -- the C ABI of libtyche_codec.so (declared in include/tyche_codec.h).
//
// Drop-in for tyche's codec boundary, src/buffer.c:159-281: buffer__compress /
// buffer__decompress keep the reference's argument checks, their order, the
// error codes, the free()-compatible ownership and the comp_length /
// comp_cost / comp_hits side effects, but the codec runs as gfx950 kernels.
// The batch entry points let the sweep (src/list.c:1039-1063) and restore
// (src/list.c:563-589) callers hand over many pages per launch, and the
// device-resident API is what bench.py measures.
//
// There is no CPU codec in this library: if the HIP device or the gfx950 code
// object is unavailable every codec entry point returns an error.
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"

#include <immintrin.h>

using namespace tyche;

namespace {
constexpr int kMaxDevices = 64;

// ------------------------------------------------------------- work counters
// One pool of device counters per device.  An entry is free, leased (between
// WorkCounter's constructor and destructor), or released: an event recorded on
// the launch stream after the kernel that claims pages from it.  A released
// entry is handed out again only when its event has completed, so a counter is
// never reset while a kernel on any stream still claims from it.
struct CounterPool {
    struct Entry {
        unsigned *p;
        hipEvent_t ev;
        int state;   // 0 free, 1 leased, 2 released (event pending)
    };
    std::mutex mu;
    std::vector<Entry> e;
    size_t cursor = 0;
    unsigned *junk = nullptr;   // shared by launches whose grid covers all their pages
};
CounterPool *const g_counters = new CounterPool[kMaxDevices];   // never destroyed (restore dispatchers may run at exit)
constexpr size_t kCounterBlock = 64;
}  // namespace

tyche::WorkCounter::WorkCounter(hipStream_t s, bool claims) : s_(s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return;
    CounterPool &P = g_counters[dev];
    std::lock_guard<std::mutex> g(P.mu);
    if (!claims) {
        // the grid covers every page: each claim returns >= gridDim.x >= count whatever the
        // counter holds, so one shared, never-reset counter serves every such launch (no
        // memset on the stream, no event)
        if (!P.junk && hipMalloc((void **)&P.junk, sizeof(unsigned)) != hipSuccess) P.junk = nullptr;
        p_ = P.junk;
        return;
    }
    const size_t n = P.e.size();
    size_t take = n;
    for (size_t k = 0; k < n; k++) {   // from the oldest release on: those are done first
        const size_t i = (P.cursor + k) % n;
        CounterPool::Entry &x = P.e[i];
        if (x.state == 1) continue;
        if (x.state == 2 && hipEventQuery(x.ev) != hipSuccess) continue;   // its kernel may still run
        take = i;
        break;
    }
    if (take == n) {   // all in use: one more block
        unsigned *blk = nullptr;
        if (hipMalloc((void **)&blk, kCounterBlock * sizeof(unsigned)) != hipSuccess) return;
        for (size_t j = 0; j < kCounterBlock; j++) {
            hipEvent_t ev;
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) break;
            P.e.push_back({blk + j, ev, 0});
        }
        if (P.e.size() == n) return;
    }
    CounterPool::Entry &x = P.e[take];
    if (hipMemsetAsync(x.p, 0, sizeof(unsigned), s) != hipSuccess) return;
    x.state = 1;
    P.cursor = take + 1;
    dev_ = dev;
    idx_ = (int)take;
    p_ = x.p;
}

tyche::WorkCounter::~WorkCounter() {
    if (idx_ < 0) return;
    CounterPool &P = g_counters[dev_];
    std::lock_guard<std::mutex> g(P.mu);
    CounterPool::Entry &x = P.e[(size_t)idx_];
    if (hipEventRecord(x.ev, s_) == hipSuccess) {
        x.state = 2;
    } else {
        (void)hipStreamSynchronize(s_);   // no event: wait for the launch instead
        x.state = 0;
    }
}

namespace {
struct ScratchPool {
    struct Entry {
        void *p;
        size_t bytes;
        hipEvent_t ev;
        int state;   // 0 free, 1 leased, 2 released (event pending)
    };
    std::mutex mu;
    std::vector<Entry> e;
};
ScratchPool *const g_scratch = new ScratchPool[kMaxDevices];   // never destroyed (restore dispatchers may run at exit)
}  // namespace

// Leases are sized by the request (1 MiB granules) and reused best-fit, never
// for a request under a quarter of their size (a small launch must not pin a
// chunked zstd decode's gigabytes).  Idle entries beyond kPoolKeep bytes per
// device are freed, largest first, whenever a lease is taken, and a failed
// allocation frees every idle entry and tries once more.
constexpr size_t kPoolKeep = size_t(2) << 30;

namespace {
bool entry_idle(ScratchPool::Entry &x) {
    return x.state == 0 || (x.state == 2 && hipEventQuery(x.ev) == hipSuccess && ((x.state = 0), true));
}
// takes idle entries (largest first) out of the pool until it holds at most `keep` bytes; under
// P.mu.  The caller frees what it returns (free_entries) after releasing P.mu: hipFree synchronises
// the device, and neither the other streams nor the other lease requests should wait on that.
std::vector<ScratchPool::Entry> pool_trim(ScratchPool &P, size_t keep) {
    std::vector<ScratchPool::Entry> out;
    size_t total = 0;
    for (auto &x : P.e) total += x.bytes;
    while (total > keep) {
        size_t best = P.e.size();
        for (size_t i = 0; i < P.e.size(); i++)
            if (entry_idle(P.e[i]) && (best == P.e.size() || P.e[i].bytes > P.e[best].bytes)) best = i;
        if (best == P.e.size()) break;
        out.push_back(P.e[best]);
        total -= P.e[best].bytes;
        P.e.erase(P.e.begin() + (long)best);
    }
    return out;
}
void free_entries(const std::vector<ScratchPool::Entry> &v) {
    for (const auto &x : v) {
        (void)hipFree(x.p);
        (void)hipEventDestroy(x.ev);
    }
}
}  // namespace

size_t tyche::scratch_idle_bytes() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 0;
    ScratchPool &P = g_scratch[dev];
    std::lock_guard<std::mutex> g(P.mu);
    size_t idle = 0;
    for (auto &x : P.e)
        if (entry_idle(x)) idle += x.bytes;
    return idle;
}

tyche::ScratchLease::ScratchLease(hipStream_t s, size_t bytes) : s_(s) {
    if (bytes == 0) return;   // nothing asked: get() is null
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return;
    ScratchPool &P = g_scratch[dev];
    const size_t want = (std::max<size_t>(bytes, 1) + 0xFFFFF) & ~size_t(0xFFFFF);
    // test hook: each new value of the SCRATCH_OOM_SEQ knob makes one lease skip the pool and see its
    // first hipMalloc fail (a real, oversized request: the HIP error slot is set as by a real OOM)
    static std::atomic<long> oom_seq{0};
    const long seq = knob("SCRATCH_OOM_SEQ", 0);
    const bool force_oom = seq != 0 && oom_seq.exchange(seq) != seq;
    auto lease = [&](size_t i) {
        P.e[i].state = 1;
        dev_ = dev;
        idx_ = (int)i;
        p_ = P.e[i].p;
    };
    // best fit among idle entries of at most 4x the request; without one, the pool is trimmed and
    // the victims freed (outside the lock: hipFree synchronises the device) BEFORE the new
    // allocation, so device memory never holds both; then a second look (another thread may have
    // released a fitting entry meanwhile) and only then hipMalloc
    for (int pass = 0; pass < 2; pass++) {
        std::vector<ScratchPool::Entry> victims;
        {
            std::lock_guard<std::mutex> g(P.mu);
            size_t take = P.e.size();
            for (size_t i = 0; i < P.e.size(); i++) {
                ScratchPool::Entry &x = P.e[i];
                if (x.state == 1 || x.bytes < want || x.bytes / 4 > want) continue;
                if (!entry_idle(x)) continue;
                if (take == P.e.size() || x.bytes < P.e[take].bytes) take = i;
            }
            if (take < P.e.size() && !force_oom) {
                lease(take);
                return;
            }
            if (pass == 0) victims = pool_trim(P, kPoolKeep > want ? kPoolKeep - want : 0);
        }
        if (victims.empty()) break;
        free_entries(victims);
    }
    ScratchPool::Entry x{nullptr, want, nullptr, 0};
    if ((force_oom ? hipMalloc(&x.p, size_t(1) << 62) : hipMalloc(&x.p, x.bytes)) != hipSuccess) {
        // out of memory: every idle entry goes, then one more try.  The failed call's error stays in
        // the thread's HIP error slot, where the launch helpers' hipGetLastError() would report a
        // recovered allocation as a failed launch: clear it.
        (void)hipGetLastError();
        std::vector<ScratchPool::Entry> all;
        {
            std::lock_guard<std::mutex> g(P.mu);
            all = pool_trim(P, 0);
        }
        free_entries(all);
        if (hipMalloc(&x.p, x.bytes) != hipSuccess) {
            (void)hipGetLastError();   // reported by get() == nullptr: the caller's own error path
            return;
        }
    }
    if (hipEventCreateWithFlags(&x.ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipFree(x.p);
        (void)hipGetLastError();
        return;
    }
    std::lock_guard<std::mutex> g(P.mu);
    P.e.push_back(x);
    lease(P.e.size() - 1);
}

tyche::ScratchLease::~ScratchLease() {
    if (idx_ < 0) return;
    ScratchPool &P = g_scratch[dev_];
    std::lock_guard<std::mutex> g(P.mu);
    // by address: pool_trim may have erased (idle) entries before this one since the lease
    size_t i = 0;
    while (i < P.e.size() && P.e[i].p != p_) i++;
    if (i == P.e.size()) return;
    ScratchPool::Entry &x = P.e[i];
    if (hipEventRecord(x.ev, s_) == hipSuccess) {
        x.state = 2;
    } else {
        (void)hipStreamSynchronize(s_);
        x.state = 0;
    }
}

size_t tyche::prepare_launch(const void *kernel) {
    static std::mutex &mu = *new std::mutex;   // never destroyed, like the pools (dispatchers at exit)
    static auto &raised = *new std::set<std::pair<int, const void *>>;
    static int cus[kMaxDevices] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= kMaxDevices) return 256;
    std::lock_guard<std::mutex> g(mu);
    if (cus[dev] == 0) {
        int n = 0;
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        cus[dev] = n > 0 ? n : 256;
    }
    if (raised.insert({dev, kernel}).second)
        (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return (size_t)cus[dev];
}

namespace {
struct KnobTable {
    std::mutex mu;
    std::map<std::string, long> over;                    // tyche_set_knob
    std::map<std::string, std::pair<bool, long>> env;    // TYCHE_<name>: (present, value)
};
KnobTable &knob_table() {
    static KnobTable *t = new KnobTable;   // never destroyed: detached pool threads may still read it at exit
    return *t;
}
}  // namespace

namespace {
// Knobs are read on every launch (a restore reads ~10).  The table's lookups (mutex, string maps) cost
// ~0.1-0.3 us each, so each thread keeps what it read, keyed by the name's address (the call sites
// pass literals), until tyche_set_knob / tyche_clear_knob bump the generation.
std::atomic<uint64_t> g_knob_gen{1};
struct KnobSeen {
    const char *name;
    uint64_t gen;
    bool present;
    long value;
};
constexpr int kKnobCache = 64;
thread_local KnobSeen t_knobs[kKnobCache];
bool knob_slow(const char *name, long &value) {
    KnobTable &T = knob_table();
    std::lock_guard<std::mutex> g(T.mu);
    const auto o = T.over.find(name);
    if (o != T.over.end()) {
        value = o->second;
        return true;
    }
    auto e = T.env.find(name);
    if (e == T.env.end()) {
        const char *v = getenv((std::string("TYCHE_") + name).c_str());
        e = T.env.emplace(name, std::make_pair(v != nullptr && *v, v ? strtol(v, nullptr, 10) : 0L)).first;
    }
    value = e->second.second;
    return e->second.first;
}
}  // namespace

long tyche::knob(const char *name, long dflt) {
    const uint64_t gen = g_knob_gen.load(std::memory_order_acquire);
    const uint32_t h = (uint32_t)(((uintptr_t)name * 0x9E3779B97F4A7C15ull) >> 58);   // 6 bits
    for (int k = 0; k < 4; k++) {   // a short probe; a miss just takes the table
        KnobSeen &c = t_knobs[(h + (uint32_t)k) % kKnobCache];
        if (c.name == name && c.gen == gen) return c.present ? c.value : dflt;
        if (c.name == nullptr || c.gen != gen || k == 3) {
            long v = 0;
            const bool present = knob_slow(name, v);
            c = KnobSeen{name, gen, present, v};
            return present ? v : dflt;
        }
    }
    return dflt;   // (unreachable)
}

namespace {
// Diagnostic builds only (-DTYCHE_PROFILE, libtyche_codec_prof.so): TYCHE_HOST_DIAG bit 0 makes the
// host batch report the results without copying the page bytes out (prices the scatter copies).  The
// product library has no such switch, so a stray setting can never report success without the data
// (ADVICE r05).
bool host_diag_no_copy() {
#ifdef TYCHE_PROFILE
    return (tyche::knob("HOST_DIAG", 0) & 1) != 0;
#else
    return false;
#endif
}
}  // namespace

namespace {

// -1: the host API spreads work over every usable device (the default);
// >= 0: tyche_set_device pinned the calling thread to that device
thread_local int t_device = -1;
thread_local std::string t_error;

// TYCHE_LOG_ERRORS=1: every engine failure is also printed to stderr (one
// "tyche-engine: ..." line), so a caller that drops the status -- list.c:1051
// keeps going on any rv but 124 -- still leaves a trace (the C1 tests fail on it).
// The line goes straight to fd 2 (one write): the reference app's stderr is a stdio
// stream it also prints progress to, and a buffered line would be lost when the
// app then crashes (the unchanged caller's lost page, test_c1_app.py).
void log_error(const std::string &m) {
    if (!knob("LOG_ERRORS", 0)) return;
    const std::string line = "tyche-engine: " + m + "\n";
    (void)!write(2, line.data(), line.size());
}
int fail(const char *what, hipError_t e) {
    t_error = std::string(what) + ": " + hipGetErrorString(e);
    log_error(t_error);
    return TYCHE_E_DEVICE;
}
int fail_msg(const std::string &m) {
    t_error = m;
    log_error(t_error);
    return TYCHE_E_DEVICE;
}

uint64_t now_ns() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

bool device_is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// The devices the host API uses when the thread is not pinned: the visible
// gfx950 devices, the first TYCHE_DEVICES of them when that is set.
struct DeviceSet {
    std::vector<int> ids;
    std::string why;   // empty when ids is non-empty
};
const DeviceSet &device_set() {
    static DeviceSet &ds = *new DeviceSet([] {
        DeviceSet d;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
            d.why = "no HIP device available (the codec runs only on the GPU)";
            return d;
        }
        // TYCHE_DEVICE_IDS: an explicit list ("0,1,2"; repeats allowed, which lets
        // one GPU rehearse the multi-device fan-out in tests)
        if (const char *ids = getenv("TYCHE_DEVICE_IDS")) {
            for (const char *p = ids; *p;) {
                char *end = nullptr;
                const long v = strtol(p, &end, 10);
                if (end == p) break;
                if (v >= 0 && v < n && v < kMaxDevices && device_is_gfx950((int)v)) d.ids.push_back((int)v);
                p = *end == ',' ? end + 1 : end;
            }
        } else {
            const char *env = getenv("TYCHE_DEVICES");
            const int want = env ? atoi(env) : n;
            for (int i = 0; i < n && (int)d.ids.size() < want && i < kMaxDevices; i++)
                if (device_is_gfx950(i)) d.ids.push_back(i);
        }
        if (d.ids.empty()) d.why = "no gfx950 device; libtyche_codec.so carries gfx950 code only";
        return d;
    }());   // never destroyed, like the pools
    return ds;
}

// Restores the calling thread's current device when it goes out of scope: the
// host entry points switch devices to run a batch, and a caller (a torch rank
// after set_device, say) must find its own device current afterwards.
struct DeviceGuard {
    int saved = -1;
    DeviceGuard() {
        if (hipGetDevice(&saved) != hipSuccess) saved = -1;
    }
    ~DeviceGuard() {
        int now = -1;
        if (saved >= 0 && hipGetDevice(&now) == hipSuccess && now != saved) (void)hipSetDevice(saved);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

// makes `dev` current on this thread after checking it (cached per device)
int ensure_device(int dev) {
    static std::atomic<int> ok[kMaxDevices];   // 0 unknown, 1 gfx950, 2 unusable
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return fail_msg("no HIP device available (the codec runs only on the GPU)");
    if (dev < 0 || dev >= n || dev >= kMaxDevices) return fail_msg("selected device out of range");
    e = hipSetDevice(dev);
    if (e != hipSuccess) return fail("hipSetDevice", e);
    if (ok[dev].load() == 0) ok[dev].store(device_is_gfx950(dev) ? 1 : 2);
    if (ok[dev].load() != 1) return fail_msg("device is not gfx950; libtyche_codec.so carries gfx950 code only");
    return TYCHE_E_OK;
}

int rank_device();

// the device for a thread's device-side work: its pinned one, the rank's, else the first of the set
int current_device(int *dev) {
    if (t_device >= 0 || rank_device() >= 0) {
        *dev = t_device >= 0 ? t_device : rank_device();
        return TYCHE_E_OK;
    }
    const DeviceSet &ds = device_set();
    if (ds.ids.empty()) return fail_msg(ds.why);
    *dev = ds.ids[0];
    return TYCHE_E_OK;
}

// codecs with a gfx950 kernel, per direction
bool valid_codec(int id) {
    return id == TYCHE_LZ4_COMPRESSOR_ID || id == TYCHE_ZLIB_COMPRESSOR_ID || id == TYCHE_ZSTD_COMPRESSOR_ID;
}

// the encoder kernel for a codec id (valid_codec)
hipError_t launch_encode(int id, const tyche_batch_t &b, uint32_t in_cap, hipStream_t s) {
    // Test hook (TYCHE_FAIL_COMPRESS_EVERY=N or the knob): every Nth encode launch
    // fails as a lost device would, so the callers' TYCHE_E_DEVICE handling
    // (list.c:1051-1060 and the INTEGRATION.md change) can be exercised.
    static std::atomic<unsigned long> launches{0};
    const long every = knob("FAIL_COMPRESS_EVERY", 0);
    if (every > 0 && (launches.fetch_add(1) + 1) % (unsigned long)every == 0) return hipErrorLaunchFailure;
    if (id == TYCHE_ZSTD_COMPRESSOR_ID) return launch_zstd_encode(b, in_cap, s);
    if (id == TYCHE_ZLIB_COMPRESSOR_ID) return launch_zlib_deflate(b, in_cap, s);
    return launch_lz4_encode(b, in_cap, s);
}
bool valid_decode_codec(int id) {
    return id == TYCHE_LZ4_COMPRESSOR_ID || id == TYCHE_ZLIB_COMPRESSOR_ID || id == TYCHE_ZSTD_COMPRESSOR_ID;
}

std::string codec_msg(int id) {
    if (id == TYCHE_ZLIB_COMPRESSOR_ID || id == TYCHE_ZSTD_COMPRESSOR_ID)
        return "compressor id " + std::to_string(id) + " has no gfx950 kernel for this direction in this build";
    return "unknown compressor id " + std::to_string(id);
}

// zlib 1.2.8 compressBound (compress.c:74-78)
inline uint32_t zlib_bound(uint32_t n) { return n + (n >> 12) + (n >> 14) + (n >> 25) + 13u; }
// zstd 1.1.2 ZSTD_compressBound (zstd_compress.c:37): FSE_compressBound(n) + 12
inline uint32_t zstd_bound(uint32_t n) { return n + (n >> 7) + 512u + 12u; }

// in_cap for a decode batch: the largest stream length (or a bound for unknown lengths)
inline uint32_t decode_in_cap(const tyche_batch_t &b, uint32_t fallback) {
    uint32_t in_cap = b.src_lengths ? b.max_src_length : b.src_length;
    if (b.src_lengths && in_cap == 0) in_cap = fallback;
    return in_cap;
}

// ---------------------------------------------------------------- host batches
// The Buffer API and the host batch entry points start and end in host memory
// (tyche's Buffer->data is malloc'd, src/buffer.c:181, 246).  A batch is cut
// into chunks of ~kChunkBytes of input that flow through a ring of kSlots
// staging slots, one HIP stream each:
//
//   host gather (thread pool memcpy into pinned) -> H2D -> kernel -> D2H -> host scatter
//
// so chunk c's gather overlaps chunk c-1's copies and kernel and chunk c-2's
// scatter; the two copy directions and the kernels of different slots run
// concurrently.  tyche calls the codec from its compressor pool and its
// worker threads at once (src/list.c:1051, 572; opts.cpu_count threads,
// src/options.c:64): the staging contexts are therefore a small per-device pool
// (TYCHE_HOST_CONTEXTS, default kContextsPerDevice) that a call borrows for its
// duration, not one per calling thread, so streams and pinned arenas stay
// bounded however many threads call in.
struct Arena {
    void *p = nullptr;
    void *dp = nullptr;   // host arenas: the device's address of the pinned buffer (zero-copy launches)
    size_t cap = 0;
    bool host = false;
    int grow(size_t need) {
        if (need <= cap) return TYCHE_E_OK;
        size_t n = std::max(need, cap * 2);
        n = (n + 4095) & ~size_t(4095);
        release();
        hipError_t e = host ? hipHostMalloc(&p, n, hipHostMallocDefault) : hipMalloc(&p, n);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(host ? "hipHostMalloc" : "hipMalloc", e);
        }
        if (host && hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) dp = nullptr;
        cap = n;
        return TYCHE_E_OK;
    }
    void release() {
        if (p) {
            if (host) (void)hipHostFree(p); else (void)hipFree(p);
        }
        p = dp = nullptr;
        cap = 0;
    }
};

constexpr int kSlots = 4;   // round 3: 4 x 32 MiB (was 3 x 64 MiB): the host path waited on streams ~30 % of a call
constexpr size_t kChunkBytes = size_t(32) << 20;
constexpr int kContextsPerDevice = 8;

struct Slot {
    hipStream_t stream = nullptr;
    Arena h_in, h_out, h_meta, d_in, d_out, d_meta;
    size_t first = 0, count = 0;   // pages of the chunk in flight
    bool busy = false;
    Slot() { h_in.host = h_out.host = h_meta.host = true; }
};

struct HostCtx {
    Slot slot[kSlots];
    int group = 0;   // hardware-queue group of slot 0's stream (see acquire_ctx)
    // waits for whatever the slots still hold and forgets it (error paths)
    void abandon() {
        for (Slot &s : slot)
            if (s.busy) {
                (void)hipStreamSynchronize(s.stream);
                s.busy = false;
            }
    }
};

struct CtxPool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<HostCtx *> all, idle;
    std::vector<int> busy;   // leased contexts per hardware-queue group
};
CtxPool *const g_ctx = new CtxPool[kMaxDevices];   // never destroyed (restore dispatchers may run at exit)

// HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default), in
// creation order; kernels of streams that share a queue run one after the
// other (tools/probes/hwq.hip: with 24 streams, stream 0 overlaps streams
// 1-6 but serializes with 7, 11, 15, ...).  Two restore batches (an LZ4 and a
// zlib one, say) on contexts whose streams share a queue therefore wait for
// each other.  So a device's contexts are created together, their streams in
// an order that puts slot s of context i in group (i + s) mod Q -- the three
// slots of one context on three queues, for the chunk pipeline -- and a call
// borrows the idle context whose group has the fewest calls running.
int hw_queues() {
    static const int q = [] {
        const char *env = getenv("GPU_MAX_HW_QUEUES");
        const int v = env ? atoi(env) : 4;
        return v > 0 ? v : 4;
    }();
    return q;
}

int context_cap() {
    static const int cap = [] {
        const char *env = getenv("TYCHE_HOST_CONTEXTS");
        const int v = env ? atoi(env) : kContextsPerDevice;
        return v > 0 ? v : kContextsPerDevice;
    }();
    return cap;
}

// creates the device's contexts (under P.mu): stream k created goes to queue
// group k mod Q, and is given to the (context, slot) pair of that group
int create_contexts(CtxPool &P) {
    const int n = context_cap(), Q = hw_queues();
    std::vector<HostCtx *> cs;
    for (int i = 0; i < n; i++) {
        cs.push_back(new HostCtx);
        cs.back()->group = i % Q;
    }
    std::vector<bool> made((size_t)n * kSlots, false);
    for (int k = 0; k < n * kSlots; k++) {
        int pick = -1;
        for (int j = 0; j < n * kSlots && pick < 0; j++)
            if (!made[j] && ((j / kSlots) + (j % kSlots)) % Q == k % Q) pick = j;
        for (int j = 0; j < n * kSlots && pick < 0; j++)
            if (!made[j]) pick = j;
        made[pick] = true;
        hipError_t e = hipStreamCreateWithFlags(&cs[pick / kSlots]->slot[pick % kSlots].stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            for (HostCtx *c : cs) {
                for (Slot &t : c->slot)
                    if (t.stream) (void)hipStreamDestroy(t.stream);
                delete c;
            }
            return fail("hipStreamCreate", e);
        }
    }
    P.all = cs;
    P.idle = cs;
    P.busy.assign((size_t)Q, 0);
    return TYCHE_E_OK;
}

// borrows a staging context of device dev (current on this thread); waits while all are busy
int acquire_ctx(int dev, HostCtx **out) {
    CtxPool &P = g_ctx[dev];
    std::unique_lock<std::mutex> g(P.mu);
    if (P.all.empty()) {
        const int rc = create_contexts(P);
        if (rc) return rc;
    }
    P.cv.wait(g, [&] { return !P.idle.empty(); });
    // least-busy group; among equals the most recently released context (its
    // pinned and device arenas are already grown -- a fresh context pays
    // hipHostMalloc/hipMalloc for its staging slots on first use)
    size_t best = P.idle.size() - 1;
    for (size_t k = best; k-- > 0;)
        if (P.busy[(size_t)P.idle[k]->group] < P.busy[(size_t)P.idle[best]->group]) best = k;
    *out = P.idle[best];
    P.idle.erase(P.idle.begin() + (long)best);
    P.busy[(size_t)(*out)->group]++;
    return TYCHE_E_OK;
}
void release_ctx(int dev, HostCtx *c) {
    CtxPool &P = g_ctx[dev];
    {
        std::lock_guard<std::mutex> g(P.mu);
        P.busy[(size_t)c->group]--;
        P.idle.push_back(c);
    }
    P.cv.notify_one();
}

inline size_t up16(size_t x) { return (x + 15) & ~size_t(15); }

// Page copies between malloc'd Buffers and the pinned staging arenas.  The host
// path is bound by these copies (r03 stage clocks: gather + scatter ~10 of the
// 15 ms of a 32K-page decompress call), and a plain memcpy of a 16 KiB page
// reads its destination's lines before writing them (read-for-ownership): three
// DRAM transfers per byte.  Non-temporal 16-byte stores skip that read; the
// caller of a pool job fences once at its end (copy_fence) before handing the
// arena to a DMA or the caller.
inline void copy_nt(void *dst, const void *src, size_t n) {
    if (n < 512 || ((uintptr_t)dst & 15u)) {
        memcpy(dst, src, n);
        return;
    }
    __m128i *d = (__m128i *)dst;
    const __m128i *p = (const __m128i *)src;
    size_t k = n >> 6;
    for (; k; k--, d += 4, p += 4) {
        const __m128i a = _mm_loadu_si128(p), b = _mm_loadu_si128(p + 1), c = _mm_loadu_si128(p + 2),
                      e = _mm_loadu_si128(p + 3);
        _mm_stream_si128(d, a);
        _mm_stream_si128(d + 1, b);
        _mm_stream_si128(d + 2, c);
        _mm_stream_si128(d + 3, e);
    }
    const size_t done = n & ~(size_t)63;
    if (done < n) memcpy((uint8_t *)dst + done, (const uint8_t *)src + done, n - done);
}
inline void copy_fence() { _mm_sfence(); }

// A persistent worker pool for the host-side page copies (memcpy of scattered
// malloc'd pages into and out of pinned staging).  Several callers (one per
// device of a fanned-out batch, concurrent tyche threads) may run jobs at once:
// each caller works on its own job and idle workers join whichever job still
// has ranges left.
class CopyPool {
  public:
    static CopyPool &get() {
        // never destroyed: its detached workers wait on its condition variable until exit
        static CopyPool *p = new CopyPool;
        return *p;
    }
    // runs f(i) for i in [0, n), in contiguous ranges, on the pool and the caller
    template <typename F>
    void run(size_t n, F f) {
        if (n < 64 || workers_.empty()) {
            for (size_t i = 0; i < n; i++) f(i);
            copy_fence();
            return;
        }
        std::function<void(size_t, size_t)> body = [&f](size_t a, size_t b) {
            for (size_t i = a; i < b; i++) f(i);
            copy_fence();   // the job's non-temporal stores are globally visible before it completes
        };
        Job j;
        j.body = &body;
        j.n = n;
        {
            std::lock_guard<std::mutex> g(mu_);
            jobs_.push_back(&j);
        }
        cv_.notify_all();
        work(j);
        std::unique_lock<std::mutex> g(mu_);
        jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &j));   // no worker joins it from now on
        done_cv_.wait(g, [&] { return j.active == 0; });
    }

  private:
    static constexpr size_t kGrain = 32;
    struct Job {
        const std::function<void(size_t, size_t)> *body = nullptr;
        size_t n = 0;
        std::atomic<size_t> next{0};
        int active = 0;   // workers inside work(); guarded by mu_
    };
    CopyPool() {
        unsigned t = std::thread::hardware_concurrency();
        const char *env = getenv("TYCHE_HOST_THREADS");
        unsigned want = env ? (unsigned)atoi(env) : std::min(16u, t ? t : 1u);
        for (unsigned i = 1; i < want; i++) workers_.emplace_back([this] { loop(); });
        for (auto &w : workers_) w.detach();
    }
    static void work(Job &j) {
        for (;;) {
            const size_t a = j.next.fetch_add(kGrain);
            if (a >= j.n) break;
            (*j.body)(a, std::min(j.n, a + kGrain));
        }
    }
    Job *open_job() {   // under mu_
        for (Job *j : jobs_)
            if (j->next.load() < j->n) return j;
        return nullptr;
    }
    void loop() {
        for (;;) {
            Job *j = nullptr;
            {
                // j->next advances outside the lock (callers and workers claim ranges with
                // fetch_add): pick the job once, in the predicate, and pin it there
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return (j = open_job()) != nullptr; });
                j->active++;
            }
            work(*j);
            {
                std::lock_guard<std::mutex> g(mu_);
                j->active--;
            }
            done_cv_.notify_all();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<Job *> jobs_;
};

std::atomic<int> g_inflight[kMaxDevices];   // host batches running per device


// run_host_batch's direct_out modes (see there)
enum { kDirectNone = 0, kDirectAlways = 1, kDirectLz4Decode = 2 };

// Host-path stage clocks (diagnostics, tyche_host_profile): ns spent by calling threads waiting for a
// slot's stream, scattering results, gathering inputs, and enqueuing copies and kernels; bytes gathered
// and scattered.
enum { kHpWait, kHpScatter, kHpGather, kHpEnqueue, kHpGatherBytes, kHpScatterBytes, kHpChunks, kHpCount };
std::atomic<uint64_t> g_hprof[kHpCount];
struct HpClock {
    int slot;
    uint64_t t0;
    explicit HpClock(int s) : slot(s), t0(now_ns()) {}
    ~HpClock() { g_hprof[slot] += now_ns() - t0; }
};

// Moves n host pages through `launch` on device dev, chunk by chunk (see
// above).  results[i] gets the kernel's per-page result; for results in
// (0, dst_cap[i]] that many output bytes land in dst[i].  On any failure the
// context's slots are drained before it goes back to the pool, so a later call
// never scatters a failed call's chunk.
// Zero-copy limit: a decompress batch of at most this many bytes (input plus
// output capacity) skips the device staging buffers -- the kernel reads the
// gathered streams and the page table from the pinned host arenas and writes
// results and pages straight back into them.  No H2D/D2H copies (two
// hipMemcpyAsync calls and two copy kernels each way saved on the restore
// path's small batches); the kernels stage their input in LDS with 16-byte
// loads and write whole 16-byte vectors, which PCIe carries well.
// TYCHE_ZERO_COPY_BYTES=0 turns it off.
size_t zero_copy_bytes() { return (size_t)std::max(0L, knob("ZERO_COPY_BYTES", 4L << 20)); }

template <typename Launch>
int run_host_batch(int dev, size_t n, const void *const *src, const uint32_t *src_len, void *const *dst,
                   const uint32_t *dst_cap, int32_t *results, Launch launch, bool zc_ok = false,
                   int direct_out = kDirectNone) {
    DeviceGuard keep;   // the caller's device is current again on every return
    int rc = ensure_device(dev);
    if (rc) return rc;
    struct Inflight {
        int d;
        explicit Inflight(int dd) : d(dd) { g_inflight[d]++; }
        ~Inflight() { g_inflight[d]--; }
    } inflight(dev);
    HostCtx *cp = nullptr;
    if ((rc = acquire_ctx(dev, &cp))) return rc;
    HostCtx &c = *cp;
    CopyPool &pool = CopyPool::get();
    hipError_t e;
    std::function<void()> before_bail;   // stops the async finisher (below) before the slots are drained
    auto bail = [&](int r) {
        if (before_bail) before_bail();
        c.abandon();
        release_ctx(dev, cp);
        return r;
    };

    // completes the chunk held by slot s: wait for its stream, scatter its outputs
    auto finish = [&](Slot &S) -> int {
        if (!S.busy) return TYCHE_E_OK;
        S.busy = false;
        {
            HpClock hc(kHpWait);
            if ((e = hipStreamSynchronize(S.stream)) != hipSuccess) return fail("hipStreamSynchronize", e);
        }
        HpClock hc(kHpScatter);
        const size_t k = S.count;
        const uint64_t *m_doff = (const uint64_t *)S.h_meta.p + k;
        const int32_t *m_res = (const int32_t *)((const uint8_t *)S.h_meta.p + k * 24);
        const uint8_t *hout = (const uint8_t *)S.h_out.p;
        const size_t f0 = S.first;
        std::atomic<uint64_t> moved{0};
        const bool no_copy = host_diag_no_copy();
        pool.run(k, [&](size_t j) {
            const int32_t r = m_res[j];
            results[f0 + j] = r;
            if (r > 0 && (uint32_t)r <= dst_cap[f0 + j] && !no_copy) {
                copy_nt(dst[f0 + j], hout + m_doff[j], (size_t)r);
                moved.fetch_add((uint64_t)r, std::memory_order_relaxed);
            }
        });
        g_hprof[kHpScatterBytes] += moved.load();
        g_hprof[kHpChunks]++;
        return TYCHE_E_OK;
    };

    if (zc_ok) {
        size_t in_bytes = 0, out_bytes = 0;
        uint32_t max_in = 0, max_out = 0;
        for (size_t j = 0; j < n; j++) {
            in_bytes += up16(src_len[j]);
            out_bytes += up16(dst_cap[j]);
            max_in = std::max(max_in, src_len[j]);
            max_out = std::max(max_out, dst_cap[j]);
        }
        if (in_bytes + out_bytes <= zero_copy_bytes()) {
            Slot &S = c.slot[0];
            const size_t meta_bytes = n * 28 + 64;
            if ((rc = S.h_in.grow(in_bytes + 16)) || (rc = S.h_out.grow(out_bytes + 16)) ||
                (rc = S.h_meta.grow(meta_bytes)))
                return bail(rc);
            if (S.h_in.dp && S.h_out.dp && S.h_meta.dp) {
                uint64_t *m_soff = (uint64_t *)S.h_meta.p;
                uint64_t *m_doff = m_soff + n;
                uint32_t *m_slen = (uint32_t *)(m_doff + n);
                uint32_t *m_dcap = m_slen + n;
                int32_t *m_res = (int32_t *)(m_dcap + n);
                size_t so = 0, dof = 0;
                for (size_t j = 0; j < n; j++) {
                    m_soff[j] = so;
                    m_doff[j] = dof;
                    m_slen[j] = src_len[j];
                    m_dcap[j] = dst_cap[j];
                    so += up16(src_len[j]);
                    dof += up16(dst_cap[j]);
                }
                uint8_t *hin = (uint8_t *)S.h_in.p;
                {
                    HpClock hc(kHpGather);
                    pool.run(n, [&](size_t j) {
                        if (m_slen[j]) copy_nt(hin + m_soff[j], src[j], m_slen[j]);
                    });
                }
                uint8_t *dm = (uint8_t *)S.h_meta.dp;
                tyche_batch_t b{};
                b.count = n;
                b.src = S.h_in.dp;
                b.src_offsets = (const uint64_t *)dm;
                b.src_lengths = (const uint32_t *)(dm + ((uint8_t *)m_slen - (uint8_t *)m_soff));
                b.max_src_length = max_in;
                b.dst = S.h_out.dp;
                b.dst_offsets = (const uint64_t *)(dm + ((uint8_t *)m_doff - (uint8_t *)m_soff));
                b.dst_capacities = (const uint32_t *)(dm + ((uint8_t *)m_dcap - (uint8_t *)m_soff));
                b.dst_capacity = max_out;
                b.results = (int32_t *)(dm + ((uint8_t *)m_res - (uint8_t *)m_soff));
                S.first = 0;
                S.count = n;
                S.busy = true;
                {
                    HpClock hc(kHpEnqueue);
                    if ((e = launch(b, S.stream, true)) != hipSuccess) return bail(fail("kernel launch", e));
                }
                S.busy = false;
                {
                    HpClock hc(kHpWait);
                    if ((e = hipStreamSynchronize(S.stream)) != hipSuccess) return bail(fail("hipStreamSynchronize", e));
                }
                const uint8_t *hout = (const uint8_t *)S.h_out.p;
                HpClock hc(kHpScatter);
                pool.run(n, [&](size_t j) {
                    const int32_t r = m_res[j];
                    results[j] = r;
                    if (r > 0 && (uint32_t)r <= dst_cap[j]) copy_nt(dst[j], hout + m_doff[j], (size_t)r);
                });
                release_ctx(dev, cp);
                return TYCHE_E_OK;
            }
        }
    }

    size_t first = 0;
    int si = 0;
    // Async finishing (round 3): with three or more chunks a helper thread waits for each slot's
    // stream and scatters its results while the caller gathers and enqueues the next chunk -- the
    // r03 stage clocks had the caller waiting on streams ~25 % of a call, between its copies.
    // A slot is reused only after the helper has scattered it (S.busy false, under fm).
    size_t nchunks_est = 0, rem_in = 0, rem_out = 0;   // rem_*: bytes of the batch not yet in a chunk
    {
        for (size_t j = 0; j < n; j++) {
            rem_in += up16(src_len[j]);
            rem_out += up16(dst_cap[j]);
        }
        nchunks_est = (rem_in + rem_out) /
                      std::max<size_t>(1, (size_t)std::max(1L, knob("HOST_CHUNK_MB", (long)(kChunkBytes >> 20))) << 20);
    }
    const bool async = nchunks_est >= 3 && knob("HOST_ASYNC_SCATTER", 1) != 0;
    std::mutex fm;
    std::condition_variable fcv;
    std::vector<int> fq;   // slots to finish, in issue order
    bool fstop = false;
    int frc = TYCHE_E_OK;
    std::string ferr;
    std::vector<std::thread> fth;
    auto finish_async = [&](Slot &S) -> int {   // helper thread: sync, scatter, then free the slot
        hipError_t fe;
        {
            HpClock hc(kHpWait);
            if ((fe = hipStreamSynchronize(S.stream)) != hipSuccess) return fail("hipStreamSynchronize", fe);
        }
        HpClock hc(kHpScatter);
        const size_t k = S.count;
        const uint64_t *m_doff = (const uint64_t *)S.h_meta.p + k;
        const int32_t *m_res = (const int32_t *)((const uint8_t *)S.h_meta.p + k * 24);
        const uint8_t *hout = (const uint8_t *)S.h_out.p;
        const size_t f0 = S.first;
        std::atomic<uint64_t> moved{0};
        const bool no_copy = host_diag_no_copy();
        pool.run(k, [&](size_t j) {
            const int32_t r = m_res[j];
            results[f0 + j] = r;
            if (r > 0 && (uint32_t)r <= dst_cap[f0 + j] && !no_copy) {
                copy_nt(dst[f0 + j], hout + m_doff[j], (size_t)r);
                moved.fetch_add((uint64_t)r, std::memory_order_relaxed);
            }
        });
        g_hprof[kHpScatterBytes] += moved.load();
        g_hprof[kHpChunks]++;
        return TYCHE_E_OK;
    };
    // HOST_FINISHERS helpers (default 1), each taking the next queued slot (chunks go to disjoint
    // destinations, so their scatters may run in any order, on the shared copy pool).  Round 5: a
    // second and third helper, so that one chunk's scatter overlaps the next one's wait, did not
    // move decompress (32K pages, best of 5 interleaved: 34.2 / 33.7 / 31.7 GiB/s for 1 / 2 / 3,
    // profiles/r05_host_probe.jsonl).
    const int nfin = async ? (int)std::min(4L, std::max(1L, knob("HOST_FINISHERS", 1))) : 0;
    for (int h = 0; h < nfin; h++) {
        fth.emplace_back([&] {
            for (;;) {
                int idx;
                {
                    std::unique_lock<std::mutex> g(fm);
                    fcv.wait(g, [&] { return !fq.empty() || fstop || frc != TYCHE_E_OK; });
                    if (fq.empty() || frc != TYCHE_E_OK) return;
                    idx = fq.front();
                    fq.erase(fq.begin());
                }
                const int r = finish_async(c.slot[idx]);
                std::lock_guard<std::mutex> g(fm);
                if (r) {
                    if (frc == TYCHE_E_OK) {
                        frc = r;
                        ferr = t_error;   // the helper's thread-local message
                    }
                    fcv.notify_all();
                    return;
                }
                c.slot[idx].busy = false;
                fcv.notify_all();
            }
        });
    }
    auto stop_helper = [&] {
        if (fth.empty()) return;
        {
            std::lock_guard<std::mutex> g(fm);
            fstop = true;
        }
        fcv.notify_all();
        for (auto &t : fth) t.join();
        fth.clear();
    };
    struct HelperJoin {   // every return path stops the helper (bail() does so before draining the streams)
        std::function<void()> f;
        ~HelperJoin() { f(); }
    } helper_join{stop_helper};
    before_bail = stop_helper;
    auto async_fail = [&]() -> int {
        stop_helper();
        t_error = ferr;
        return frc;
    };
    // chunks hold ~chunk_bytes of input AND of output capacity: a decompress batch's
    // output is ~2.6x its input, so cutting by input alone made 3 chunks of 170 MiB
    // of D2H each out of a 32K-page batch, too few to overlap the two copy directions
    const size_t chunk_bytes = (size_t)std::max(1L, knob("HOST_CHUNK_MB", (long)(kChunkBytes >> 20))) << 20;
    // ramp (HOST_RAMP, default on): the first and the last chunk are a quarter chunk, so the
    // pipeline fills (H2D + kernel before the first D2H) and drains (the last D2H + scatter,
    // which nothing overlaps) on small chunks
    const bool ramp = knob("HOST_RAMP", 1) != 0 && nchunks_est >= 3;
    const size_t quarter = std::max<size_t>(chunk_bytes / 4, 1u << 20);
    size_t nchunk = 0;
    while (first < n) {
        // ---- chunk [first, last)
        size_t limit = chunk_bytes;
        if (ramp) {
            const size_t rem = std::max(rem_in, rem_out);
            if (nchunk == 0) limit = quarter;
            else if (rem <= chunk_bytes + quarter && rem > quarter) limit = rem - quarter;
        }
        nchunk++;
        size_t last = first, in_bytes = 0, out_bytes = 0;
        uint32_t max_in = 0, max_out = 0;
        while (last < n && (last == first || (in_bytes + up16(src_len[last]) <= limit &&
                                              out_bytes + up16(dst_cap[last]) <= limit))) {
            in_bytes += up16(src_len[last]);
            out_bytes += up16(dst_cap[last]);
            max_in = std::max(max_in, src_len[last]);
            max_out = std::max(max_out, dst_cap[last]);
            last++;
        }
        const size_t k = last - first;
        rem_in -= in_bytes;
        rem_out -= out_bytes;
        Slot &S = c.slot[si];
        if (async) {   // the helper has scattered the slot's previous chunk
            std::unique_lock<std::mutex> g(fm);
            fcv.wait(g, [&] { return !S.busy || frc != TYCHE_E_OK; });
            if (frc != TYCHE_E_OK) {
                g.unlock();
                return bail(async_fail());
            }
        } else if ((rc = finish(S))) {
            return bail(rc);   // the slot's previous chunk
        }
        // meta layout: soff[k] u64, doff[k] u64, slen[k] u32, dcap[k] u32, res[k] i32
        const size_t meta_bytes = k * 28 + 64;
        if ((rc = S.h_in.grow(in_bytes + 16)) || (rc = S.h_out.grow(out_bytes + 16)) ||
            (rc = S.h_meta.grow(meta_bytes)) || (rc = S.d_in.grow(in_bytes + 16)) ||
            (rc = S.d_out.grow(out_bytes + 16)) || (rc = S.d_meta.grow(meta_bytes)))
            return bail(rc);
        uint64_t *m_soff = (uint64_t *)S.h_meta.p;
        uint64_t *m_doff = m_soff + k;
        uint32_t *m_slen = (uint32_t *)(m_doff + k);
        uint32_t *m_dcap = m_slen + k;
        int32_t *m_res = (int32_t *)(m_dcap + k);
        size_t so = 0, dof = 0;
        for (size_t j = 0; j < k; j++) {
            m_soff[j] = so;
            m_doff[j] = dof;
            m_slen[j] = src_len[first + j];
            m_dcap[j] = dst_cap[first + j];
            so += up16(src_len[first + j]);
            dof += up16(dst_cap[first + j]);
        }
        uint8_t *hin = (uint8_t *)S.h_in.p;
        {
            HpClock hc(kHpGather);
            pool.run(k, [&](size_t j) {
                if (m_slen[j]) copy_nt(hin + m_soff[j], src[first + j], m_slen[j]);
            });
            g_hprof[kHpGatherBytes] += so;
        }
        HpClock enq(kHpEnqueue);
        // ---- H2D -> kernel -> D2H on the slot's stream
        uint8_t *dmeta = (uint8_t *)S.d_meta.p;
        const size_t head_bytes = (uint8_t *)m_res - (uint8_t *)m_soff;
        S.first = first;
        S.count = k;
        {
            std::lock_guard<std::mutex> g(fm);
            S.busy = true;   // from the first enqueued copy on, the slot must be drained on failure
        }
        if ((e = hipMemcpyAsync(dmeta, S.h_meta.p, head_bytes, hipMemcpyHostToDevice, S.stream)) != hipSuccess)
            return bail(fail("hipMemcpyAsync(meta)", e));
        if (so && (e = hipMemcpyAsync(S.d_in.p, hin, so, hipMemcpyHostToDevice, S.stream)) != hipSuccess)
            return bail(fail("hipMemcpyAsync(in)", e));
        tyche_batch_t b{};
        b.count = k;
        b.src = S.d_in.p;
        b.src_offsets = (const uint64_t *)dmeta;
        b.src_lengths = (const uint32_t *)(dmeta + ((uint8_t *)m_slen - (uint8_t *)m_soff));
        b.max_src_length = max_in;
        // direct_out: the kernel writes its results straight into the pinned arena over PCIe, as
        // posted writes that overlap its own work, and no D2H of the arena follows.  LZ4 compress
        // (kDirectAlways): only the compressed bytes cross the link -- a D2H of the arena would move
        // every page's full capacity (16 KiB+ per 16 KiB page at ratio 2.6).  LZ4 decompress
        // (kDirectLz4Decode): the jump and wave decoders write each page once, whole, from LDS; the
        // lane decoder (chunks of >= kLaneMin pages) reads its own output back, so it keeps the D2H;
        // TYCHE_HOST_DIRECT_DECODE_MAX: chunks of more pages than this stage through HBM too.  The
        // choice is made once here and handed to the launch (host_dst), so a knob changed meanwhile
        // cannot put the lane decoder on a host destination.
        const bool direct = S.h_out.dp != nullptr &&
                            (direct_out == kDirectAlways ||
                             (direct_out == kDirectLz4Decode && !lz4_lane_decode_wanted(k, max_in, max_out) &&
                              (long)k <= knob("HOST_DIRECT_DECODE_MAX", 1L << 30)));
        b.dst = direct ? S.h_out.dp : S.d_out.p;
        b.dst_offsets = (const uint64_t *)(dmeta + ((uint8_t *)m_doff - (uint8_t *)m_soff));
        b.dst_capacities = (const uint32_t *)(dmeta + ((uint8_t *)m_dcap - (uint8_t *)m_soff));
        b.dst_capacity = max_out;
        b.results = (int32_t *)(dmeta + head_bytes);
        if ((e = launch(b, S.stream, direct)) != hipSuccess) return bail(fail("kernel launch", e));
        if ((e = hipMemcpyAsync(m_res, b.results, k * 4, hipMemcpyDeviceToHost, S.stream)) != hipSuccess)
            return bail(fail("hipMemcpyAsync(results)", e));
        if (dof && !direct && (e = hipMemcpyAsync(S.h_out.p, S.d_out.p, dof, hipMemcpyDeviceToHost, S.stream)) != hipSuccess)
            return bail(fail("hipMemcpyAsync(out)", e));
        if (async) {
            std::lock_guard<std::mutex> g(fm);
            fq.push_back(si);
            fcv.notify_all();
        }
        first = last;
        si = (si + 1) % kSlots;
    }
    if (async) {   // the helper drains the queue, then stops
        stop_helper();
        if (frc != TYCHE_E_OK) {
            t_error = ferr;
            return bail(frc);
        }
        release_ctx(dev, cp);
        return TYCHE_E_OK;
    }
    // drain in issue order
    for (int j = 0; j < kSlots; j++)
        if ((rc = finish(c.slot[(si + j) % kSlots]))) return bail(rc);
    release_ctx(dev, cp);
    return TYCHE_E_OK;
}

// minimum input bytes per device before a host batch is split across devices
uint64_t fanout_min_bytes() { return (uint64_t)std::max(0L, knob("FANOUT_MIN_BYTES", 64L << 20)); }

// A process launched one per GPU (torch.distributed.run sets LOCAL_RANK and
// LOCAL_WORLD_SIZE) keeps its host work on its own device -- LOCAL_RANK modulo
// the visible devices, torch's convention, whichever thread calls.  Only
// LOCAL_RANK engages it (a launcher that sets WORLD_SIZE alone gets the
// fan-out, not device 0), a LOCAL_WORLD_SIZE of 1 does not (the node's only
// process may use every device), and TYCHE_DEVICES / TYCHE_DEVICE_IDS or the
// RANK_PIN knob (0, at any time through tyche_set_knob) turn it off, e.g. for a
// helper process that inherited a worker's environment.  -1: not pinned.
int rank_device() {
    static const int d = [] {
        if (getenv("TYCHE_DEVICES") || getenv("TYCHE_DEVICE_IDS")) return -1;
        const char *lr = getenv("LOCAL_RANK"), *lw = getenv("LOCAL_WORLD_SIZE");
        if (!lr || !*lr || (lw && atoi(lw) == 1)) return -1;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -1;
        return std::max(0, atoi(lr)) % n;
    }();
    return d >= 0 && knob("RANK_PIN", 1) != 0 ? d : -1;
}

// the device with the fewest host batches in flight (ties rotate)
int pick_device(const std::vector<int> &ids) {
    static std::atomic<unsigned> rot{0};
    const unsigned r = rot++;
    int best = ids[r % ids.size()];
    for (size_t k = 0; k < ids.size(); k++) {
        const int d = ids[(r + k) % ids.size()];
        if (g_inflight[d].load() < g_inflight[best].load()) best = d;
    }
    return best;
}

// Host batch over the calling thread's devices: its pinned device, or the
// device set.  Batches of at least two parts' worth of input
// (tyche_plan_split) are cut into contiguous page ranges of about equal input
// bytes, one per device, run concurrently; smaller ones go whole to the least
// busy device, so concurrent small calls (tyche's per-page compressor pool and
// restores) spread over all devices.
template <typename Launch>
int run_host(size_t n, const void *const *src, const uint32_t *src_len, void *const *dst, const uint32_t *dst_cap,
             int32_t *results, Launch launch, bool zc_ok = false, int direct_out = kDirectNone) {
    if (t_device >= 0) return run_host_batch(t_device, n, src, src_len, dst, dst_cap, results, launch, zc_ok, direct_out);
    if (rank_device() >= 0)   // one process per GPU: its own device only
        return run_host_batch(rank_device(), n, src, src_len, dst, dst_cap, results, launch, zc_ok, direct_out);
    const DeviceSet &ds = device_set();
    if (ds.ids.empty()) return fail_msg(ds.why);
    std::vector<size_t> cuts(ds.ids.size() + 1);
    const size_t parts = tyche_plan_split(n, src_len, (int)ds.ids.size(), fanout_min_bytes(), cuts.data());
    if (parts <= 1)
        return run_host_batch(pick_device(ds.ids), n, src, src_len, dst, dst_cap, results, launch, zc_ok, direct_out);
    std::vector<int> rcs(parts, TYCHE_E_OK);
    std::vector<std::string> errs(parts);
    std::vector<std::thread> th;
    auto part = [&](size_t p) {
        const size_t a = cuts[p], m = cuts[p + 1] - cuts[p];
        rcs[p] = run_host_batch(ds.ids[p], m, src + a, src_len + a, dst + a, dst_cap + a, results + a, launch, zc_ok,
                                direct_out);
        if (rcs[p]) errs[p] = t_error;
    };
    for (size_t p = 1; p < parts; p++) th.emplace_back(part, p);
    part(0);
    for (auto &t : th) t.join();
    for (size_t p = 0; p < parts; p++)
        if (rcs[p]) {
            t_error = errs[p];
            return rcs[p];
        }
    return TYCHE_E_OK;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ runtime
int tyche_host_profile(uint64_t *out, int n) {
    const int k = std::min(n, (int)kHpCount);
    for (int i = 0; i < k; i++) out[i] = g_hprof[i].exchange(0);
    return k;
}

int tyche_set_knob(const char *name, long value) {
    if (!name || !*name) return TYCHE_E_BAD_ARGS;
    KnobTable &T = knob_table();
    std::lock_guard<std::mutex> g(T.mu);
    T.over[name] = value;
    g_knob_gen.fetch_add(1, std::memory_order_acq_rel);
    return TYCHE_E_OK;
}

int tyche_clear_knob(const char *name) {
    if (!name || !*name) return TYCHE_E_BAD_ARGS;
    KnobTable &T = knob_table();
    std::lock_guard<std::mutex> g(T.mu);
    T.over.erase(name);
    g_knob_gen.fetch_add(1, std::memory_order_acq_rel);
    return TYCHE_E_OK;
}

int tyche_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int tyche_set_device(int device) {
    if (device < TYCHE_ALL_DEVICES) return TYCHE_E_BAD_ARGS;
    t_device = device;
    return TYCHE_E_OK;
}

int tyche_active_devices(void) {
    if (t_device >= 0 || rank_device() >= 0) return 1;
    return (int)device_set().ids.size();
}

size_t tyche_plan_split(size_t n, const uint32_t *src_lengths, int ndev, uint64_t min_part_bytes, size_t *cuts) {
    cuts[0] = 0;
    uint64_t total = 0;
    for (size_t i = 0; i < n; i++) total += src_lengths[i];
    uint64_t parts = ndev > 0 ? (uint64_t)ndev : 1u;
    if (min_part_bytes > 0) parts = std::min<uint64_t>(parts, total / min_part_bytes);
    parts = std::min<uint64_t>(std::max<uint64_t>(parts, 1u), std::max<size_t>(n, 1u));
    size_t i = 0;
    uint64_t acc = 0;
    for (uint64_t p = 1; p < parts; p++) {   // part p-1 ends where the input bytes pass p/parts of the total
        const uint64_t goal = total / parts * p + (total % parts) * p / parts;
        while (i < n && acc < goal) acc += src_lengths[i++];
        cuts[p] = i;
    }
    cuts[parts] = n;
    size_t k = 1;   // drop empty parts
    for (uint64_t p = 1; p <= parts; p++)
        if (cuts[p] > cuts[k - 1]) cuts[k++] = cuts[p];
    if (k == 1) cuts[k++] = n;   // n == 0: one empty part
    return k - 1;
}

const char *tyche_last_error(void) { return t_error.c_str(); }

int tyche_device_ready(void) {
    DeviceGuard keep;
    int dev = 0;
    int rc = current_device(&dev);
    if (rc == TYCHE_E_OK) rc = ensure_device(dev);
    return rc == TYCHE_E_OK ? 1 : 0;
}

uint32_t tyche_compress_bound(int compressor_id, uint32_t n) {
    if (compressor_id == TYCHE_LZ4_COMPRESSOR_ID) return lz4_bound(n);
    if (compressor_id == TYCHE_ZLIB_COMPRESSOR_ID) return zlib_bound(n);
    if (compressor_id == TYCHE_ZSTD_COMPRESSOR_ID) return zstd_bound(n);
    return 0;
}

// ------------------------------------------------------- device-resident API
// Launches, counters and scratch follow the current device (hipGetDevice); a
// stream created on another device makes that device current for the call
// (DeviceGuard puts the caller's back).
static int stream_device(hipStream_t s) {
    if (!s) return TYCHE_E_OK;
    int sd = -1, cur = -1;
    if (hipStreamGetDevice(s, &sd) != hipSuccess || sd < 0) return TYCHE_E_OK;
    if (hipGetDevice(&cur) == hipSuccess && cur == sd) return TYCHE_E_OK;
    hipError_t e = hipSetDevice(sd);
    return e == hipSuccess ? TYCHE_E_OK : fail("hipSetDevice (stream's device)", e);
}

int tyche_compress_batch(int compressor_id, int compressor_level, const tyche_batch_t *batch, void *stream) {
    (void)compressor_level;   // level is fixed at 1 by tyche (src/options.c:68); LZ4 has no level
    if (!batch) return TYCHE_E_BAD_ARGS;
    if (!valid_codec(compressor_id)) { t_error = codec_msg(compressor_id); return TYCHE_E_BAD_ARGS; }
    if (batch->count == 0) return TYCHE_E_OK;
    if (!batch->src || !batch->dst || !batch->results) return TYCHE_E_BAD_ARGS;
    uint32_t in_cap = batch->src_lengths ? batch->max_src_length : batch->src_length;
    if (batch->src_lengths && in_cap == 0) in_cap = 65535;
    if (in_cap > 65535) { t_error = "pages above 64 KiB are not supported by the device encoders"; return TYCHE_E_BAD_ARGS; }
    DeviceGuard keep;
    if (int rc = stream_device((hipStream_t)stream)) return rc;
    hipError_t e = launch_encode(compressor_id, *batch, in_cap, (hipStream_t)stream);
    if (e != hipSuccess) return fail("encode launch", e);
    return TYCHE_E_OK;
}

int tyche_decompress_batch(int compressor_id, const tyche_batch_t *batch, void *stream) {
    if (!batch) return TYCHE_E_BAD_ARGS;
    if (!valid_decode_codec(compressor_id)) { t_error = codec_msg(compressor_id); return TYCHE_E_BAD_ARGS; }
    if (batch->count == 0) return TYCHE_E_OK;
    if (!batch->src || !batch->dst || !batch->results) return TYCHE_E_BAD_ARGS;
    DeviceGuard keep;
    if (int rc = stream_device((hipStream_t)stream)) return rc;
    uint32_t out_cap = batch->dst_capacity;
    if (compressor_id == TYCHE_ZLIB_COMPRESSOR_ID) {
        hipError_t e = launch_zlib_inflate(*batch, out_cap, (hipStream_t)stream);
        if (e != hipSuccess) return fail("zlib inflate launch", e);
        return TYCHE_E_OK;
    }
    if (compressor_id == TYCHE_ZSTD_COMPRESSOR_ID) {
        hipError_t e = launch_zstd_decode(*batch, decode_in_cap(*batch, zstd_bound(out_cap)), out_cap,
                                          (hipStream_t)stream);
        if (e != hipSuccess) return fail("zstd decode launch", e);
        return TYCHE_E_OK;
    }
    hipError_t e = launch_lz4_decode(*batch, decode_in_cap(*batch, lz4_bound(out_cap)), out_cap, (hipStream_t)stream);
    if (e != hipSuccess) return fail("lz4 decode launch", e);
    return TYCHE_E_OK;
}

// ----------------------------------------------------------- host batch API
int tyche_compress_host(int compressor_id, int compressor_level, size_t n, const void *const *src,
                        const uint32_t *src_lengths, void *const *dst, const uint32_t *dst_capacities,
                        int32_t *results) {
    (void)compressor_level;
    if (!valid_codec(compressor_id)) { t_error = codec_msg(compressor_id); return TYCHE_E_BAD_ARGS; }
    if (n == 0) return TYCHE_E_OK;
    for (size_t i = 0; i < n; i++)
        if (src_lengths[i] > 65535u) { t_error = "pages above 64 KiB are not supported by the device encoders"; return TYCHE_E_BAD_ARGS; }
    // LZ4's encoders only store to their destination (never read it back), so their streams may go
    // straight into the pinned staging arena (HOST_DIRECT_OUT=0: stage through HBM and D2H instead)
    const int direct = compressor_id == TYCHE_LZ4_COMPRESSOR_ID && knob("HOST_DIRECT_OUT", 1) ? kDirectAlways : kDirectNone;
    return run_host(n, src, src_lengths, dst, dst_capacities, results,
                          [compressor_id](const tyche_batch_t &b, hipStream_t s, bool) {
                              return launch_encode(compressor_id, b, std::max(b.max_src_length, 1u), s);
                          }, false, direct);
}

int tyche_decompress_host(int compressor_id, size_t n, const void *const *src, const uint32_t *src_lengths,
                          void *const *dst, const uint32_t *dst_capacities, int32_t *results) {
    if (!valid_decode_codec(compressor_id)) { t_error = codec_msg(compressor_id); return TYCHE_E_BAD_ARGS; }
    if (n == 0) return TYCHE_E_OK;
    if (compressor_id == TYCHE_ZLIB_COMPRESSOR_ID)
        return run_host(n, src, src_lengths, dst, dst_capacities, results,
                              [](const tyche_batch_t &b, hipStream_t s, bool) {
                                  return launch_zlib_inflate(b, b.dst_capacity, s);
                              }, true);
    if (compressor_id == TYCHE_ZSTD_COMPRESSOR_ID)
        return run_host(n, src, src_lengths, dst, dst_capacities, results,
                              [](const tyche_batch_t &b, hipStream_t s, bool) {
                                  return launch_zstd_decode(b, b.max_src_length, b.dst_capacity, s);
                              }, true);
    return run_host(n, src, src_lengths, dst, dst_capacities, results,
                          [](const tyche_batch_t &b, hipStream_t s, bool host_dst) {
                              return launch_lz4_decode(b, b.max_src_length, b.dst_capacity, s, !host_dst);
                          }, true, knob("HOST_DIRECT_OUT", 1) ? kDirectLz4Decode : kDirectNone);
}

// ------------------------------------------------------- Buffer entry points
int buffer__initialize(Buffer **buf, bufferid_t id, uint32_t size, void *data, char *page_filespec) {
    // src/buffer.c:61-109
    *buf = (Buffer *)malloc(sizeof(Buffer));
    if (*buf == NULL) return TYCHE_E_NO_MEMORY;
    memset(*buf, 0, sizeof(Buffer));
    pthread_mutex_init(&(*buf)->lock, NULL);
    (*buf)->id = id;
    if (page_filespec == NULL && size == 0 && data == NULL) return TYCHE_E_OK;
    if ((page_filespec != NULL) == (size > 0 || data != NULL)) return TYCHE_E_BAD_ARGS;
    if (page_filespec == NULL) {
        (*buf)->data = data;
        (*buf)->data_length = size;
        return TYCHE_E_OK;
    }
    FILE *fh = fopen(page_filespec, "rb");
    if (fh == NULL) return TYCHE_E_GENERIC;
    fseek(fh, 0, SEEK_END);
    (*buf)->data_length = (uint32_t)ftell(fh);
    rewind(fh);
    (*buf)->data = malloc((*buf)->data_length);
    if ((*buf)->data == NULL) { fclose(fh); return TYCHE_E_NO_MEMORY; }
    if (fread((*buf)->data, (*buf)->data_length, 1, fh) == 0) { fclose(fh); return TYCHE_E_GENERIC; }
    fclose(fh);
    return TYCHE_E_OK;
}

void buffer__destroy(Buffer *buf, const bool destroy_data) {
    // src/buffer.c:116-124
    if (destroy_data) free(buf->data);
    free(buf);
}

void buffer__lock(Buffer *buf) { pthread_mutex_lock(&buf->lock); }
void buffer__unlock(Buffer *buf) { pthread_mutex_unlock(&buf->lock); }
void buffer__release_pin(Buffer *buf) { __sync_fetch_and_add(&buf->ref_count, (uint16_t)-1); }

void buffer__copy(Buffer *src, Buffer *dst, bool copy_data) {
    // src/buffer.c:287-310
    dst->id = src->id;
    dst->ref_count = src->ref_count;
    dst->popularity = src->popularity;
    dst->comp_cost = src->comp_cost;
    dst->comp_hits = src->comp_hits;
    dst->data_length = src->data_length;
    dst->comp_length = src->comp_length;
    if (copy_data) {
        size_t n = src->comp_length > 0 ? src->comp_length : src->data_length;
        free(dst->data);
        dst->data = malloc(n);
        memcpy(dst->data, src->data, n);
    }
    dst->next = NULL;
}

// Pre-codec checks of buffer__compress, src/buffer.c:161-174, in the same order.
// Returns -1 when the buffer should go to the codec.
static int compress_precheck(Buffer *buf, int compressor_id) {
    if (compressor_id == TYCHE_NO_COMPRESSOR_ID) {
        if (buf == NULL) return TYCHE_E_BUFFER_NOT_FOUND;   // the reference dereferences NULL here
        buf->comp_length = buf->data_length;
        return TYCHE_E_OK;
    }
    if (buf == NULL) return TYCHE_E_BUFFER_NOT_FOUND;
    if (buf->data == NULL || buf->data_length == 0) return TYCHE_E_BUFFER_MISSING_DATA;
    if (buf->comp_length != 0) return TYCHE_E_BUFFER_ALREADY_COMPRESSED;
    return -1;
}

// src/buffer.c:229-240
static int decompress_precheck(Buffer *buf, int compressor_id) {
    if (compressor_id == TYCHE_NO_COMPRESSOR_ID) {
        if (buf == NULL) return TYCHE_E_BUFFER_NOT_FOUND;
        buf->comp_length = 0;
        return TYCHE_E_OK;
    }
    if (buf == NULL) return TYCHE_E_BUFFER_NOT_FOUND;
    if (buf->data == NULL || buf->data_length == 0) return TYCHE_E_BUFFER_MISSING_DATA;
    if (buf->comp_length == 0) return TYCHE_E_BUFFER_ALREADY_DECOMPRESSED;
    return -1;
}

int tyche_buffers_compress(Buffer **bufs, void **compressed, int *status, size_t n, int compressor_id,
                           int compressor_level) {
    std::vector<size_t> idx;
    idx.reserve(n);
    for (size_t i = 0; i < n; i++) {
        status[i] = compress_precheck(bufs[i], compressor_id);
        if (status[i] == -1) {
            if (!valid_codec(compressor_id) && compressor_id >= 1 && compressor_id <= 3) {
                t_error = codec_msg(compressor_id);
                status[i] = TYCHE_E_BUFFER_COMPRESSION_PROBLEM;
            } else if (!valid_codec(compressor_id)) {
                status[i] = TYCHE_E_OK;   // unknown id: the reference's if-chain falls through (buffer.c:176-218)
            } else {
                idx.push_back(i);
            }
        }
    }
    if (idx.empty()) return TYCHE_E_OK;
    const size_t m = idx.size();
    std::vector<const void *> src(m);
    std::vector<void *> dst(m);
    std::vector<uint32_t> slen(m), dcap(m);
    std::vector<int32_t> res(m);
    for (size_t k = 0; k < m; k++) {
        Buffer *b = bufs[idx[k]];
        src[k] = b->data;
        slen[k] = b->data_length;
        dcap[k] = tyche_compress_bound(compressor_id, b->data_length);   // the codec's bound (buffer.c:179, 191, 204)
        dst[k] = malloc(dcap[k]);
        if (!dst[k]) {
            for (size_t j = 0; j < k; j++) free(dst[j]);
            for (size_t j = 0; j < m; j++) {
                status[idx[j]] = TYCHE_E_NO_MEMORY;
                compressed[idx[j]] = NULL;
            }
            return TYCHE_E_NO_MEMORY;
        }
    }
    uint64_t t0 = now_ns();
    int rc = tyche_compress_host(compressor_id, compressor_level, m, src.data(), slen.data(), dst.data(),
                                 dcap.data(), res.data());
    uint64_t per = (now_ns() - t0) / m;
    for (size_t k = 0; k < m; k++) {
        Buffer *b = bufs[idx[k]];
        size_t i = idx[k];
        if (rc != TYCHE_E_OK || res[k] < 1) {
            // The reference leaks its output block here (buffer.c:185-186) and leaves
            // *compressed_data pointing at it; this frees it and sets NULL, so a caller
            // that ignores the status (list.c:1050-1058 installs the pointer on any
            // status but 124) never installs memory it does not own.
            free(dst[k]);
            compressed[i] = NULL;
            status[i] = rc != TYCHE_E_OK ? TYCHE_E_DEVICE : TYCHE_E_BUFFER_COMPRESSION_PROBLEM;
            continue;
        }
        compressed[i] = dst[k];
        b->comp_length = (uint32_t)res[k];
        b->comp_cost += (uint32_t)per;
        status[i] = TYCHE_E_OK;
    }
    return rc;
}

int tyche_buffers_decompress(Buffer **bufs, int *status, size_t n, int compressor_id) {
    std::vector<size_t> idx;
    idx.reserve(n);
    for (size_t i = 0; i < n; i++) {
        status[i] = decompress_precheck(bufs[i], compressor_id);
        if (status[i] == -1) {
            if (!valid_decode_codec(compressor_id) && compressor_id >= 1 && compressor_id <= 3) {
                t_error = codec_msg(compressor_id);
                status[i] = TYCHE_E_BUFFER_COMPRESSION_PROBLEM;
            } else if (!valid_decode_codec(compressor_id)) {
                // unknown id: the reference swaps in an unfilled malloc(data_length) block and
                // reports success (buffer.c:244-279); mirrored, with the block zeroed.
                Buffer *b = bufs[i];
                void *fresh = calloc(1, b->data_length);
                if (!fresh) { status[i] = TYCHE_E_NO_MEMORY; continue; }
                free(b->data);
                b->data = fresh;
                b->comp_hits++;
                b->comp_length = 0;
                status[i] = TYCHE_E_OK;
            } else {
                idx.push_back(i);
            }
        }
    }
    if (idx.empty()) return TYCHE_E_OK;
    const size_t m = idx.size();
    std::vector<const void *> src(m);
    std::vector<void *> dst(m);
    std::vector<uint32_t> slen(m), dcap(m);
    std::vector<int32_t> res(m);
    for (size_t k = 0; k < m; k++) {
        Buffer *b = bufs[idx[k]];
        src[k] = b->data;
        slen[k] = b->comp_length;
        dcap[k] = b->data_length;
        dst[k] = malloc(b->data_length);                             // buffer.c:246
        if (!dst[k]) {
            for (size_t j = 0; j < k; j++) free(dst[j]);
            for (size_t j = 0; j < m; j++) status[idx[j]] = TYCHE_E_NO_MEMORY;
            return TYCHE_E_NO_MEMORY;
        }
    }
    uint64_t t0 = now_ns();
    int rc = tyche_decompress_host(compressor_id, m, src.data(), slen.data(), dst.data(), dcap.data(), res.data());
    uint64_t per = (now_ns() - t0) / m;
    for (size_t k = 0; k < m; k++) {
        Buffer *b = bufs[idx[k]];
        size_t i = idx[k];
        // LZ4 accepts any rv >= 0 (buffer.c:251-253); zlib needs Z_OK and the exact length (:257-260);
        // zstd only !ZSTD_isError (:264-266)
        const bool bad = res[k] < 0 || (compressor_id == TYCHE_ZLIB_COMPRESSOR_ID && (uint32_t)res[k] != b->data_length);
        if (rc != TYCHE_E_OK || bad) {
            free(dst[k]);                           // the reference leaks here
            status[i] = rc != TYCHE_E_OK ? TYCHE_E_DEVICE : TYCHE_E_BUFFER_COMPRESSION_PROBLEM;
            continue;
        }
        free(b->data);
        b->data = dst[k];
        b->comp_hits++;
        b->comp_length = 0;
        b->comp_cost += (uint32_t)per;
        status[i] = TYCHE_E_OK;
    }
    return rc;
}

int buffer__compress(Buffer *buf, void **compressed_data, int compressor_id, int compressor_level) {
    int status = TYCHE_E_OK;
    tyche_buffers_compress(&buf, compressed_data, &status, 1, compressor_id, compressor_level);
    return status;
}

int buffer__decompress(Buffer *buf, int compressor_id) {
    int status = TYCHE_E_OK;
    tyche_buffers_decompress(&buf, &status, 1, compressor_id);
    return status;
}

// ---------------------------------------------------------- restore queue
// list__search restores one page per hit, synchronously, under the buffer's
// lock (src/list.c:563-589).  The queue lets those concurrent per-hit restores
// share GPU launches: a caller enqueues its Buffer and blocks; a dispatcher
// thread takes whatever is queued (up to max_batch, after waiting at most
// max_wait_us for company once the first request arrives), runs one
// tyche_buffers_decompress over the batch, and wakes each caller with its
// buffer__decompress status.  Per-buffer semantics are unchanged.
//
// Each codec has its own queue and dispatchers (TYCHE_RESTORE_DISPATCHERS per
// codec, default two per device): a batch's latency is that of its slowest
// page (~0.04 ms for a 16 KiB LZ4 page on the single-page decoder, ~0.3 ms for
// zlib, tools/latency.c), so LZ4 restores never wait behind a zlib batch, and a
// second dispatcher collects the next batch while one runs: 2.53 vs 2.06 GiB/s of
// tools/cycle.c restores (round 5, r05_restore_dispatch.log; with the jump
// decoder and a shared wake-up round 2 had measured 1.70 vs 1.32 on one box and
// 1.12-1.24 vs 1.32-1.36 on another, r02_restore_dispatch.jsonl); 3-4 per codec
// oversubscribed the hardware queues then.
namespace {
constexpr int kQueueHistBuckets = 11;
// A restorer waits on its own request word (spin briefly, then futex), so a finished batch wakes
// exactly its callers -- a shared condition variable woke every blocked restorer (64 in the C5
// cycle) to re-take the queue mutex and find its request still pending.
// A request lives on its caller's stack; the futex word it is woken through does not: it is the
// caller's thread_local word (reset on entry), so the FUTEX_WAKE that follows the store -- which
// the waiter may already have seen and returned on -- still lands on a live word of that thread,
// never on a reused stack frame.  A wake that finds no waiter is a no-op, and every
// waiter re-checks its word in a loop, so a late wake is harmless.
struct RestoreReq {
    Buffer *buf;
    int status;
    std::atomic<int> *done;
    void wait() {
        for (int i = 0; i < 64; i++) {   // (a batch takes ~0.1 ms: spinning longer only takes CPU from the others)
            if (done->load(std::memory_order_acquire)) return;
            _mm_pause();
        }
        while (!done->load(std::memory_order_acquire))
            syscall(SYS_futex, (int *)done, FUTEX_WAIT_PRIVATE, 0, nullptr, nullptr, 0);
    }
    void wake() {
        std::atomic<int> *w = done;   // read before the store: the request may be gone after it
        w->store(1, std::memory_order_release);
        syscall(SYS_futex, (int *)w, FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
    }
};
thread_local std::atomic<int> t_restore_word{0};
struct RestoreQueue {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<RestoreReq *> q[4];   // by codec id (NO is restored by the caller)
    bool collecting[4] = {false, false, false, false};
    bool running = false, stop = false;
    int max_batch = 1024, max_wait_us = 50, device = -1;
    uint64_t batches = 0, buffers = 0;
    uint64_t hist[kQueueHistBuckets] = {};   // launches by batch size (power-of-two buckets)
    std::vector<std::thread> th;
    void loop(int codec) {
        (void)tyche_set_device(device);
        std::vector<RestoreReq *> take;
        std::vector<Buffer *> bufs;
        std::vector<int> st;
        std::vector<RestoreReq *> &cq = q[codec];
        // TYCHE_RESTORE_WAIT_IDLE (default 1): the wait for company applies only when this
        // dispatcher found its queue empty -- requests that queued up while its last batch ran
        // have waited a whole batch already and go out at once (0: every batch waits)
        const bool wait_idle_only = knob("RESTORE_WAIT_IDLE", 1) != 0;
        bool idle = true;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu);
                if (cq.empty()) idle = true;
                cv.wait(g, [&] { return (stop && cq.empty()) || (!cq.empty() && !collecting[codec]); });
                if (cq.empty()) return;   // stopping
                collecting[codec] = true;
                if ((idle || !wait_idle_only) && (int)cq.size() < max_batch && max_wait_us > 0)
                    cv.wait_for(g, std::chrono::microseconds(max_wait_us),
                                [&] { return stop || (int)cq.size() >= max_batch; });
                const size_t k = std::min(cq.size(), (size_t)max_batch);
                take.assign(cq.begin(), cq.begin() + k);
                cq.erase(cq.begin(), cq.begin() + k);
                collecting[codec] = false;
            }
            cv.notify_all();   // the next dispatcher of this codec may collect
            bufs.resize(take.size());
            st.resize(take.size());
            for (size_t i = 0; i < take.size(); i++) bufs[i] = take[i]->buf;
            tyche_buffers_decompress(bufs.data(), st.data(), bufs.size(), codec);
            {
                std::lock_guard<std::mutex> g(mu);
                batches++;
                buffers += take.size();
                hist[std::min(kQueueHistBuckets - 1, 31 - __builtin_clz((unsigned)take.size()))]++;
                idle = cq.empty();
            }
            for (size_t i = 0; i < take.size(); i++) {
                take[i]->status = st[i];
                take[i]->wake();   // (the request lives on its caller's stack: not touched after this)
            }
        }
    }
};
// never destroyed: a process may exit without tyche_restore_queue_stop (the reference app's
// list__destroy can hang before it gets there), and destroying joinable dispatcher threads (or the
// mutex they wait on) at exit would abort the process in std::terminate
RestoreQueue &g_rq = *new RestoreQueue;
}  // namespace

int tyche_restore_queue_start(int max_batch, int max_wait_us) {
    std::lock_guard<std::mutex> g(g_rq.mu);
    if (g_rq.running) return TYCHE_E_OK;
    g_rq.max_batch = max_batch > 0 ? max_batch : 1024;
    g_rq.max_wait_us = max_wait_us >= 0 ? max_wait_us : 50;
    g_rq.device = t_device;
    g_rq.stop = false;
    for (bool &c : g_rq.collecting) c = false;
    g_rq.running = true;
    int k = (int)knob("RESTORE_DISPATCHERS", 2 * std::max(1, tyche_active_devices()));
    k = std::max(1, std::min(k, 64));
    for (int codec = 1; codec <= 3; codec++)
        for (int i = 0; i < k; i++) g_rq.th.emplace_back([codec] { g_rq.loop(codec); });
    return TYCHE_E_OK;
}

void tyche_restore_queue_stop(void) {
    {
        std::lock_guard<std::mutex> g(g_rq.mu);
        if (!g_rq.running) return;
        g_rq.stop = true;
    }
    g_rq.cv.notify_all();
    for (auto &t : g_rq.th) t.join();
    std::lock_guard<std::mutex> g(g_rq.mu);
    g_rq.th.clear();
    g_rq.running = false;
}

int tyche_buffer_restore(Buffer *buf, int compressor_id) {
    // NO and unknown ids need no GPU batch: the direct path gives the reference's answer
    if (compressor_id < 1 || compressor_id > 3) return buffer__decompress(buf, compressor_id);
    RestoreReq r;
    r.buf = buf;
    r.status = TYCHE_E_OK;
    t_restore_word.store(0, std::memory_order_relaxed);
    r.done = &t_restore_word;
    {
        std::unique_lock<std::mutex> g(g_rq.mu);
        if (!g_rq.running || g_rq.stop) {
            g.unlock();
            return buffer__decompress(buf, compressor_id);   // no queue: the direct path
        }
        g_rq.q[compressor_id].push_back(&r);
    }
    g_rq.cv.notify_all();   // the collecting dispatcher, whichever it is
    r.wait();
    return r.status;
}

void tyche_restore_queue_stats(uint64_t *batches, uint64_t *buffers) {
    std::lock_guard<std::mutex> g(g_rq.mu);
    if (batches) *batches = g_rq.batches;
    if (buffers) *buffers = g_rq.buffers;
}

int tyche_restore_queue_hist(uint64_t *counts, int n) {
    if (!counts || n <= 0) return 0;
    std::lock_guard<std::mutex> g(g_rq.mu);
    const int k = std::min(n, kQueueHistBuckets);
    for (int i = 0; i < k; i++) counts[i] = g_rq.hist[i];
    return k;
}

// ---------------------------------------------------------- synthetic input
int tyche_pagegen(void *dst, uint64_t stride, uint32_t page_len, uint64_t seed, uint64_t first, size_t count,
                  uint32_t dist, void *stream) {
    // device-resident like the batch API: runs on the caller's current device
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail_msg("no HIP device available (the codec runs only on the GPU)");
    int rc = ensure_device(dev);
    if (rc) return rc;
    hipError_t e = launch_pagegen(dst, stride, page_len, seed, first, count, dist, (hipStream_t)stream);
    if (e != hipSuccess) return fail("pagegen launch", e);
    return TYCHE_E_OK;
}

}  // extern "C"
