// okm_engine.hip — host side of the counting context (C ABI in orion_kmer.h).
//
// One okm_ctx = one device + one HIP stream.  Work per okm_count():
//
//   add_batch*:  L1 pass per batch (extract_hist -> host offsets ->
//                extract_scatter): the batch's canonical k-mers land in 2^l1
//                key-range partitions ("runs"; one run per batch).
//   okm_count:   split every partition whose size could exceed the LDS table
//                (rounds of part_hist/part_scatter, each consuming more key
//                bits, per-partition bit budget), then count_items (LDS table
//                + sort per partition), then compact to one dense sorted
//                (key, count) table.
//
// Replaces run_count's map (count.rs:48), its per-record fill
// (count.rs:68-72 -> process_sequence_chunk count.rs:23-38) and its
// drain/filter/sort (count.rs:106-119).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "okm_arena.h"
#include "okm_hip_try.h"
#include "okm_internal.h"
#include "okm_key.h"
#include "orion_kmer_testing.h"

namespace okm {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

okm_status fail(okm_status s, const std::string &msg) {
    g_last_error = msg;
    return s;
}

// ---------------------------------------------------------------------------
// Device memory: one virtual-memory arena per context (okm_arena.h), under
// ONE budget for every context of the process on a device.
// ---------------------------------------------------------------------------
struct DevPool;
static std::mutex g_pools_mu;
static std::vector<DevPool *> g_pools;  // every live context's pool (cross-pool trim, the budget)
static constexpr size_t kArenaChunk = size_t(1) << 30;  // 1 GiB: 64 MiB chunks cost the streaming kernels TLB reach
// Per device: the bytes every pool has mapped plus the communicators' device
// buffers (okm_dist.hip DevBuf) -- what the budget compares against.  An
// atomic, so that a pool holding its own lock never takes g_pools_mu (the
// lock order is g_pools_mu, then a pool's mu: trim_others / trim_device_pools).
static std::atomic<int64_t> g_dev_bytes[64];
void device_bytes_add(int device, int64_t delta) { g_dev_bytes[device & 63].fetch_add(delta, std::memory_order_relaxed); }

// The device memory the process's contexts may map together: OKM_HBM_CAP, a
// fraction of HBM (<= 1, default 0.9) or a byte count (> 1; "16e9" or with a
// K/M/G/T suffix, powers of 1024), or the OKM_TEST_HBM_BUDGET_BYTES test hook.
// A hard limit: past it the arena first unmaps idle chunks (its own, then the
// other contexts'), and an allocation that still does not fit fails with
// OKM_E_NOMEM -- which the counting paths plan around (key-range groups,
// folding, tables moved to host memory: DESIGN.md §5).
// A byte count: "28.8e9", "24G" (K/M/G/T: powers of 1024); < 0 when unparsable.
static double parse_bytes(const char *e) {
    char *end = nullptr;
    double v = strtod(e, &end);
    if (end == e || !(v >= 0)) return -1.0;
    if (end && *end) {
        const char u = (char)(*end | 0x20);
        v *= u == 'k' ? 1024.0 : u == 'm' ? 1048576.0 : u == 'g' ? 1073741824.0 : u == 't' ? 1099511627776.0 : 1.0;
    }
    return v;
}
static double parse_budget(const char *e, double total) {
    if (!e || !*e) return 0.9 * total;
    const double v = parse_bytes(e);
    if (!(v > 0)) return 0.9 * total;
    return v <= 1.0 ? v * total : std::min(v, total);
}
static double device_total_bytes(int device) {
    static std::atomic<size_t> totals[64];
    const int d = device & 63;
    size_t t = totals[d].load(std::memory_order_relaxed);
    if (!t) {
        if (hipDeviceTotalMem(&t, device) != hipSuccess) {
            (void)hipGetLastError();
            return 0.0;
        }
        totals[d] = t;
    }
    return (double)t;
}
static double hbm_budget(int device) {
    const double total = device_total_bytes(device);
    const int64_t t = test_knob(OKM_TEST_HBM_BUDGET_BYTES);
    if (t > 0) return std::min((double)t, total);
    static const std::string env = getenv("OKM_HBM_CAP") ? getenv("OKM_HBM_CAP") : "";
    return parse_budget(env.c_str(), total);
}

struct DevPool {
    int device = 0;
    bool ready = false;
    VmmArena arena;
    std::atomic<size_t> mapped_bytes{0};  // arena.mapped, readable without mu (the budget sums every pool)
    size_t peak_in_use = 0;               // high-water mark of live ranges (okm_engine_info.device_peak_bytes)
    std::mutex mu;  // the owning context's thread, or another pool trimming this one

    void attach(int dev) {
        device = dev;
        std::lock_guard<std::mutex> g(g_pools_mu);
        g_pools.push_back(this);
    }
    void detach() {
        std::lock_guard<std::mutex> g(g_pools_mu);
        g_pools.erase(std::remove(g_pools.begin(), g_pools.end(), this), g_pools.end());
    }
    bool init_locked() {  // mu held
        if (!ready) ready = arena.init(device, kArenaChunk);
        return ready;
    }
    bool owns(const void *p) const {
        const char *q = static_cast<const char *>(p);
        return arena.base && q >= arena.base && q < arena.base + arena.reserved;
    }
    // Bytes every pool on this device has mapped (+ communicator buffers); lock-free.
    static size_t device_mapped(int device) {
        const int64_t b = g_dev_bytes[device & 63].load(std::memory_order_relaxed);
        return b > 0 ? (size_t)b : 0;
    }
    void set_mapped(size_t m) {
        const size_t old = mapped_bytes.exchange(m, std::memory_order_relaxed);
        device_bytes_add(device, (int64_t)m - (int64_t)old);
    }
    // Would `bytes` more mapped memory take the device's pools past the budget?
    bool over_budget(size_t bytes) const { return (double)device_mapped(device) + (double)bytes > hbm_budget(device); }

    // A best-fit address range, then physical chunks for the parts of it that
    // are not mapped yet.  Past the budget, idle chunks of this arena (then of
    // the other pools on the device) are unmapped first -- after a device
    // sync, since a freed range's last kernel may still be in flight.
    okm_status get(size_t bytes, void **out) {
        std::lock_guard<std::mutex> lk(mu);
        if (!init_locked()) return fail(OKM_E_DEVICE, "device arena: no virtual memory management on this device");
        bytes = VmmArena::round_up(std::max<size_t>(bytes, 256), 256);
        const size_t off = arena.take(bytes);
        if (off == ~size_t(0))
            return fail(OKM_E_NOMEM, "device arena: no free range of " + std::to_string(bytes) + " B");
        const size_t c0 = arena.first_chunk(off), c1 = arena.last_chunk(off, bytes);
        size_t missing = 0;
        for (size_t i = c0; i <= c1; ++i) {
            arena.chunks[i].users++;  // reserved: nobody unmaps them from here on
            missing += !arena.chunks[i].mapped;
        }
        auto undo = [&]() {
            for (size_t i = c0; i <= c1; ++i) arena.chunks[i].users--;
            arena.give_back(off);
        };
        if (missing) {
            const size_t need = missing * arena.chunk;
            if (over_budget(need) && arena.idle()) {
                (void)hipDeviceSynchronize();
                arena.unmap_idle(need);
                set_mapped(arena.mapped);
            }
            if (over_budget(need)) {  // other contexts' idle chunks (their locks, not ours)
                mu.unlock();
                trim_others();
                mu.lock();
            }
            hipError_t e = over_budget(need) ? hipErrorOutOfMemory : hipSuccess;
            for (size_t i = c0; i <= c1 && e == hipSuccess; ++i)
                if (!arena.chunks[i].mapped) e = arena.map_chunk(i);
            if (e != hipSuccess && !over_budget(need)) {  // HBM full (other allocations): everything idle back, once more
                (void)hipGetLastError();
                (void)hipDeviceSynchronize();
                arena.unmap_idle(~size_t(0));
                set_mapped(arena.mapped);
                mu.unlock();
                trim_others();
                mu.lock();
                e = hipSuccess;
                for (size_t i = c0; i <= c1 && e == hipSuccess; ++i)
                    if (!arena.chunks[i].mapped) e = arena.map_chunk(i);
            }
            set_mapped(arena.mapped);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                undo();
                size_t fr = 0, tot = 0;
                (void)hipMemGetInfo(&fr, &tot);
                (void)hipGetLastError();
                return fail(OKM_E_NOMEM, "device arena: mapping " + std::to_string(bytes) + " B: " +
                                             (over_budget(need) ? std::string("over the device budget of ") +
                                                                      std::to_string((uint64_t)hbm_budget(device)) + " B"
                                                                : std::string(hipGetErrorString(e))) +
                                             " (context maps " + std::to_string(arena.mapped) + " B, " +
                                             std::to_string(arena.in_use) + " B in use; device free " +
                                             std::to_string(fr) + " of " + std::to_string(tot) + " B)");
            }
        }
        peak_in_use = std::max(peak_in_use, arena.in_use);
        *out = arena.base + off;
        return OKM_OK;
    }
    void put(void *p) {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu);
        if (!owns(p)) return;
        const size_t off = static_cast<char *>(p) - arena.base;
        auto it = arena.live.find(off);
        if (it == arena.live.end()) return;  // a pointer inside a block (e.g. a table's counts)
        for (size_t i = arena.first_chunk(off); i <= arena.last_chunk(off, it->second); ++i) arena.chunks[i].users--;
        arena.give_back(off);
    }
    // Keep the first `bytes` of the allocation at p (its tail returns to the
    // arena, nothing moves); false when p is not an allocation of this pool.
    bool shrink(void *p, size_t bytes) {
        std::lock_guard<std::mutex> g(mu);
        if (!owns(p)) return false;
        const size_t off = static_cast<char *>(p) - arena.base;
        if (!arena.live.count(off)) return false;
        arena.shrink(off, VmmArena::round_up(std::max<size_t>(bytes, 256), 256));
        return true;
    }
    size_t size_of(const void *p) {
        std::lock_guard<std::mutex> g(mu);
        if (!owns(p)) return 0;
        auto it = arena.live.find(static_cast<const char *>(p) - arena.base);
        return it == arena.live.end() ? 0 : it->second;
    }
    size_t held() {
        std::lock_guard<std::mutex> g(mu);
        return arena.mapped;
    }
    size_t in_use() {
        std::lock_guard<std::mutex> g(mu);
        return arena.in_use;
    }
    size_t peak() {
        std::lock_guard<std::mutex> g(mu);
        return peak_in_use;
    }
    void reset_peak() {
        std::lock_guard<std::mutex> g(mu);
        peak_in_use = arena.in_use;
    }
    // Bytes mapped but not in use (reusable without new device memory).
    size_t cached() {
        std::lock_guard<std::mutex> g(mu);
        return arena.mapped - std::min(arena.mapped, arena.in_use);
    }
    void trim() {
        std::lock_guard<std::mutex> g(mu);
        if (arena.idle()) {
            (void)hipDeviceSynchronize();
            arena.unmap_idle(~size_t(0));
            set_mapped(arena.mapped);
        }
    }
    void trim_others() {
        std::lock_guard<std::mutex> g(g_pools_mu);
        for (DevPool *o : g_pools)
            if (o != this && o->device == device) o->trim();
    }
    void release_all() {
        std::lock_guard<std::mutex> g(mu);
        arena.release();
        set_mapped(0);
        ready = false;
    }
};

bool device_over_budget(int device, size_t bytes) {
    return (double)DevPool::device_mapped(device) + (double)bytes > hbm_budget(device);
}

void trim_device_pools(int device) {
    std::lock_guard<std::mutex> g(g_pools_mu);
    for (DevPool *o : g_pools)
        if (o->device == device) o->trim();
}

template <typename T>
static okm_status pool_get(DevPool &pool, size_t n, T **out) {
    void *p = nullptr;
    OKM_TRY(pool.get(n * sizeof(T), &p));
    *out = static_cast<T *>(p);
    return OKM_OK;
}

static bool debug_sync() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("OKM_DEBUG_SYNC");
        v = (e && *e && *e != '0') ? 1 : 0;
    }
    return v == 1;
}

// OKM_PROFILE_HOST=1: wall time of host phases (incl. the syncs inside them),
// printed to stderr by okm_count.
struct HostProf {
    bool on = false;
    std::vector<std::pair<std::string, double>> acc;
    std::chrono::steady_clock::time_point last;
    HostProf() {
        const char *e = getenv("OKM_PROFILE_HOST");
        on = e && *e && *e != '0';
        last = std::chrono::steady_clock::now();
    }
    void mark(const char *name) {
        if (!on) return;
        auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - last).count();
        last = now;
        for (auto &kv : acc)
            if (kv.first == name) {
                kv.second += ms;
                return;
            }
        acc.emplace_back(name, ms);
    }
    void dump(const char *tag) {
        if (!on) return;
        fprintf(stderr, "[okm host %s]", tag);
        for (auto &kv : acc) fprintf(stderr, " %s=%.3f", kv.first.c_str(), kv.second);
        fprintf(stderr, "\n");
        acc.clear();
    }
};

// ---------------------------------------------------------------------------
// HIP-event kernel timing (okm_set_timing / okm_kernel_stats)
// ---------------------------------------------------------------------------
struct KernelTimer {
    bool on = false;
    struct Pending {
        int id;
        hipEvent_t a, b;
        double bytes;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> spare;
    std::vector<std::string> names;
    std::vector<okm_kernel_stat> stats;
    hipEvent_t cur_a = nullptr;

    int id_of(const char *name) {
        for (size_t i = 0; i < names.size(); ++i)
            if (names[i] == name) return (int)i;
        names.emplace_back(name);
        okm_kernel_stat st{};
        stats.push_back(st);
        return (int)names.size() - 1;
    }
    hipEvent_t ev() {
        if (!spare.empty()) {
            hipEvent_t e = spare.back();
            spare.pop_back();
            return e;
        }
        hipEvent_t e;
        (void)hipEventCreate(&e);
        return e;
    }
    void begin(hipStream_t s) {
        if (!on) return;
        cur_a = ev();
        (void)hipEventRecord(cur_a, s);
    }
    void end(hipStream_t s, const char *name, double bytes) {
        if (debug_sync()) {  // OKM_DEBUG_SYNC=1: serialise and name every kernel
            hipError_t e = hipStreamSynchronize(s);
            fprintf(stderr, "[okm] %s done: %s\n", name, hipGetErrorString(e));
        }
        if (!on) return;
        hipEvent_t b = ev();
        (void)hipEventRecord(b, s);
        pending.push_back({id_of(name), cur_a, b, bytes});
    }
    // algorithmic bytes of an already-timed launch known only after a sync
    void add_bytes(const char *name, double bytes) {
        if (on) stats[id_of(name)].alg_bytes += bytes;
    }
    // call after the stream is synchronised
    void flush() {
        for (auto &p : pending) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, p.a, p.b);
            stats[p.id].launches += 1;
            stats[p.id].total_ms += ms;
            stats[p.id].alg_bytes += p.bytes;
            spare.push_back(p.a);
            spare.push_back(p.b);
        }
        pending.clear();
    }
    void reset() {
        flush();
        for (auto &s : stats) s = okm_kernel_stat{};
    }
    void destroy() {
        flush();
        for (auto e : spare) (void)hipEventDestroy(e);
        spare.clear();
    }
};

// L1-partitioned keys of one batch (or one add_pairs call).
struct Run {
    uint64_t *keys = nullptr;
    uint64_t *counts = nullptr;  // null: every key weighs 1
    std::vector<uint64_t> off;   // nbins + 1 offsets
    std::vector<uint64_t> end;   // per-bin ends (line padded) when bins do not abut (sampled L1)
    uint64_t n = 0;              // keys (sorted runs)
    bool sorted = false;         // strictly ascending unique keys (okm_add_sorted_pairs_device)
    bool borrowed = false;       // caller-owned memory: never returned to the pool
    bool folded = false;         // a counted table kept as a weighted L1 run (fold(), bins by binary search)
    bool host = false;           // keys / counts in page-locked HOST memory (a folded table moved off a full device)
    uint64_t len(uint32_t b) const { return (end.empty() ? off[b + 1] : end[b]) - off[b]; }
};

}  // namespace okm

using namespace okm;

static const size_t kHpinBytes = size_t(4) << 20;
static const size_t kHresWords = 8192;  // [0, 4096): L1 readback (3 nb + 2 words, nb <= 1024); [4096, 4112): count readback
static const size_t kHresCount = 4096;

struct okm_ctx {
    int device = 0;
    uint8_t k = 0;
    okm_mode mode = OKM_MODE_COUNT;
    hipStream_t stream = nullptr;
    uint32_t l1_bits = 0, nbins = 1, shift1 = 64;
    bool l1_fold = false;  // extract with the folding geometry (extract_l1_bits): set by the first fold, kept by reset
    bool wide = false;   // k > 32: K128 keys (two u64 per key)
    uint32_t kw = 1;     // u64 words per key

    // density hint for the next sorted-run count (set_sorted_hint): pairs per
    // top-hint_bits key bin; empty = none
    std::vector<unsigned long long> sorted_hint;
    uint32_t sorted_hint_bits = 0;
    std::unique_ptr<DevPool> pool{new DevPool};  // heap-held: a merge at one rank hands the whole pool over (adopt_result)
    std::vector<Run> runs;
    KernelTimer timer;
    HostProf hprof;

    // small persistent scratch
    uint32_t *HC = nullptr;
    size_t HC_cap = 0;
    unsigned long long *Hg = nullptr, *cursor = nullptr;
    size_t Hg_cap = 0;
    unsigned long long *flag = nullptr;  // overflow word
    unsigned long long *l1cap = nullptr; // sampled L1: cap_end | start | overflow
    unsigned long long *curpad = nullptr;  // sampled L1 claim cursors, kL1CurStride apart
    uint8_t *staging = nullptr;          // device copy of a host batch
    size_t staging_cap = 0;
    uint8_t *pinned = nullptr;           // pinned host staging
    size_t pinned_cap = 0;
    uint8_t *hpin = nullptr;             // pinned staging of small host->device tables (recycled at sync)
    size_t hpin_used = 0;
    unsigned long long *hres = nullptr;  // pinned landing area of small device->host reads

    // fold: once the uncounted L1 runs hold more than this many bytes, they are
    // counted and replaced by their sorted table (memory grows with distinct keys)
    uint64_t fold_bytes = 0;
    uint32_t folds = 0;
    double l1_ratio = 0;  // largest windows-per-byte ratio of a batch so far (L1 run sizing)

    // result
    bool counted = false;
    // the result stands for every input added so far: the runs it was
    // counted from are gone (borrowed runs are dropped once counted, since
    // their memory belongs to the caller); the next add keeps it as a table
    bool res_is_input = false;
    // the count in progress is the runs' last use (do_count releases them, a
    // fold replaces them): its staged keys may go into a run's block (C2: the
    // L1 run's 3.2 GB, instead of a block of their own)
    bool may_take_runs = false;
    bool took_runs = false;    // ... and it did
    bool input_lost = false;   // a count failed after overwriting a run: only okm_reset recovers
    // the result goes to the caller (okm_count), not into a kept table: it may
    // take the dead level array's block (keys, then counts) instead of blocks
    // of its own (C2: 1.8 GB fewer held; a table kept later is moved by
    // result_to_folded_run's shrink)
    bool share_result = false;
    // A count whose items were counted in place (count_parts, one child per
    // item) leaves its table as the items' sorted runs: keys over the items'
    // own keys in the level array, u32 / u64 counts at each item's out_off,
    // n_out[i] entries per item, items in key order (count.rs:106-119's
    // sorted drain, segment by segment).  The dense (keys, counts) copy is
    // made by the first reader that needs one (ensure_dense: okm_result_device,
    // the fetch / drain, folding, the multi-GPU merge), so a count whose table
    // is only drained pays one gather, not two.
    struct Pending {
        bool on = false;
        DevItem *items = nullptr;
        uint32_t nitems = 0;
        unsigned long long *n_out = nullptr, *dense_off = nullptr;
        uint64_t *sk = nullptr;  // the staged runs' keys (nullptr: staged in place, over the items' own keys)
        uint64_t *sc = nullptr;
        bool narrow = false;
        std::vector<void *> hold;  // freed with it: level arrays, segments, items, n_out, offsets, counts
    } pend;
    uint64_t *res_keys = nullptr, *res_counts = nullptr;
    uint64_t n_res = 0;
    bool res_host = false;     // the result lies in page-locked HOST memory (too big to stay beside its inputs)
    uint64_t host_bytes = 0;   // host memory held by host runs and a host result
    uint32_t spills = 0;       // tables moved to host memory
    okm_engine_info info{};
};

namespace okm {

int ctx_device(const okm_ctx *c) { return c->device; }
bool ctx_is_wide(const okm_ctx *c) { return c->wide; }
uint32_t ctx_k(const okm_ctx *c) { return c->k; }
void set_sorted_hint(okm_ctx *c, const unsigned long long *fine, uint32_t fine_bits) {
    c->sorted_hint.clear();
    c->sorted_hint_bits = 0;
    if (!fine || fine_bits > 24) return;
    c->sorted_hint.assign(fine, fine + (size_t(1) << fine_bits));
    c->sorted_hint_bits = fine_bits;
}
bool ctx_is_set(const okm_ctx *c) { return c->mode == OKM_MODE_SET; }

void *host_pinned_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return p;
}

void host_pinned_free(void *p) {
    if (p) (void)hipHostFree(p);
}

okm_status memcpy_d2h_on(int device, void *dst, const void *src, size_t bytes) {
    HIP_TRY(hipSetDevice(device));
    if (bytes) HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return OKM_OK;
}

static okm_status ensure_hc(okm_ctx *c, size_t n_u32) {
    if (n_u32 <= c->HC_cap) return OKM_OK;
    if (c->HC) (void)hipFree(c->HC);
    c->HC = nullptr;
    size_t cap = std::max(n_u32, size_t(1) << 20);
    HIP_TRY(hipMalloc(&c->HC, cap * sizeof(uint32_t)));
    c->HC_cap = cap;
    return OKM_OK;
}

static okm_status ensure_hg(okm_ctx *c, size_t n) {
    if (n <= c->Hg_cap) return OKM_OK;
    if (c->Hg) (void)hipFree(c->Hg);
    if (c->cursor) (void)hipFree(c->cursor);
    c->Hg = c->cursor = nullptr;
    size_t cap = std::max(n, size_t(1) << 16);
    HIP_TRY(hipMalloc(&c->Hg, cap * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc(&c->cursor, cap * sizeof(unsigned long long)));
    c->Hg_cap = cap;
    return OKM_OK;
}

static okm_status ensure_pinned(okm_ctx *c, size_t bytes) {
    if (bytes <= c->pinned_cap) return OKM_OK;
    if (c->pinned) (void)hipHostFree(c->pinned);
    c->pinned = nullptr;
    size_t cap = std::max(bytes, size_t(1) << 20);
    HIP_TRY(hipHostMalloc(&c->pinned, cap, hipHostMallocDefault));
    c->pinned_cap = cap;
    return OKM_OK;
}

static okm_status ensure_staging(okm_ctx *c, size_t bytes) {
    if (bytes <= c->staging_cap) return OKM_OK;
    if (c->staging) (void)hipFree(c->staging);
    c->staging = nullptr;
    size_t cap = std::max(bytes + 64, size_t(1) << 20);
    HIP_TRY(hipMalloc(&c->staging, cap));
    c->staging_cap = cap;
    return OKM_OK;
}

static void host_table_free(okm_ctx *c, uint64_t *keys, uint64_t *counts, uint64_t n) {
    host_pinned_free(keys);
    host_pinned_free(counts);
    const uint64_t b = n * 8 * c->kw + (counts ? n * 8 : 0);
    c->host_bytes -= std::min(c->host_bytes, b);
}

static void drop_pending(okm_ctx *c) {
    for (void *p : c->pend.hold) c->pool->put(p);
    c->pend = okm_ctx::Pending{};
}

static void invalidate_result(okm_ctx *c) {
    drop_pending(c);
    if (c->res_host) {
        host_table_free(c, c->res_keys, c->res_counts, c->n_res);
    } else {
        if (c->res_keys) c->pool->put(c->res_keys);
        if (c->res_counts) c->pool->put(c->res_counts);
    }
    c->res_host = false;
    c->res_keys = c->res_counts = nullptr;
    c->n_res = 0;
    c->counted = false;
    c->res_is_input = false;
}

// Device memory this context may still use: the budget (OKM_HBM_CAP) less
// what every pool on the device maps, plus this pool's cached (idle) part --
// and no more than the device's free memory plus that cached part.
static double device_room(okm_ctx *c) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        free_b = 0;
    }
    const double cached = (double)c->pool->cached();
    const double room = std::min((double)free_b + cached,
                                 hbm_budget(c->device) - (double)DevPool::device_mapped(c->device) + cached);
    return std::max(room, 0.0);
}

static okm_status sync(okm_ctx *c) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipGetLastError());
    c->timer.flush();
    c->hpin_used = 0;  // every copy out of the pinned staging has completed
    return OKM_OK;
}

// The dense (keys, counts) copy of a table left as the items' sorted runs
// (okm_ctx::Pending): one gather in key order (k_compact_items), then the
// runs' memory goes back to the pool.  A no-op for a dense result.
static okm_status ensure_dense(okm_ctx *c) {
    if (!c->pend.on) return OKM_OK;
    const uint64_t nd = c->n_res;
    const uint64_t kb = std::max<uint64_t>(nd, 1) * 8 * c->kw, cb = std::max<uint64_t>(nd, 1) * 8;
    uint64_t *dk = nullptr, *dc = nullptr, *hk = nullptr, *hc = nullptr;
    okm_status st = pool_get(*c->pool, kb / 8, &dk);
    if (st == OKM_OK) st = pool_get(*c->pool, cb / 8, &dc);
    if (st == OKM_E_NOMEM) {
        // no room on the device for the dense copy: the gather writes it
        // straight into page-locked, device-mapped host memory (the host tier)
        c->pool->put(dk);
        dk = dc = nullptr;
        if (hipHostMalloc(reinterpret_cast<void **>(&hk), kb, hipHostMallocMapped) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void **>(&hc), cb, hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            host_pinned_free(hk);
            return fail(OKM_E_NOMEM, "the dense copy of a " + std::to_string(nd) +
                                         "-entry table fits neither the device nor page-locked host memory");
        }
        st = OKM_OK;
        if (hipHostGetDevicePointer(reinterpret_cast<void **>(&dk), hk, 0) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void **>(&dc), hc, 0) != hipSuccess)
            st = fail(OKM_E_DEVICE, "hipHostGetDevicePointer");
    }
    if (st == OKM_OK) {
        c->timer.begin(c->stream);
        launch_compact_items(c->stream, c->pend.items, c->pend.nitems, c->pend.n_out, c->pend.dense_off, c->pend.sk,
                             c->pend.sc, dk, dc, c->wide, c->pend.narrow, nullptr, nullptr, nullptr);
        c->timer.end(c->stream, "compact_items",
                     (8.0 * c->kw + (c->pend.narrow ? 4.0 : 8.0) + 8.0 * c->kw + 8.0) * (double)nd);
        st = hipGetLastError() == hipSuccess ? sync(c) : fail(OKM_E_DEVICE, "compact_items launch");
    }
    if (st != OKM_OK) {
        if (hk) {
            host_pinned_free(hk);
            host_pinned_free(hc);
        } else {
            c->pool->put(dk);
            c->pool->put(dc);
        }
        return st;
    }
    for (void *p : c->pend.hold) c->pool->put(p);
    c->pend = okm_ctx::Pending{};
    if (hk) {
        c->res_keys = hk;
        c->res_counts = hc;
        c->res_host = true;
        c->host_bytes += kb + cb;
    } else {
        c->res_keys = dk;
        c->res_counts = dc;
    }
    c->hprof.mark("dense");
    return OKM_OK;
}

// Several small host tables laid out in one buffer (256-B aligned), so that
// they reach the device in a single copy.
struct TablePack {
    std::vector<uint8_t> bytes;
    template <typename T> size_t add(const std::vector<T> &v) {
        const size_t at = (bytes.size() + 255) & ~size_t(255);
        bytes.resize(at + v.size() * sizeof(T));
        if (!v.empty()) memcpy(bytes.data() + at, v.data(), v.size() * sizeof(T));
        return at;
    }
};

// Host-to-device copy of a small table, staged in pinned memory so that the
// DMA reads it directly (a pageable source takes a bounce copy and a blit).
static okm_status h2d(okm_ctx *c, void *dst, const void *src, size_t bytes) {
    if (!bytes) return OKM_OK;
    const size_t at = (c->hpin_used + 255) & ~size_t(255);
    if (at + bytes <= kHpinBytes) {
        memcpy(c->hpin + at, src, bytes);
        c->hpin_used = at + bytes;
        HIP_TRY(hipMemcpyAsync(dst, c->hpin + at, bytes, hipMemcpyHostToDevice, c->stream));
    } else {
        HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    }
    return OKM_OK;
}

// Host prefix sum of a device histogram -> offsets (host) and device cursor.
// align > 1: every bin's slot is rounded up to `align` keys (starts on a
// 128-B line for align 16); *exact (if given) receives the unpadded total.
static okm_status hist_to_offsets(okm_ctx *c, size_t nb, std::vector<uint64_t> &off, uint64_t align = 1,
                                  uint64_t *exact = nullptr) {
    std::vector<unsigned long long> h(nb);
    HIP_TRY(hipMemcpyAsync(h.data(), c->Hg, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    OKM_TRY(sync(c));
    off.assign(nb + 1, 0);
    uint64_t tot = 0;
    for (size_t b = 0; b < nb; ++b) {
        off[b + 1] = off[b] + (h[b] + align - 1) / align * align;
        tot += h[b];
    }
    if (exact) *exact = tot;
    HIP_TRY(hipMemcpyAsync(c->cursor, off.data(), nb * sizeof(unsigned long long), hipMemcpyHostToDevice, c->stream));
    return OKM_OK;
}

// Tile sampling stride of the sampled L1 placement.
static constexpr uint32_t kL1SampleStride = 16;

// Sampled L1 placement: histogram every S-th tile, size each bin from that
// sample (launch_l1_capacity), scatter with per-tile claims.  One host sync,
// after the scatter, reads the bins' ends and the overflow flag; *placed is
// false (nothing recorded) when some bin outgrew its capacity.
static okm_status l1_sampled(okm_ctx *c, const uint8_t *d_seq, uint64_t n, const ExtractGeom &g, uint32_t S,
                             bool *placed) {
    *placed = false;
    const uint64_t tile = extract_tile();
    const uint64_t tiles = (n + tile - 1) / tile;
    const uint32_t nb = c->nbins, align = 16 / c->kw;
    ExtractGeom gs{n, c->k, c->shift1, nb, (uint32_t)((tiles + S - 1) / S), tile, S};
    const uint64_t last = (uint64_t)(gs.nblocks - 1) * S * tile;  // the only sampled tile that can be short
    const uint64_t sbytes = (uint64_t)(gs.nblocks - 1) * tile + std::min(tile, n - last);
    const double scale = (double)n / (double)sbytes;
    const int64_t dbg = test_knob(OKM_TEST_L1_CAP_PERMILLE);  // tests: shrink capacities to force the exact redo
    const double mul = dbg >= 0 ? (double)dbg / 1000.0 : 1.0;
    // sum_b scale s_b <= w n (windows <= bytes; w = the windows-per-byte ratio
    // seen so far on this context, 1 before the first batch: the run is sized
    // for the keys it gets, not for the bytes); sum_b sqrt(s_b) <= sqrt(nb * w * sbytes).
    // A batch with more windows than that overflows its sampled placement and
    // is redone exactly (correct, just slower).
    const double w = c->l1_ratio > 0 ? std::min(1.0, c->l1_ratio * 1.02 + 0.002) : 1.0;
    const uint64_t limit = (uint64_t)(1.01 * (w * (double)n + 6.0 * scale * std::sqrt((double)nb * w * (double)sbytes) +
                                              9.0 * scale * nb) +
                                      (double)nb * (256.0 + align)) + 64;
    OKM_TRY(ensure_hg(c, nb));
    HIP_TRY(hipMemsetAsync(c->Hg, 0, nb * sizeof(unsigned long long), c->stream));
    c->timer.begin(c->stream);
    launch_extract_hist(c->stream, d_seq, gs, nullptr, c->Hg);
    c->timer.end(c->stream, "extract_sample", (double)sbytes);
    // l1cap: cap_end[nb] | start[nb + 1] | overflow; the claim cursors stay in
    // their own (line-aligned) array: placing them beside the other words slowed
    // the claims by 25 %
    unsigned long long *cur = c->curpad;
    launch_l1_capacity(c->stream, c->Hg, nb, scale, mul, align, limit, cur, c->l1cap);
    HIP_TRY(hipGetLastError());
    Run run;
    OKM_TRY(pool_get(*c->pool, limit * c->kw, &run.keys));
    c->timer.begin(c->stream);
    launch_extract_scatter(c->stream, d_seq, g, nullptr, cur, run.keys, c->l1cap, c->l1cap + 2 * nb + 1);
    c->timer.end(c->stream, "extract_scatter", (double)n);
    launch_fill_line_tails(c->stream, cur, nb, run.keys, c->wide, c->l1cap);
    HIP_TRY(hipGetLastError());
    unsigned long long *cap = c->hres, *ends = c->hres + 2 * nb + 2;  // 3 nb + 2 <= kHresCount words
    HIP_TRY(hipMemcpyAsync(cap, c->l1cap, (2 * nb + 2) * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipMemcpy2DAsync(ends, sizeof(unsigned long long), cur, kL1CurStride * sizeof(unsigned long long),
                             sizeof(unsigned long long), nb, hipMemcpyDeviceToHost, c->stream));
    OKM_TRY(sync(c));
    if (cap[2 * nb + 1]) {  // some bin outgrew its sampled capacity: redo exactly
        c->pool->put(run.keys);
        c->hprof.mark("l1.sampled_overflow");
        return OKM_OK;
    }
    uint64_t total = 0;
    run.off.assign(cap + nb, cap + 2 * nb + 1);
    run.end.resize(nb);
    for (uint32_t b = 0; b < nb; ++b) {
        total += ends[b] - run.off[b];
        run.end[b] = (ends[b] + align - 1) / align * align;
    }
    c->timer.add_bytes("extract_scatter", 8.0 * c->kw * (double)total);
    c->l1_ratio = std::max(c->l1_ratio, (double)total / (double)n);
    *placed = true;
    if (total == 0) {
        c->pool->put(run.keys);
        return OKM_OK;
    }
    c->runs.push_back(std::move(run));
    c->info.kmers += total;
    c->hprof.mark("l1.sampled");
    return OKM_OK;
}

static okm_status do_count(okm_ctx *c);

static okm_status shrink_table(okm_ctx *c, uint64_t **keys, uint64_t **counts, uint64_t n, double slack);
static okm_status count_general(okm_ctx *c);

static void set_l1_geometry(okm_ctx *c) {
    c->l1_bits = std::min<uint32_t>(extract_l1_bits(c->wide, c->l1_fold), 2u * c->k);
    c->nbins = 1u << c->l1_bits;
    c->shift1 = 2u * c->k - c->l1_bits;
}

// L1 bin bounds of a sorted run by binary search (a sorted table is already
// partitioned by key range: nothing moves).
// L1 bin b of a key: its top l1 bits (the same cut as k_bin_bounds).
static uint64_t key_bin_host(const okm_ctx *c, const uint64_t *keys, uint64_t i) {
    if (c->wide) {
        const uint64_t lo = keys[2 * i], hi = keys[2 * i + 1];
        const uint32_t sh = c->shift1;
        return sh >= 128 ? 0 : sh >= 64 ? hi >> (sh - 64) : sh == 0 ? lo : (hi << (64 - sh)) | (lo >> sh);
    }
    return c->shift1 >= 64 ? 0 : keys[i] >> c->shift1;
}

static okm_status sorted_run_bins(okm_ctx *c, Run &run) {
    if (run.host) {  // a table in host memory: the bin starts by binary search on the host
        run.off.assign(c->nbins + 1, run.n);
        for (uint32_t b = 0; b <= c->nbins; ++b) {
            uint64_t lo = 0, hi = run.n;  // first i with bin(i) >= b
            while (lo < hi) {
                const uint64_t mid = (lo + hi) / 2;
                if (key_bin_host(c, run.keys, mid) < b) lo = mid + 1; else hi = mid;
            }
            run.off[b] = lo;
        }
        run.off[c->nbins] = run.n;
        return OKM_OK;
    }
    OKM_TRY(ensure_hg(c, c->nbins + 1));
    launch_bin_bounds(c->stream, run.keys, run.n, c->shift1, c->nbins, c->Hg, c->wide);
    HIP_TRY(hipGetLastError());
    run.off.assign(c->nbins + 1, 0);
    HIP_TRY(hipMemcpyAsync(run.off.data(), c->Hg, (c->nbins + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    OKM_TRY(sync(c));
    return OKM_OK;
}

// The counted result becomes a folded run: a sorted weighted table owned by
// the context, at its exact size (the count sized it by its instances).
static okm_status result_to_folded_run(okm_ctx *c, Run *out) {
    OKM_TRY(ensure_dense(c));
    if (!c->res_host) OKM_TRY(shrink_table(c, &c->res_keys, &c->res_counts, c->n_res, 1.25));
    Run run;
    run.keys = c->res_keys;
    run.counts = c->res_counts;
    run.n = c->n_res;
    run.sorted = true;
    run.folded = true;
    run.host = c->res_host;
    c->res_keys = c->res_counts = nullptr;
    c->res_host = false;
    c->n_res = 0;
    c->counted = false;
    if (run.n) OKM_TRY(sorted_run_bins(c, run));
    *out = std::move(run);
    return OKM_OK;
}

// Before new input: drop the result, unless it is the only record of the
// input so far (res_is_input: its borrowed runs were released once counted),
// in which case it stays as a folded run that the next count merges with the
// new input (count.rs:48: one map across every add).
static okm_status before_add(okm_ctx *c) {
    if (c->input_lost) return fail(OKM_E_STATE, "a failed count overwrote this context's input: okm_reset it");
    if (!(c->counted && c->res_is_input)) {
        invalidate_result(c);
        return OKM_OK;
    }
    c->res_is_input = false;
    Run t;
    OKM_TRY(result_to_folded_run(c, &t));
    if (t.n) {
        c->runs.push_back(std::move(t));
    } else {
        c->pool->put(t.keys);
        c->pool->put(t.counts);
    }
    return OKM_OK;
}

// A run's memory back to the pool (device) or the host (host runs); borrowed
// runs belong to the caller.
static void free_run(okm_ctx *c, Run &r) {
    if (r.borrowed) return;
    if (r.host) {  // (a batch run moved there by spill_runs: its whole capacity)
        host_table_free(c, r.keys, r.counts, r.sorted ? r.n : (r.off.empty() ? 0 : r.off.back()));
    } else {
        c->pool->put(r.keys);
        c->pool->put(r.counts);
    }
    r.keys = r.counts = nullptr;
}

static void release_runs(okm_ctx *c, std::vector<Run> &runs) {
    for (auto &r : runs) free_run(c, r);
    runs.clear();
}

// Count the context's unsorted runs (batches) alone into one sorted table and
// keep it, as a folded run, beside the sorted runs already there.
static okm_status count_unsorted_to_table(okm_ctx *c) {
    std::vector<Run> keep, batches;  // (batch runs in host memory stay for count_spilled)
    for (auto &r : c->runs) (r.sorted || r.host ? keep : batches).push_back(std::move(r));
    c->runs = std::move(batches);
    c->counted = false;
    const bool outer = !c->may_take_runs, shared = c->share_result;
    c->may_take_runs = true;  // the batches are released below
    c->share_result = false;  // ... and the table is kept
    okm_status st = c->runs.empty() ? OKM_OK : count_general(c);
    if (outer) c->may_take_runs = false;
    c->share_result = shared;
    if (st != OKM_OK) {
        // the batches are intact (a count reads them until it succeeds; a
        // count that wrote into one set input_lost): they stay, so the
        // caller's fallback (do_count: the host tier) can count them
        for (auto &r : keep) c->runs.push_back(std::move(r));
        return st;
    }
    Run t;
    if (!c->runs.empty()) st = result_to_folded_run(c, &t);
    release_runs(c, c->runs);
    for (auto &r : keep) c->runs.push_back(std::move(r));
    if (st != OKM_OK) return st;
    if (t.n) {
        c->runs.push_back(std::move(t));
    } else if (t.keys) {
        c->pool->put(t.keys);
        c->pool->put(t.counts);
    }
    return OKM_OK;
}

// Fold (memory bounded by distinct keys, not by input): the batches added
// since the last fold are counted into a sorted (key, count) table that
// replaces their L1 runs; every kFoldMergeRuns tables are merged into one
// (k-way LDS merge, okm_merge.hip).  okm_count merges the tables with the
// last batches' table.  The reference's DashMap grows with distinct k-mers
// only (count.rs:48); without folding every batch's instances would stay
// resident until okm_count.
// Device bytes a run holds (borrowed and host runs: none).
static uint64_t run_device_bytes(okm_ctx *c, const Run &r) {
    if (r.borrowed || r.host) return 0;
    return c->pool->size_of(r.keys) + c->pool->size_of(r.counts);
}

// Move folded tables to page-locked host memory, oldest first, until the
// device has `need` bytes of room (or no table is left on it).  The
// reference's DashMap grows in host RAM until the machine runs out
// (count.rs:48); here a table that no longer fits beside the next count's
// working set waits in host memory, and okm_count merges every table key
// range by key range (count_spilled), the host ones streamed back in slices.
static okm_status spill_tables(okm_ctx *c, double need) {
    for (auto &r : c->runs) {
        if (device_room(c) >= need) break;
        if (!r.folded || r.host || r.borrowed || r.n == 0) continue;
        const uint64_t kb = r.n * 8 * c->kw, cb = r.counts ? r.n * 8 : 0;
        uint64_t *hk = static_cast<uint64_t *>(host_pinned_alloc(kb));
        uint64_t *hc = cb ? static_cast<uint64_t *>(host_pinned_alloc(cb)) : nullptr;
        if (!hk || (cb && !hc)) {
            host_pinned_free(hk);
            host_pinned_free(hc);
            return fail(OKM_E_NOMEM, "moving a " + std::to_string(kb + cb) +
                                         " B table off the device: page-locked host allocation failed");
        }
        HIP_TRY(hipMemcpyAsync(hk, r.keys, kb, hipMemcpyDeviceToHost, c->stream));
        if (cb) HIP_TRY(hipMemcpyAsync(hc, r.counts, cb, hipMemcpyDeviceToHost, c->stream));
        OKM_TRY(sync(c));
        c->pool->put(r.keys);
        c->pool->put(r.counts);  // (inside the keys' block when shrink_table joined them: ignored)
        r.keys = hk;
        r.counts = hc;
        r.host = true;
        c->host_bytes += kb + cb;
        c->spills += 1;
        c->hprof.mark("spill");
    }
    return OKM_OK;
}

// Move every uncounted batch run (L1-partitioned keys, no table yet) to
// page-locked host memory: the last resort when even one count's working set
// does not fit beside them.  count_spilled then counts the key space in
// groups of L1 bins, each group's slices uploaded and counted on the device.
static okm_status spill_runs(okm_ctx *c) {
    for (auto &r : c->runs) {
        if (r.sorted || r.host || r.borrowed || r.off.empty()) continue;
        const uint64_t words = r.off.back() * c->kw;
        const uint64_t kb = words * 8, cb = r.counts ? r.off.back() * 8 : 0;
        uint64_t *hk = static_cast<uint64_t *>(host_pinned_alloc(std::max<uint64_t>(kb, 8)));
        uint64_t *hc = cb ? static_cast<uint64_t *>(host_pinned_alloc(cb)) : nullptr;
        if (!hk || (cb && !hc)) {
            host_pinned_free(hk);
            host_pinned_free(hc);
            return fail(OKM_E_NOMEM, "moving a " + std::to_string(kb + cb) +
                                         " B batch run off the device: page-locked host allocation failed");
        }
        if (kb) HIP_TRY(hipMemcpyAsync(hk, r.keys, kb, hipMemcpyDeviceToHost, c->stream));
        if (cb) HIP_TRY(hipMemcpyAsync(hc, r.counts, cb, hipMemcpyDeviceToHost, c->stream));
        OKM_TRY(sync(c));
        c->pool->put(r.keys);
        c->pool->put(r.counts);
        r.keys = hk;
        r.counts = hc;
        r.host = true;
        c->host_bytes += kb + cb;
        c->spills += 1;
        c->hprof.mark("spill_run");
    }
    return OKM_OK;
}

// Device bytes of the uncounted batch runs (their count needs ~4.5x that:
// level array, staged runs, the exact table).
static double uncounted_bytes(okm_ctx *c) {
    double b = 0;
    for (auto &r : c->runs)
        if (!r.sorted) b += (double)run_device_bytes(c, r);
    return b;
}

static okm_status fold(okm_ctx *c) {
    OKM_TRY(spill_tables(c, 4.5 * uncounted_bytes(c)));
    OKM_TRY(count_unsorted_to_table(c));
    c->folds += 1;
    if (c->hprof.on)
        fprintf(stderr, "[okm fold] #%u counted: peak in use so far %.1f GB\n", c->folds + 0u, c->pool->peak() / 1e9);
    // A context that folds takes 10 L1 bits from here on (and after okm_reset):
    // a fold counts ~3.6 G instances, whose 9-bit parts are too big for one
    // 2048-child pass and go through the fan-out split; 10-bit parts do not
    // (C3 on one GPU: 414 vs 461 ms; a batch-by-batch C2 count stays at 9 bits,
    // its extraction writes longer runs: 5.23 vs 5.44 ms).  Only sorted runs
    // (tables) are left here, and their bins come from a binary search.
    if (!c->l1_fold && !c->wide) {
        bool all_sorted = true;
        for (auto &r : c->runs) all_sorted &= r.sorted;
        if (all_sorted) {
            c->l1_fold = true;
            set_l1_geometry(c);
            for (auto &r : c->runs)
                if (r.n) OKM_TRY(sorted_run_bins(c, r));
        }
    }
    // four tables merge into one (3: 438-448 ms per C3 job, 6: 446-451, 8: 499,
    // 4: 409-412; profiles/AB_LOG.md round 4)
    // Tables in host memory wait for okm_count; the device ones merge when
    // the merge's exact table fits beside them, else they go to host memory too.
    constexpr uint32_t merge_runs = 4;
    uint32_t tables = 0;
    bool only_folded = true;
    double dev_pairs = 0;
    for (auto &r : c->runs) {
        tables += r.folded && !r.host;
        only_folded &= r.folded;
        if (!r.host) dev_pairs += (double)r.n;
    }
    if (tables >= merge_runs && only_folded) {
        if (device_room(c) < 1.5 * (8.0 * c->kw + 8.0) * dev_pairs) {
            OKM_TRY(spill_tables(c, INFINITY));
        } else {
            std::vector<Run> host_runs, dev_runs;
            for (auto &r : c->runs) (r.host ? host_runs : dev_runs).push_back(std::move(r));
            c->runs = std::move(dev_runs);
            okm_status st = do_count(c);
            if (st == OKM_OK) release_runs(c, c->runs);
            Run t;
            if (st == OKM_OK) st = result_to_folded_run(c, &t);
            for (auto &r : host_runs) c->runs.push_back(std::move(r));
            OKM_TRY(st);
            if (t.n) c->runs.push_back(std::move(t));
        }
    }
    c->hprof.mark("fold");
    if (c->hprof.on) {
        uint64_t tb = 0, tn = 0;
        for (auto &r : c->runs) {
            tb += c->pool->size_of(r.keys) + c->pool->size_of(r.counts);
            tn += r.n;
        }
        fprintf(stderr, "[okm fold] #%u: %zu runs of %.3f G keys holding %.1f GB; pool held %.1f GB, cached %.1f GB; "
                        "peak in use so far %.1f GB\n",
                c->folds, c->runs.size(), tn / 1e9, tb / 1e9, c->pool->held() / 1e9, c->pool->cached() / 1e9,
                c->pool->peak() / 1e9);
    }
    return OKM_OK;
}

// Fold before a batch of n bytes (<= n windows, 8 B per key word each) would
// take the uncounted L1 runs past the context's fold threshold.
static okm_status maybe_fold(okm_ctx *c, uint64_t n) {
    if (!c->fold_bytes) return OKM_OK;  // OKM_FOLD_BYTES=0: folding off
    uint64_t held = 0;
    bool uncounted = false;
    for (auto &r : c->runs) {
        if (r.borrowed || r.folded || r.host) continue;
        held += c->pool->size_of(r.keys) + c->pool->size_of(r.counts);  // allocations, not keys
        uncounted = true;
    }
    const double w = c->l1_ratio > 0 ? std::min(1.0, c->l1_ratio * 1.03) : 1.0;
    if (!uncounted) return OKM_OK;
    if (held + (uint64_t)(w * (double)n) * 8 * c->kw <= c->fold_bytes) return OKM_OK;
    return fold(c);
}

// L1 pass over a device-resident batch (whitespace-free records joined by
// OKM_RECORD_SEPARATOR, 16-byte aligned).
static okm_status l1_batch(okm_ctx *c, const uint8_t *d_seq, uint64_t n) {
    if (n == 0) return OKM_OK;
    OKM_TRY(maybe_fold(c, n));
    c->hprof.mark("idle");
    const uint64_t tile = extract_tile();
    uint64_t tiles = (n + tile - 1) / tile;
    // extraction workgroups: 8192 (C2: ~4 tiles each) against 2048: extract_scatter
    // 1.438 vs 1.484 ms over 4 interleaved runs, 4096 1.447 (profiles/r04_ab_extract_blocks.txt)
    constexpr uint64_t max_blocks = 8192;
    uint32_t nblocks = (uint32_t)std::min<uint64_t>(tiles, max_blocks);
    uint64_t chunk = ((tiles + nblocks - 1) / nblocks) * tile;
    nblocks = (uint32_t)((n + chunk - 1) / chunk);
    ExtractGeom g{n, c->k, c->shift1, c->nbins, nblocks, chunk, 1};
    const uint32_t S = kL1SampleStride;
    if (S > 1 && tiles >= 64ull * S && c->nbins > 1) {
        bool placed = false;
        OKM_TRY(l1_sampled(c, d_seq, n, g, S, &placed));
        if (placed) return OKM_OK;
    }

    OKM_TRY(ensure_hc(c, (size_t)nblocks * c->nbins));
    OKM_TRY(ensure_hg(c, c->nbins));
    HIP_TRY(hipMemsetAsync(c->Hg, 0, c->nbins * sizeof(unsigned long long), c->stream));
    c->timer.begin(c->stream);
    launch_extract_hist(c->stream, d_seq, g, c->HC, c->Hg);
    c->timer.end(c->stream, "extract_hist", (double)n);
    HIP_TRY(hipGetLastError());

    Run run;
    uint64_t total = 0;  // bins start on 128-B lines; slot tails hold the empty key
    OKM_TRY(hist_to_offsets(c, c->nbins, run.off, 16 / c->kw, &total));
    c->l1_ratio = std::max(c->l1_ratio, (double)total / (double)n);
    c->hprof.mark("l1.hist+sync");
    if (total == 0) return OKM_OK;
    OKM_TRY(pool_get(*c->pool, run.off.back() * c->kw, &run.keys));
    c->timer.begin(c->stream);
    launch_extract_scatter(c->stream, d_seq, g, c->HC, c->cursor, run.keys, nullptr, nullptr);
    c->timer.end(c->stream, "extract_scatter", (double)n + 8.0 * c->kw * (double)total);
    HIP_TRY(hipGetLastError());
    launch_fill_line_tails(c->stream, c->cursor, c->nbins, run.keys, c->wide);
    HIP_TRY(hipGetLastError());
    c->runs.push_back(std::move(run));
    c->info.kmers += total;
    c->hprof.mark("l1.scatter_launch");
    return OKM_OK;
}

struct Part {
    uint32_t seg_begin, seg_count;  // into the host segment table
    uint64_t len;
    unsigned __int128 prefix;       // absolute key prefix at `consumed` bits (2k <= 128)
    uint32_t consumed;
};

static constexpr uint64_t kChunkKeys = 65536;  // keys per partition chunk (a multiple of the scatter tiles)

// Output of one partition pass: a level array whose bins are the children, in
// key order, of the parts that took part (offsets stay on the device).
struct Level {
    unsigned long long *d_offs = nullptr;  // nout + 1 exclusive offsets (line padded)
    unsigned long long *d_ends = nullptr;  // sampled placement: per-bin ends (else bins abut)
    unsigned long long *d_ovf = nullptr;   // sampled placement: overflow word
    uint64_t *lk = nullptr, *lc = nullptr;
    uint32_t nout = 0;
    uint64_t padded = 0;                   // keys of address space (offsets' total)
    uint64_t total = 0;                    // input keys of the pass
    std::vector<uint32_t> out_base;        // first output bin of each participating part
};

// One partition pass: split every part in `todo` by its own number of bits
// (0 bits = gather the part as one bin).
static okm_status split_launch_sampled(okm_ctx *c, const std::vector<DevSeg> &psegs,
                                       const std::vector<DevChunk> &chunks, const std::vector<uint32_t> &todo,
                                       const std::vector<uint32_t> &bits, bool weighted, uint32_t max_local,
                                       std::vector<void *> &level_bufs, Level &L, unsigned long long *ovf);

// Tile sampling stride of the sampled partition placement.
static constexpr uint32_t kPartSampleStride = 16;

// ovf (sampled mode): size the children from a histogram of 1/S of every
// chunk (launch_part_capacity) instead of an exact pass, so no host sync
// sits between the passes; *ovf becomes nonzero when a child outgrew its
// slot (the level is then invalid and must be redone exactly).
static okm_status split_launch(okm_ctx *c, const std::vector<DevSeg> &segtab, const std::vector<Part> &parts,
                               const std::vector<uint32_t> &todo, const std::vector<uint32_t> &bits, bool weighted,
                               std::vector<void *> &level_bufs, Level &L, unsigned long long *ovf = nullptr) {
    const uint32_t twok = 2u * c->k;
    std::vector<DevSeg> psegs;      // pass segments (one per input segment)
    std::vector<DevChunk> chunks;
    L.out_base.assign(todo.size(), 0);
    uint32_t nout = 0, max_local = 1;
    uint64_t total = 0;
    for (size_t t = 0; t < todo.size(); ++t) {
        const Part &p = parts[todo[t]];
        const uint32_t b = bits[t];
        const uint32_t nl = 1u << b;
        L.out_base[t] = nout;
        nout += nl;
        max_local = std::max(max_local, nl);
        for (uint32_t s = 0; s < p.seg_count; ++s) {
            DevSeg d = segtab[p.seg_begin + s];
            d.shift = b ? twok - p.consumed - b : kSingleBin;
            d.key_base = (uint64_t)(p.prefix << b);  // local_bin works modulo 2^64
            d.out_base = L.out_base[t];
            d.nlocal = nl;
            const uint32_t sid = (uint32_t)psegs.size();
            psegs.push_back(d);
            for (uint64_t o = 0; o < d.len; o += kChunkKeys)
                chunks.push_back(DevChunk{sid, 0, o, std::min(kChunkKeys, d.len - o)});
        }
        total += p.len;
    }
    L.nout = nout;
    L.total = total;
    OKM_TRY(ensure_hg(c, nout + 1));
    if (ovf) return split_launch_sampled(c, psegs, chunks, todo, bits, weighted, max_local, level_bufs, L, ovf);
    OKM_TRY(ensure_hc(c, chunks.size() * (size_t)max_local));
    DevSeg *d_segs;
    DevChunk *d_chunks;
    unsigned long long *scan_tmp;
    OKM_TRY(pool_get(*c->pool, psegs.size(), &d_segs));
    OKM_TRY(pool_get(*c->pool, chunks.size(), &d_chunks));
    OKM_TRY(pool_get(*c->pool, (size_t)nout + 1, &L.d_offs));
    OKM_TRY(pool_get(*c->pool, scan_tmp_elems(nout + 1), &scan_tmp));
    level_bufs.push_back(d_segs);
    level_bufs.push_back(d_chunks);
    level_bufs.push_back(L.d_offs);
    level_bufs.push_back(scan_tmp);
    OKM_TRY(h2d(c, d_segs, psegs.data(), psegs.size() * sizeof(DevSeg)));
    OKM_TRY(h2d(c, d_chunks, chunks.data(), chunks.size() * sizeof(DevChunk)));
    HIP_TRY(hipMemsetAsync(c->Hg, 0, ((size_t)nout + 1) * sizeof(unsigned long long), c->stream));
    const double kb = weighted ? 16.0 : 8.0;
    c->timer.begin(c->stream);
    launch_part_hist(c->stream, d_segs, d_chunks, (uint32_t)chunks.size(), max_local, c->HC, c->Hg, c->wide);
    c->timer.end(c->stream, "part_hist", 8.0 * c->kw * (double)total);
    HIP_TRY(hipGetLastError());
    // bin offsets on the device; only the total crosses to the host
    launch_exclusive_scan(c->stream, c->Hg, L.d_offs, (uint64_t)nout + 1, scan_tmp);
    HIP_TRY(hipMemcpyAsync(c->cursor, L.d_offs, (size_t)nout * sizeof(unsigned long long), hipMemcpyDeviceToDevice, c->stream));
    unsigned long long padded = 0;
    HIP_TRY(hipMemcpyAsync(&padded, L.d_offs + nout, sizeof(padded), hipMemcpyDeviceToHost, c->stream));
    c->hprof.mark("split.prep+hist_launch");
    OKM_TRY(sync(c));
    c->hprof.mark("split.hist_sync");
    L.padded = padded;  // bins start on 128-B lines (okm_partition.hip)
    OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(padded, 1) * c->kw, &L.lk));
    level_bufs.push_back(L.lk);
    if (weighted) {
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(padded, 1), &L.lc));
        level_bufs.push_back(L.lc);
    }
    c->timer.begin(c->stream);
    launch_part_scatter(c->stream, d_segs, d_chunks, (uint32_t)chunks.size(), max_local, c->HC, c->cursor, L.lk, L.lc,
                        c->wide);
    c->timer.end(c->stream, "part_scatter", 2.0 * (kb + 8.0 * (c->kw - 1)) * (double)total);
    HIP_TRY(hipGetLastError());
    c->info.levels += 1;
    return OKM_OK;
}

static okm_status split_launch_sampled(okm_ctx *c, const std::vector<DevSeg> &psegs,
                                       const std::vector<DevChunk> &chunks, const std::vector<uint32_t> &todo,
                                       const std::vector<uint32_t> &bits, bool weighted, uint32_t max_local,
                                       std::vector<void *> &level_bufs, Level &L, unsigned long long *ovf) {
    const uint32_t S = kPartSampleStride, nout = L.nout;
    L.d_ovf = ovf;
    const uint64_t piece = kChunkKeys / S;
    // sample = the first 1/S of every chunk; per parent: keys / sampled keys
    std::vector<DevChunk> sample;
    sample.reserve(chunks.size());
    std::vector<uint64_t> seg_sampled(psegs.size(), 0);
    for (const DevChunk &ch : chunks) {
        const uint64_t l = std::min(piece, ch.len);
        sample.push_back(DevChunk{ch.seg, 0, ch.begin, l});
        seg_sampled[ch.seg] += l;
    }
    std::vector<DevCapParent> cp(todo.size());
    double limit = 64.0 + 2.0 * nout;
    for (size_t t = 0, sg = 0; t < todo.size(); ++t) {
        uint64_t len = 0, sl = 0;
        for (; sg < psegs.size() && psegs[sg].out_base == L.out_base[t]; ++sg) {
            len += psegs[sg].len;
            sl += seg_sampled[sg];
        }
        const double scale = sl ? (double)len / (double)sl : 1.0;
        cp[t] = DevCapParent{L.out_base[t], 0, scale};
        // sum_b scale (sqrt(s_b) + 3)^2 <= scale (sl + 6 sqrt(2^bits * sl) + 9 * 2^bits) (s_b sum to <= sl);
        // + 80 per bin (64 + rounding)
        const double nl = (double)(1u << bits[t]);
        limit += 1.01 * scale * ((double)sl + 6.0 * std::sqrt(nl * (double)sl) + 9.0 * nl) + 80.0 * nl;
    }
    const int64_t dbg = test_knob(OKM_TEST_PART_CAP_PERMILLE);  // tests: shrink capacities to force the exact redo
    const double mul = dbg >= 0 ? (double)dbg / 1000.0 : 1.0;
    // the four host tables travel in one copy
    TablePack pack;
    const size_t o_segs = pack.add(psegs), o_chunks = pack.add(chunks), o_sample = pack.add(sample),
                 o_cp = pack.add(cp);
    uint8_t *blob;
    unsigned long long *scan_tmp;
    OKM_TRY(pool_get(*c->pool, pack.bytes.size(), &blob));
    OKM_TRY(pool_get(*c->pool, (size_t)nout + 1, &L.d_offs));
    OKM_TRY(pool_get(*c->pool, (size_t)nout, &L.d_ends));
    OKM_TRY(pool_get(*c->pool, scan_tmp_elems(nout + 1), &scan_tmp));
    for (void *p : {(void *)blob, (void *)L.d_offs, (void *)L.d_ends, (void *)scan_tmp}) level_bufs.push_back(p);
    DevSeg *d_segs = reinterpret_cast<DevSeg *>(blob + o_segs);
    DevChunk *d_chunks = reinterpret_cast<DevChunk *>(blob + o_chunks);
    DevChunk *d_sample = reinterpret_cast<DevChunk *>(blob + o_sample);
    DevCapParent *d_cp = reinterpret_cast<DevCapParent *>(blob + o_cp);
    L.padded = (uint64_t)limit;
    OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(L.padded, 1) * c->kw, &L.lk));
    level_bufs.push_back(L.lk);
    if (weighted) {
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(L.padded, 1), &L.lc));
        level_bufs.push_back(L.lc);
    }
    OKM_TRY(h2d(c, blob, pack.bytes.data(), pack.bytes.size()));
    HIP_TRY(hipMemsetAsync(c->Hg, 0, ((size_t)nout + 1) * sizeof(unsigned long long), c->stream));
    uint64_t sampled_keys = 0;
    for (const DevChunk &ch : sample) sampled_keys += ch.len;
    c->timer.begin(c->stream);
    launch_part_hist(c->stream, d_segs, d_sample, (uint32_t)sample.size(), max_local, nullptr, c->Hg, c->wide);
    c->timer.end(c->stream, "part_sample", 8.0 * c->kw * (double)sampled_keys);
    launch_part_capacity(c->stream, c->Hg, nout, d_cp, (uint32_t)cp.size(), mul);
    launch_exclusive_scan(c->stream, c->Hg, L.d_offs, (uint64_t)nout + 1, scan_tmp);
    HIP_TRY(hipMemcpyAsync(L.d_ends, L.d_offs, (size_t)nout * sizeof(unsigned long long), hipMemcpyDeviceToDevice,
                           c->stream));
    HIP_TRY(hipGetLastError());
    const double kb = weighted ? 16.0 : 8.0;
    c->timer.begin(c->stream);
    launch_part_scatter(c->stream, d_segs, d_chunks, (uint32_t)chunks.size(), max_local, nullptr, L.d_ends, L.lk,
                        L.lc, c->wide, L.d_offs + 1, L.d_ovf);
    c->timer.end(c->stream, "part_scatter", 2.0 * (kb + 8.0 * (c->kw - 1)) * (double)L.total);
    HIP_TRY(hipGetLastError());
    c->hprof.mark("split.sampled_launch");
    c->info.levels += 1;
    return OKM_OK;
}

// Host view of a level: replace each participating part by its non-empty
// children (rare path: a child is still too big for one LDS item).
static okm_status split_children_host(okm_ctx *c, const Level &L, std::vector<DevSeg> &segtab,
                                      std::vector<Part> &parts, const std::vector<uint32_t> &todo,
                                      const std::vector<uint32_t> &bits) {
    std::vector<uint64_t> off((size_t)L.nout + 1), end;
    HIP_TRY(hipMemcpyAsync(off.data(), L.d_offs, off.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    if (L.d_ends) {
        end.resize(L.nout);
        HIP_TRY(hipMemcpyAsync(end.data(), L.d_ends, end.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    }
    OKM_TRY(sync(c));
    std::vector<Part> next;
    next.reserve(parts.size() + L.nout);
    size_t t = 0;
    for (uint32_t i = 0; i < parts.size(); ++i) {
        if (t < todo.size() && todo[t] == i) {
            const Part &p = parts[i];
            const uint32_t b = bits[t];
            for (uint32_t l = 0; l < (1u << b); ++l) {
                const uint32_t ob = L.out_base[t] + l;
                const uint64_t len = (end.empty() ? off[ob + 1] : end[ob]) - off[ob];
                if (!len) continue;
                DevSeg d{};
                d.keys = L.lk + off[ob] * c->kw;
                d.counts = L.lc ? L.lc + off[ob] : nullptr;
                d.len = len;
                d.shift = kSingleBin;
                d.nlocal = 1;
                Part ch{(uint32_t)segtab.size(), 1, len, (p.prefix << b) | l, p.consumed + b};
                segtab.push_back(d);
                next.push_back(ch);
            }
            ++t;
        } else {
            next.push_back(parts[i]);
        }
    }
    parts.swap(next);
    return OKM_OK;
}

static uint32_t log2_floor(uint64_t x) {
    uint32_t r = 0;
    while (x > 1) {
        x >>= 1;
        ++r;
    }
    return r;
}

// Move a (keys, counts) table of n entries into exact-size allocations when
// its current ones are more than `slack` times larger (bound-sized result
// tables hold one slot per instance).
static okm_status shrink_table(okm_ctx *c, uint64_t **keys, uint64_t **counts, uint64_t n, double slack) {
    const uint64_t kb = std::max<uint64_t>(n, 1) * 8 * c->kw, cb = std::max<uint64_t>(n, 1) * 8;
    const double held = (double)c->pool->size_of(*keys) + (double)c->pool->size_of(*counts);
    if (held <= slack * (double)(kb + cb) + (64u << 20)) return OKM_OK;
    // arena: the table stays where it is and the allocations' tails go back
    // (counts inside the keys' block, as count_and_compact lays a shared
    // result out, or two allocations of their own)
    {
        const size_t kpad = (kb + 255) & ~size_t(255);
        uint8_t *kbase = reinterpret_cast<uint8_t *>(*keys);
        if (reinterpret_cast<uint8_t *>(*counts) == kbase + kpad && c->pool->size_of(*keys) >= kpad + cb &&
            c->pool->shrink(*keys, kpad + cb))
            return OKM_OK;
        if (c->pool->size_of(*keys) && c->pool->size_of(*counts) && c->pool->shrink(*keys, kb) &&
            c->pool->shrink(*counts, cb))
            return OKM_OK;
    }
    // keys and counts in ONE block (the counts pointer lies inside it, and the
    // pool ignores it on put): a table kept for long (a folded run, a group's
    // table) then takes one cached block of its total size, where two requests
    // each took a block left by an instance-bound count result (C3 on one GPU:
    // 3.4 G keys of folded tables in 127 GB of blocks instead of 54 GB)
    const uint64_t kpad = (kb + 255) & ~255ull;
    uint8_t *blk;
    OKM_TRY(pool_get(*c->pool, kpad + cb, &blk));
    uint64_t *nk = reinterpret_cast<uint64_t *>(blk), *nc = reinterpret_cast<uint64_t *>(blk + kpad);
    if (n) {
        HIP_TRY(hipMemcpyAsync(nk, *keys, kb, hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(nc, *counts, cb, hipMemcpyDeviceToDevice, c->stream));
    }
    OKM_TRY(sync(c));
    c->pool->put(*keys);
    c->pool->put(*counts);
    *keys = nk;
    *counts = nc;
    return OKM_OK;
}

// A result table owned by the caller (key-range groups, do_count): entries
// go to [off, off + distinct).
struct ResDst {
    uint64_t *keys, *counts;
    uint64_t off;
    // pipelined groups: the table's next entry lives on the device (d_base),
    // and the count's readback words land in hslot ([0] distinct, [1] error
    // word, [2..4] guard words) without a host sync (count_grouped)
    unsigned long long *d_base = nullptr;
    unsigned long long *hslot = nullptr;
};

// Count the items in LDS (okm_count.hip), then gather their sorted runs into
// the dense result table.  One host sync sits between the two: it reads the
// distinct total (and the guard words), so the table is allocated at its exact
// size -- after the level arrays went back to the pool, whose blocks it then
// reuses (the count's working set: level + staged keys + u32 staged counts;
// an instance-bound table would hold 16 B per instance instead of per
// distinct key, 3.6x more at C2).  Into a caller's table (dst: key-range
// groups) the compaction is launched with the count, before the sync.
// Releases level_bufs, d_items and d_segs.
// last_use: no run is read after this count (its items lie in level arrays,
// and c->may_take_runs: the runs are released once counted); the staged keys
// then go into the smallest run block that holds them, when one does.
// guard (a speculative launch over round-0 items, make_items' flags): the
// kernels return at once when guard[0] or guard[1] is set; then *aborted is
// set, hguard[0..2] receives the flags, and the caller keeps level_bufs,
// d_items and d_segs.
static okm_status count_and_compact(okm_ctx *c, DevItem *d_items, DevSeg *d_segs, uint32_t nitems,
                                    uint64_t out_total, uint64_t in_total, bool weighted,
                                    std::vector<void *> &level_bufs, const unsigned long long *guard = nullptr,
                                    unsigned long long *hguard = nullptr, bool *aborted = nullptr,
                                    const unsigned long long *d_nitems = nullptr, const ResDst *dst = nullptr,
                                    bool last_use = false, bool in_place = false) {
    uint64_t *sk = nullptr, *sc = nullptr;
    unsigned long long *n_out, *dense_off, *scan_tmp;
    // wide keys into a caller's table: the count kernel writes the table
    // itself (okm_count.hip launch_count_direct: items in order, each at its
    // look-back prefix) -- no staged runs, no compaction pass
    const bool direct = dst && c->wide;
    // staged counts: u32 (okm_count.hip store_count) -- for weighted launches
    // too when their input survives the count (no in-place staging, no
    // caller's table), which is then redone with u64 counts in the rare case
    // that one does not fit (a C3 merge of four folded tables: 17 GB less)
    bool narrow = !direct && (!weighted || (!in_place && !dst));
    const uint64_t sc_words = narrow ? (std::max<uint64_t>(out_total, 1) + 1) / 2 : std::max<uint64_t>(out_total, 1);
    if (last_use && c->may_take_runs && !dst && !in_place) {
        const size_t need = std::max<uint64_t>(out_total, 1) * 8 * c->kw;
        size_t best = 0;
        for (auto &r : c->runs) {
            const size_t b = r.borrowed ? 0 : c->pool->size_of(r.keys);
            if (b >= need && (!best || b < best)) best = b, sk = r.keys;
        }
    }
    const bool donated = sk != nullptr;
    // a failure once the count may have written into a run: the input is gone
    struct Lost {
        okm_ctx *c;
        bool on;
        ~Lost() {
            if (on) c->input_lost = true;
        }
    } lost{c, false};
    if (!donated && !in_place && !direct) OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(out_total, 1) * c->kw, &sk));
    if (!direct) OKM_TRY(pool_get(*c->pool, sc_words, &sc));
    OKM_TRY(pool_get(*c->pool, nitems + 1, &n_out));
    OKM_TRY(pool_get(*c->pool, nitems + 1, &dense_off));
    OKM_TRY(pool_get(*c->pool, scan_tmp_elems(nitems + 1), &scan_tmp));
    uint32_t *defer = nullptr;             // deferred items (tag kernel)
    unsigned long long *status = nullptr;  // per-item look-back words (direct)
    if (direct)
        OKM_TRY(pool_get(*c->pool, nitems, &status));
    else
        OKM_TRY(pool_get(*c->pool, nitems, &defer));
    auto release_own = [&]() {
        for (void *p : {(void *)sk, (void *)sc, (void *)n_out, (void *)dense_off, (void *)scan_tmp, (void *)defer,
                        (void *)status})
            if (p && !(donated && p == (void *)sk)) c->pool->put(p);
    };
    auto release_level = [&]() {
        for (void *p : level_bufs) c->pool->put(p);
        level_bufs.clear();
        c->pool->put(d_segs);
    };
    if (c->hprof.on) {
        uint64_t rb = 0;
        for (auto &r : c->runs) rb += run_device_bytes(c, r);
        size_t lb = 0;
        for (void *p : level_bufs) lb += c->pool->size_of(p);
        fprintf(stderr, "[okm count] %u items, %.3f G keys: in use %.1f GB (runs %.1f, level %.1f, staged counts %.1f, "
                        "staged keys %.1f GB)\n", nitems, in_total / 1e9, c->pool->in_use() / 1e9, rb / 1e9, lb / 1e9,
                c->pool->size_of(sc) / 1e9, (sk && !donated ? c->pool->size_of(sk) : 0) / 1e9);
    }
    HIP_TRY(hipMemsetAsync(c->flag, 0, 2 * sizeof(unsigned long long), c->stream));
    // items past a device-side count (d_nitems) must scan as empty
    HIP_TRY(hipMemsetAsync(d_nitems ? n_out : n_out + nitems, 0,
                           (d_nitems ? nitems + 1 : 1) * sizeof(unsigned long long), c->stream));
    if (direct) HIP_TRY(hipMemsetAsync(status, 0, (size_t)nitems * sizeof(unsigned long long), c->stream));
    c->timer.begin(c->stream);
    c->hprof.mark("items.h2d");
    lost.on = donated;
    if (direct)
        launch_count_direct(c->stream, d_items, nitems, d_segs, n_out, c->flag, weighted, guard, d_nitems, status,
                            dst->d_base ? dst->keys : dst->keys + dst->off * c->kw,
                            dst->d_base ? dst->counts : dst->counts + dst->off, dst->d_base);
    else
        launch_count_items(c->stream, d_items, nitems, d_segs, sk, sc, n_out, c->flag, defer, weighted, c->wide, guard,
                           d_nitems, false, narrow);
    c->timer.end(c->stream, "count_items", (8.0 * c->kw + (weighted ? 8.0 : 0.0)) * (double)in_total);
    HIP_TRY(hipGetLastError());
    launch_exclusive_scan(c->stream, n_out, dense_off, nitems + 1, scan_tmp);
    HIP_TRY(hipGetLastError());
    if (dst && !direct) {  // a key-range group: straight into the caller's table (sized by the instance bound)
        c->timer.begin(c->stream);
        if (dst->d_base)
            launch_compact_items(c->stream, d_items, nitems, n_out, dense_off, sk, sc, dst->keys, dst->counts, c->wide,
                                 !weighted, guard, c->flag, d_nitems, dst->d_base);
        else
            launch_compact_items(c->stream, d_items, nitems, n_out, dense_off, sk, sc, dst->keys + dst->off * c->kw,
                                 dst->counts + dst->off, c->wide, !weighted, guard, c->flag, d_nitems);
        c->timer.end(c->stream, "compact_items", 0.0);  // bytes added once the total is known
        HIP_TRY(hipGetLastError());
    }
    if (dst && dst->d_base) {
        // pipelined group: the table's next entry advances on the device, the
        // readback waits for the groups' one sync, and every buffer goes back
        // to the pool now (the next group's kernels reuse them in stream order)
        launch_advance_base(c->stream, dst->d_base, dense_off + nitems, guard, c->flag);
        HIP_TRY(hipGetLastError());
        unsigned long long *hs = dst->hslot;
        for (int i = 0; i < 6; ++i) hs[i] = 0;
        HIP_TRY(hipMemcpyAsync(&hs[0], dense_off + nitems, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(&hs[1], c->flag, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
        if (guard) HIP_TRY(hipMemcpyAsync(&hs[2], guard, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
        lost.on = false;  // (groups never write into a run)
        release_own();
        release_level();
        c->pool->put(d_items);
        if (aborted) *aborted = false;  // (known at the sync: count_grouped recounts every group then)
        c->n_res = 0;
        return OKM_OK;
    }
    // [0] distinct, [1] error word, [2..4] guard words, [5] items kept (d_nitems)
    unsigned long long *hv = c->hres + kHresCount;
    HIP_TRY(hipMemcpyAsync(&hv[0], dense_off + nitems, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&hv[1], c->flag, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    if (guard)
        HIP_TRY(hipMemcpyAsync(&hv[2], guard, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    if (d_nitems) HIP_TRY(hipMemcpyAsync(&hv[5], d_nitems, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    if (c->hprof.on)  // deferred items (tag kernel) / tickets taken (direct)
        HIP_TRY(hipMemcpyAsync(&hv[6], c->flag + 1, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    OKM_TRY(sync(c));
    c->hprof.mark("count+scan+sync");
    if (c->hprof.on && !c->wide)
        fprintf(stderr, "[okm count] %u items, %llu deferred to the slow kernel\n", nitems,
                (unsigned long long)(hv[6] & 0xFFFFFFFFull));
    if (guard) {
        for (int i = 0; i < 3; ++i) hguard[i] = hv[2 + i];
        *aborted = (hv[2] | hv[3]) != 0;
        if (*aborted) {  // the kernels returned at once: nothing was written
            lost.on = false;
            release_own();
            return OKM_OK;
        }
    }
    if (weighted && narrow && hv[1] == 8) {
        // a count past 2^32 in the u32 staging: count again with u64 counts
        // (the input is intact: staging was separate, nothing was compacted)
        c->hprof.mark("count.narrow_overflow");
        c->pool->put(sc);
        sc = nullptr;
        narrow = false;
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(out_total, 1), &sc));
        HIP_TRY(hipMemsetAsync(c->flag, 0, 2 * sizeof(unsigned long long), c->stream));
        HIP_TRY(hipMemsetAsync(d_nitems ? n_out : n_out + nitems, 0,
                               (d_nitems ? nitems + 1 : 1) * sizeof(unsigned long long), c->stream));
        launch_count_items(c->stream, d_items, nitems, d_segs, sk, sc, n_out, c->flag, defer, weighted, c->wide, guard,
                           d_nitems, false, false);
        HIP_TRY(hipGetLastError());
        launch_exclusive_scan(c->stream, n_out, dense_off, nitems + 1, scan_tmp);
        HIP_TRY(hipMemcpyAsync(&hv[0], dense_off + nitems, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(&hv[1], c->flag, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
        OKM_TRY(sync(c));
    }
    if (hv[1]) {  // give every buffer of the step back before failing (long-lived contexts)
        release_own();
        release_level();
        c->pool->put(d_items);
        return fail(OKM_E_DEVICE, "count_items invariant violated (code " + std::to_string(hv[1]) + ")");
    }
    const uint64_t nd = hv[0];
    const uint32_t nkept = d_nitems ? (uint32_t)std::min<unsigned long long>(nitems, hv[5]) : nitems;
    const double staged = 8.0 * c->kw + (narrow ? 4.0 : 8.0);  // per distinct key: staged (key, count)
    const double dense = 8.0 * c->kw + 8.0;                      // ... and its dense result entry
    if (!c->timer.stats.empty()) {
        c->timer.stats[c->timer.id_of("count_items")].alg_bytes += (direct ? dense : staged) * (double)nd;
        if (dst && !direct) c->timer.add_bytes("compact_items", (staged + dense) * (double)nd);
    }
    // nothing is in flight: the level arrays (and the item flags the kernels
    // read) are dead -- unless they hold the in-place runs the compaction
    // reads -- and their blocks may hold the result; in place, a dead run
    // block may (the runs' last use: their keys went into the level arrays)
    const size_t kpad = (std::max<uint64_t>(nd, 1) * 8 * c->kw + 255) & ~(size_t)255;
    const size_t need = kpad + std::max<uint64_t>(nd, 1) * 8;
    uint8_t *blk = nullptr;
    if (!dst && in_place && last_use && c->may_take_runs) {
        // the runs are dead (their keys were partitioned into the level
        // arrays, where the compaction reads the staged runs): their blocks go
        // back to the pool before the result is allocated, and neighbouring
        // ones coalesce (a fold's table then fits where its batches were)
        for (auto &r : c->runs) {
            if (r.borrowed || r.host) continue;
            c->pool->put(r.keys);
            c->pool->put(r.counts);
            r.keys = r.counts = nullptr;
        }
        c->took_runs = true;  // (the runs are released after the count)
    } else if (!dst && !in_place && c->share_result) {  // the smallest level block that holds keys and counts
        size_t best = 0, at = 0;
        for (size_t i = 0; i < level_bufs.size(); ++i) {
            const size_t b = c->pool->size_of(level_bufs[i]);
            if (b >= need && (!best || b < best)) best = b, at = i;
        }
        if (best) {
            blk = static_cast<uint8_t *>(level_bufs[at]);
            level_bufs.erase(level_bufs.begin() + at);
        }
    }
    if (!dst && !donated && c->share_result) {
        // the table stays as the items' sorted runs (okm_ctx::Pending): the
        // dense copy is made by its first reader (ensure_dense).  In place,
        // the runs lie over the items' keys in the level arrays, which stay;
        // otherwise in the staging array sk, and the level arrays go now.
        drop_pending(c);
        if (!in_place) release_level();
        okm_ctx::Pending &p = c->pend;
        p.on = true;
        p.items = d_items;
        p.nitems = nkept;
        p.n_out = n_out;
        p.dense_off = dense_off;
        p.sk = in_place ? nullptr : sk;
        p.sc = sc;
        p.narrow = narrow;
        p.hold = level_bufs;
        for (void *q : {(void *)d_segs, (void *)d_items, (void *)n_out, (void *)dense_off, (void *)sc, (void *)p.sk})
            if (q && !(q == (void *)d_segs && !in_place)) p.hold.push_back(q);
        level_bufs.clear();
        sc = nullptr;
        sk = nullptr;
        n_out = dense_off = nullptr;
        release_own();
        c->n_res = nd;
        c->info.distinct = nd;
        c->counted = true;
        c->hprof.mark("count (runs kept)");
        c->hprof.dump("count");
        return OKM_OK;
    }
    if (!in_place) release_level();
    if (!dst) {
        if (blk) {
            c->res_keys = reinterpret_cast<uint64_t *>(blk);
            c->res_counts = reinterpret_cast<uint64_t *>(blk + kpad);  // inside the block: the pool ignores it on put
        } else {
            OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(nd, 1) * c->kw, &c->res_keys));
            OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(nd, 1), &c->res_counts));
        }
        c->timer.begin(c->stream);
        launch_compact_items(c->stream, d_items, nkept, n_out, dense_off, sk, sc, c->res_keys, c->res_counts, c->wide,
                             narrow, nullptr, nullptr, nullptr);
        c->timer.end(c->stream, "compact_items", (staged + dense) * (double)nd);
        HIP_TRY(hipGetLastError());
    }
    OKM_TRY(sync(c));  // the result is complete (and a group's buffers may serve the next group)
    if (in_place) release_level();
    c->pool->put(d_items);
    release_own();
    lost.on = false;
    c->took_runs |= donated;
    c->n_res = nd;
    c->info.distinct = nd;
    c->counted = true;
    c->hprof.mark("compact+sync");
    c->hprof.dump("count");
    return OKM_OK;
}
// L1-partition (key, count) pairs in device memory with the generic pass (one
// segment, 2^l1 bins) into an owned run.
static okm_status partition_pairs(okm_ctx *c, const uint64_t *d_keys, const uint64_t *d_counts, uint64_t n,
                                  Run &run) {
    DevSeg s{};
    s.keys = d_keys;
    s.counts = d_counts;
    s.len = n;
    s.key_base = 0;
    s.out_base = 0;
    s.shift = c->shift1;
    s.nlocal = c->nbins;
    std::vector<DevChunk> chunks;
    for (uint64_t o = 0; o < n; o += kChunkKeys) chunks.push_back(DevChunk{0, 0, o, std::min(kChunkKeys, n - o)});
    DevSeg *d_seg;
    DevChunk *d_chunks;
    OKM_TRY(pool_get(*c->pool, 1, &d_seg));
    OKM_TRY(pool_get(*c->pool, chunks.size(), &d_chunks));
    HIP_TRY(hipMemcpyAsync(d_seg, &s, sizeof(DevSeg), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_chunks, chunks.data(), chunks.size() * sizeof(DevChunk), hipMemcpyHostToDevice, c->stream));
    OKM_TRY(ensure_hc(c, chunks.size() * (size_t)c->nbins));
    OKM_TRY(ensure_hg(c, c->nbins));
    HIP_TRY(hipMemsetAsync(c->Hg, 0, c->nbins * sizeof(unsigned long long), c->stream));
    c->timer.begin(c->stream);
    launch_part_hist(c->stream, d_seg, d_chunks, (uint32_t)chunks.size(), c->nbins, c->HC, c->Hg, c->wide);
    c->timer.end(c->stream, "part_hist", 8.0 * c->kw * (double)n);
    HIP_TRY(hipGetLastError());
    OKM_TRY(hist_to_offsets(c, c->nbins, run.off));
    OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(run.off.back(), 1) * c->kw, &run.keys));
    OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(run.off.back(), 1), &run.counts));
    c->timer.begin(c->stream);
    launch_part_scatter(c->stream, d_seg, d_chunks, (uint32_t)chunks.size(), c->nbins, c->HC, c->cursor, run.keys,
                        run.counts, c->wide);
    c->timer.end(c->stream, "part_scatter", (16.0 + 16.0 * c->kw) * (double)n);
    HIP_TRY(hipGetLastError());
    OKM_TRY(sync(c));
    c->pool->put(d_seg);
    c->pool->put(d_chunks);
    return OKM_OK;
}


// The k-way merge of sorted runs (okm_merge.hip) in two passes: distinct
// keys per item, exclusive scan, then the merge writes every item's keys and
// summed counts straight into the exact-size result table (no staging, no
// compaction).  Releases bufs, d_items and d_segs.
static okm_status merge_sorted_items(okm_ctx *c, DevItem *d_items, DevSeg *d_segs, uint32_t nitems, uint64_t in_total,
                                     bool weighted, std::vector<void *> &bufs) {
    unsigned long long *n_out, *dense_off, *scan_tmp;
    OKM_TRY(pool_get(*c->pool, (size_t)nitems + 1, &n_out));
    OKM_TRY(pool_get(*c->pool, (size_t)nitems + 1, &dense_off));
    OKM_TRY(pool_get(*c->pool, scan_tmp_elems(nitems + 1), &scan_tmp));
    for (void *p : {(void *)n_out, (void *)dense_off, (void *)scan_tmp, (void *)d_items, (void *)d_segs})
        bufs.push_back(p);
    auto release = [&]() {
        for (void *p : bufs) c->pool->put(p);
        bufs.clear();
    };
    HIP_TRY(hipMemsetAsync(c->flag, 0, 2 * sizeof(unsigned long long), c->stream));
    HIP_TRY(hipMemsetAsync(n_out + nitems, 0, sizeof(unsigned long long), c->stream));
    c->timer.begin(c->stream);
    launch_merge_items(c->stream, d_items, nitems, d_segs, n_out, nullptr, nullptr, nullptr, c->flag, weighted,
                       c->wide, false);
    c->timer.end(c->stream, "merge_count", 8.0 * c->kw * (double)in_total);
    HIP_TRY(hipGetLastError());
    launch_exclusive_scan(c->stream, n_out, dense_off, nitems + 1, scan_tmp);
    HIP_TRY(hipGetLastError());
    unsigned long long *hv = c->hres + kHresCount;
    HIP_TRY(hipMemcpyAsync(&hv[0], dense_off + nitems, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&hv[1], c->flag, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    OKM_TRY(sync(c));
    if (hv[1]) {
        release();
        return fail(OKM_E_DEVICE, "merge_items invariant violated (code " + std::to_string(hv[1]) + ")");
    }
    const uint64_t nd = hv[0];
    OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(nd, 1) * c->kw, &c->res_keys));
    OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(nd, 1), &c->res_counts));
    c->timer.begin(c->stream);
    launch_merge_items(c->stream, d_items, nitems, d_segs, n_out, dense_off, c->res_keys, c->res_counts, c->flag,
                       weighted, c->wide, true);
    c->timer.end(c->stream, "merge_write",
                 (8.0 * c->kw + (weighted ? 8.0 : 0.0)) * (double)in_total + (8.0 * c->kw + 8.0) * (double)nd);
    HIP_TRY(hipGetLastError());
    OKM_TRY(sync(c));  // borrowed runs (okm_add_sorted_pairs_device) may be freed once okm_count returns
    release();
    c->n_res = nd;
    c->info.distinct = nd;
    c->counted = true;
    c->hprof.mark("merge");
    return OKM_OK;
}

// Weighted sorted runs at the memory limit (a context's own folded tables,
// C3 on one GPU): the count kernels in two passes -- each item's distinct
// keys (nothing written), an exclusive scan, then the same items counted
// again straight into the exact-size result table at their scanned offsets.
// Same memory as the k-way merge kernel (no instance-bound staging, no
// compaction) at the count kernels' speed.  Releases bufs, d_items, d_segs.
static okm_status count_sorted_two_pass(okm_ctx *c, DevItem *d_items, DevSeg *d_segs, uint32_t nitems,
                                        uint64_t in_total, std::vector<void *> &bufs) {
    bufs.push_back(d_items);
    bufs.push_back(d_segs);
    auto release = [&]() {
        for (void *p : bufs) c->pool->put(p);
        bufs.clear();
    };
    unsigned long long *n_out = nullptr, *dense_off = nullptr, *scan_tmp = nullptr;
    uint32_t *defer = nullptr;
    okm_status st = pool_get(*c->pool, (size_t)nitems + 1, &n_out);
    if (st == OKM_OK) bufs.push_back(n_out), st = pool_get(*c->pool, (size_t)nitems + 1, &dense_off);
    if (st == OKM_OK) bufs.push_back(dense_off), st = pool_get(*c->pool, scan_tmp_elems(nitems + 1), &scan_tmp);
    if (st == OKM_OK) bufs.push_back(scan_tmp), st = pool_get(*c->pool, (size_t)nitems, &defer);
    if (st != OKM_OK) {
        release();
        return st;
    }
    bufs.push_back(defer);
    const double in_bytes = (8.0 * c->kw + 8.0) * (double)in_total;
    HIP_TRY(hipMemsetAsync(c->flag, 0, 2 * sizeof(unsigned long long), c->stream));
    HIP_TRY(hipMemsetAsync(n_out + nitems, 0, sizeof(unsigned long long), c->stream));
    c->timer.begin(c->stream);
    launch_count_items(c->stream, d_items, nitems, d_segs, nullptr, nullptr, n_out, c->flag, defer, true, c->wide,
                       nullptr, nullptr, true);
    c->timer.end(c->stream, "count_distinct", in_bytes);
    HIP_TRY(hipGetLastError());
    launch_exclusive_scan(c->stream, n_out, dense_off, nitems + 1, scan_tmp);
    HIP_TRY(hipGetLastError());
    unsigned long long *hv = c->hres + kHresCount;
    HIP_TRY(hipMemcpyAsync(&hv[0], dense_off + nitems, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&hv[1], c->flag, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    OKM_TRY(sync(c));
    if (hv[1]) {
        release();
        return fail(OKM_E_DEVICE, "count_items invariant violated (code " + std::to_string(hv[1]) + ")");
    }
    const uint64_t nd = hv[0];
    st = pool_get(*c->pool, std::max<uint64_t>(nd, 1) * c->kw, &c->res_keys);
    if (st == OKM_OK) st = pool_get(*c->pool, std::max<uint64_t>(nd, 1), &c->res_counts);
    if (st != OKM_OK) {
        release();
        invalidate_result(c);
        return st;
    }
    launch_set_out_off(c->stream, d_items, nitems, dense_off);
    HIP_TRY(hipMemsetAsync(c->flag, 0, 2 * sizeof(unsigned long long), c->stream));
    c->timer.begin(c->stream);
    launch_count_items(c->stream, d_items, nitems, d_segs, c->res_keys, c->res_counts, n_out, c->flag, defer, true,
                       c->wide);
    c->timer.end(c->stream, "count_write", in_bytes + (8.0 * c->kw + 8.0) * (double)nd);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(&hv[1], c->flag, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    OKM_TRY(sync(c));  // borrowed runs (okm_add_sorted_pairs_device) may be freed once okm_count returns
    release();
    if (hv[1]) return fail(OKM_E_DEVICE, "count_items invariant violated (code " + std::to_string(hv[1]) + ")");
    c->n_res = nd;
    c->info.distinct = nd;
    c->counted = true;
    c->hprof.mark("count_two_pass");
    return OKM_OK;
}

// All runs sorted (okm_add_sorted_pairs_device, e.g. the per-rank slices an
// owner receives in the multi-GPU merge): every L1 part is split into
// key-range children by binary search in each run — no key moves — and each
// child is one multi-segment item.  *fallback: a child is still too big for
// one item (a hot key); the caller takes the partitioning path instead.
static okm_status count_sorted_plan(okm_ctx *c, bool *fallback, std::vector<uint32_t> &add_bits);

// Split bits for one L1 part from its fine-bin pair counts f[0 .. 2^sub):
// the fewest bits whose largest child stays within `target`, a child being
// a window of 2^(sub - bits) fine bins (bits <= sub) or a 2^(bits - sub)-th of
// one fine bin (keys spread evenly inside a fine bin: canonical-key density
// changes smoothly, not inside 1/2^16 of the key space).
static uint32_t hint_part_bits(const unsigned long long *f, uint32_t sub, uint64_t target) {
    const uint32_t nf = 1u << sub;
    for (uint32_t bits = 0; bits <= sub; ++bits) {
        const uint32_t w = nf >> bits;
        uint64_t worst = 0;
        for (uint32_t c0 = 0; c0 < nf; c0 += w) {
            uint64_t sum = 0;
            for (uint32_t j = 0; j < w; ++j) sum += f[c0 + j];
            worst = std::max<uint64_t>(worst, sum);
        }
        if (worst <= target) return bits;
    }
    uint64_t fmax = 0;
    for (uint32_t j = 0; j < nf; ++j) fmax = std::max<uint64_t>(fmax, f[j]);
    uint32_t more = 0;
    while (more < 20 && (fmax + (1ull << more) - 1) >> more > target) ++more;
    return sub + more;
}

// All runs sorted (see count_sorted_plan).  A child above one item's capacity
// (canonical-key density gradients inside an L1 bin, a dense run) re-plans
// with one more key bit for every part, up to 4 times, before giving up to
// the partitioning path.
static okm_status count_sorted(okm_ctx *c, bool *fallback) {
    // per part: key bits added to its split after a plan left a child above
    // one item (count_sorted_plan) -- only the parts that overflowed, e.g. an
    // owner's first and last L1 bins, which its key range covers in part
    std::vector<uint32_t> add_bits(c->nbins, 0);
    okm_status st = OKM_OK;
    for (uint32_t attempt = 0;; ++attempt) {
        const std::vector<uint32_t> before = add_bits;
        st = count_sorted_plan(c, fallback, add_bits);
        // no part can split further (its bits are at the cap: keys crowded
        // into a sliver of the key space): the partitioning path, at once
        if (st != OKM_OK || !*fallback || attempt == 6 || add_bits == before) break;
        c->hprof.mark("sorted.replan");
    }
    set_sorted_hint(c, nullptr, 0);  // one count's
    return st;
}

static okm_status count_sorted_plan(okm_ctx *c, bool *fallback, std::vector<uint32_t> &add_bits) {
    *fallback = false;
    const uint32_t R = (uint32_t)c->runs.size();
    const uint64_t item_max = count_item_capacity();
    const uint32_t capbits = count_dense_bits();
    // children by key bits: half an item on average, so the density gradient
    // inside an L1 bin of canonical keys stays below one item
#ifndef OKM_SORTED_TARGET_Q
#define OKM_SORTED_TARGET_Q 2
#endif
    const uint64_t target = item_max * OKM_SORTED_TARGET_Q / 4;
    bool weighted = false;
    for (auto &r : c->runs) weighted |= r.counts != nullptr;
    // fine bins per L1 bin of the density hint (-1: no usable hint)
    const int hint_sub = !c->sorted_hint.empty() && c->sorted_hint_bits >= c->l1_bits &&
                                 c->sorted_hint_bits <= 2 * c->k
                             ? (int)(c->sorted_hint_bits - c->l1_bits)
                             : -1;
    std::vector<DevSortedPart> parts;
    std::vector<DevSeg> rbins;
    uint32_t nitems = 0;
    uint64_t in_total = 0;
    for (uint32_t b = 0; b < c->nbins; ++b) {
        uint64_t len = 0;
        for (auto &r : c->runs) len += r.len(b);
        if (!len) continue;
        uint32_t bits = 0;
        if (len > item_max && c->shift1 > capbits) {
            if (hint_sub >= 0)
                // (the densest child is known, not guessed from the mean:
                // it may come to 3/4 of an item)
                bits = hint_part_bits(c->sorted_hint.data() + ((size_t)b << hint_sub), (uint32_t)hint_sub,
                                      item_max * 3 / 4);
            else
                while (bits < 20 && bits < c->shift1 && (len >> bits) > target) ++bits;
            bits = std::min<uint32_t>(bits, std::min<uint32_t>(20u, c->shift1));
        }
        if (bits || add_bits[b])
            bits = std::min<uint32_t>(std::min<uint32_t>(bits + add_bits[b], 20u), c->shift1);
        parts.push_back(DevSortedPart{b, bits, nitems, (uint32_t)parts.size()});
        nitems += 1u << bits;
        in_total += len;
        for (auto &r : c->runs) {
            DevSeg d{};
            d.keys = r.keys + r.off[b] * c->kw;
            d.counts = r.counts ? r.counts + r.off[b] : nullptr;
            d.len = r.len(b);
            d.shift = kSingleBin;
            d.nlocal = 1;
            rbins.push_back(d);
        }
    }
    c->info.l1_bits = c->l1_bits;
    c->info.levels = 0;
    c->info.work_items = nitems;
    if (nitems == 0) {
        c->counted = true;
        c->n_res = 0;
        c->info.distinct = 0;
        return OKM_OK;
    }
    std::vector<void *> bufs;
    DevSortedPart *d_parts;
    DevSeg *d_rbins, *d_segs;
    DevItem *d_items;
    unsigned long long *itemtot, *offs, *tmp, *flags;
    OKM_TRY(pool_get(*c->pool, parts.size(), &d_parts));
    OKM_TRY(pool_get(*c->pool, rbins.size(), &d_rbins));
    OKM_TRY(pool_get(*c->pool, (size_t)nitems * R, &d_segs));
    OKM_TRY(pool_get(*c->pool, nitems, &d_items));
    OKM_TRY(pool_get(*c->pool, (size_t)nitems + 1, &itemtot));
    OKM_TRY(pool_get(*c->pool, (size_t)nitems + 1, &offs));
    OKM_TRY(pool_get(*c->pool, scan_tmp_elems(nitems + 1), &tmp));
    OKM_TRY(pool_get(*c->pool, 2, &flags));
    unsigned long long *bounds, *part_max;
    OKM_TRY(pool_get(*c->pool, std::max<size_t>((size_t)nitems * R, 1), &bounds));
    OKM_TRY(pool_get(*c->pool, parts.size(), &part_max));
    for (void *p : {(void *)d_parts, (void *)d_rbins, (void *)itemtot, (void *)offs, (void *)tmp, (void *)flags,
                    (void *)bounds, (void *)part_max})
        bufs.push_back(p);
    OKM_TRY(h2d(c, d_parts, parts.data(), parts.size() * sizeof(DevSortedPart)));
    OKM_TRY(h2d(c, d_rbins, rbins.data(), rbins.size() * sizeof(DevSeg)));
    HIP_TRY(hipMemsetAsync(flags, 0, 2 * sizeof(unsigned long long), c->stream));
    HIP_TRY(hipMemsetAsync(part_max, 0, parts.size() * sizeof(unsigned long long), c->stream));
    HIP_TRY(hipMemsetAsync(itemtot + nitems, 0, sizeof(unsigned long long), c->stream));
    c->timer.begin(c->stream);
    launch_sorted_items(c->stream, d_parts, (uint32_t)parts.size(), nitems, d_rbins, R, c->shift1, d_items, d_segs,
                        itemtot, item_max, capbits, flags, c->wide, bounds, part_max);
    launch_exclusive_scan(c->stream, itemtot, offs, (uint64_t)nitems + 1, tmp);
    launch_set_out_off(c->stream, d_items, nitems, offs);
    c->timer.end(c->stream, "sorted_items", 0.0);
    HIP_TRY(hipGetLastError());
    unsigned long long hf[2];
    HIP_TRY(hipMemcpyAsync(hf, flags, sizeof(hf), hipMemcpyDeviceToHost, c->stream));
    std::vector<unsigned long long> pmax(parts.size());
    HIP_TRY(hipMemcpyAsync(pmax.data(), part_max, pmax.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           c->stream));
    OKM_TRY(sync(c));
    if (hf[0]) {
        // only the parts with a child above one item split further: by the
        // bits that bring their largest child below the target
        for (size_t p = 0; p < parts.size(); ++p) {
            if (pmax[p] <= item_max) continue;
            uint32_t more = 1;
            while (more < 8 && (pmax[p] >> more) > target) ++more;
            // (only while the part's bits can still grow: capped at 20 and at
            // the key bits below the L1 prefix)
            const uint32_t cap = std::min<uint32_t>(20u, c->shift1);
            if (parts[p].bits < cap) add_bits[parts[p].bin] += std::min<uint32_t>(more, cap - parts[p].bits);
        }
        if (c->hprof.on) {
            uint64_t maxlen = 0, maxbits = 0;
            for (auto &p : parts) maxbits = std::max<uint64_t>(maxbits, p.bits);
            for (uint32_t b = 0; b < c->nbins; ++b) {
                uint64_t len = 0;
                for (auto &r : c->runs) len += r.len(b);
                maxlen = std::max(maxlen, len);
            }
            fprintf(stderr, "[okm sorted] %llu children too big (max %llu); %u runs, %zu parts, %u items, "
                            "largest part %llu, max bits %llu\n",
                    (unsigned long long)hf[0], (unsigned long long)hf[1], R, parts.size(), nitems,
                    (unsigned long long)maxlen, (unsigned long long)maxbits);
            for (auto &r : c->runs)
                fprintf(stderr, "[okm sorted]   run n=%llu sorted=%d folded=%d borrowed=%d off.back=%llu\n",
                        (unsigned long long)r.n, r.sorted, r.folded, r.borrowed,
                        (unsigned long long)(r.off.empty() ? 0 : r.off.back()));
        }
        for (void *p : bufs) c->pool->put(p);
        c->pool->put(d_segs);
        c->pool->put(d_items);
        *fallback = true;
        return OKM_OK;
    }
    c->info.max_partition = hf[1];
    // k-way LDS merge of the runs' sorted slices; the hashing count kernel
    // only for more runs than one merge workgroup tracks
    // The count kernel over these multi-segment items measured faster than the
    // k-way merge kernel at every run count (C3 owner slices,
    // tools/merge8_cost.py: 2 runs 3.9 vs 4.3 ms, 4 runs 7.2 vs 13.1, 8 runs
    // 27.0 vs 53.4 ms), but it needs instance-bound slots and result (~2 x 16 B
    // per pair) where the merge kernel writes the table once at its exact size:
    // the merge kernel when that does not fit (the last folds of C3 on one GPU),
    // or on request (test hook OKM_TEST_SORTED_PATH = 1)
    // The staged path holds 16 B of staged pairs per instance and then the
    // exact table beside them; a context's own folded tables take it too when
    // that fits (C3 on one GPU, two merges of ~5 G pairs: 497 vs 559 ms per
    // job against the exact two-pass count, at the same peak memory)
    // OKM_TEST_SORTED_PATH: 1 the merge kernel, 2 the two-pass count (tests)
    const int64_t mkv = test_knob(OKM_TEST_SORTED_PATH);
    const double need = 2.0 * (8.0 * c->kw + 8.0) * (double)in_total;
    const bool tight = need > 0.9 * device_room(c);
    // weighted runs at the limit: the count kernels in two passes
    // (tools/merge8_cost.py, 8 runs: see DESIGN.md §8)
    if (weighted && (mkv == 2 || (tight && mkv != 1)))
        return count_sorted_two_pass(c, d_items, d_segs, nitems, in_total, bufs);
    const bool merge = (mkv == 1 || tight) && R <= merge_max_runs() && item_max <= merge_item_capacity();
    if (merge) return merge_sorted_items(c, d_items, d_segs, nitems, in_total, weighted, bufs);
    return count_and_compact(c, d_items, d_segs, nitems, in_total, in_total, weighted, bufs);
}

struct CountPlan {
    uint32_t twok;
    uint64_t item_max;
    uint32_t capbits;
    uint64_t target;
    uint32_t maxb;
};
static okm_status count_parts(okm_ctx *c, std::vector<DevSeg> &segtab, std::vector<Part> &parts, bool weighted,
                              const CountPlan &cp, const ResDst *dst);
static okm_status count_grouped(okm_ctx *c, std::vector<DevSeg> &segtab, std::vector<Part> &parts, bool weighted,
                                const CountPlan &cp);

static okm_status count_general(okm_ctx *c);
static okm_status count_unsorted_to_table(okm_ctx *c);

static okm_status do_count_runs(okm_ctx *c);

// Count the runs; afterwards no run may still point at caller memory: the
// caller may free a borrowed run (okm_add_sorted_pairs_device) once okm_count
// returns, so those runs are released and the result stands for the input.
static okm_status do_count(okm_ctx *c) {
    if (c->counted) return OKM_OK;
    if (c->input_lost) return fail(OKM_E_STATE, "a failed count overwrote this context's input: okm_reset it");
    // the runs are released once counted, so the count may stage into their blocks
    const bool outer = !c->may_take_runs;
    if (outer) c->took_runs = false;
    c->may_take_runs = true;
    if (outer) c->share_result = true;
    okm_status st = do_count_runs(c);
    if (st == OKM_E_NOMEM && !c->input_lost && outer) {
        // out of device memory: every table to host memory, then the key-range
        // grouped count of count_spilled (the reference's map just grows)
        // (batch runs too: with no folded table to move, the batches' L1
        // runs go to host memory and are counted group by group from there)
        bool movable = false;
        for (auto &r : c->runs) movable |= !r.host && !r.borrowed && (r.folded || !r.sorted);
        if (movable) {
            c->hprof.mark("count_nomem");
            st = spill_tables(c, INFINITY);
            if (st == OKM_OK) st = spill_runs(c);
            if (st == OKM_OK) st = do_count_runs(c);
        }
    }
    if (outer) c->may_take_runs = c->share_result = false;
    OKM_TRY(st);
    bool borrowed = false;
    for (auto &r : c->runs) borrowed |= r.borrowed;
    if ((borrowed || c->took_runs) && c->counted) {
        release_runs(c, c->runs);
        c->res_is_input = true;
    }
    return OKM_OK;
}

static okm_status count_spilled(okm_ctx *c);

// Every run sorted: split by binary search into key-range items (count_sorted),
// or -- a key range too dense for one item -- partition the runs first.
static okm_status count_all_sorted(okm_ctx *c) {
    bool fallback = false;
    OKM_TRY(count_sorted(c, &fallback));
    if (!fallback) return OKM_OK;
    for (auto &r : c->runs) {
        Run owned;
        OKM_TRY(partition_pairs(c, r.keys, r.counts, r.n, owned));
        free_run(c, r);
        r = std::move(owned);
    }
    return count_general(c);
}

static okm_status do_count_runs(okm_ctx *c) {
    invalidate_result(c);
    bool any_host = false;
    for (auto &r : c->runs) any_host |= r.host;
    if (any_host && !(c->runs.size() == 1 && c->runs[0].folded)) return count_spilled(c);
    if (c->runs.size() == 1 && c->runs[0].folded) {  // nothing added since the fold: its table is the result
        Run &r = c->runs[0];
        c->res_keys = r.keys;
        c->res_counts = r.counts;
        c->res_host = r.host;
        c->n_res = r.n;
        c->info.distinct = r.n;
        c->runs.clear();
        c->counted = true;
        c->res_is_input = true;  // the fold's table was the input: kept on the next add
        return OKM_OK;
    }
    bool any_sorted = false, all_sorted = !c->runs.empty();
    for (auto &r : c->runs) {
        any_sorted |= r.sorted;
        all_sorted &= r.sorted;
    }
    if (any_sorted && !all_sorted) {
        // sorted tables beside batches: count the batches into one more sorted
        // table, then merge all of them (no key of a sorted table moves)
        OKM_TRY(count_unsorted_to_table(c));
        if (c->runs.size() == 1 && c->runs[0].folded) return do_count(c);
        all_sorted = !c->runs.empty();
    }
    if (all_sorted && c->runs.size() == 1 && c->runs[0].counts) {
        // one sorted weighted table (e.g. the only slice a multi-GPU owner
        // holds): it already is the result — copied, since it may be borrowed
        Run &r = c->runs[0];
        const uint64_t n = r.n;
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(n, 1) * c->kw, &c->res_keys));
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(n, 1), &c->res_counts));
        c->timer.begin(c->stream);
        if (n) {
            HIP_TRY(hipMemcpyAsync(c->res_keys, r.keys, n * c->kw * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                                   c->stream));
            HIP_TRY(hipMemcpyAsync(c->res_counts, r.counts, n * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                                   c->stream));
        }
        c->timer.end(c->stream, "sorted_copy", 2.0 * (8.0 * c->kw + 8.0) * (double)n);
        OKM_TRY(sync(c));  // a borrowed run may be freed once okm_count returns
        free_run(c, r);
        c->runs.clear();
        c->n_res = n;
        c->info.distinct = n;
        c->info.levels = 0;
        c->info.work_items = 0;
        c->counted = true;
        c->res_is_input = true;  // its run is gone: the copy is kept on the next add
        return OKM_OK;
    }
    if (all_sorted) return count_all_sorted(c);
    return count_general(c);
}

// okm_count with tables in host memory (spill_tables): the batches are
// counted into one more table first -- unless batch runs lie in host memory
// too (spill_runs: no count's working set fitted beside them), in which case
// every batch run goes there and is counted group by group with the tables;
// then the key space is counted in groups of L1 bins sized to the device's
// room -- each group's slices of the device runs in place and of the host
// runs copied in, counted (and merged with the tables' slices) on the device
// -- and the groups' tables, in key order, are the result: on the device when
// it fits there, else in page-locked host memory (okm_fetch_counts / the TSV
// writer stream it; okm_result_device uploads it or fails with OKM_E_NOMEM).
static okm_status count_spilled(okm_ctx *c) {
    bool unsorted_dev = false, unsorted_host = false;
    for (auto &r : c->runs)
        if (!r.sorted) (r.host ? unsorted_host : unsorted_dev) = true;
    if (unsorted_host) {
        if (unsorted_dev) OKM_TRY(spill_runs(c));
    } else if (unsorted_dev) {
        OKM_TRY(spill_tables(c, 4.5 * uncounted_bytes(c)));
        OKM_TRY(count_unsorted_to_table(c));
    }
    const uint32_t nb = c->nbins;
    const uint64_t kw = c->kw;
    bool weighted = false;
    std::vector<uint64_t> binlen(nb, 0);
    for (auto &r : c->runs) {
        weighted |= r.counts != nullptr;
        for (uint32_t b = 0; b < nb; ++b) binlen[b] += r.len(b);
    }
    // per input pair of a group: its upload (host slices), the sorted count's
    // staged slots and exact table (count_sorted_plan: ~2 x 16 B), slack
    const double per_pair = 4.0 * (8.0 * kw + 8.0);
    const uint64_t gmax = std::max<uint64_t>(1, (uint64_t)(0.6 * device_room(c) / per_pair));
    std::vector<uint64_t> hk, hc;  // the groups' tables, in key order
    std::vector<Run> all = std::move(c->runs);
    c->runs.clear();
    okm_status st = OKM_OK;
    uint32_t groups = 0;
    for (uint32_t b0 = 0; b0 < nb && st == OKM_OK;) {
        uint32_t b1 = b0;
        uint64_t pairs = 0;
        while (b1 < nb && (b1 == b0 || pairs + binlen[b1] <= gmax)) pairs += binlen[b1++];
        uint64_t host_pairs = 0;  // (batch runs: their bins' capacities, gaps included)
        for (auto &r : all)
            if (r.host) host_pairs += r.off[b1] - r.off[b0];
        uint64_t *uk = nullptr, *uc = nullptr;
        if (host_pairs) {
            st = pool_get(*c->pool, host_pairs * kw, &uk);
            if (st == OKM_OK && weighted) st = pool_get(*c->pool, host_pairs, &uc);
        }
        std::vector<Run> grp;
        uint64_t at = 0;
        for (auto &r : all) {
            if (st != OKM_OK) break;
            const uint64_t a = r.off[b0], e = r.off[b1];
            uint64_t data = 0;  // keys in the group's bins
            for (uint32_t b = b0; b < b1; ++b) data += r.len(b);
            if (a == e || data == 0) continue;
            Run t;
            t.sorted = r.sorted;
            t.borrowed = true;
            t.n = r.sorted ? e - a : 0;
            if (r.host) {
                t.keys = uk + at * kw;
                t.counts = r.counts ? uc + at : nullptr;
                if (hipMemcpyAsync(t.keys, r.keys + a * kw, (e - a) * 8 * kw, hipMemcpyHostToDevice, c->stream) !=
                        hipSuccess ||
                    (r.counts &&
                     hipMemcpyAsync(t.counts, r.counts + a, (e - a) * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess))
                    st = fail(OKM_E_DEVICE, "count_spilled: host-to-device copy");
                at += e - a;
            } else {
                t.keys = r.keys + a * kw;
                t.counts = r.counts ? r.counts + a : nullptr;
            }
            t.off.assign(nb + 1, 0);
            for (uint32_t b = 0; b <= nb; ++b) t.off[b] = std::min(std::max(r.off[b], a), e) - a;
            if (!r.end.empty()) {  // a batch run's bins end before their sampled capacities
                t.end.assign(nb, 0);
                for (uint32_t b = 0; b < nb; ++b)
                    t.end[b] = (b >= b0 && b < b1) ? std::min(std::max(r.end[b], a), e) - a : t.off[b];
            }
            grp.push_back(std::move(t));
        }
        if (st == OKM_OK && !grp.empty()) {
            bool grp_sorted = true;
            for (auto &t : grp) grp_sorted &= t.sorted;
            c->runs = std::move(grp);
            c->counted = false;
            // (batch slices: partitioned and counted, merged with the tables' slices)
            st = grp_sorted ? count_all_sorted(c) : do_count_runs(c);
            // (borrowed slices are skipped; runs a fallback partitioned into
            // owned memory go back to the pool)
            release_runs(c, c->runs);
            if (st == OKM_OK) st = ensure_dense(c);
            if (st == OKM_OK && c->n_res) {  // the group's table off the device, appended in key order
                const size_t o = hk.size() / kw;
                hk.resize((o + c->n_res) * kw);
                hc.resize(o + c->n_res);
                if (hipMemcpyAsync(hk.data() + o * kw, c->res_keys, c->n_res * 8 * kw, hipMemcpyDeviceToHost,
                                   c->stream) != hipSuccess ||
                    hipMemcpyAsync(hc.data() + o, c->res_counts, c->n_res * 8, hipMemcpyDeviceToHost, c->stream) !=
                        hipSuccess)
                    st = fail(OKM_E_DEVICE, "count_spilled: device-to-host copy");
                if (st == OKM_OK) st = sync(c);
            }
            invalidate_result(c);
        }
        c->pool->put(uk);
        c->pool->put(uc);
        ++groups;
        b0 = b1;
    }
    c->runs = std::move(all);
    OKM_TRY(st);
    release_runs(c, c->runs);
    // the result: on the device when it fits beside what is left, else on the host
    const uint64_t nd = hc.size();
    if ((double)nd * (8.0 * kw + 8.0) <= 0.8 * device_room(c)) {
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(nd, 1) * kw, &c->res_keys));
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(nd, 1), &c->res_counts));
        if (nd) {
            HIP_TRY(hipMemcpyAsync(c->res_keys, hk.data(), nd * 8 * kw, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(hipMemcpyAsync(c->res_counts, hc.data(), nd * 8, hipMemcpyHostToDevice, c->stream));
        }
        OKM_TRY(sync(c));
    } else {
        uint64_t *pk = static_cast<uint64_t *>(host_pinned_alloc(std::max<uint64_t>(nd, 1) * 8 * kw));
        uint64_t *pc = static_cast<uint64_t *>(host_pinned_alloc(std::max<uint64_t>(nd, 1) * 8));
        if (!pk || !pc) {
            host_pinned_free(pk);
            host_pinned_free(pc);
            return fail(OKM_E_NOMEM, "count_spilled: page-locked host memory for a " + std::to_string(nd) +
                                         "-entry table");
        }
        std::memcpy(pk, hk.data(), nd * 8 * kw);
        std::memcpy(pc, hc.data(), nd * 8);
        c->res_keys = pk;
        c->res_counts = pc;
        c->res_host = true;
        c->host_bytes += nd * 8 * kw + nd * 8;
    }
    c->n_res = nd;
    c->info.distinct = nd;
    c->info.groups = groups;
    c->counted = true;
    c->res_is_input = true;  // every run is gone: the table is kept on the next add
    c->hprof.mark("count_spilled");
    return OKM_OK;
}

// Every run an L1-partitioned batch (or partitioned pairs): key-range passes
// + LDS counting + compaction.
static okm_status count_general(okm_ctx *c) {
    const uint32_t twok = 2u * c->k;
    bool weighted = false;
    for (auto &r : c->runs) weighted |= (r.counts != nullptr);
    // sort-mode items hold at most count_item_capacity() instances; items with
    // at most count_dense_bits() remaining key bits are counted by direct
    // address and may be any size (okm_count.hip)
    const uint64_t item_max = count_item_capacity();   // split parts larger than this
    const uint32_t capbits = count_dense_bits();
    // Items are sized in instances, assuming some duplication (reads cover
    // the genome several times); an item with more distinct keys than one
    // pass holds is still counted exactly, in several passes (okm_count.hip).
    const uint64_t target = item_max * 3 / 4;          // aim below it after a split (canonical-key density
                                                       // gradients and line padding must still fit)
    uint32_t maxb = log2_floor(part_max_bins(weighted, c->wide));  // bits one pass can split
    if (const int64_t e = test_knob(OKM_TEST_PART_MAX_BITS); e > 0)  // tests: small passes (fan-out, host rounds)
        maxb = std::max<uint32_t>(1, std::min<uint32_t>(maxb, (uint32_t)e));
    c->hprof.mark("pre_count");

    // initial parts: the L1 bins, each a list of per-run segments
    std::vector<DevSeg> segtab;
    std::vector<Part> parts;
    const CountPlan cp{twok, item_max, capbits, target, maxb};
    for (uint32_t b = 0; b < c->nbins; ++b) {
        Part p{(uint32_t)segtab.size(), 0, 0, b, c->l1_bits};
        for (auto &r : c->runs) {
            const uint64_t len = r.len(b);
            if (!len) continue;
            DevSeg d{};
            d.keys = r.keys + r.off[b] * c->kw;
            d.counts = r.counts ? r.counts + r.off[b] : nullptr;
            d.len = len;
            d.shift = kSingleBin;
            d.nlocal = 1;
            segtab.push_back(d);
            p.seg_count++;
            p.len += len;
        }
        if (p.len) parts.push_back(p);
    }
    c->info.l1_bits = c->l1_bits;
    c->info.l2_bits = 0;
    c->info.levels = 0;
    c->info.max_partition = 0;
    return count_grouped(c, segtab, parts, weighted, cp);
}

// Count `parts` (key-range parts over segtab, in key order) into c->res_*, or
// into *dst (then only c->n_res is set: this part's distinct keys).
static okm_status count_parts(okm_ctx *c, std::vector<DevSeg> &segtab, std::vector<Part> &parts, bool weighted,
                              const CountPlan &cp, const ResDst *dst) {
    const uint32_t twok = cp.twok, capbits = cp.capbits, maxb = cp.maxb;
    const uint64_t item_max = cp.item_max, target = cp.target;
    // bits to split part i by (0: keep).  eager (the host rounds, which only
    // see parts the device round could not bring to one item -- mostly a hot
    // key, which no split shrinks): a whole pass, so that the key bits run out
    // in ~(2k - 11) / maxb rounds rather than one bit per round
    auto plan = [&](uint32_t i, bool eager) -> uint32_t {
        const Part &p = parts[i];
        const uint32_t rem = twok - p.consumed;
        if (p.len <= item_max || rem <= capbits) return 0;
        uint32_t b = eager ? maxb : 1;
        while (b < maxb && (p.len >> b) > target) ++b;
        return std::min(b, rem);
    };

    std::vector<void *> level_bufs;
    DevItem *d_items = nullptr;
    DevSeg *d_segs = nullptr;
    uint32_t nitems = 0;
    uint64_t out_total = 0, in_total = 0;

    // Round 0 on the device: every part takes part (0 bits = gathered as one
    // bin), so the level's bins are the count work list in key order and are
    // turned into items without the offsets ever reaching the host.
    {
        std::vector<uint32_t> all, bits;
        bool any = false;
        for (uint32_t i = 0; i < parts.size(); ++i) {
            all.push_back(i);
            bits.push_back(plan(i, false));
            any |= bits.back() != 0;
        }
        if (any) {
            c->info.l2_bits = *std::max_element(bits.begin(), bits.end());
            // Fan-out: when the pass cannot bring some parts' children down to
            // one item (the bits it can split are capped), every child gets
            // 2^fan item slots and an oversized child is split once more in
            // place on the device (k_fan_split) -- no host round.  Sized for
            // twice the average child of the biggest part (canonical keys are
            // not uniform inside a part).
            FanOut fan;
            const bool fan_in_place = !weighted && !c->wide;
            {
                uint32_t fb = 0;
                for (uint32_t i = 0; i < parts.size(); ++i) {
                    const uint64_t child = 2 * (parts[i].len >> bits[i]);
                    if (!bits[i] || (parts[i].len >> bits[i]) <= target) continue;
                    uint32_t f = 1;
                    while (f < 4 && (child >> f) > target) ++f;
                    fb = std::max(fb, f);
                }
                fan.bits = fb;
                fan.target = target;
                // unweighted u64 keys: oversized children are split in place
                // (no second level array: a C3 fold's is ~45 GB); a child too
                // big for the register variant then takes a host round
                fan.split_max = fan_in_place ? fan_split_max_in_place() : fan_split_max();
            }
            c->hprof.mark("split.plan");
            uint64_t keys_in = 0;
            for (const Part &p : parts) keys_in += p.len;
            const bool try_sampled = keys_in >= (1ull << 22);
            // The level's bins become the items and are counted at once
            // (speculatively: the count kernels check make_items' flags), so
            // the first host sync of the round comes after the compaction.
            for (int attempt = 0;; ++attempt) {
                unsigned long long *flags;  // [0] children too big, [1] 1: slot overflow | 2: 64-bit counts, [2] max,
                                            // [3] / [4] fan-out jobs (small / large)
                OKM_TRY(pool_get(*c->pool, 5, &flags));
                level_bufs.push_back(flags);
                HIP_TRY(hipMemsetAsync(flags, 0, 5 * sizeof(unsigned long long), c->stream));
                Level L;
                OKM_TRY(split_launch(c, segtab, parts, all, bits, weighted, level_bufs, L,
                                     try_sampled && !attempt ? flags + 1 : nullptr));
                std::vector<DevParent> par(parts.size());
                for (uint32_t i = 0; i < parts.size(); ++i)
                    par[i] = DevParent{L.out_base[i], twok - parts[i].consumed - bits[i]};
                DevParent *d_par;
                OKM_TRY(pool_get(*c->pool, par.size(), &d_par));
                const uint32_t nslots = L.nout << fan.bits;
                const unsigned long long *d_nitems = nullptr;  // fan-out: items kept, on the device
                OKM_TRY(pool_get(*c->pool, nslots, &d_items));
                OKM_TRY(pool_get(*c->pool, nslots, &d_segs));
                level_bufs.push_back(d_par);
                if (fan.bits) {
                    OKM_TRY(pool_get(*c->pool, L.nout, &fan.jobs));
                    level_bufs.push_back(fan.jobs);
                }
                OKM_TRY(h2d(c, d_par, par.data(), par.size() * sizeof(DevParent)));
                // items stage their runs densely: slots = the pass's keys, not the
                // level's sampled capacity (~1.5x the keys at C2)
                unsigned long long *doff, *dtmp;
                OKM_TRY(pool_get(*c->pool, (size_t)L.nout + 1, &doff));
                OKM_TRY(pool_get(*c->pool, scan_tmp_elems(L.nout + 1), &dtmp));
                level_bufs.push_back(doff);
                level_bufs.push_back(dtmp);
                launch_child_offsets(c->stream, L.d_offs, L.d_ends, L.nout, doff, dtmp);
                launch_make_items(c->stream, L.d_offs, L.d_ends, L.nout, d_par, (uint32_t)par.size(), L.lk, L.lc,
                                  d_items, d_segs, item_max, capbits, flags, c->kw, fan, doff);
                HIP_TRY(hipGetLastError());
                if (fan.bits) {  // oversized children split into a second level array (same offsets), or in place
                    uint64_t *fk = L.lk, *fc = nullptr;
                    if (!fan_in_place) {
                        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(L.padded, 1) * c->kw, &fk));
                        level_bufs.push_back(fk);
                    }
                    if (L.lc) {
                        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(L.padded, 1), &fc));
                        level_bufs.push_back(fc);
                    }
                    c->timer.begin(c->stream);
                    launch_fan_split(c->stream, fan.jobs, L.nout, flags, L.lk, L.lc, fk, fc, d_items, d_segs, item_max,
                                     capbits, flags, c->wide);
                    c->timer.end(c->stream, "fan_split", 0.0);
                    HIP_TRY(hipGetLastError());
                    // drop the empty slots, so the count kernels deal real items only
                    DevItem *dense_items;
                    unsigned long long *iflags, *ipos, *itmp;
                    OKM_TRY(pool_get(*c->pool, nslots, &dense_items));
                    OKM_TRY(pool_get(*c->pool, (size_t)nslots + 1, &iflags));
                    OKM_TRY(pool_get(*c->pool, (size_t)nslots + 1, &ipos));
                    OKM_TRY(pool_get(*c->pool, scan_tmp_elems(nslots + 1), &itmp));
                    for (void *p : {(void *)d_items, (void *)iflags, (void *)ipos, (void *)itmp}) level_bufs.push_back(p);
                    launch_item_compact(c->stream, d_items, nslots, dense_items, iflags, ipos, itmp);
                    HIP_TRY(hipGetLastError());
                    d_items = dense_items;
                    d_nitems = ipos + nslots;
                }
                c->hprof.mark("split.round_launch");
                c->info.work_items = nslots;
                unsigned long long hf[3] = {0, 0, 0};
                bool aborted = false;
                // every item lies in the level arrays: the runs are not read again
                // every item is one child in a level array (lk, or fk after the
                // fan-out): its sorted run is staged in place, over its keys
                OKM_TRY(count_and_compact(c, d_items, d_segs, nslots, L.total, L.total, weighted, level_bufs, flags,
                                          hf, &aborted, d_nitems, dst, true, true));
                if (!aborted) {
                    c->info.max_partition = hf[2];
                    return OKM_OK;
                }
                c->pool->put(d_items);
                c->pool->put(d_segs);
                d_items = nullptr;
                d_segs = nullptr;
                if (hf[1] & 1) {  // a child outgrew its sampled slot: redo the pass exactly
                    c->info.levels -= 1;
                    continue;
                }
                if (hf[0]) {  // children still too big for one item: host rounds below
                    OKM_TRY(split_children_host(c, L, segtab, parts, all, bits));
                    break;
                }
                weighted = true;  // a child of >= 2^32 instances: 64-bit counting
                c->info.levels -= 1;
            }
        }
    }

    // Further rounds on the host view (only when a child is still too big:
    // skewed or adversarial key distributions).
    for (int round = 1; round < 64; ++round) {
        std::vector<uint32_t> todo, bits;
        for (uint32_t i = 0; i < parts.size(); ++i) {
            const uint32_t b = plan(i, true);
            if (!b) continue;
            todo.push_back(i);
            bits.push_back(b);
        }
        if (todo.empty()) break;
        Level L;
        OKM_TRY(split_launch(c, segtab, parts, todo, bits, weighted, level_bufs, L));
        OKM_TRY(split_children_host(c, L, segtab, parts, todo, bits));
    }

    // items on the host view: the parts themselves
    std::vector<DevItem> items;
    nitems = (uint32_t)parts.size();
    items.resize(nitems);
    bool one_seg = true;  // every part one child in a level array: its run is staged in place
    for (uint32_t i = 0; i < nitems; ++i) {
        one_seg &= parts[i].seg_count == 1;
        // distinct <= instances, and <= 2^remaining-bits
        const uint32_t rem = twok - parts[i].consumed;
        const uint64_t bound = rem >= 63 ? parts[i].len : std::min<uint64_t>(parts[i].len, 1ull << rem);
        const DevSeg &s0 = segtab[parts[i].seg_begin];
        items[i] = DevItem{parts[i].seg_begin, parts[i].seg_count, out_total, rem, 0, parts[i].len, s0.keys, s0.counts};
        out_total += bound;
        in_total += parts[i].len;
        c->info.max_partition = std::max(c->info.max_partition, parts[i].len);
        if (parts[i].len >= (1ull << 32)) weighted = true;  // u32 LDS counts could overflow
    }
    c->info.work_items = nitems;
    if (nitems == 0) {
        for (void *p : level_bufs) c->pool->put(p);
        c->counted = true;
        c->n_res = 0;
        c->info.distinct = 0;
        return OKM_OK;
    }
    OKM_TRY(pool_get(*c->pool, segtab.size(), &d_segs));
    OKM_TRY(pool_get(*c->pool, nitems, &d_items));
    OKM_TRY(h2d(c, d_segs, segtab.data(), segtab.size() * sizeof(DevSeg)));
    OKM_TRY(h2d(c, d_items, items.data(), nitems * sizeof(DevItem)));
    c->hprof.mark("items.build");
    // (parts that never took part in a split round keep their run segments:
    // those are staged in a separate array)
    return count_and_compact(c, d_items, d_segs, nitems, out_total, in_total, weighted, level_bufs, nullptr, nullptr,
                             nullptr, nullptr, dst, false, one_seg && !level_bufs.empty());
}

// Memory-bounded counting.  The working set of a count (level array, fan-out
// copy, per-item staging: ~4 key words + a count per instance) is bounded by
// counting the L1 parts in key-range groups, one after the other; the result
// is the groups' tables in order.  Either every group compacts straight into
// one table sized by the instance bound (when it fits beside the runs), or
// each group gets an exact table and the tables are joined at the end.
// Needed from ~4 G instances on one GPU (e.g. BASELINE configs[3], k=63 over
// 5.4 Gbases: 85 GB of L1 runs + 127 GB of result); OKM_TEST_GROUP_KEYS /
// OKM_TEST_GROUP_EXACT (0: bound table, 1: exact tables) force it in tests.
static okm_status count_grouped(okm_ctx *c, std::vector<DevSeg> &segtab, std::vector<Part> &parts, bool weighted,
                                const CountPlan &cp) {
    uint64_t total = 0;
    for (const Part &p : parts) total += p.len;
    // per instance: level + fan-out copy (+ slack) + staged counts (u32
    // unweighted) (+ weights of both levels); the keys' runs are staged in
    // place, over the level array
    const double ws_key = 8.0 * c->kw * 3 + (weighted ? 8.0 : 4.0) + (weighted ? 16.0 : 0.0);
    const double res_key = 8.0 * c->kw + 8.0;     // result entry (instance bound)
    // one group: the exact result is allocated after the level arrays went
    // back to the pool, beside the staged runs only (count_and_compact)
    const double one_key = std::max(ws_key, 8.0 * c->kw + (weighted ? 8.0 : 4.0) + res_key);
    // 3/4 of what is free: sampled capacities, line padding and the pool's size
    // classes make a pass hold more than its keys
    const double room = device_room(c);
    const double avail = 0.75 * room;
    uint64_t group_keys = total;
    int mode = 0;  // 0: one group (no grouping)
    // The table's keys can be written over the batch's own L1 run (below):
    // one batch run, unweighted, and no run needed after this count
    // (may_take_runs).  Then only the counts are instance-bound new memory.
    bool over_ok = false;
    if (!weighted && c->may_take_runs && c->runs.size() == 1) {
        const Run &r = c->runs[0];
        over_ok = !r.sorted && !r.folded && !r.host && !r.borrowed && !r.counts && r.keys &&
                  c->pool->size_of(r.keys) >= std::max<uint64_t>(total, 1) * 8 * c->kw;
    }
    if (test_knob(OKM_TEST_GROUP_OVER) == 0) over_ok = false;
    bool use_over = false;
    const int64_t ge = test_knob(OKM_TEST_GROUP_KEYS);
    if (ge > 0) {
        group_keys = (uint64_t)ge;
        mode = test_knob(OKM_TEST_GROUP_EXACT) == 1 ? 2 : 1;
    } else if ((double)total * one_key > avail) {
        // beside a bound-sized table: the 3/4 margin over both (room_a), or —
        // the last resort below, when per-group tables could not be joined —
        // over the groups' working sets only (room_l: the table's size is exact)
        const double room_a = avail - (double)total * res_key;
        const double room_l = 0.75 * (std::max(room, 0.0) - (double)total * res_key);
        // a bound-sized table is only worth it when it is a small share of HBM
        // (dense inputs such as k=63 long reads); with duplicated keys (a fold
        // of covered reads) exact per-group tables hold a fraction of it
        // ... and when the exact tables could not be joined anyway (their
        // worst case is the bound itself, twice over while joining)
        // (then even at up to 256 groups: slower, but the join is what fails)
        const double bound = (double)total * res_key;
        const bool a_fits = room_a >= (double)total * ws_key / 64.0;
        const bool a_last = 2.0 * bound > avail && room_l >= (double)total * ws_key / 256.0;
        // the keys over the run (below): the bound-sized table is its counts
        // only, so groups get the key array's room too.  Groups hold 52 B of
        // working set per instance at k > 32 and larger ones gain little
        // (C4, 5.36 Gbases: 18 groups 188 ms at 228.5 GB with a separate key
        // array; over the run 5 groups of <= 2^30 instances 180-186 ms at
        // 175 GB, 4 of <= 1.4 G 179-183 ms at 185 GB, 3 of <= 1.8 G 177-180 ms
        // at 203 GB: profiles/r06_c4_over.txt, r06_c4_groups.txt)
        constexpr uint64_t kGroupKeysMax = 1400000000ull;
        const double room_o = avail - (double)total * 8.0;
        const bool o_fits = over_ok && room_o >= (double)total * ws_key / 64.0;
        if (o_fits) {
            mode = 1;
            use_over = true;
            group_keys = std::min<uint64_t>((uint64_t)(room_o / ws_key), kGroupKeysMax);
        } else if (a_fits && (bound <= 0.5 * avail || 2.0 * bound > avail)) {
            mode = 1;
            group_keys = (uint64_t)(room_a / ws_key);
        } else if (a_last) {
            mode = 1;
            group_keys = (uint64_t)(room_l / ws_key);
        } else {
            mode = 2;  // a bound-sized table per group, plus the finished groups' exact tables
            group_keys = (uint64_t)(avail * 0.6 / (ws_key + res_key));
        }
        group_keys = std::max<uint64_t>(group_keys, 1);
    }
    // wide keys that fit beside an instance-bound table count straight into
    // it as one group (the direct count: no staged runs, no compaction pass),
    // and the table then gives its tail back
    const bool direct_one = c->wide && mode == 0 && (double)total * (ws_key + res_key) <= avail;
    if (direct_one) {
        mode = 1;
        use_over = over_ok;  // (one group: its keys over its own run, read by then)
    }
    if (mode == 0 || (group_keys >= total && !direct_one)) return count_parts(c, segtab, parts, weighted, cp, nullptr);
    // The table's keys over the batch's own L1 run: with one batch run, the
    // groups in key order and the runs no longer needed after this count
    // (may_take_runs), group g's keys -- at most as many as the instances of
    // groups 0..g -- end before group g + 1's run starts, and group g's own
    // run was read by its partition pass before its count writes.  The
    // instance-bound key array (16 B per instance at k > 32: 85 GB at C4)
    // is then never allocated.
    // forced by the test hook too (knob group_over), so the small test
    // inputs take the path
    if (mode == 1 && over_ok && test_knob(OKM_TEST_GROUP_OVER) == 1) use_over = true;
    Run *over = use_over ? &c->runs[0] : nullptr;
    // every group reads the runs: none may hold a group's staged keys
    struct Keep {
        okm_ctx *c;
        bool saved, shared;
        ~Keep() {
            c->may_take_runs = saved;
            c->share_result = shared;
        }
    } keep{c, c->may_take_runs, c->share_result};
    c->may_take_runs = c->share_result = false;

    ResDst d{nullptr, nullptr, 0};
    struct Tab {
        uint64_t *keys, *counts, n;
    };
    std::vector<Tab> tabs;
    // every table block goes back to the pool on any error path (a stranded
    // block would make the caller's retry run out of memory sooner)
    struct Guard {
        okm_ctx *c;
        ResDst *d;
        std::vector<Tab> *tabs;
        bool armed = true;
        bool keys_are_run = false;  // (the run's block: it stays with the run)
        ~Guard() {
            if (!armed) return;
            if (!keys_are_run) c->pool->put(d->keys);
            c->pool->put(d->counts);
            for (auto &t : *tabs) {
                c->pool->put(t.keys);
                c->pool->put(t.counts);
            }
        }
    } guard{c, &d, &tabs};
    if (mode == 1) {
        if (over) {
            d.keys = over->keys;
            guard.keys_are_run = true;
        } else {
            OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(total, 1) * c->kw, &d.keys));
        }
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(total, 1), &d.counts));
    }
    // once a group wrote over the run, a failure leaves no input to count again
    struct Lost {
        okm_ctx *c;
        bool on = false;
        ~Lost() {
            if (on) c->input_lost = true;
        }
    } lost{c};
    const okm_engine_info info0 = c->info;
    okm_engine_info agg = info0;
    agg.work_items = 0;
    agg.max_partition = 0;
    uint32_t ngroups = 0;
    std::vector<size_t> cuts{0};  // group g: parts [cuts[g], cuts[g + 1])
    for (size_t g0 = 0; g0 < parts.size();) {
        size_t g1 = g0;
        uint64_t keys = 0;
        while (g1 < parts.size() && (g1 == g0 || keys + parts[g1].len <= group_keys)) keys += parts[g1++].len;
        cuts.push_back(g1);
        g0 = g1;
    }
    // Mode 1, pipelined: every group's kernels queue behind the previous
    // group's with no host sync in between (the table's next entry advances
    // on the device); one sync at the end reads every group's words.  A group
    // whose speculative count was abandoned (a sampled slot overflowed, a
    // child too big for one item) left nothing in the table and moved nothing,
    // and poisoned the device-side base, so no later group wrote either: then
    // the groups from the first abandoned one on are counted again, one sync
    // each, from the base the groups before it reached (their entries are in
    // place, and the runs of the groups from there on are intact).
    struct Slots {
        okm_ctx *c;
        unsigned long long *p = nullptr, *d_base = nullptr;
        ~Slots() {
            host_pinned_free(p);
            c->pool->put(d_base);
        }
    } slots{c};
    unsigned long long *&d_base = slots.d_base;
    const size_t G = cuts.size() - 1;
    bool pipelined = mode == 1 && G > 1;
    if (pipelined) {
        slots.p = static_cast<unsigned long long *>(host_pinned_alloc(G * 8 * sizeof(unsigned long long)));
        pipelined = slots.p && pool_get(*c->pool, 1, &d_base) == OKM_OK;
        if (pipelined) HIP_TRY(hipMemsetAsync(d_base, 0, sizeof(unsigned long long), c->stream));
    }
    size_t g_from = 0;  // the first group of this pass
    for (int pass = 0; pass < 2; ++pass) {
        bool redo = false;
        if (pass == 0) {
            d.off = 0;
            agg = info0;
            agg.work_items = 0;
            agg.max_partition = 0;
            ngroups = 0;
        }
        d.d_base = pipelined ? d_base : nullptr;
        for (size_t g = g_from; g < G; ++g) {
            std::vector<Part> sub(parts.begin() + cuts[g], parts.begin() + cuts[g + 1]);
            c->info.levels = 0;
            c->info.l2_bits = 0;
            if (pipelined) d.hslot = slots.p + 8 * g;
            OKM_TRY(count_parts(c, segtab, sub, weighted, cp, mode == 1 ? &d : nullptr));
            lost.on = over != nullptr;  // (this group's keys are written, or queued)
            agg.levels = std::max(agg.levels, c->info.levels);
            agg.l2_bits = std::max(agg.l2_bits, c->info.l2_bits);
            agg.work_items += c->info.work_items;
            agg.max_partition = std::max(agg.max_partition, c->info.max_partition);
            if (mode == 1) {
                d.off += c->n_res;
            } else {
            // keep the group's table at its exact size: the bound-sized one goes
            // back to the pool and serves the next group
                OKM_TRY(ensure_dense(c));
                OKM_TRY(shrink_table(c, &c->res_keys, &c->res_counts, c->n_res, 1.0));
                tabs.push_back(Tab{c->res_keys, c->res_counts, c->n_res});
                c->res_keys = c->res_counts = nullptr;
            }
            ++ngroups;
        }
        if (!pipelined) break;
        unsigned long long base = 0;
        HIP_TRY(hipMemcpyAsync(&c->hres[kHresCount], d_base, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                               c->stream));
        OKM_TRY(sync(c));
        base = c->hres[kHresCount];
        size_t first_bad = G;
        for (size_t g = 0; g < G; ++g) {
            const unsigned long long *hs = slots.p + 8 * g;
            if (hs[1]) return fail(OKM_E_DEVICE, "count_items invariant violated (code " + std::to_string(hs[1]) + ")");
            if ((hs[2] | hs[3]) != 0 && first_bad == G) first_bad = g;
            agg.max_partition = std::max<uint64_t>(agg.max_partition, hs[4]);
        }
        redo = first_bad < G;
        if (redo != ((base & kBasePoison) != 0))
            return fail(OKM_E_DEVICE, "pipelined key-range groups: table base and group flags disagree");
        d.off = base & ~kBasePoison;
        if (!redo) break;
        c->hprof.mark("groups.redo");
        pipelined = false;  // the groups from the first abandoned one, one sync each
        g_from = first_bad;
        ngroups = (uint32_t)first_bad;
    }
    lost.on = false;
    uint64_t nd = d.off;
    if (mode == 1) {
        guard.armed = false;
        c->res_keys = d.keys;
        c->res_counts = d.counts;
        if (over) {  // the run's block is the table's now; the run is gone (released after the count)
            over->keys = nullptr;
            c->took_runs = true;
            OKM_TRY(shrink_table(c, &c->res_keys, &c->res_counts, nd, 1.0));
        }
        if (direct_one) {
            OKM_TRY(shrink_table(c, &c->res_keys, &c->res_counts, nd, 1.0));
            ngroups = 0;  // (one pass: no grouping)
        }
    } else {
        nd = 0;
        for (auto &t : tabs) nd += t.n;
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(nd, 1) * c->kw, &c->res_keys));
        OKM_TRY(pool_get(*c->pool, std::max<uint64_t>(nd, 1), &c->res_counts));
        uint64_t o = 0;
        for (auto &t : tabs) {
            if (t.n) {
                HIP_TRY(hipMemcpyAsync(c->res_keys + o * c->kw, t.keys, t.n * 8 * c->kw, hipMemcpyDeviceToDevice,
                                       c->stream));
                HIP_TRY(hipMemcpyAsync(c->res_counts + o, t.counts, t.n * 8, hipMemcpyDeviceToDevice, c->stream));
            }
            o += t.n;
        }
        OKM_TRY(sync(c));  // the guard returns the groups' tables (and only them: d is unused in mode 2)
    }
    agg.distinct = nd;
    agg.groups = ngroups;
    c->info = agg;
    c->n_res = nd;
    c->counted = true;
    return OKM_OK;
}

static bool device_ok(int device, std::string *why) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        *why = "no HIP device visible (the engine has no CPU fallback)";
        return false;
    }
    if (device < 0 || device >= n) {
        *why = "device ordinal " + std::to_string(device) + " out of range (" + std::to_string(n) + " visible)";
        return false;
    }
    return true;
}

}  // namespace okm

// l1_batch, once more after making room when the device is out of memory:
// what is pending is folded into a table and the tables go to host memory.
// l1_batch, and when its L1 run does not fit: the pending batches folded
// into a table (or, when even that count does not fit, moved to host memory),
// the tables moved to host memory, and the batch again; when the batch alone
// still does not fit (a single batch past the device budget), its two halves
// one after the other -- the first [0, q + k - 1) holds every window that
// starts before the 16-B aligned q, the second [q, n) every one from q on, so
// no window is lost or counted twice (a window needs k bytes: one starting
// at or past q ends past the first half) -- down to 1 MiB pieces.  The
// reference's map grows in host RAM (count.rs:48); this never fails for lack
// of device memory while host memory lasts.
static okm_status l1_batch_or_spill(okm_ctx *c, const uint8_t *d_seq, uint64_t n) {
    okm_status st = l1_batch(c, d_seq, n);
    if (st != OKM_E_NOMEM || c->input_lost) return st;
    bool pending = false;
    for (auto &r : c->runs) pending |= !r.sorted && !r.host;
    if (pending) {
        st = fold(c);
        if (st == OKM_E_NOMEM && !c->input_lost) st = spill_runs(c);
        OKM_TRY(st);
    }
    OKM_TRY(spill_tables(c, INFINITY));
    st = l1_batch(c, d_seq, n);
    if (st != OKM_E_NOMEM || c->input_lost || n < (uint64_t(1) << 20)) return st;
    OKM_TRY(spill_runs(c));
    c->hprof.mark("batch_split");
    const uint64_t q = (n / 2) & ~uint64_t(15);
    OKM_TRY(l1_batch_or_spill(c, d_seq, std::min<uint64_t>(n, q + c->k - 1)));
    return l1_batch_or_spill(c, d_seq + q, n - q);
}

namespace okm {
// okm_merge_owned at one rank: the owner's key range is the whole key space
// and its only slice the local table, so the owner takes that table as it
// stands (dense, or still the items' sorted runs) instead of copying it
// (do_count_runs' copy of a single borrowed sorted run).  The two contexts
// swap their device pools -- one device, and every pool is one arena of
// that device -- so the table stays where it is and is later returned to
// the pool that holds it; the local context is left reset (its input runs
// are released first); *adopted says whether it happened.
okm_status adopt_result(okm_ctx *owner, okm_ctx *local, bool *adopted) {
    *adopted = false;
    if (owner == local || owner->device != local->device || owner->k != local->k || owner->mode != local->mode ||
        owner->wide != local->wide)
        return OKM_OK;
    HIP_TRY(hipSetDevice(local->device));
    OKM_TRY(do_count(local));
    if (local->input_lost) return OKM_OK;
    OKM_TRY(okm_reset(owner));  // (synchronises the owner's stream)
    OKM_TRY(sync(local));
    // the counted input is no longer needed (the local is left reset, and no
    // result ever points into a run: a folded table that became the result
    // left the run list): its memory goes back before the pools swap
    release_runs(local, local->runs);
    std::swap(owner->pool, local->pool);
    owner->pend = std::move(local->pend);
    local->pend = okm_ctx::Pending{};
    owner->res_keys = local->res_keys;
    owner->res_counts = local->res_counts;
    owner->res_host = local->res_host;
    owner->n_res = local->n_res;
    owner->counted = true;
    owner->res_is_input = true;  // the table stands for the owner's input (kept on its next add)
    owner->info = local->info;
    if (local->res_host) {
        const uint64_t b = local->n_res * (8 * local->kw + 8);
        owner->host_bytes += b;
        local->host_bytes -= std::min(local->host_bytes, b);
    }
    local->res_keys = local->res_counts = nullptr;
    local->res_host = false;
    local->n_res = 0;
    local->counted = false;
    local->res_is_input = false;
    OKM_TRY(okm_reset(local));
    owner->hprof.mark("adopt_result");
    *adopted = true;
    return OKM_OK;
}

okm_status result_view(okm_ctx *c, const uint64_t **keys, const uint64_t **counts, uint64_t *n, bool *on_host) {
    OKM_TRY(okm_count(c, nullptr));
    OKM_TRY(ensure_dense(c));
    *keys = c->res_keys;
    *counts = c->res_counts;
    *n = c->n_res;
    *on_host = c->res_host;
    return OKM_OK;
}
}  // namespace okm

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int okm_abi_version(void) { return OKM_ABI_VERSION; }

const char *okm_status_string(okm_status s) {
    switch (s) {
    case OKM_OK: return "ok";
    case OKM_E_INVALID_K: return "invalid k";
    case OKM_E_NOMEM: return "out of memory";
    case OKM_E_DEVICE: return "device error";
    case OKM_E_COMM: return "communication error";
    case OKM_E_ARG: return "invalid argument";
    case OKM_E_OVERFLOW: return "capacity exceeded";
    case OKM_E_IO: return "i/o error";
    case OKM_E_PARSE: return "parse error";
    case OKM_E_RECORD: return "record error";
    case OKM_E_STATE: return "invalid state";
    case OKM_E_FORMAT: return "format error";
    }
    return "unknown";
}

const char *okm_last_error(void) { return okm::g_last_error.c_str(); }

int okm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

const char *okm_device_arch(int device) {
    static thread_local char buf[64];
    buf[0] = 0;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) {
        (void)hipGetLastError();
        return buf;
    }
    std::snprintf(buf, sizeof(buf), "%s", p.gcnArchName);
    char *colon = std::strchr(buf, ':');
    if (colon) *colon = 0;
    return buf;
}

okm_status okm_create(okm_ctx **out, uint8_t k, okm_mode mode, int device, uint64_t distinct_hint) {
    if (!out) return fail(OKM_E_ARG, "okm_create: out is NULL");
    *out = nullptr;
    const bool wide_ok = (mode & OKM_MODE_WIDE) != 0;  // opt-in two-u64 extension (k <= 64)
    mode = (okm_mode)(mode & ~OKM_MODE_WIDE);
    if (k == 0 || k > 32) {
        if (!wide_ok || k == 0 || k > 64)
            return fail(OKM_E_INVALID_K, "Invalid K-mer size: " + std::to_string(k) + ". Must be between 1 and " +
                                             (wide_ok ? "64." : "32."));
    }
    if (mode != OKM_MODE_COUNT && mode != OKM_MODE_SET) return fail(OKM_E_ARG, "okm_create: bad mode");
    std::string why;
    if (!device_ok(device, &why)) return fail(OKM_E_DEVICE, why);
    HIP_TRY(hipSetDevice(device));
    okm_ctx *c = new okm_ctx();
    c->device = device;
    c->k = k;
    c->mode = mode;
    c->wide = k > 32;
    c->kw = c->wide ? 2 : 1;
    c->l1_fold = !c->wide && distinct_hint >= (1ull << 30);  // a table this big is built by folding
    set_l1_geometry(c);
    {
        // fold threshold: OKM_FOLD_BYTES, else a ninth of the device budget (10 %
        // of HBM at the default 0.9; the count of the folded runs needs ~4.5x their
        // bytes of working set; C3 on one GPU: 8 % 596 ms, 10 % 569 ms; 12 % needs
        // key-range groups: 2.5 s)
        const char *fe = getenv("OKM_FOLD_BYTES");
        const double fv = fe && *fe ? parse_bytes(fe) : -1.0;
        c->fold_bytes = fv >= 0 ? (uint64_t)fv : (uint64_t)(hbm_budget(device) / 9.0);
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->flag, 2 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->l1cap, (2 * (size_t)extract_max_bins(c->wide) + 2) * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->curpad, (size_t)extract_max_bins(c->wide) * kL1CurStride * sizeof(unsigned long long)) !=
            hipSuccess ||
        hipHostMalloc(&c->hpin, kHpinBytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&c->hres, kHresWords * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        delete c;
        return fail(OKM_E_DEVICE, "okm_create: stream/alloc failed");
    }
    c->pool->attach(device);
    *out = c;
    return OKM_OK;
}

void okm_destroy(okm_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->timer.destroy();
    invalidate_result(c);  // host tables are freed here; device memory goes with the arena
    release_runs(c, c->runs);
    c->pool->detach();
    c->pool->release_all();
    if (c->HC) (void)hipFree(c->HC);
    if (c->Hg) (void)hipFree(c->Hg);
    if (c->cursor) (void)hipFree(c->cursor);
    if (c->flag) (void)hipFree(c->flag);
    if (c->l1cap) (void)hipFree(c->l1cap);
    if (c->curpad) (void)hipFree(c->curpad);
    if (c->hpin) (void)hipHostFree(c->hpin);
    if (c->hres) (void)hipHostFree(c->hres);
    if (c->staging) (void)hipFree(c->staging);
    if (c->pinned) (void)hipHostFree(c->pinned);
    (void)hipStreamDestroy(c->stream);
    delete c;
}


okm_status okm_trim(okm_ctx *c) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    OKM_TRY(sync(c));
    c->pool->trim();
    return OKM_OK;
}

okm_status okm_reset(okm_ctx *c) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    OKM_TRY(sync(c));
    invalidate_result(c);
    release_runs(c, c->runs);
    c->info = okm_engine_info{};
    c->spills = 0;
    c->folds = 0;
    c->pool->reset_peak();
    c->input_lost = false;
    set_sorted_hint(c, nullptr, 0);
    c->hprof.mark("reset");
    return OKM_OK;
}

static bool is_ws(uint8_t ch) { return ch == ' ' || ch == '\t' || ch == '\r' || ch == '\n'; }

okm_status okm_add_batch(okm_ctx *c, const uint8_t *seq, const uint64_t *offsets, uint64_t n_records,
                         int normalized) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    if (n_records == 0) return OKM_OK;
    if (!offsets) return fail(OKM_E_ARG, "okm_add_batch: null offsets");
    const uint64_t total = offsets[n_records] - offsets[0];
    if (total == 0) return OKM_OK;  // only empty records (e.g. header-only FASTA)
    if (!seq) return fail(OKM_E_ARG, "okm_add_batch: null seq");
    HIP_TRY(hipSetDevice(c->device));
    OKM_TRY(sync(c));  // pinned buffer reuse
    OKM_TRY(ensure_pinned(c, total + n_records + 16));
    // device batch layout: whitespace-free records + separator
    uint8_t *dst = c->pinned;
    uint64_t o = 0;
    for (uint64_t r = 0; r < n_records; ++r) {
        const uint8_t *s = seq + offsets[r];
        const uint64_t len = offsets[r + 1] - offsets[r];
        if (normalized) {
            std::memcpy(dst + o, s, len);
            o += len;
        } else {
            for (uint64_t i = 0; i < len; ++i)
                if (!is_ws(s[i])) dst[o++] = s[i];
        }
        dst[o++] = OKM_RECORD_SEPARATOR;
    }
    OKM_TRY(ensure_staging(c, o));
    HIP_TRY(hipMemcpyAsync(c->staging, dst, o, hipMemcpyHostToDevice, c->stream));
    OKM_TRY(before_add(c));
    return l1_batch_or_spill(c, c->staging, o);
}

okm_status okm_add_batch_device(okm_ctx *c, const uint8_t *d_seq, uint64_t n_bytes) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    if (n_bytes == 0) return OKM_OK;
    if (!d_seq) return fail(OKM_E_ARG, "okm_add_batch_device: null pointer");
    HIP_TRY(hipSetDevice(c->device));
    OKM_TRY(before_add(c));
    if ((reinterpret_cast<uintptr_t>(d_seq) & 15u) != 0) {
        OKM_TRY(ensure_staging(c, n_bytes));
        HIP_TRY(hipMemcpyAsync(c->staging, d_seq, n_bytes, hipMemcpyDeviceToDevice, c->stream));
        return l1_batch_or_spill(c, c->staging, n_bytes);
    }
    return l1_batch_or_spill(c, d_seq, n_bytes);
}

okm_status okm_add_pairs_device(okm_ctx *c, const uint64_t *d_keys, const uint64_t *d_counts, uint64_t n) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    if (n == 0) return OKM_OK;
    if (!d_keys) return fail(OKM_E_ARG, "okm_add_pairs_device: null keys");
    HIP_TRY(hipSetDevice(c->device));
    OKM_TRY(before_add(c));
    Run run;
    OKM_TRY(partition_pairs(c, d_keys, d_counts, n, run));
    c->runs.push_back(std::move(run));
    return OKM_OK;
}

okm_status okm_add_sorted_pairs_device(okm_ctx *c, const uint64_t *d_keys, const uint64_t *d_counts, uint64_t n) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    if (n == 0) return OKM_OK;
    if (!d_keys) return fail(OKM_E_ARG, "okm_add_sorted_pairs_device: null keys");
    HIP_TRY(hipSetDevice(c->device));
    OKM_TRY(before_add(c));
    Run run;
    run.keys = const_cast<uint64_t *>(d_keys);
    run.counts = const_cast<uint64_t *>(d_counts);
    run.n = n;
    run.sorted = true;
    run.borrowed = true;
    // L1 bin boundaries by binary search: the run stays where it is
    OKM_TRY(sorted_run_bins(c, run));
    c->runs.push_back(std::move(run));
    return OKM_OK;
}

okm_status okm_add_pairs(okm_ctx *c, const uint64_t *keys, const uint64_t *counts, uint64_t n) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    if (n == 0) return OKM_OK;
    if (!keys) return fail(OKM_E_ARG, "okm_add_pairs: null keys");
    HIP_TRY(hipSetDevice(c->device));
    uint64_t *dk = nullptr, *dc = nullptr;
    OKM_TRY(pool_get(*c->pool, n * c->kw, &dk));
    if (counts) OKM_TRY(pool_get(*c->pool, n, &dc));
    HIP_TRY(hipMemcpyAsync(dk, keys, n * 8 * c->kw, hipMemcpyHostToDevice, c->stream));
    if (counts) HIP_TRY(hipMemcpyAsync(dc, counts, n * 8, hipMemcpyHostToDevice, c->stream));
    okm_status s = okm_add_pairs_device(c, dk, dc, n);
    c->pool->put(dk);
    c->pool->put(dc);
    return s;
}

okm_status okm_count(okm_ctx *c, uint64_t *n_distinct) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    OKM_TRY(do_count(c));
    if (n_distinct) *n_distinct = c->n_res;
    return OKM_OK;
}

// A result in host memory (count_spilled) moved to the device, when it fits.
static okm_status result_to_device(okm_ctx *c) {
    if (!c->res_host) return OKM_OK;
    const uint64_t n = c->n_res;
    uint64_t *dk = nullptr, *dc = nullptr;
    okm_status st = pool_get(*c->pool, std::max<uint64_t>(n, 1) * c->kw, &dk);
    if (st == OKM_OK) st = pool_get(*c->pool, std::max<uint64_t>(n, 1), &dc);
    if (st != OKM_OK) {
        c->pool->put(dk);
        return fail(OKM_E_NOMEM, "the counted table (" + std::to_string(n) +
                                     " entries) lies in host memory and does not fit on the device: read it with "
                                     "okm_fetch_counts / okm_finish_counts");
    }
    if (n) {
        HIP_TRY(hipMemcpyAsync(dk, c->res_keys, n * 8 * c->kw, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(dc, c->res_counts, n * 8, hipMemcpyHostToDevice, c->stream));
    }
    OKM_TRY(sync(c));
    host_table_free(c, c->res_keys, c->res_counts, n);
    c->res_keys = dk;
    c->res_counts = dc;
    c->res_host = false;
    return OKM_OK;
}

okm_status okm_result_device(okm_ctx *c, const uint64_t **d_keys, const uint64_t **d_counts, uint64_t *n) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    OKM_TRY(okm_count(c, nullptr));
    OKM_TRY(ensure_dense(c));
    OKM_TRY(result_to_device(c));
    if (d_keys) *d_keys = c->res_keys;
    if (d_counts) *d_counts = c->res_counts;
    if (n) *n = c->n_res;
    return OKM_OK;
}

// count.rs:106-116 over a device range of the result: the entries with count
// >= min_count (min_count <= 1: all) copied to keys / counts (device or host
// memory) at most `cap` of them; *m = how many there are (cap == 0 and no
// outputs: only counted).
static okm_status fetch_range(okm_ctx *c, const uint64_t *dk, const uint64_t *dc, uint64_t n, uint64_t min_count,
                              uint64_t *keys, uint64_t *counts, uint64_t cap, uint64_t *m, bool dst_on_device) {
    *m = 0;
    if (!n) return OKM_OK;
    const uint64_t *src_k = dk, *src_c = dc;
    uint64_t cnt = n;
    uint64_t *tk = nullptr, *tc = nullptr;
    if (min_count > 1) {
        const uint32_t nb = filter_blocks(n);
        unsigned long long *bc, *bo, *tmp;
        OKM_TRY(pool_get(*c->pool, nb + 1, &bc));
        OKM_TRY(pool_get(*c->pool, nb + 1, &bo));
        OKM_TRY(pool_get(*c->pool, scan_tmp_elems(nb + 1), &tmp));
        HIP_TRY(hipMemsetAsync(bc, 0, (nb + 1) * sizeof(unsigned long long), c->stream));
        launch_filter_count(c->stream, dc, n, min_count, bc, nb);
        launch_exclusive_scan(c->stream, bc, bo, nb + 1, tmp);
        unsigned long long tot = 0;
        HIP_TRY(hipMemcpyAsync(&tot, bo + nb, sizeof(tot), hipMemcpyDeviceToHost, c->stream));
        OKM_TRY(sync(c));
        cnt = tot;
        if ((keys || counts) && cnt > cap) {
            c->pool->put(bc); c->pool->put(bo); c->pool->put(tmp);
            return fail(OKM_E_OVERFLOW, "okm_fetch_counts: buffer too small");
        }
        if (cnt && (keys || counts)) {
            OKM_TRY(pool_get(*c->pool, cnt * c->kw, &tk));
            OKM_TRY(pool_get(*c->pool, cnt, &tc));
            launch_filter_scatter(c->stream, dk, dc, n, min_count, bo, tk, tc, c->wide);
            HIP_TRY(hipGetLastError());
        }
        c->pool->put(bc); c->pool->put(bo); c->pool->put(tmp);
        src_k = tk;
        src_c = tc;
    } else if ((keys || counts) && cnt > cap) {
        return fail(OKM_E_OVERFLOW, "okm_fetch_counts: buffer too small");
    }
    if (cnt && (keys || counts)) {
        const hipMemcpyKind kind = dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        if (keys) HIP_TRY(hipMemcpyAsync(keys, src_k, cnt * 8 * c->kw, kind, c->stream));
        if (counts) HIP_TRY(hipMemcpyAsync(counts, src_c, cnt * 8, kind, c->stream));
        OKM_TRY(sync(c));
    }
    if (tk) c->pool->put(tk);
    if (tc) c->pool->put(tc);
    *m = cnt;
    return OKM_OK;
}

// fetch_range over the whole result; a host-resident result goes through the
// device filter in slices of `kSlice` entries.
static okm_status fetch_result(okm_ctx *c, uint64_t min_count, uint64_t *keys, uint64_t *counts, uint64_t cap,
                               uint64_t *n, bool dst_on_device) {
    *n = 0;
    if (c->n_res == 0) return OKM_OK;
    OKM_TRY(ensure_dense(c));
    if (!c->res_host)
        return fetch_range(c, c->res_keys, c->res_counts, c->n_res, min_count, keys, counts, cap, n, dst_on_device);
    constexpr uint64_t kSlice = uint64_t(1) << 26;
    const uint64_t sl = std::min<uint64_t>(kSlice, c->n_res);
    uint64_t *dk = nullptr, *dc = nullptr;
    OKM_TRY(pool_get(*c->pool, sl * c->kw, &dk));
    okm_status st = pool_get(*c->pool, sl, &dc);
    uint64_t done = 0;
    for (uint64_t o = 0; o < c->n_res && st == OKM_OK; o += sl) {
        const uint64_t len = std::min(sl, c->n_res - o);
        if (hipMemcpyAsync(dk, c->res_keys + o * c->kw, len * 8 * c->kw, hipMemcpyHostToDevice, c->stream) !=
                hipSuccess ||
            hipMemcpyAsync(dc, c->res_counts + o, len * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
            st = fail(OKM_E_DEVICE, "okm_fetch_counts: host-to-device copy");
            break;
        }
        uint64_t got = 0;
        const bool out = keys || counts;
        st = fetch_range(c, dk, dc, len, min_count, out && keys ? keys + done * c->kw : nullptr,
                         out && counts ? counts + done : nullptr, out ? cap - done : 0, &got, dst_on_device);
        done += got;
    }
    c->pool->put(dk);
    c->pool->put(dc);
    OKM_TRY(st);
    *n = done;
    return OKM_OK;
}

okm_status okm_result_size(okm_ctx *c, uint64_t min_count, uint64_t *n) {
    if (!c || !n) return fail(OKM_E_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    OKM_TRY(okm_count(c, nullptr));
    if (min_count <= 1 || c->n_res == 0) {
        *n = c->n_res;
        return OKM_OK;
    }
    return fetch_result(c, min_count, nullptr, nullptr, 0, n, false);
}

okm_status okm_fetch_counts(okm_ctx *c, uint64_t min_count, uint64_t *keys, uint64_t *counts, uint64_t cap,
                            uint64_t *n, int dst_on_device) {
    if (!c || !n) return fail(OKM_E_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    OKM_TRY(okm_count(c, nullptr));
    *n = 0;
    return fetch_result(c, min_count, keys, counts, cap, n, dst_on_device != 0);
}

okm_status okm_finish_counts(okm_ctx *c, uint64_t min_count, uint64_t **keys, uint64_t **counts, uint64_t *n) {
    if (!c || !keys || !n) return fail(OKM_E_ARG, "null argument");
    *keys = nullptr;
    if (counts) *counts = nullptr;
    uint64_t m = 0;
    OKM_TRY(okm_result_size(c, min_count, &m));
    uint64_t *hk = (uint64_t *)std::malloc(std::max<uint64_t>(m, 1) * 8 * c->kw);
    uint64_t *hc = counts ? (uint64_t *)std::malloc(std::max<uint64_t>(m, 1) * 8) : nullptr;
    if (!hk || (counts && !hc)) {
        std::free(hk);
        std::free(hc);
        return fail(OKM_E_NOMEM, "okm_finish_counts: host allocation");
    }
    okm_status s = okm_fetch_counts(c, min_count, hk, hc, m, n, 0);
    if (s != OKM_OK) {
        std::free(hk);
        std::free(hc);
        return s;
    }
    *keys = hk;
    if (counts) *counts = hc;
    return OKM_OK;
}

okm_status okm_finish_set(okm_ctx *c, uint64_t **keys, uint64_t *n) {
    return okm_finish_counts(c, 1, keys, nullptr, n);
}

void okm_free_result(void *p) { std::free(p); }

okm_status okm_set_intersection_size(const uint64_t *a, uint64_t na, const uint64_t *b, uint64_t nb, int device,
                                     uint64_t *out) {
    if (!out) return fail(OKM_E_ARG, "null out");
    *out = 0;
    if (na == 0 || nb == 0) return OKM_OK;
    if (!a || !b) return fail(OKM_E_ARG, "null input");
    std::string why;
    if (!device_ok(device, &why)) return fail(OKM_E_DEVICE, why);
    HIP_TRY(hipSetDevice(device));
    uint64_t *da = nullptr, *db = nullptr;
    unsigned long long *dout = nullptr;
    hipStream_t st;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    okm_status status = OKM_OK;
    do {
        // probe the smaller set into the larger (compare.rs:58)
        const bool swap = na > nb;
        const uint64_t *sa = swap ? b : a, *sb = swap ? a : b;
        const uint64_t sna = swap ? nb : na, snb = swap ? na : nb;
        if (hipMalloc(&da, sna * 8) != hipSuccess || hipMalloc(&db, snb * 8) != hipSuccess ||
            hipMalloc(&dout, 8) != hipSuccess) {
            status = fail(OKM_E_NOMEM, "okm_set_intersection_size: device allocation");
            break;
        }
        if (hipMemcpyAsync(da, sa, sna * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(db, sb, snb * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemsetAsync(dout, 0, 8, st) != hipSuccess) {
            status = fail(OKM_E_DEVICE, "okm_set_intersection_size: copy");
            break;
        }
        launch_intersect_count(st, da, sna, db, snb, dout, false);
        unsigned long long h = 0;
        if (hipMemcpyAsync(&h, dout, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            status = fail(OKM_E_DEVICE, "okm_set_intersection_size: kernel");
            break;
        }
        *out = h;
    } while (0);
    (void)hipGetLastError();
    if (da) (void)hipFree(da);
    if (db) (void)hipFree(db);
    if (dout) (void)hipFree(dout);
    (void)hipStreamDestroy(st);
    return status;
}

okm_status okm_set_intersection_size_device(const uint64_t *d_a, uint64_t na, const uint64_t *d_b, uint64_t nb,
                                            int device, uint64_t *out) {
    if (!out) return fail(OKM_E_ARG, "null out");
    *out = 0;
    if (na == 0 || nb == 0) return OKM_OK;
    if (!d_a || !d_b) return fail(OKM_E_ARG, "null input");
    std::string why;
    if (!device_ok(device, &why)) return fail(OKM_E_DEVICE, why);
    HIP_TRY(hipSetDevice(device));
    unsigned long long *dout = nullptr;
    hipStream_t st;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    okm_status status = OKM_OK;
    const bool swap = na > nb;  // probe the smaller set into the larger (compare.rs:58)
    unsigned long long h = 0;
    if (hipMalloc(&dout, 8) != hipSuccess) {
        status = fail(OKM_E_NOMEM, "okm_set_intersection_size_device: device allocation");
    } else if (hipMemsetAsync(dout, 0, 8, st) != hipSuccess) {
        status = fail(OKM_E_DEVICE, "okm_set_intersection_size_device: memset");
    } else {
        launch_intersect_count(st, swap ? d_b : d_a, swap ? nb : na, swap ? d_a : d_b, swap ? na : nb, dout, false);
        if (hipMemcpyAsync(&h, dout, 8, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
            status = fail(OKM_E_DEVICE, "okm_set_intersection_size_device: kernel");
    }
    if (status == OKM_OK) *out = h;
    (void)hipGetLastError();
    if (dout) (void)hipFree(dout);
    (void)hipStreamDestroy(st);
    return status;
}

okm_status okm_synchronize(okm_ctx *c) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    return sync(c);
}

okm_status okm_set_timing(okm_ctx *c, int enable) {
    if (!c) return fail(OKM_E_ARG, "null ctx");
    OKM_TRY(sync(c));
    c->timer.on = enable != 0;
    c->timer.reset();
    return OKM_OK;
}

okm_status okm_kernel_stats(okm_ctx *c, okm_kernel_stat *stats, int cap, int *n) {
    if (!c || !n) return fail(OKM_E_ARG, "null argument");
    OKM_TRY(sync(c));
    const int m = (int)c->timer.stats.size();
    for (int i = 0; i < m && i < cap; ++i) {
        stats[i] = c->timer.stats[i];
        stats[i].name = c->timer.names[i].c_str();
    }
    *n = m;
    return OKM_OK;
}

okm_status okm_engine_info_get(okm_ctx *c, okm_engine_info *info) {
    if (!c || !info) return fail(OKM_E_ARG, "null argument");
    *info = c->info;
    info->folds = c->folds;
    info->device_bytes = c->pool->held() + c->HC_cap * 4 + c->Hg_cap * 16 + c->staging_cap;
    info->device_peak_bytes = c->pool->peak() + c->HC_cap * 4 + c->Hg_cap * 16 + c->staging_cap;
    info->host_bytes = c->host_bytes;
    info->spills = c->spills;
    return OKM_OK;
}

okm_status okm_device_alloc(int device, uint64_t bytes, void **d_ptr) {
    if (!d_ptr) return fail(OKM_E_ARG, "null out");
    std::string why;
    if (!device_ok(device, &why)) return fail(OKM_E_DEVICE, why);
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipMalloc(d_ptr, bytes ? bytes : 1));
    return OKM_OK;
}

okm_status okm_device_free(void *d_ptr) {
    if (d_ptr) HIP_TRY(hipFree(d_ptr));
    return OKM_OK;
}

okm_status okm_memcpy_h2d(void *d_dst, const void *src, uint64_t bytes) {
    if (bytes) HIP_TRY(hipMemcpy(d_dst, src, bytes, hipMemcpyHostToDevice));
    return OKM_OK;
}

okm_status okm_memcpy_d2h(void *dst, const void *d_src, uint64_t bytes) {
    if (bytes) HIP_TRY(hipMemcpy(dst, d_src, bytes, hipMemcpyDeviceToHost));
    return OKM_OK;
}

}  // extern "C"
