// okm_probe.hip — device hash sets / maps of canonical k-mers and the probe
// kernels of the two read-only callers of the counting path:
//
//   query    (commands/query.rs:24-134): the DB's unified k-mer set
//            (db_types.rs:43-48 get_all_kmers_unified -> HashSet<u64>) and, per
//            read, the number of windows whose canonical k-mer is in it
//            (query.rs:81-99: seq_to_u64 on the RAW record.sequence(), no
//            normalize, so U/u and line breaks kill windows).
//   classify (commands/classify.rs:215-308): per reference, how many of the
//            filtered input k-mers it holds and the sum of their counts, and
//            the same over the union of the database's references.
//
// Tables are open-addressing arrays of u64 keys (or {key, value} pairs) at
// load <= 1/2, linear probing from the top bits of a murmur3 fmix64 of the
// key.  ~0 is the empty slot; it is never a canonical k-mer, and
// a stray ~0 in a database lives in a side flag word at slots[cap].
//
// The query kernel is the extraction scan of okm_extract.hip with a probe in
// place of the partition emit: one thread walks SEG window starts, issues all
// of their first-slot loads back to back (SEG loads in flight per thread), then
// resolves and sums the hits per record.  A record's index is the number of
// separators before it: per-tile separator counts are scanned on the device,
// and a block scan gives each thread its first record, so no offsets array is
// needed and a device batch is consumed in place.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "okm_internal.h"
#include "okm_scan.h"

namespace okm {

constexpr ull kEmpty = ~0ull;

__device__ __forceinline__ uint64_t slot_hash(uint64_t x) {  // murmur3 fmix64
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

struct SetTab {
    ull *slots;      // cap + 1 words (slots[cap]: the ~0 flag)
    uint64_t mask;   // cap - 1
    uint32_t shift;  // 64 - log2(cap)
};

struct MapTab {
    ulonglong2 *slots;  // {key, value}
    uint64_t mask;
    uint32_t shift;
};

__device__ __forceinline__ uint64_t home_slot(uint64_t key, uint32_t shift) { return slot_hash(key) >> shift; }

// HashSet::insert: true iff the key was not there yet.
__device__ __forceinline__ bool set_insert(const SetTab &t, ull key) {
    if (key == kEmpty) return atomicCAS(&t.slots[t.mask + 1], 0ull, 1ull) == 0ull;
    uint64_t s = home_slot(key, t.shift);
    for (;;) {
        ull v = t.slots[s];
        if (v == kEmpty) {
            v = atomicCAS(&t.slots[s], kEmpty, key);
            if (v == kEmpty) return true;
        }
        if (v == key) return false;
        s = (s + 1) & t.mask;
    }
}

// Continue a probe whose home slot held `first` (neither key nor empty).
__device__ __noinline__ bool set_probe_rest(const SetTab &t, ull key, uint64_t s) {
    for (;;) {
        s = (s + 1) & t.mask;
        const ull v = t.slots[s];
        if (v == key) return true;
        if (v == kEmpty) return false;
    }
}

__device__ __forceinline__ bool set_contains(const SetTab &t, ull key) {
    if (key == kEmpty) return t.slots[t.mask + 1] != 0ull;
    const uint64_t s = home_slot(key, t.shift);
    const ull v = t.slots[s];
    if (v == key) return true;
    if (v == kEmpty) return false;
    return set_probe_rest(t, key, s);
}

// Map lookup: value of key, or 0 when absent (stored values are >= 1).
__device__ __forceinline__ ull map_get(const MapTab &t, ull key) {
    if (key == kEmpty) return 0;  // never an input k-mer
    uint64_t s = home_slot(key, t.shift);
    for (;;) {
        const ulonglong2 v = t.slots[s];
        if (v.x == key) return v.y;
        if (v.x == kEmpty) return 0;
        s = (s + 1) & t.mask;
    }
}

// ---------------------------------------------------------------------------
// Set build / rehash / membership
// ---------------------------------------------------------------------------
constexpr int kProbeBlock = 256;

__global__ __launch_bounds__(kProbeBlock) void k_set_insert(SetTab t, const ull *__restrict__ keys, uint64_t n,
                                                            ull *__restrict__ n_new) {
    const uint64_t stride = (uint64_t)gridDim.x * kProbeBlock;
    ull mine = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kProbeBlock + threadIdx.x; i < n; i += stride)
        mine += set_insert(t, keys[i]) ? 1u : 0u;
    // one atomic per wave
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) mine += __shfl_xor(mine, d, 64);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd(n_new, mine);
}

// Re-insert every key of an old table (growth).
__global__ __launch_bounds__(kProbeBlock) void k_set_rehash(SetTab t, const ull *__restrict__ old, uint64_t old_cap) {
    const uint64_t stride = (uint64_t)gridDim.x * kProbeBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kProbeBlock + threadIdx.x; i <= old_cap; i += stride) {
        const ull v = old[i];
        if (i == old_cap) {
            if (v) t.slots[t.mask + 1] = 1ull;
        } else if (v != kEmpty) {
            set_insert(t, v);
        }
    }
}

__global__ __launch_bounds__(kProbeBlock) void k_set_contains(SetTab t, const ull *__restrict__ keys, uint64_t n,
                                                              uint8_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * kProbeBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kProbeBlock + threadIdx.x; i < n; i += stride)
        out[i] = set_contains(t, keys[i]) ? 1 : 0;
}

// ---------------------------------------------------------------------------
// query: per-record hit counts over a batch (records joined by separators)
// ---------------------------------------------------------------------------
constexpr int kQSeg = 16;                      // window starts per thread
constexpr int kQTile = kProbeBlock * kQSeg;    // 4096 bytes per block

// Number of separator bytes in a little-endian word.
__device__ __forceinline__ uint32_t sep_bytes(uint32_t w) {
    const uint32_t x = w ^ (0x01010101u * OKM_RECORD_SEPARATOR);
    const uint32_t y = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    return __popc(y);  // exact zero-byte count
}

__device__ __forceinline__ uint32_t sep_mask16(const uint32_t *w) {  // bit j: byte j is a separator
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < kQSeg; ++i) m |= (((w[i >> 2] >> ((i & 3) * 8)) & 0xFFu) == OKM_RECORD_SEPARATOR ? 1u : 0u) << i;
    return m;
}

__global__ __launch_bounds__(kProbeBlock) void k_sep_count(const uint8_t *__restrict__ seq, uint64_t n,
                                                           ull *__restrict__ tile_cnt) {
    __shared__ ull wsum[kProbeBlock / 64];
    const uint64_t w0 = (uint64_t)blockIdx.x * kQTile + (uint64_t)threadIdx.x * kQSeg;
    uint32_t c = 0;
    if (w0 + kQSeg <= n) {
        const uint4 v = *reinterpret_cast<const uint4 *>(seq + w0);
        c = sep_bytes(v.x) + sep_bytes(v.y) + sep_bytes(v.z) + sep_bytes(v.w);
    } else {
        for (uint64_t i = w0; i < n; ++i) c += seq[i] == OKM_RECORD_SEPARATOR;
    }
    ull tot;
    block_excl_scan<kProbeBlock>((ull)c, wsum, &tot);
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

__device__ __forceinline__ void flush_hits(uint32_t *hits, uint64_t nrec, ull rec, uint32_t cur) {
    if (cur && rec < nrec) atomicAdd(&hits[rec], cur);
}

// The compiler may not keep values derived from the codes alive across the
// probe loads (it would: they are cheaper to keep than to recompute, and they
// cost the occupancy): the codes are "changed" here, so they are recomputed.
template <int NP>
__device__ __forceinline__ void opaque_codes(Codes<NP> &c) {
#pragma unroll
    for (int i = 0; i < NP; ++i) asm volatile("" : "+v"(c.p[i]), "+v"(c.q[i]));
}

// Keys of the thread's SEG windows stay in registers and their home-slot
// loads are all in flight together.  K > 0: k known at compile time; K = 0:
// runtime k.
template <int K>
__global__ __launch_bounds__(kProbeBlock) void k_query_hits(const uint8_t *__restrict__ seq, uint64_t n,
                                                            const ull *__restrict__ tile_pre, SetTab t,
                                                            uint32_t k_rt, uint32_t *__restrict__ hits,
                                                            uint64_t nrec) {
    __shared__ ull wsum[kProbeBlock / 64];
    const uint64_t w0 = (uint64_t)blockIdx.x * kQTile + (uint64_t)threadIdx.x * kQSeg;
    WinWords<kQSeg> ww;
    load_windows<kQSeg>(seq, n, w0, ww);
    const uint32_t *w = ww.w;
    const uint32_t sepm = w0 < n ? sep_mask16(w) : 0u;  // bytes past n read as 0
    ull tot;
    const ull rec0 = tile_pre[blockIdx.x] + block_excl_scan<kProbeBlock>((ull)__popc(sepm), wsum, &tot);
    if (w0 >= n) return;

    const uint32_t k = K ? (uint32_t)K : k_rt;
    constexpr int NP = WinWords<kQSeg>::kLoad / 16;
    Codes<NP> c;
    make_codes<NP, true>(w, c);  // query.rs: raw bytes, U invalid
    const uint32_t vmask = ~invalid_windows<kQSeg, NP>(c, k) & 0xFFFFu;
    // every valid window's home slot load in flight before any is consumed;
    // only the loaded words stay live across the loads (keys and homes are
    // recomputed from the codes afterwards), so 8 waves fit a SIMD and twice
    // the probes are in flight per CU
    ull first[kQSeg];
#pragma unroll
    for (int j = 0; j < kQSeg; ++j)
        first[j] = (vmask >> j) & 1u ? t.slots[home_slot(window_key_nv(c, j, k), t.shift)] : kEmpty;
    opaque_codes(c);
    ull rec = rec0;
    uint32_t cur = 0;
#pragma unroll
    for (int j = 0; j < kQSeg; ++j) {
        if ((sepm >> j) & 1u) {  // window j starts a new record (and is itself invalid)
            flush_hits(hits, nrec, rec, cur);
            cur = 0;
            ++rec;
        }
        if (first[j] != kEmpty) {  // a valid window whose home slot holds a key
            const ull key = window_key_nv(c, j, k);
            const bool hit = first[j] == key || set_probe_rest(t, key, home_slot(key, t.shift));
            cur += hit ? 1u : 0u;
        }
    }
    flush_hits(hits, nrec, rec, cur);
}

// ---------------------------------------------------------------------------
// classify: map of the filtered input counts, probed by every reference key
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kProbeBlock) void k_map_build(MapTab t, const ull *__restrict__ keys,
                                                           const ull *__restrict__ counts, uint64_t n,
                                                           uint64_t min_count, ull *__restrict__ n_ins) {
    const uint64_t stride = (uint64_t)gridDim.x * kProbeBlock;
    ull mine = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kProbeBlock + threadIdx.x; i < n; i += stride) {
        const ull c = counts ? counts[i] : 1ull;
        if (c < min_count) continue;  // classify.rs:195-199
        const ull key = keys[i];      // distinct, canonical (never ~0)
        uint64_t s = home_slot(key, t.shift);
        while (atomicCAS(&t.slots[s].x, kEmpty, key) != kEmpty) s = (s + 1) & t.mask;
        t.slots[s].y = c;
        ++mine;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) mine += __shfl_xor(mine, d, 64);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd(n_ins, mine);
}

constexpr int kCPer = 8;  // reference keys per thread

// Reference r owns keys[ref_off[r], ref_off[r+1]).  per_ref[r] = {input k-mers
// it holds, sum of their counts} (classify.rs:228-236); tot = {|union|,
// |input ∩ union|, sum of counts over it} (classify.rs:237, :268-272,
// db_types.rs:50-53).
__device__ __forceinline__ uint64_t ref_of(const ull *__restrict__ ref_off, uint64_t nrefs, uint64_t i) {
    uint64_t lo = 0, hi = nrefs;  // last r with ref_off[r] <= i
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (ref_off[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kProbeBlock) void k_classify(const ull *__restrict__ keys, uint64_t nkeys,
                                                          const ull *__restrict__ ref_off, uint64_t nrefs,
                                                          MapTab m, SetTab u, ulonglong2 *__restrict__ per_ref,
                                                          ull *__restrict__ tot) {
    __shared__ ull red[5];
    if (threadIdx.x < 5) red[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * kProbeBlock * kCPer;
    const uint64_t base = b0 + (uint64_t)threadIdx.x * kCPer;
    // a block's keys usually all belong to one reference (references hold
    // millions): its per-reference sums then leave as ONE pair of atomics
    // instead of one pair per thread on the same 32 counters
    const uint64_t blast = min(b0 + (uint64_t)kProbeBlock * kCPer, nkeys) - 1;
    const uint64_t rb = ref_of(ref_off, nrefs, b0);
    const bool one_ref = ref_off[rb + 1] > blast;  // block-uniform
    ull un = 0, um = 0, us = 0, hm = 0, hs = 0;
    if (base < nkeys) {
        uint64_t r = one_ref ? rb : ref_of(ref_off, nrefs, base), rend = ref_off[r + 1];
        for (int j = 0; j < kCPer; ++j) {
            const uint64_t i = base + j;
            if (i >= nkeys) break;
            while (i >= rend) {  // next reference (skipping empty ones); never in a one-reference block
                if (hm) {
                    atomicAdd(&per_ref[r].x, hm);
                    atomicAdd(&per_ref[r].y, hs);
                }
                hm = hs = 0;
                ++r;
                rend = ref_off[r + 1];
            }
            const ull key = keys[i];
            const ull c = map_get(m, key);
            if (c) {
                ++hm;
                hs += c;
            }
            if (set_insert(u, key)) {
                ++un;
                if (c) {
                    ++um;
                    us += c;
                }
            }
        }
        if (hm && !one_ref) {
            atomicAdd(&per_ref[r].x, hm);
            atomicAdd(&per_ref[r].y, hs);
        }
    }
    if (!one_ref) hm = hs = 0;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {  // wave sums, then one LDS add per wave
        un += __shfl_xor(un, d, 64);
        um += __shfl_xor(um, d, 64);
        us += __shfl_xor(us, d, 64);
        hm += __shfl_xor(hm, d, 64);
        hs += __shfl_xor(hs, d, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (un) atomicAdd(&red[0], un);
        if (um) atomicAdd(&red[1], um);
        if (us) atomicAdd(&red[2], us);
        if (hm) atomicAdd(&red[3], hm);
        if (hs) atomicAdd(&red[4], hs);
    }
    __syncthreads();
    if (threadIdx.x < 3 && red[threadIdx.x]) atomicAdd(&tot[threadIdx.x], red[threadIdx.x]);
    if (one_ref && threadIdx.x == 0 && red[3]) {
        atomicAdd(&per_ref[rb].x, red[3]);
        atomicAdd(&per_ref[rb].y, red[4]);
    }
}

static uint32_t grid_for(uint64_t n) {
    uint64_t g = (n + kProbeBlock - 1) / kProbeBlock;
    if (g > 65536) g = 65536;
    return (uint32_t)(g ? g : 1);
}

}  // namespace okm

using namespace okm;

// ===========================================================================
// Host side
// ===========================================================================
namespace {

#define PHIP(expr)                                                                             \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(e_ == hipErrorOutOfMemory ? OKM_E_NOMEM : OKM_E_DEVICE,                \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                    \
    } while (0)

#define PTRY(expr)                   \
    do {                             \
        okm_status s_ = (expr);      \
        if (s_ != OKM_OK) return s_; \
    } while (0)

uint64_t pow2_at_least(uint64_t x) {
    uint64_t c = 1024;
    while (c < x) c <<= 1;
    return c;
}

uint32_t log2_exact(uint64_t c) {
    uint32_t l = 0;
    while ((1ull << l) < c) ++l;
    return l;
}

bool device_usable(int device, std::string *why) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        *why = "no HIP device visible (the engine has no CPU fallback)";
        return false;
    }
    if (device < 0 || device >= n) {
        *why = "device ordinal " + std::to_string(device) + " out of range";
        return false;
    }
    return true;
}

// Growable device scratch.
struct Scratch {
    void *p = nullptr;
    size_t cap = 0;
    okm_status ensure(size_t bytes) {
        if (bytes <= cap) return OKM_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 8 + 256;
        PHIP(hipMalloc(&p, want));
        cap = want;
        return OKM_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

struct okm_kset {
    int device = 0;
    uint8_t k = 0;
    hipStream_t st = nullptr;
    ull *slots = nullptr;
    uint64_t cap = 0;
    uint64_t size = 0;
    ull *d_ctr = nullptr;  // [0]: new keys of the last insert
    Scratch keys, batch, tiles, hits;
    std::vector<uint8_t> host_batch;

    SetTab tab() const { return SetTab{slots, cap - 1, 64u - log2_exact(cap)}; }
};

struct okm_classifier {
    int device = 0;
    hipStream_t st = nullptr;
    ulonglong2 *slots = nullptr;
    uint64_t cap = 0;
    uint64_t n_input = 0;
    ull *d_ctr = nullptr;
    Scratch keys, offs, uset, per_ref;
    uint8_t *stage[2] = {nullptr, nullptr};  // pinned host staging of the database keys (okm_classifier_probe_db)
    hipEvent_t staged[2] = {nullptr, nullptr};

    MapTab tab() const { return MapTab{slots, cap - 1, 64u - log2_exact(cap)}; }
};

namespace {

okm_status set_alloc(okm_kset *s, uint64_t cap) {
    ull *p = nullptr;
    PHIP(hipMalloc(&p, (cap + 1) * sizeof(ull)));
    PHIP(hipMemsetAsync(p, 0xFF, cap * sizeof(ull), s->st));
    PHIP(hipMemsetAsync(p + cap, 0, sizeof(ull), s->st));
    if (s->slots) {
        const ull *old = s->slots;
        const uint64_t old_cap = s->cap;
        s->slots = p;
        s->cap = cap;
        hipLaunchKernelGGL(k_set_rehash, dim3(grid_for(old_cap + 1)), dim3(kProbeBlock), 0, s->st, s->tab(), old,
                           old_cap);
        PHIP(hipGetLastError());
        PHIP(hipStreamSynchronize(s->st));
        (void)hipFree((void *)old);
    } else {
        s->slots = p;
        s->cap = cap;
    }
    return OKM_OK;
}

// Load stays <= 1/2 even if all n keys are new.
okm_status set_reserve(okm_kset *s, uint64_t n) {
    const uint64_t need = 2 * (s->size + n);
    if (need <= s->cap) return OKM_OK;
    return set_alloc(s, pow2_at_least(need));
}

okm_status set_insert_device(okm_kset *s, const uint64_t *d_keys, uint64_t n, uint64_t *n_new) {
    PTRY(set_reserve(s, n));
    PHIP(hipMemsetAsync(s->d_ctr, 0, sizeof(ull), s->st));
    hipLaunchKernelGGL(k_set_insert, dim3(grid_for(n)), dim3(kProbeBlock), 0, s->st, s->tab(),
                       (const ull *)d_keys, n, s->d_ctr);
    PHIP(hipGetLastError());
    ull h = 0;
    PHIP(hipMemcpyAsync(&h, s->d_ctr, sizeof(ull), hipMemcpyDeviceToHost, s->st));
    PHIP(hipStreamSynchronize(s->st));
    s->size += h;
    if (n_new) *n_new = h;
    return OKM_OK;
}

template <int K>
void launch_query_k(okm_kset *s, const uint8_t *d_seq, uint64_t n, const ull *pre, uint32_t *d_hits, uint64_t nrec,
                    uint32_t ntiles) {
    hipLaunchKernelGGL(k_query_hits<K>, dim3(ntiles), dim3(kProbeBlock), 0, s->st, d_seq, n, pre, s->tab(),
                       (uint32_t)s->k, d_hits, nrec);
}

okm_status query_device(okm_kset *s, const uint8_t *d_seq, uint64_t n, uint64_t nrec, uint32_t *d_hits) {
    PHIP(hipMemsetAsync(d_hits, 0, nrec * sizeof(uint32_t), s->st));
    if (n == 0 || s->size == 0) return OKM_OK;
    const uint64_t ntiles = (n + kQTile - 1) / kQTile;
    if (ntiles > 0x7FFFFFFFull) return fail(OKM_E_ARG, "okm_query_hits: batch too large");
    const size_t tmp = scan_tmp_elems(ntiles);
    PTRY(s->tiles.ensure((2 * ntiles + tmp) * sizeof(ull)));
    ull *cnt = (ull *)s->tiles.p, *pre = cnt + ntiles, *scr = pre + ntiles;
    hipLaunchKernelGGL(k_sep_count, dim3((uint32_t)ntiles), dim3(kProbeBlock), 0, s->st, d_seq, n, cnt);
    launch_exclusive_scan(s->st, cnt, pre, ntiles, scr);
    switch (s->k) {
    case 21: launch_query_k<21>(s, d_seq, n, pre, d_hits, nrec, (uint32_t)ntiles); break;
    case 25: launch_query_k<25>(s, d_seq, n, pre, d_hits, nrec, (uint32_t)ntiles); break;
    case 27: launch_query_k<27>(s, d_seq, n, pre, d_hits, nrec, (uint32_t)ntiles); break;
    case 31: launch_query_k<31>(s, d_seq, n, pre, d_hits, nrec, (uint32_t)ntiles); break;
    case 32: launch_query_k<32>(s, d_seq, n, pre, d_hits, nrec, (uint32_t)ntiles); break;
    default: launch_query_k<0>(s, d_seq, n, pre, d_hits, nrec, (uint32_t)ntiles); break;
    }
    PHIP(hipGetLastError());
    return OKM_OK;
}

}  // namespace

extern "C" {

okm_status okm_kset_create(okm_kset **out, uint8_t k, int device, uint64_t capacity_hint) {
    if (!out) return fail(OKM_E_ARG, "null out");
    *out = nullptr;
    if (k == 0 || k > 32) return fail(OKM_E_INVALID_K, "Invalid K-mer size: " + std::to_string(k) + ". Must be between 1 and 32.");
    std::string why;
    if (!device_usable(device, &why)) return fail(OKM_E_DEVICE, why);
    PHIP(hipSetDevice(device));
    okm_kset *s = new okm_kset();
    s->device = device;
    s->k = k;
    okm_status st = OKM_OK;
    if (hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&s->d_ctr, 8 * sizeof(ull)) != hipSuccess)
        st = fail(OKM_E_DEVICE, "okm_kset_create: stream/counter allocation");
    if (st == OKM_OK) st = set_alloc(s, pow2_at_least(2 * capacity_hint));
    if (st == OKM_OK && hipStreamSynchronize(s->st) != hipSuccess) st = fail(OKM_E_DEVICE, "okm_kset_create: sync");
    if (st != OKM_OK) {
        okm_kset_destroy(s);
        return st;
    }
    *out = s;
    return OKM_OK;
}

void okm_kset_destroy(okm_kset *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->st) (void)hipStreamSynchronize(s->st);
    if (s->slots) (void)hipFree(s->slots);
    if (s->d_ctr) (void)hipFree(s->d_ctr);
    s->keys.release();
    s->batch.release();
    s->tiles.release();
    s->hits.release();
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
}

okm_status okm_kset_insert(okm_kset *s, const uint64_t *keys, uint64_t n, int keys_on_device, uint64_t *n_new) {
    if (!s) return fail(OKM_E_ARG, "null set");
    if (n_new) *n_new = 0;
    if (n == 0) return OKM_OK;
    if (!keys) return fail(OKM_E_ARG, "okm_kset_insert: null keys");
    PHIP(hipSetDevice(s->device));
    if (keys_on_device) return set_insert_device(s, keys, n, n_new);
    const uint64_t chunk = 64ull << 20;  // keys per upload (512 MB)
    uint64_t total = 0;
    for (uint64_t o = 0; o < n; o += chunk) {
        const uint64_t m = n - o < chunk ? n - o : chunk;
        PTRY(s->keys.ensure(m * sizeof(uint64_t)));
        PHIP(hipMemcpyAsync(s->keys.p, keys + o, m * sizeof(uint64_t), hipMemcpyHostToDevice, s->st));
        uint64_t got = 0;
        PTRY(set_insert_device(s, (const uint64_t *)s->keys.p, m, &got));
        total += got;
    }
    if (n_new) *n_new = total;
    return OKM_OK;
}

okm_status okm_kset_size(const okm_kset *s, uint64_t *n) {
    if (!s || !n) return fail(OKM_E_ARG, "null argument");
    *n = s->size;
    return OKM_OK;
}

okm_status okm_kset_contains(okm_kset *s, const uint64_t *keys, uint64_t n, uint8_t *out) {
    if (!s || (!keys && n) || (!out && n)) return fail(OKM_E_ARG, "null argument");
    if (n == 0) return OKM_OK;
    PHIP(hipSetDevice(s->device));
    PTRY(s->keys.ensure(n * sizeof(uint64_t) + n + 16));
    ull *dk = (ull *)s->keys.p;
    uint8_t *dout = (uint8_t *)(dk + n);
    PHIP(hipMemcpyAsync(dk, keys, n * sizeof(uint64_t), hipMemcpyHostToDevice, s->st));
    hipLaunchKernelGGL(k_set_contains, dim3(grid_for(n)), dim3(kProbeBlock), 0, s->st, s->tab(), dk, n, dout);
    PHIP(hipGetLastError());
    PHIP(hipMemcpyAsync(out, dout, n, hipMemcpyDeviceToHost, s->st));
    PHIP(hipStreamSynchronize(s->st));
    return OKM_OK;
}

okm_status okm_query_hits_device(okm_kset *s, const uint8_t *d_seq, uint64_t n_bytes, uint64_t n_records,
                                 uint32_t *d_hits) {
    if (!s) return fail(OKM_E_ARG, "null set");
    if (n_records == 0) return OKM_OK;
    if (!d_hits || (!d_seq && n_bytes)) return fail(OKM_E_ARG, "okm_query_hits_device: null pointer");
    PHIP(hipSetDevice(s->device));
    const uint8_t *src = d_seq;
    if ((reinterpret_cast<uintptr_t>(d_seq) & 15u) != 0) {  // the scan loads 16-B words
        PTRY(s->batch.ensure(n_bytes + 16));
        PHIP(hipMemcpyAsync(s->batch.p, d_seq, n_bytes, hipMemcpyDeviceToDevice, s->st));
        src = (const uint8_t *)s->batch.p;
    }
    PTRY(query_device(s, src, n_bytes, n_records, d_hits));
    PHIP(hipStreamSynchronize(s->st));
    return OKM_OK;
}

okm_status okm_query_hits(okm_kset *s, const uint8_t *seq, const uint64_t *offsets, uint64_t n_records,
                          uint32_t *hits) {
    if (!s) return fail(OKM_E_ARG, "null set");
    if (n_records == 0) return OKM_OK;
    if (!offsets || !hits) return fail(OKM_E_ARG, "okm_query_hits: null pointer");
    const uint64_t total = offsets[n_records] - offsets[0];
    if (total && !seq) return fail(OKM_E_ARG, "okm_query_hits: null seq");
    PHIP(hipSetDevice(s->device));
    // device layout: raw bytes, anything but A/C/G/T (either case) -> 'N' (so a
    // line break inside a multi-line FASTA record kills windows without ending
    // the record), one separator after each record (query.rs:81-88)
    static uint8_t lut[256];
    static bool lut_init = false;
    if (!lut_init) {
        for (int c = 0; c < 256; ++c) lut[c] = 'N';
        for (const char *p = "ACGTacgt"; *p; ++p) lut[(uint8_t)*p] = (uint8_t)*p;
        lut_init = true;
    }
    const uint64_t nb = total + n_records;
    s->host_batch.resize(nb);
    uint8_t *d = s->host_batch.data();
    uint64_t o = 0;
    for (uint64_t r = 0; r < n_records; ++r) {
        const uint8_t *src = seq + offsets[r];
        const uint64_t len = offsets[r + 1] - offsets[r];
        for (uint64_t i = 0; i < len; ++i) d[o + i] = lut[src[i]];
        o += len;
        d[o++] = OKM_RECORD_SEPARATOR;
    }
    PTRY(s->batch.ensure(nb + 16));
    PTRY(s->hits.ensure(n_records * sizeof(uint32_t)));
    PHIP(hipMemcpyAsync(s->batch.p, d, nb, hipMemcpyHostToDevice, s->st));
    PTRY(query_device(s, (const uint8_t *)s->batch.p, nb, n_records, (uint32_t *)s->hits.p));
    PHIP(hipMemcpyAsync(hits, s->hits.p, n_records * sizeof(uint32_t), hipMemcpyDeviceToHost, s->st));
    PHIP(hipStreamSynchronize(s->st));
    return OKM_OK;
}

// ---------------------------------------------------------------------------
// classify
// ---------------------------------------------------------------------------
okm_status okm_classifier_create(okm_classifier **out, okm_ctx *input, uint64_t min_kmer_frequency,
                                 uint64_t *n_input_kmers) {
    if (!out || !input) return fail(OKM_E_ARG, "null argument");
    *out = nullptr;
    uint64_t nd = 0;
    PTRY(okm_count(input, &nd));  // idempotent when already counted
    const uint64_t *dk = nullptr, *dc = nullptr;
    uint64_t n = 0;
    PTRY(okm_result_device(input, &dk, &dc, &n));
    if (ctx_is_wide(input)) return fail(OKM_E_INVALID_K, "classify needs k <= 32 (classify.rs:79-80)");
    const int device = ctx_device(input);
    PHIP(hipSetDevice(device));
    okm_classifier *c = new okm_classifier();
    c->device = device;
    okm_status st = OKM_OK;
    do {
        if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&c->d_ctr, 8 * sizeof(ull)) != hipSuccess) {
            st = fail(OKM_E_DEVICE, "okm_classifier_create: stream/counter allocation");
            break;
        }
        c->cap = pow2_at_least(2 * n);
        if (hipMalloc(&c->slots, c->cap * sizeof(ulonglong2)) != hipSuccess) {
            st = fail(OKM_E_NOMEM, "okm_classifier_create: table allocation");
            break;
        }
        if (hipMemsetAsync(c->slots, 0xFF, c->cap * sizeof(ulonglong2), c->st) != hipSuccess ||
            hipMemsetAsync(c->d_ctr, 0, 8 * sizeof(ull), c->st) != hipSuccess) {
            st = fail(OKM_E_DEVICE, "okm_classifier_create: memset");
            break;
        }
        if (n)
            hipLaunchKernelGGL(k_map_build, dim3(grid_for(n)), dim3(kProbeBlock), 0, c->st, c->tab(), (const ull *)dk,
                               (const ull *)dc, n, min_kmer_frequency, c->d_ctr);
        ull h = 0;
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(&h, c->d_ctr, sizeof(ull), hipMemcpyDeviceToHost, c->st) != hipSuccess ||
            hipStreamSynchronize(c->st) != hipSuccess) {
            st = fail(OKM_E_DEVICE, "okm_classifier_create: map build");
            break;
        }
        c->n_input = h;
    } while (0);
    if (st != OKM_OK) {
        okm_classifier_destroy(c);
        return st;
    }
    if (n_input_kmers) *n_input_kmers = c->n_input;
    *out = c;
    return OKM_OK;
}

void okm_classifier_destroy(okm_classifier *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->st) (void)hipStreamSynchronize(c->st);
    if (c->slots) (void)hipFree(c->slots);
    if (c->d_ctr) (void)hipFree(c->d_ctr);
    c->keys.release();
    c->offs.release();
    c->uset.release();
    c->per_ref.release();
    for (int i = 0; i < 2; ++i) {
        if (c->stage[i]) (void)hipHostFree(c->stage[i]);
        if (c->staged[i]) (void)hipEventDestroy(c->staged[i]);
    }
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
}

}  // extern "C"

namespace {

constexpr size_t kStageBytes = size_t(64) << 20;  // per pinned staging buffer

// Database keys (pageable host memory) to the device: 64 MiB pieces copied
// into two pinned buffers by host threads in parallel, each piece's DMA
// overlapping the copy of the next (a single pageable hipMemcpy moves the
// 880 MB of 110 M keys at a few GB/s).
okm_status stage_keys(okm_classifier *c, const uint64_t *keys, uint64_t nkeys, uint64_t *d_keys) {
    for (int i = 0; i < 2; ++i) {
        if (!c->stage[i]) PHIP(hipHostMalloc(reinterpret_cast<void **>(&c->stage[i]), kStageBytes, hipHostMallocDefault));
        if (!c->staged[i]) PHIP(hipEventCreateWithFlags(&c->staged[i], hipEventDisableTiming));
    }
    const uint8_t *src = reinterpret_cast<const uint8_t *>(keys);
    uint8_t *dst = reinterpret_cast<uint8_t *>(d_keys);
    const size_t bytes = nkeys * sizeof(uint64_t);
    const unsigned nthr = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    for (size_t off = 0, piece = 0; off < bytes; off += kStageBytes, ++piece) {
        const int b = (int)(piece & 1);
        const size_t len = std::min(kStageBytes, bytes - off);
        PHIP(hipEventSynchronize(c->staged[b]));  // the DMA that last read this buffer is done
        const size_t part = (len + nthr - 1) / nthr;
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nthr && (size_t)t * part < len; ++t) {
            const size_t o = (size_t)t * part, l = std::min(part, len - o);
            th.emplace_back([=] { memcpy(c->stage[b] + o, src + off + o, l); });
        }
        for (auto &x : th) x.join();
        PHIP(hipMemcpyAsync(dst + off, c->stage[b], len, hipMemcpyHostToDevice, c->st));
        PHIP(hipEventRecord(c->staged[b], c->st));
    }
    return OKM_OK;
}

// classify.rs:215-308 over device-resident database keys (ref_offsets and
// the outputs on the host).
okm_status probe_db(okm_classifier *c, const ull *d_keys, const uint64_t *ref_offsets, uint64_t n_refs,
                    uint64_t *ref_matched, uint64_t *ref_sum_depth, uint64_t *db_union, uint64_t *db_matched,
                    uint64_t *db_sum_depth) {
    const uint64_t nkeys = ref_offsets[n_refs] - ref_offsets[0];
    const uint64_t ucap = pow2_at_least(2 * nkeys);
    PTRY(c->offs.ensure((n_refs + 1) * sizeof(uint64_t)));
    PTRY(c->uset.ensure((ucap + 1) * sizeof(ull)));
    PTRY(c->per_ref.ensure(n_refs * sizeof(ulonglong2)));
    std::vector<uint64_t> off(ref_offsets, ref_offsets + n_refs + 1);
    for (auto &v : off) v -= ref_offsets[0];
    ull *uslots = (ull *)c->uset.p;
    PHIP(hipMemcpyAsync(c->offs.p, off.data(), off.size() * sizeof(uint64_t), hipMemcpyHostToDevice, c->st));
    PHIP(hipMemsetAsync(uslots, 0xFF, ucap * sizeof(ull), c->st));
    PHIP(hipMemsetAsync(uslots + ucap, 0, sizeof(ull), c->st));
    PHIP(hipMemsetAsync(c->per_ref.p, 0, n_refs * sizeof(ulonglong2), c->st));
    PHIP(hipMemsetAsync(c->d_ctr, 0, 3 * sizeof(ull), c->st));
    const SetTab u{uslots, ucap - 1, 64u - log2_exact(ucap)};
    const uint64_t threads = (nkeys + kCPer - 1) / kCPer;
    const uint64_t blocks = (threads + kProbeBlock - 1) / kProbeBlock;
    if (blocks > 0x7FFFFFFFull) return fail(OKM_E_ARG, "okm_classifier_probe_db: too many keys");
    hipLaunchKernelGGL(k_classify, dim3((uint32_t)blocks), dim3(kProbeBlock), 0, c->st, d_keys, nkeys,
                       (const ull *)c->offs.p, n_refs, c->tab(), u, (ulonglong2 *)c->per_ref.p, c->d_ctr);
    PHIP(hipGetLastError());
    std::vector<ulonglong2> pr(n_refs);
    ull tot[3];
    PHIP(hipMemcpyAsync(pr.data(), c->per_ref.p, n_refs * sizeof(ulonglong2), hipMemcpyDeviceToHost, c->st));
    PHIP(hipMemcpyAsync(tot, c->d_ctr, 3 * sizeof(ull), hipMemcpyDeviceToHost, c->st));
    PHIP(hipStreamSynchronize(c->st));
    for (uint64_t r = 0; r < n_refs; ++r) {
        ref_matched[r] = pr[r].x;
        ref_sum_depth[r] = pr[r].y;
    }
    *db_union = tot[0];
    *db_matched = tot[1];
    *db_sum_depth = tot[2];
    return OKM_OK;
}

// Argument checks shared by both entry points; *nkeys = the database's keys.
okm_status probe_args(okm_classifier *c, const uint64_t *ref_offsets, uint64_t n_refs, uint64_t *ref_matched,
                      uint64_t *ref_sum_depth, uint64_t *db_union, uint64_t *db_matched, uint64_t *db_sum_depth,
                      uint64_t *nkeys) {
    *nkeys = 0;
    if (!c || !db_union || !db_matched || !db_sum_depth) return fail(OKM_E_ARG, "null argument");
    *db_union = *db_matched = *db_sum_depth = 0;
    if (n_refs == 0) return OKM_OK;
    if (!ref_offsets || !ref_matched || !ref_sum_depth) return fail(OKM_E_ARG, "null argument");
    for (uint64_t r = 0; r < n_refs; ++r) {
        if (ref_offsets[r + 1] < ref_offsets[r]) return fail(OKM_E_ARG, "ref_offsets not ascending");
        ref_matched[r] = ref_sum_depth[r] = 0;
    }
    *nkeys = ref_offsets[n_refs] - ref_offsets[0];
    return OKM_OK;
}

}  // namespace

extern "C" {

okm_status okm_classifier_probe_db(okm_classifier *c, const uint64_t *keys, const uint64_t *ref_offsets,
                                   uint64_t n_refs, uint64_t *ref_matched, uint64_t *ref_sum_depth,
                                   uint64_t *db_union, uint64_t *db_matched, uint64_t *db_sum_depth) {
    uint64_t nkeys = 0;
    PTRY(probe_args(c, ref_offsets, n_refs, ref_matched, ref_sum_depth, db_union, db_matched, db_sum_depth, &nkeys));
    if (nkeys == 0) return OKM_OK;
    if (!keys) return fail(OKM_E_ARG, "null keys");
    PHIP(hipSetDevice(c->device));
    PTRY(c->keys.ensure(nkeys * sizeof(uint64_t)));
    PTRY(stage_keys(c, keys + ref_offsets[0], nkeys, (uint64_t *)c->keys.p));
    return probe_db(c, (const ull *)c->keys.p, ref_offsets, n_refs, ref_matched, ref_sum_depth, db_union, db_matched,
                    db_sum_depth);
}

okm_status okm_classifier_probe_db_device(okm_classifier *c, const uint64_t *d_keys, const uint64_t *ref_offsets,
                                          uint64_t n_refs, uint64_t *ref_matched, uint64_t *ref_sum_depth,
                                          uint64_t *db_union, uint64_t *db_matched, uint64_t *db_sum_depth) {
    uint64_t nkeys = 0;
    PTRY(probe_args(c, ref_offsets, n_refs, ref_matched, ref_sum_depth, db_union, db_matched, db_sum_depth, &nkeys));
    if (nkeys == 0) return OKM_OK;
    if (!d_keys) return fail(OKM_E_ARG, "null keys");
    PHIP(hipSetDevice(c->device));
    return probe_db(c, (const ull *)d_keys + ref_offsets[0], ref_offsets, n_refs, ref_matched, ref_sum_depth,
                    db_union, db_matched, db_sum_depth);
}

}  // extern "C"
