// okm_count.hip — LDS counting of key-range partitions ("items").
//
// Replaces the DashMap RMW of count.rs:31-34 and the sort of count.rs:119 for
// one key range at a time.  One workgroup per item (items dealt to blocks by
// blockIdx stride; an LDS-broadcast dynamic queue deadlocked under hipcc's
// structuriser).
//
// An item is a contiguous key range whose keys share all bits above its
// `rem_bits` remaining bits.  Its "home" is the next kHomeBits bits (monotone in
// the key), so homes are key sub-ranges in order.  Three modes:
//
//  tag mode (rem_bits > kHomeBits, at most kCapI instances — the planner
//  guarantees it): every home has a TAG slot.  One 64-bit LDS CAS per
//  instance: the first key to reach a home claims the tag, and every instance
//  of the tag key just adds to the home's packed counter.  At 4x-coverage
//  reads ~88 % of instances end there (a home holds 0.3 distinct keys on
//  average).  Only the other ("rest") instances are counting-sorted by home
//  into LDS; each thread then owns 4 consecutive homes, insertion-sorts its
//  (small) rest slice and emits, per home in order, the rest keys merged with
//  the tag key.  Two block scans (rest offsets, distinct counts) place
//  everything.  Per-thread loops run over REST instances only, which is what
//  keeps the wave's slowest lane — that a divergent loop waits for — short.
//
//  full mode (fallback: more rest instances than the rest buffer holds, e.g.
//  inputs whose keys are all distinct): all instances counting-sorted by home,
//  per-thread insertion sort + run-length encoding over the same LDS.
//
//  dense mode (rem_bits <= kHomeBits): the key IS its slot; direct-address
//  counters in LDS take any number of instances (small k, or keys the planner
//  could not split further).
#include "okm_dev_common.h"

namespace okm {

constexpr int kCountWpe = 8;  // waves per EU floor of the unweighted tag kernel: 4 blocks/CU (64 VGPRs)
constexpr int kFullHomeBitsW = 12;  // full mode, K128 keys: 4096 homes (~1 key each at 4096 instances)

// Threads per counting workgroup: 512, 4096-instance items (256 threads and
// 1024 homes measured count -9 % but partition +8 %, profiles/AB_LOG.md)
constexpr int kCB = 512;
constexpr int kPer = 8;                   // instances per thread (tag / full modes)
constexpr int kCapI = kCB * kPer;         // instances per tag/full-mode item (4096)
constexpr int kHomeBits = kCB == 512 ? 11 : 10;
constexpr int kHomes = 1 << kHomeBits;    // 2048 homes
constexpr int kHomesPer = kHomes / kCB;   // homes owned by one thread (4)
constexpr int kDenseBits = kHomeBits;     // dense mode: rem_bits <= this
constexpr int kLoadU = 4;                 // dense mode: loads in flight per thread

// LDS carve-up (bytes).  Tag mode: tag[kHomes] u64, tag counts (u16 pairs /
// u64), three u16-pair per-home arrays (rest counts -> rest offsets, rest
// distinct -> output offsets, rest keys below the tag), then the rest buffer
// (keys, weights, first-occurrence flags).  Unweighted: 40,896 + 32 B of scan
// scratch, so that 3-4 workgroups fit in 160 KiB.
constexpr int kTagBytes = kHomes * 8;
constexpr int kPairBytes = kHomes * 2;  // one u16 per home, packed in pairs
template <bool W> struct Lds {
    static constexpr int kTcntBytes = W ? kHomes * 8 : kPairBytes;
    static constexpr int kRc = kTagBytes + kTcntBytes;   // byte offsets of the u16-pair arrays
    static constexpr int kHd = kRc + kPairBytes;
    static constexpr int kLt = kHd + kPairBytes;
    static constexpr int kFixed = kLt + kPairBytes;
    static constexpr int kRestEntry = W ? 17 : 9;        // key (+ weight) + first flag
    static constexpr int kFullBytes = kCapI * 8 * (W ? 2 : 1) + kPairBytes;  // full mode: keys (+w) + counters
    static constexpr int kBytes = W ? kFixed + 2048 * kRestEntry : 40896 / (512 / kCB);
    static constexpr int kRest = ((kBytes - kFixed) / kRestEntry) & ~15;
    static constexpr int kRestIters = (kRest + kCB - 1) / kCB;
    static_assert(kFullBytes <= kBytes, "full mode must fit the carve-up");
    static_assert(kHomes * 12 <= kBytes, "dense mode must fit the carve-up");
};

uint32_t count_item_capacity() { return kCapI; }
uint32_t count_dense_bits() { return kDenseBits; }

template <bool W>
struct CountType {
    typedef uint32_t T;
};
template <>
struct CountType<true> {
    typedef ull T;
};

__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// Block-wide exclusive scan (u32); returns the block total in *total.  Two
// barriers (LDS-only ones when LDS_ONLY: see lds_only_sync).
__device__ __forceinline__ void lds_only_sync();
template <bool LDS_ONLY = false>
__device__ __forceinline__ uint32_t block_excl_scan32(uint32_t v, uint32_t *wsum, uint32_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan32(v);
    if (lane == 63) wsum[wid] = inc;
    if (LDS_ONLY) lds_only_sync(); else lds_sync();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kCB / 64; ++w) {
        const uint32_t s = wsum[w];
        wbase += w < wid ? s : 0u;
        tot += s;
    }
    if (LDS_ONLY) lds_only_sync(); else lds_sync();
    *total = tot;
    return wbase + inc - v;
}

// Per-item output counts: u32 (the compaction widens them) -- every count of
// an unweighted launch is < 2^32; a weighted launch stages u32 too when
// `narrow` (the caller redoes it with u64 counts if a count did not fit:
// ctl[0] bit 8) -- else u64.
template <bool W>
__device__ __forceinline__ void store_count(uint64_t *out_counts, uint64_t o, uint64_t c, bool narrow, ull *ctl) {
    if (W && !narrow) {
        out_counts[o] = c;
        return;
    }
    if (W && c > 0xFFFFFFFFull) atomicOr(reinterpret_cast<unsigned int *>(ctl), 8u);
    reinterpret_cast<uint32_t *>(out_counts)[o] = (uint32_t)c;
}

// Top kHomeBits of the r remaining bits (r > kHomeBits): monotone in the key.
__device__ __forceinline__ uint32_t home_of(uint64_t key, uint32_t r) {
    return (uint32_t)(key >> (r - kHomeBits)) & (kHomes - 1);
}
__device__ __forceinline__ uint32_t home_of(const K128 &key, uint32_t r) {
    return (uint32_t)KeyOps<K128>::shr(key, r - kHomeBits) & (kHomes - 1);
}

// Packed u16 pair helpers (home h lives in word h >> 1, half h & 1).
__device__ __forceinline__ uint32_t half_shift(uint32_t h) { return (h & 1u) << 4; }
__device__ __forceinline__ uint32_t half_of(uint32_t word, uint32_t h) { return (word >> half_shift(h)) & 0xFFFFu; }

// Where an item's sorted (key, count) run goes: its slot of the staging array
// at out_off, or -- out_keys == nullptr, "in place" -- over its own input: a
// single-segment item in a level array (okm_engine.hip count_parts) reads all
// its keys before it writes any and has at least as many instances as it
// writes keys, so its run replaces its keys (counts stay at out_counts +
// out_off).  No other item reads that range.
template <typename KT>
__device__ __forceinline__ KT *out_slot_keys(const DevItem &it, uint64_t *out_keys) {
    return out_keys ? reinterpret_cast<KT *>(out_keys) + it.out_off
                    : const_cast<KT *>(reinterpret_cast<const KT *>(it.keys0));
}

// Instances of an item (scalar loop over its segments: block-uniform).
__device__ __forceinline__ uint64_t item_total(const DevItem &it, const DevSeg *__restrict__) {
    return it.total;
}

// Load a tag/full-mode item's instances into registers (flat index over its
// segments; such items hold <= kCapI instances, so 32-bit indices).
template <bool W, typename KT = ull>
__device__ __forceinline__ void load_item(const DevItem &it, const DevSeg *__restrict__ segs, KT (&kk)[kPer],
                                          ull (&ww)[kPer]) {
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        kk[u] = KeyOps<KT>::empty();
        ww[u] = 1;
    }
    if (it.seg_count == 1) {  // one segment: straight from the item (no dependent segment load)
        const uint32_t len = (uint32_t)it.total;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            if ((uint32_t)u * kCB >= len) break;  // block-uniform
            const uint32_t f = (uint32_t)u * kCB + t;
            if (f < len) {
                kk[u] = gload(reinterpret_cast<const KT *>(it.keys0) + f);
                if (W && it.counts0) ww[u] = gload(it.counts0 + f);
            }
        }
        return;
    }
    if (it.seg_count <= 4) {  // a key range of <= 4 sorted runs (k_sorted_items): the descriptors load together
        const uint32_t R = it.seg_count;
        const KT *kb[4];
        const uint64_t *cb[4];
        uint32_t st[5];
        st[0] = 0;
#pragma unroll
        for (uint32_t sg = 0; sg < 4; ++sg) {
            const DevSeg s = segs[it.seg_begin + (sg < R ? sg : 0u)];
            kb[sg] = reinterpret_cast<const KT *>(s.keys);
            cb[sg] = s.counts;
            st[sg + 1] = st[sg] + (sg < R ? (uint32_t)s.len : 0u);
        }
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            if ((uint32_t)u * kCB >= st[4]) break;  // block-uniform
            const uint32_t f = (uint32_t)u * kCB + t;
            if (f < st[4]) {
                const uint32_t sg = (f >= st[1] ? 1u : 0u) + (f >= st[2] ? 1u : 0u) + (f >= st[3] ? 1u : 0u);
                const uint32_t p = f - (sg == 0 ? 0u : sg == 1 ? st[1] : sg == 2 ? st[2] : st[3]);
                const KT *kp = sg == 0 ? kb[0] : sg == 1 ? kb[1] : sg == 2 ? kb[2] : kb[3];
                kk[u] = gload(kp + p);
                if (W) {
                    const uint64_t *cp = sg == 0 ? cb[0] : sg == 1 ? cb[1] : sg == 2 ? cb[2] : cb[3];
                    if (cp) ww[u] = gload(cp + p);
                }
            }
        }
        return;
    }
    uint32_t sbase = 0;
    for (uint32_t sg = 0; sg < it.seg_count; ++sg) {
        const DevSeg s = segs[it.seg_begin + sg];
        const uint32_t len = (uint32_t)s.len;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            if ((uint32_t)u * kCB >= sbase + len) break;  // block-uniform: rows past the segment
            const uint32_t f = (uint32_t)u * kCB + t - sbase;  // wraps for f < sbase
            if (f < len) {
                kk[u] = gload(reinterpret_cast<const KT *>(s.keys) + f);
                if (W && s.counts) ww[u] = gload(s.counts + f);
            }
        }
        sbase += len;
    }
}

// A multi-segment item (sorted runs: every run's slice of one key range) with
// its segment descriptors staged in LDS first — one parallel load instead of
// seg_count dependent ones before the keys can be fetched.  Block-uniform
// call (it contains barriers); seg_count <= kSegCache.
constexpr int kSegCache = 64;
template <bool W, typename KT = ull>
__device__ __forceinline__ void load_item_segs(const DevItem &it, const DevSeg *__restrict__ segs, KT (&kk)[kPer],
                                               ull (&ww)[kPer], const uint64_t **ck, const uint64_t **cc,
                                               uint32_t *coff) {
    const uint32_t t = threadIdx.x;
    const uint32_t R = __builtin_amdgcn_readfirstlane(it.seg_count);
    lds_sync();  // the previous tag item's last step may still read the rest buffer
    if (t < R) {
        const DevSeg s = segs[it.seg_begin + t];
        ck[t] = s.keys;
        cc[t] = s.counts;
        coff[t + 1] = (uint32_t)s.len;
    }
    lds_sync();
    if (t == 0) {
        coff[0] = 0;
        for (uint32_t r = 0; r < R; ++r) coff[r + 1] += coff[r];
    }
    lds_sync();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        kk[u] = KeyOps<KT>::empty();
        ww[u] = 1;
        const uint32_t f = (uint32_t)u * kCB + t;
        if (f < coff[R]) {
            uint32_t lo = 0, hi = R;  // segment of f: last r with coff[r] <= f
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (coff[mid] <= f) lo = mid; else hi = mid;
            }
            const uint32_t p = f - coff[lo];
            kk[u] = gload(reinterpret_cast<const KT *>(ck[lo]) + p);
            if (W && cc[lo]) ww[u] = gload(cc[lo] + p);
        }
    }
}

// Tag-mode LDS state between items: all tags empty, all counters zero.
template <bool W>
__device__ __forceinline__ void tag_reset(ull *lds) {
    uint32_t *p = reinterpret_cast<uint32_t *>(lds);
    lds_sync();
    for (int j = threadIdx.x; j < kHomes; j += kCB) lds[j] = kEmptyKey;
    for (int j = kTagBytes / 4 + threadIdx.x; j < Lds<W>::kFixed / 4; j += kCB) p[j] = 0;
    lds_sync();
}

// ---------------------------------------------------------------------------
// direct output (k_count_slow<KT, W, true>): no staging, no compaction
// ---------------------------------------------------------------------------
//
// Items are taken in index (= key) order from a ticket counter, and each one,
// once it knows its distinct count D, finds its exclusive prefix over the
// items before it with a decoupled look-back over per-item status words
// (aggregate D published at once, inclusive prefix once known), then writes
// its sorted run straight into the caller's table with u64 counts.  A ticket
// is only taken by a running workgroup, and an item waits only on smaller
// tickets, so every wait ends.  A look-back that has waited on one
// predecessor for kLookbackTicks of the device's constant-rate wall clock
// (~15 s at its 100 MHz: a broken invariant, never a slow predecessor) flags
// ctl[0] bit 16 and moves on instead of hanging the device.
struct Direct {
    ull *status;               // [nitems], zero before the launch
    uint64_t *keys, *counts;   // the table (KT keys, u64 counts)
    const ull *base;           // device-side first entry (pipelined groups) or nullptr
    uint32_t item;
    ull *bcast;                // LDS word: the item's first table entry
};
constexpr ull kStAgg = 1ull << 62, kStPre = 2ull << 62, kStVal = kStAgg - 1;
constexpr uint64_t kLookbackTicks = 1500000000ull;

// A barrier that orders LDS only (a workgroup fence on the local address
// space): a look-back load issued before it stays in flight across it.
__device__ __forceinline__ void lds_only_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ ull status_window(const Direct &dir, int64_t hi) {
    const int64_t p = hi - (int64_t)(threadIdx.x & 63u);  // lane t reads hi - t
    return p >= 0 ? __hip_atomic_load(dir.status + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kStPre;
}

// Look-back, first half (wave 0): publish the item's aggregate D and put the
// nearest 64 predecessors' status words in flight.  Other waves get 0.
__device__ __forceinline__ ull lookback_begin(const Direct &dir, uint32_t D) {
    ull v = 0;
    if (threadIdx.x < 64) {
        if (threadIdx.x == 0)
            __hip_atomic_store(dir.status + dir.item, (dir.item ? kStAgg : kStPre) | (ull)D, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        v = status_window(dir, (int64_t)dir.item - 1);
    }
    return v;
}

// Second half: sum the window's aggregates back to the nearest inclusive
// prefix (64 predecessors per round trip, waiting on any not yet published),
// publish this item's prefix.  Block-uniform call (a barrier); returns the
// item's first table entry.
__device__ __forceinline__ uint64_t lookback_end(const Direct &dir, uint32_t D, ull v, ull *ctl) {
    const uint32_t t = threadIdx.x;
    if (t < 64) {
        const uint32_t item = dir.item;
        ull excl = 0;
        int64_t hi = (int64_t)item - 1;
        uint64_t wait_from = 0;  // wall clock at the first wait on the current window
        bool waiting = false;
        while (hi >= 0) {
            const uint64_t pre = __ballot((v >> 62) == 2);
            const uint64_t wait = __ballot((v >> 62) == 0);
            const uint64_t upto = ((pre & (~pre + 1)) << 1) - 1;  // lanes up to the nearest prefix (all if none)
            if (wait & upto) {
                const uint64_t now = wall_clock64();
                if (!waiting) {
                    waiting = true;
                    wait_from = now;
                } else if (now - wait_from > kLookbackTicks) {
                    if (t == 0) atomicOr(reinterpret_cast<unsigned int *>(ctl), 16u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                v = status_window(dir, hi);
                continue;
            }
            waiting = false;
            ull a = ((upto >> t) & 1ull) ? (v & kStVal) : 0ull;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) a += __shfl_xor(a, d, 64);
            excl += a;
            if (pre) break;
            hi -= 64;
            v = status_window(dir, hi);
        }
        if (t == 0) {
            if (item)
                __hip_atomic_store(dir.status + item, kStPre | (excl + D), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            *dir.bcast = excl + (dir.base ? *dir.base : 0ull);
        }
    }
    lds_sync();
    const ull o = *dir.bcast;
    // (readfirstlane returns int: widen through uint32_t, never sign-extend)
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(o >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)o);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t lookback(const Direct &dir, uint32_t D, ull *ctl) {
    return lookback_end(dir, D, lookback_begin(dir, D), ctl);
}

// ---------------------------------------------------------------------------
// full mode (fallback): every instance counting-sorted by home
// ---------------------------------------------------------------------------

// Full-mode LDS bytes: keys (+ weights), then the home counters, which the
// run starts (u16 [kCapI + 1]) reuse once the homes are dead.
template <bool W, typename KT, int HB>
constexpr int full_lds_bytes() {
    return kCapI * ((int)sizeof(KT) + (W ? 8 : 0)) + ((1 << HB) * 2 > (kCapI + 16) * 2 ? (1 << HB) * 2 : (kCapI + 16) * 2);
}

// HB: home bits.  K128 items (k > 32, ~all keys distinct) take 4096 homes, so
// a home holds ~1 key and each instance's rank scan reads ~1 key (random
// 16-B LDS reads are the kernel's most bank-conflicted accesses).
// DIRECT (dir): the item's distinct count is taken from the rank pass, so its
// aggregate is published and the look-back's first loads fly while the
// sorted run is built (LDS-only barriers until the run is written).
template <bool W, typename KT, int HB = kHomeBits, bool DIRECT = false>
__device__ __forceinline__ uint32_t full_item(const DevItem &it, uint32_t nrows, const KT (&kk)[kPer],
                                              const ull (&ww)[kPer], ull *lds, uint32_t *wsum,
                                              uint64_t *__restrict__ out_keys_raw, uint64_t *__restrict__ out_counts,
                                              bool nowrite, bool narrow, ull *ctl, const Direct *dir = nullptr) {
    constexpr uint32_t kH = 1u << HB;         // homes (key sub-ranges in order)
    constexpr uint32_t kHW = kH / 2 / kCB;    // u16-pair counter words per thread (2 or 4)
    static_assert(kHW >= 1 && kH / 2 == kHW * kCB, "whole counter words per thread");
    const uint32_t t = threadIdx.x;
    const uint32_t r = it.rem_bits;
    const uint64_t out_off = it.out_off;
    KT *okeys = out_slot_keys<KT>(it, out_keys_raw);
    KT *sk = reinterpret_cast<KT *>(lds);
    ull *sw = reinterpret_cast<ull *>(sk + kCapI);
    uint32_t *hc = reinterpret_cast<uint32_t *>(sw + (W ? kCapI : 0));
    uint16_t *first = reinterpret_cast<uint16_t *>(hc);  // [D + 1]: run starts in sk (the homes are dead by then)
    lds_sync();  // the previous item's LDS state is dead
#pragma unroll
    for (uint32_t q = 0; q < kHW; ++q) hc[kHW * t + q] = 0;
    if (DIRECT && t == 0) wsum[kCB / 64] = 0;  // first occurrences (the rank pass)
    lds_sync();
    uint32_t hp[kPer];  // home << 16 | pos
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        if ((uint32_t)u >= nrows) break;  // block-uniform
        hp[u] = 0;
        if (!KeyOps<KT>::is_empty(kk[u])) {
            const uint32_t h = (uint32_t)KeyOps<KT>::shr(kk[u], r - HB) & (kH - 1u);  // r > kDenseBits >= HB - 1
            const uint32_t o = atomicAdd(&hc[h >> 1], 1u << half_shift(h));
            hp[u] = (h << 16) | half_of(o, h);
        }
    }
    lds_sync();
    uint32_t wv[kHW];
    uint32_t n = 0;
#pragma unroll
    for (uint32_t q = 0; q < kHW; ++q) {
        wv[q] = hc[kHW * t + q];
        n += (wv[q] & 0xFFFFu) + (wv[q] >> 16);
    }
    uint32_t ntot;
    const uint32_t a = block_excl_scan32(n, wsum, &ntot);
    {
        uint32_t run = a;
#pragma unroll
        for (uint32_t q = 0; q < kHW; ++q) {
            const uint32_t lo = run;
            run += wv[q] & 0xFFFFu;
            hc[kHW * t + q] = lo | (run << 16);
            run += wv[q] >> 16;
        }
    }
    lds_sync();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        if ((uint32_t)u >= nrows) break;
        if (!KeyOps<KT>::is_empty(kk[u])) {
            const uint32_t h = hp[u] >> 16;
            const uint32_t dst = half_of(hc[h >> 1], h) + (hp[u] & 0xFFFFu);
            sk[dst] = kk[u];
            if (W) sw[dst] = ww[u];
        }
    }
    lds_sync();
    uint32_t m = 0;  // run-start flags of positions p0 .. p0 + 7 (p0 = 8t)
    constexpr int kPerT = kCapI / kCB;  // 8 positions per thread
    static_assert(kPerT == 8, "8 flag bits per thread");
    const uint32_t p0 = t * kPerT;
    // every instance ranks itself inside its home (keys below it, and equal
    // keys at earlier positions) and moves there: homes are key ranges in
    // order, so this sorts the item; loops run over one home's keys (~2 at
    // k=63, whose keys are ~98 % distinct) instead of a thread's whole slice
    uint32_t dst[kPer];
    uint32_t nfirst = 0;  // DIRECT: instances with no equal key before them (= distinct keys)
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        dst[u] = ~0u;
        if ((uint32_t)u >= nrows) break;
        if (!KeyOps<KT>::is_empty(kk[u])) {
            const uint32_t h = hp[u] >> 16;
            const uint32_t hs = half_of(hc[h >> 1], h);
            const uint32_t he = h + 1 < kH ? half_of(hc[(h + 1) >> 1], h + 1) : ntot;
            const uint32_t me = hs + (hp[u] & 0xFFFFu);
            uint32_t rank = hs;
            bool dup = false;
            for (uint32_t q = hs; q < he; ++q) {
                const KT y = sk[q];
                const bool before = q < me && KeyOps<KT>::eq(y, kk[u]);
                rank += (KeyOps<KT>::lt(y, kk[u]) || before) ? 1u : 0u;
                dup = dup || before;
            }
            dst[u] = rank;
            nfirst += dup ? 0u : 1u;
        }
    }
    if (DIRECT) {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) nfirst += __shfl_xor(nfirst, d, 64);
        if ((t & 63u) == 0) atomicAdd(&wsum[kCB / 64], nfirst);
    }
    lds_sync();  // every read of the home-ordered keys is done
    uint32_t De = 0;
    ull lbv = 0;
    if (DIRECT) {
        De = __builtin_amdgcn_readfirstlane(wsum[kCB / 64]);
        lbv = lookback_begin(*dir, De);
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        if ((uint32_t)u >= nrows) break;
        if (dst[u] != ~0u) {
            sk[dst[u]] = kk[u];
            if (W) sw[dst[u]] = ww[u];
        }
    }
    if (DIRECT) lds_only_sync(); else lds_sync();
    // count.rs:33: a key's count = its run's length (weight); flag run starts.
    // The flags are taken in rows of lane-contiguous positions (conflict-free
    // LDS reads; a thread's own 8 consecutive keys sit 128 B apart from its
    // neighbours' and read 8-way bank-conflicted as K128) into one ballot
    // word per wave and row, in the dead home counters
    uint64_t *fm = reinterpret_cast<uint64_t *>(hc);  // [kCapI / 64] run-start masks
    static_assert(kCapI / 64 * 8 <= (int)kH * 2, "run-start masks fit the home counters");
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const uint32_t p = (uint32_t)i * kCB + t;
        bool f = false;
        if (p < ntot) f = p == 0 || !KeyOps<KT>::eq(sk[p], sk[p - 1]);
        const uint64_t b = __ballot(f);
        if ((t & 63u) == 0) fm[(uint32_t)i * (kCB / 64) + (t >> 6)] = b;
    }
    if (DIRECT) lds_only_sync(); else lds_sync();
    const uint32_t rp = p0 % kCB;
    m = (uint32_t)(fm[(p0 / kCB) * (kCB / 64) + rp / 64] >> (rp % 64)) & 0xFFu;
    uint32_t D;
    {
        uint32_t q = block_excl_scan32<DIRECT>((uint32_t)__builtin_popcount(m), wsum, &D);
#pragma unroll
        for (int j = 0; j < kPerT; ++j)
            if (m & (1u << j)) first[q++] = (uint16_t)(p0 + j);
        if (t == 0) first[D] = (uint16_t)ntot;  // ntot <= kCapI fits u16
    }
    if (DIRECT) lds_only_sync(); else lds_sync();
    if (DIRECT) {  // straight into the table at the item's prefix
        if (De != D && t == 0) atomicOr(reinterpret_cast<unsigned int *>(ctl), 32u);  // never: both count runs
        const uint64_t o0 = lookback_end(*dir, De, lbv, ctl);
        KT *dk = reinterpret_cast<KT *>(dir->keys) + o0;
        for (uint32_t p = t; p < D; p += kCB) {
            const uint32_t b = first[p], e = first[p + 1];
            dk[p] = sk[b];
            ull c = 0;
            if (W)
                for (uint32_t i = b; i < e; ++i) c += sw[i];
            else
                c = e - b;
            dir->counts[o0 + p] = c;
        }
        return __builtin_amdgcn_readfirstlane(D);
    }
    for (uint32_t p = t; p < (nowrite ? 0u : D); p += kCB) {
        const uint32_t b = first[p], e = first[p + 1];
        okeys[p] = sk[b];
        ull c = 0;
        if (W)
            for (uint32_t i = b; i < e; ++i) c += sw[i];
        else
            c = e - b;
        store_count<W>(out_counts, out_off + p, c, narrow, ctl);
    }
    return __builtin_amdgcn_readfirstlane(D);
}

// ---------------------------------------------------------------------------
// tag mode
// ---------------------------------------------------------------------------

constexpr uint32_t kDeferred = ~0u;

template <bool W, bool NW = false>
__device__ __forceinline__ uint32_t tag_item(const DevItem &it, const DevSeg *__restrict__ segs, uint32_t nrows,
                                             const ull (&kk)[kPer], const ull (&ww)[kPer], ull *lds, uint32_t *wsum,
                                             uint64_t *__restrict__ out_keys, uint64_t *__restrict__ out_counts,
                                             bool narrow, ull *ctl) {
    const uint32_t r = it.rem_bits;
    const uint64_t out_off = it.out_off;
    ull *okeys = out_slot_keys<ull>(it, out_keys);
    typedef Lds<W> L;
    typedef typename CountType<W>::T CT;
    const uint32_t t = threadIdx.x;
    char *base = reinterpret_cast<char *>(lds);
    ull *tag = lds;
    uint32_t *tc16 = reinterpret_cast<uint32_t *>(lds + kHomes);
    ull *tc64 = lds + kHomes;
    uint32_t *rc = reinterpret_cast<uint32_t *>(base + L::kRc);  // rest counts, then rest offsets
    uint32_t *hd = reinterpret_cast<uint32_t *>(base + L::kHd);  // rest distinct, then output offsets
    uint32_t *lt = reinterpret_cast<uint32_t *>(base + L::kLt);  // rest distinct keys below the tag
    ull *rk = reinterpret_cast<ull *>(base + L::kFixed);
    ull *rw = rk + L::kRest;
    uint8_t *rf = reinterpret_cast<uint8_t *>(rk + (W ? 2 : 1) * L::kRest);

    // 1. claim / count tags; rest instances take a slot in their home's run
    //    (row by row: batching the rows' CASes before consuming them measured
    //    slower, 1.66 -> 1.71-1.78 ms on C2 at 2 / 4 rows per batch)
    uint32_t hp[kPer];  // rest: home << 16 | pos; otherwise ~0
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        if ((uint32_t)u >= nrows) break;  // block-uniform
        hp[u] = ~0u;
        const ull x = kk[u];
        if (x != kEmptyKey) {
            const uint32_t h = home_of(x, r);
            const ull old = atomicCAS(&tag[h], kEmptyKey, x);
            if (old == kEmptyKey || old == x) {  // DashMap entry().or_insert().fetch_add() (count.rs:31-34)
                if (W)
                    atomicAdd(&tc64[h], ww[u]);
                else
                    atomicAdd(&tc16[h >> 1], 1u << half_shift(h));  // <= 4096 per item: no carry
            } else {
                const uint32_t o = atomicAdd(&rc[h >> 1], 1u << half_shift(h));
                hp[u] = (h << 16) | half_of(o, h);
            }
        }
    }
    lds_sync();
    // 2. rest offsets: thread t owns homes [4t, 4t+4) = words 2t, 2t+1
    //    (late reset: the previous item's home offsets, read by its last step
    //    before this item's first barrier, are cleared here)
    hd[2 * t] = hd[2 * t + 1] = 0;
    {
        const uint32_t w0 = rc[2 * t], w1 = rc[2 * t + 1];
        const uint32_t c0 = w0 & 0xFFFFu, c1 = w0 >> 16, c2 = w1 & 0xFFFFu;
        uint32_t rtot;
        const uint32_t a = block_excl_scan32(c0 + c1 + c2 + (w1 >> 16), wsum, &rtot);
        if (__builtin_amdgcn_readfirstlane(rtot) > (uint32_t)L::kRest) {  // block-uniform
            tag_reset<W>(lds);
            return kDeferred;  // too many rest instances: k_count_slow takes the item
        }
        rc[2 * t] = a | ((a + c0) << 16);
        rc[2 * t + 1] = (a + c0 + c1) | ((a + c0 + c1 + c2) << 16);
        if (t == 0) wsum[kCB / 64] = rtot;  // rest total, read by every rest position below
    }
    lds_sync();
    // 3. scatter rest instances into home order
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        if ((uint32_t)u >= nrows) break;
        if (hp[u] != ~0u) {
            const uint32_t h = hp[u] >> 16;
            const uint32_t dst = half_of(rc[h >> 1], h) + (hp[u] & 0xFFFFu);
            rk[dst] = kk[u];
            if (W) rw[dst] = ww[u];
        }
    }
    lds_sync();
    // 4. rest positions, one per lane: count, first occurrence in the home's
    //    run, and what the home's distinct count / tag rank must include
    const uint32_t rtot = __builtin_amdgcn_readfirstlane(wsum[kCB / 64]);
    ull px[L::kRestIters];
    CT pc[L::kRestIters];
    uint32_t prange[L::kRestIters];  // hs << 16 | he; 0 = not a first occurrence
#pragma unroll
    for (int k = 0; k < L::kRestIters; ++k) {
        prange[k] = 0;
        if ((uint32_t)k * kCB >= rtot) break;  // block-uniform
        const uint32_t p = (uint32_t)k * kCB + t;
        if (p < rtot) {
            const ull x = rk[p];
            const uint32_t h = home_of(x, r);
            const uint32_t hs = half_of(rc[h >> 1], h);
            const uint32_t he = h + 1 < (uint32_t)kHomes ? half_of(rc[(h + 1) >> 1], h + 1) : rtot;
            CT c = 0;
            bool first = true;
            for (uint32_t q = hs; q < he; ++q) {
                const bool eq = rk[q] == x;
                c += eq ? (W ? (CT)rw[q] : (CT)1) : (CT)0;
                first = first && !(eq && q < p);
            }
            rf[p] = first ? 1 : 0;
            px[k] = x;
            pc[k] = c;
            if (first) {
                // bit 31: the home's tag sorts below x (a rest key never equals its
                // home's tag), so step 6b need not read the tags again
                const ull tgh = tag[h];
                prange[k] = (hs << 16) | he | (tgh < x ? 0x80000000u : 0u);
                atomicAdd(&hd[h >> 1], 1u << half_shift(h));
                if (x < tgh) atomicAdd(&lt[h >> 1], 1u << half_shift(h));
            }
        }
    }
    lds_sync();
    // 5. output offsets per home: [tag] + rest distinct keys
    ull tg[kHomesPer];
    uint32_t ho[kHomesPer];
    uint32_t D;
    // late reset: this thread's homes are read here for the last time (step 4,
    // the last reader of other threads' tags and rest offsets, is behind the
    // barrier above), so they are cleared at once for the next item
    uint32_t nw0 = 0, nw1 = 0;  // tag counts (u16 pairs)
    ull tw[W ? kHomesPer : 1];   // tag weights (weighted launches)
    const uint32_t lw0 = lt[2 * t], lw1 = lt[2 * t + 1];  // rest keys below the tag
    lt[2 * t] = lt[2 * t + 1] = 0;
    rc[2 * t] = rc[2 * t + 1] = 0;
    if (W) {
#pragma unroll
        for (int q = 0; q < kHomesPer; ++q) {
            tw[q] = tc64[kHomesPer * t + q];
            tc64[kHomesPer * t + q] = 0;
        }
    } else {
        nw0 = tc16[2 * t];
        nw1 = tc16[2 * t + 1];
        tc16[2 * t] = tc16[2 * t + 1] = 0;
    }
    {
        const uint32_t w0 = hd[2 * t], w1 = hd[2 * t + 1];
        uint32_t dq[kHomesPer] = {w0 & 0xFFFFu, w0 >> 16, w1 & 0xFFFFu, w1 >> 16};
        uint32_t d = 0;
#pragma unroll
        for (int q = 0; q < kHomesPer; ++q) {
            tg[q] = tag[kHomesPer * t + q];
            tag[kHomesPer * t + q] = kEmptyKey;
            dq[q] += tg[q] != kEmptyKey;
            ho[q] = d;
            d += dq[q];
        }
        const uint32_t od = block_excl_scan32(d, wsum, &D);
#pragma unroll
        for (int q = 0; q < kHomesPer; ++q) ho[q] += od;
        hd[2 * t] = ho[0] | (ho[1] << 16);
        hd[2 * t + 1] = ho[2] | (ho[3] << 16);
    }
    lds_sync();
    // 6a. tags: rank = home offset + rest distinct keys below the tag
    {
        const uint32_t lq[kHomesPer] = {lw0 & 0xFFFFu, lw0 >> 16, lw1 & 0xFFFFu, lw1 >> 16};
        uint32_t nq[kHomesPer];
        if (!W) {
            nq[0] = nw0 & 0xFFFFu;
            nq[1] = nw0 >> 16;
            nq[2] = nw1 & 0xFFFFu;
            nq[3] = nw1 >> 16;
        }
#pragma unroll
        for (int q = 0; q < kHomesPer; ++q) {
            if (!NW && tg[q] != kEmptyKey) {
                const uint64_t o = out_off + ho[q] + lq[q];
                okeys[o - out_off] = tg[q];
                const uint64_t cq = W ? (uint64_t)tw[q] : (uint64_t)nq[q];
                store_count<W>(out_counts, o, cq, narrow, ctl);
            }
        }
    }
    // 6b. rest keys: rank = home offset + rest distinct keys below + [tag below]
#pragma unroll
    for (int k = 0; k < L::kRestIters; ++k) {
        if (NW || (uint32_t)k * kCB >= rtot) break;
        if (prange[k]) {
            const ull x = px[k];
            const uint32_t hs = (prange[k] >> 16) & 0x7FFFu, he = prange[k] & 0xFFFFu;
            uint32_t less = 0;
            for (uint32_t q = hs; q < he; ++q) less += (rf[q] && rk[q] < x) ? 1u : 0u;
            const uint32_t h = home_of(x, r);
            const uint32_t tag_below = prange[k] >> 31;
            const uint64_t o = out_off + half_of(hd[h >> 1], h) + less + tag_below;
            okeys[o - out_off] = x;
            store_count<W>(out_counts, o, (uint64_t)pc[k], narrow, ctl);
        }
    }
    // late reset: everything but the home offsets (hd, cleared in the next
    // item's step 2) was cleared in step 5, and nothing read here is written
    // before the next item's first barrier: no trailing barriers, the next
    // item's loads overlap this step
    return __builtin_amdgcn_readfirstlane(D);
}

// ---------------------------------------------------------------------------
// dense mode: direct-address counters (rem_bits <= kDenseBits)
// ---------------------------------------------------------------------------

template <bool W, typename KT>
__device__ __forceinline__ uint32_t dense_item(const DevItem &it, const DevSeg *__restrict__ segs,
                                               uint64_t *__restrict__ out_keys_raw, uint64_t *__restrict__ out_counts,
                                               ull *lds, uint32_t *wsum, bool nowrite, bool narrow, ull *ctl,
                                               const Direct *dir = nullptr) {
    typedef typename CountType<W>::T CT;
    const uint32_t t = threadIdx.x;
    const uint32_t r = it.rem_bits;
    const uint32_t nslots = 1u << r;
    const ull mask = (ull)nslots - 1ull;
    KT *okeys = out_slot_keys<KT>(it, out_keys_raw);
    KT *slot_key = reinterpret_cast<KT *>(lds);               // [kHomes]
    CT *cnt = reinterpret_cast<CT *>(slot_key + kHomes);      // [kHomes]
    lds_sync();  // the previous item's LDS state is dead
    for (uint32_t j = t; j < nslots; j += kCB) cnt[j] = 0;
    lds_sync();
    for (uint32_t sg = 0; sg < it.seg_count; ++sg) {
        const DevSeg s = segs[it.seg_begin + sg];
        const KT *keys = reinterpret_cast<const KT *>(s.keys);
        for (uint64_t base = 0; base < s.len; base += (uint64_t)kCB * kLoadU) {
            KT kk[kLoadU];
            CT ww[kLoadU];
#pragma unroll
            for (int u = 0; u < kLoadU; ++u) {
                const uint64_t idx = base + (uint64_t)u * kCB + t;
                kk[u] = idx < s.len ? gload(keys + idx) : KeyOps<KT>::empty();
                ww[u] = (W && s.counts && idx < s.len) ? (CT)gload(s.counts + idx) : (CT)1;
            }
#pragma unroll
            for (int u = 0; u < kLoadU; ++u) {
                if (!KeyOps<KT>::is_empty(kk[u])) {
                    const uint32_t h = (uint32_t)(KeyOps<KT>::shr(kk[u], 0) & mask);  // the key's remaining bits
                    atomicAdd(&cnt[h], ww[u]);
                    slot_key[h] = kk[u];  // all writers of a slot store the same key
                }
            }
        }
    }
    lds_sync();
    uint32_t d = 0;
    for (uint32_t q = 0; q < kHomesPer; ++q) {
        const uint32_t j = t * kHomesPer + q;
        d += (j < nslots && cnt[j] != 0) ? 1u : 0u;
    }
    uint32_t D;
    uint64_t o = it.out_off + block_excl_scan32(d, wsum, &D);
    if (dir) {  // straight into the table at the item's prefix
        o += lookback(*dir, D, ctl) - it.out_off;
        KT *dk = reinterpret_cast<KT *>(dir->keys);
        for (uint32_t q = 0; q < kHomesPer; ++q) {
            const uint32_t j = t * kHomesPer + q;
            if (j < nslots && cnt[j] != 0) {
                dk[o] = slot_key[j];
                dir->counts[o] = (uint64_t)cnt[j];
                ++o;
            }
        }
        return __builtin_amdgcn_readfirstlane(D);
    }
    for (uint32_t q = 0; q < kHomesPer; ++q) {
        const uint32_t j = t * kHomesPer + q;
        if (!nowrite && j < nslots && cnt[j] != 0) {
            okeys[o - it.out_off] = slot_key[j];
            store_count<W>(out_counts, o, (uint64_t)cnt[j], narrow, ctl);
            ++o;
        }
    }
    return __builtin_amdgcn_readfirstlane(D);
}

// Tag-mode kernel.  Items it cannot take (dense-mode items, rest overflow)
// go to the deferred list defer[ctl[1]++] for k_count_slow, which runs right
// after it: separate kernels keep the rare paths' registers out of this one.
// NW (weighted launches only): count each item's distinct keys into n_out and
// write nothing -- the first pass of an exact-size two-pass count.
template <bool W, bool NW = false, bool NARROW = !W>
__global__ __launch_bounds__(kCB) __attribute__((amdgpu_waves_per_eu(W ? 1 : kCountWpe)))
void k_count_items(const DevItem *__restrict__ items, uint32_t nitems, const DevSeg *__restrict__ segs,
                   uint64_t *__restrict__ out_keys, uint64_t *__restrict__ out_counts, ull *__restrict__ n_out,
                   ull *__restrict__ ctl, uint32_t *__restrict__ defer, const ull *__restrict__ guard,
                   const ull *__restrict__ d_nitems) {
    if (guard && (guard[0] | guard[1])) return;  // speculative launch whose items were not valid
    if (d_nitems) nitems = __builtin_amdgcn_readfirstlane((uint32_t)min((ull)nitems, *d_nitems));
    // items dealt by stride (item = block + k * grid)
    __shared__ __attribute__((aligned(16))) ull lds[Lds<W>::kBytes / 8];
    __shared__ uint32_t wsum[kCB / 64 + 1];
    // multi-segment items: their descriptors are staged in the rest buffer,
    // which is free until tag_item's step 3 (the keys are in registers by then)
    const uint64_t **seg_k = reinterpret_cast<const uint64_t **>(reinterpret_cast<char *>(lds) + Lds<W>::kFixed);
    const uint64_t **seg_c = seg_k + kSegCache;
    uint32_t *seg_off = reinterpret_cast<uint32_t *>(seg_c + kSegCache);
    static_assert(kSegCache * 20 + 4 <= Lds<W>::kRest * 8, "segment cache fits the rest buffer");
    const uint32_t t = threadIdx.x;
    tag_reset<W>(lds);
    // Block-uniform values that steer code containing barriers come from
    // blockIdx / scalar loads (see DESIGN.md on the structuriser).
    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        const DevItem it = items[item];
        const uint64_t total = it.pad == kItemEmpty ? 0 : item_total(it, segs);
        if (total == 0) {  // an empty fan-out slot (block-uniform)
            if (t == 0) n_out[item] = 0;
            continue;
        }
        uint32_t written = kDeferred;
        if (it.rem_bits > (uint32_t)kDenseBits && total <= (uint64_t)kCapI) {
            ull kk[kPer];
            ull ww[kPer];
            // (weighted launches only: the unweighted kernel sits at its 64-VGPR
            // cap and the staged load costs it spills)
            if (W && it.seg_count > 1 && it.seg_count <= (uint32_t)kSegCache)
                load_item_segs<W>(it, segs, kk, ww, seg_k, seg_c, seg_off);
            else
                load_item<W>(it, segs, kk, ww);
            const uint32_t nrows = (uint32_t)((total + kCB - 1) / kCB);  // rows of kk in use (block-uniform)
            written = tag_item<W, NW>(it, segs, nrows, kk, ww, lds, wsum, out_keys, out_counts, NARROW, ctl);
        }
        if (t == 0) {
            if (written == kDeferred)
                defer[atomicAdd(reinterpret_cast<unsigned int *>(ctl + 1), 1u)] = item;
            else
                n_out[item] = written;
        }
    }
}

// Deferred items (defer != nullptr: the ctl[1] items listed there), or every
// item (defer == nullptr: wide keys, which have no tag mode — LDS has no
// 128-bit CAS): dense mode, or full mode (every instance counting-sorted).
// DIRECT (defer == nullptr): items by ticket (ctl[1]) in order, each run
// written straight into the table (fin_*) at its look-back prefix.
template <typename KT, bool W, bool DIRECT = false>
__global__ __launch_bounds__(kCB) __attribute__((amdgpu_waves_per_eu((W && sizeof(KT) > 8) ? 1 : 4))) void k_count_slow(const DevItem *__restrict__ items, uint32_t nitems,
                                                    const DevSeg *__restrict__ segs,
                                                    uint64_t *__restrict__ out_keys,
                                                    uint64_t *__restrict__ out_counts, ull *__restrict__ n_out,
                                                    ull *__restrict__ ctl, const uint32_t *__restrict__ defer,
                                                    const ull *__restrict__ guard, const ull *__restrict__ d_nitems,
                                                    bool nowrite, bool narrow, ull *__restrict__ status,
                                                    uint64_t *__restrict__ fin_keys, uint64_t *__restrict__ fin_counts,
                                                    const ull *__restrict__ fin_base) {
    if (guard && (guard[0] | guard[1])) return;
    // a poisoned table base: an earlier pipelined key-range group was
    // abandoned, so this one is counted again too (nothing may be written;
    // checked once here -- a per-item check in the write path measured 8 %
    // slower on C4)
    if (DIRECT && fin_base && (*fin_base & kBasePoison)) return;
    if (d_nitems) nitems = __builtin_amdgcn_readfirstlane((uint32_t)min((ull)nitems, *d_nitems));
    constexpr int kHB = sizeof(KT) > 8 ? kFullHomeBitsW : kHomeBits;  // full-mode home bits
    // full_item shifts a key by rem_bits - kHB with rem_bits > kDenseBits: the
    // shift stays non-negative only while kHB <= kDenseBits + 1
    static_assert(kHB <= kDenseBits + 1, "full-mode home bits exceed kDenseBits + 1");
    constexpr int kFull = full_lds_bytes<W, KT, kHB>();
    constexpr int kDense = kHomes * ((int)sizeof(KT) + (W ? 8 : 4));
    constexpr int kBytes = kFull > kDense ? kFull : kDense;
    __shared__ __attribute__((aligned(16))) ull lds[kBytes / 8];
    __shared__ uint32_t wsum[kCB / 64 + 1];
    const uint32_t ndefer = defer ? *reinterpret_cast<volatile const unsigned int *>(ctl + 1) : nitems;
    struct Next {
        uint32_t item;
        DevItem it;
        uint64_t total;
    };
    __shared__ uint32_t s_ticket;
    __shared__ ull s_bcast;
    auto next_ticket = [&]() -> uint32_t {
        lds_sync();  // every thread has read the previous ticket
        if (threadIdx.x == 0) s_ticket = atomicAdd(reinterpret_cast<unsigned int *>(ctl + 1), 1u);
        lds_sync();
        return __builtin_amdgcn_readfirstlane(s_ticket);  // (see DESIGN.md on the structuriser)
    };
    for (uint32_t j = DIRECT ? next_ticket() : blockIdx.x; j < ndefer; j = DIRECT ? next_ticket() : j + gridDim.x) {
        Next cur;
        cur.item = defer ? defer[j] : j;
        cur.it = items[cur.item];
        cur.total = cur.it.pad == kItemEmpty ? 0 : item_total(cur.it, segs);
        KT kk[kPer];
        ull ww[kPer];
        if (cur.total != 0 && cur.it.rem_bits > (uint32_t)kDenseBits && cur.total <= (uint64_t)kCapI)
            load_item<W, KT>(cur.it, segs, kk, ww);
        const uint32_t item = cur.item;
        const DevItem it = cur.it;
        const uint64_t total = cur.total;
        const Direct dsc{status, fin_keys, fin_counts, fin_base, item, &s_bcast};
        const Direct *dir = DIRECT ? &dsc : nullptr;
        uint32_t written = 0;
        if (total == 0) {  // an empty fan-out slot (block-uniform)
            if (threadIdx.x == 0) n_out[item] = 0;
            if (DIRECT) (void)lookback(dsc, 0, ctl);  // its successors wait for its status
            continue;
        }
        if (it.rem_bits <= (uint32_t)kDenseBits) {
            written = dense_item<W, KT>(it, segs, out_keys, out_counts, lds, wsum, nowrite, narrow, ctl, dir);
        } else if (total <= (uint64_t)kCapI) {
            written = full_item<W, KT, kHB, DIRECT>(it, (uint32_t)((total + kCB - 1) / kCB), kk, ww, lds, wsum,
                                                    out_keys, out_counts, nowrite, narrow, ctl, dir);
        } else {
            if (threadIdx.x == 0) atomicOr(reinterpret_cast<unsigned int *>(ctl), 2u);  // planner invariant broken
            if (DIRECT) (void)lookback(dsc, 0, ctl);
        }
        if (threadIdx.x == 0) n_out[item] = written;
        lds_sync();  // LDS reuse by the next item
    }
}

void launch_count_items(void *stream, const DevItem *items, uint32_t nitems, const DevSeg *segs,
                        uint64_t *out_keys, uint64_t *out_counts, unsigned long long *n_out,
                        unsigned long long *ctl, uint32_t *defer, bool weighted, bool wide,
                        const unsigned long long *guard, const unsigned long long *d_nitems, bool nowrite,
                        bool narrow) {
    if (!nitems) return;
    hipStream_t s = (hipStream_t)stream;
    // wide (full-mode) count: 8191 workgroups against 4095, k=63 at 1 Gbases
    // count_items 8.61-8.62 vs 8.75-8.78 ms over 3 interleaved runs (16383: 8.60-8.65);
    // the weighted tag kernel (C3's merges) showed no difference at 1023 / 16383
    constexpr uint32_t wide_cap = 8191, weighted_cap = 4095;
    if (wide) {  // every item through the full / dense modes
        const uint32_t grid = nitems < wide_cap ? nitems : wide_cap;  // odd: fan-out slots spread over blocks
        if (weighted)
            hipLaunchKernelGGL((k_count_slow<K128, true>), dim3(grid), dim3(kCB), 0, s, items, nitems, segs, out_keys,
                               out_counts, n_out, ctl, (const uint32_t *)nullptr, guard, d_nitems, nowrite, narrow,
                               (ull *)nullptr, (uint64_t *)nullptr, (uint64_t *)nullptr, (const ull *)nullptr);
        else
            hipLaunchKernelGGL((k_count_slow<K128, false>), dim3(grid), dim3(kCB), 0, s, items, nitems, segs,
                               out_keys, out_counts, n_out, ctl, (const uint32_t *)nullptr, guard, d_nitems, nowrite,
                               narrow, (ull *)nullptr, (uint64_t *)nullptr, (uint64_t *)nullptr, (const ull *)nullptr);
        return;
    }
    // workgroups of the unweighted tag kernel (odd, so fan-out slots spread
    // over blocks).  16383 (~11 C2 items each, 16 generations of the 1024
    // resident workgroups) against 4095: count_items 1.550 vs 1.590-1.600 ms;
    // 2047 1.653, 8191 1.568, 32767 1.563, 65535 1.589, one per item 1.802
    // (profiles/r04_ab_count_grid.txt)
    constexpr uint32_t grid_cap = 16383;
    const uint32_t grid = nitems < grid_cap ? nitems : grid_cap;
    const uint32_t wgrid = nitems < weighted_cap ? nitems : weighted_cap;  // weighted: one workgroup per CU resident
    const uint32_t sgrid = nitems < 1023u ? nitems : 1023u;  // exits at once when nothing was deferred
    if (weighted) {
        if (nowrite)
            hipLaunchKernelGGL((k_count_items<true, true>), dim3(wgrid), dim3(kCB), 0, s, items, nitems, segs,
                               out_keys, out_counts, n_out, ctl, defer, guard, d_nitems);
        else if (narrow)
            hipLaunchKernelGGL((k_count_items<true, false, true>), dim3(wgrid), dim3(kCB), 0, s, items, nitems, segs,
                               out_keys, out_counts, n_out, ctl, defer, guard, d_nitems);
        else
            hipLaunchKernelGGL((k_count_items<true, false, false>), dim3(wgrid), dim3(kCB), 0, s, items, nitems,
                               segs, out_keys, out_counts, n_out, ctl, defer, guard, d_nitems);
        hipLaunchKernelGGL((k_count_slow<ull, true>), dim3(sgrid), dim3(kCB), 0, s, items, nitems, segs, out_keys,
                           out_counts, n_out, ctl, (const uint32_t *)defer, guard, d_nitems, nowrite, narrow,
                           (ull *)nullptr, (uint64_t *)nullptr, (uint64_t *)nullptr, (const ull *)nullptr);
    } else {
        hipLaunchKernelGGL(k_count_items<false>, dim3(grid), dim3(kCB), 0, s, items, nitems, segs, out_keys,
                           out_counts, n_out, ctl, defer, guard, d_nitems);
        hipLaunchKernelGGL((k_count_slow<ull, false>), dim3(sgrid), dim3(kCB), 0, s, items, nitems, segs, out_keys,
                           out_counts, n_out, ctl, (const uint32_t *)defer, guard, d_nitems, nowrite, narrow,
                           (ull *)nullptr, (uint64_t *)nullptr, (uint64_t *)nullptr, (const ull *)nullptr);
    }
}

// Wide keys straight into a caller's table (no staging, no compaction):
// fin_keys / fin_counts are the table at its next entry, or its start when
// fin_base holds the next entry on the device; status: nitems words, zeroed
// by the caller (as is ctl[0..1]).
void launch_count_direct(void *stream, const DevItem *items, uint32_t nitems, const DevSeg *segs,
                         unsigned long long *n_out, unsigned long long *ctl, bool weighted,
                         const unsigned long long *guard, const unsigned long long *d_nitems,
                         unsigned long long *status, uint64_t *fin_keys, uint64_t *fin_counts,
                         const unsigned long long *fin_base) {
    if (!nitems) return;
    hipStream_t s = (hipStream_t)stream;
    // a workgroup takes items until the tickets run out: about the resident count
    const uint32_t grid = nitems < 2048u ? nitems : 2048u;
    if (weighted)
        hipLaunchKernelGGL((k_count_slow<K128, true, true>), dim3(grid), dim3(kCB), 0, s, items, nitems, segs,
                           (uint64_t *)nullptr, (uint64_t *)nullptr, n_out, ctl, (const uint32_t *)nullptr, guard,
                           d_nitems, false, false, status, fin_keys, fin_counts, fin_base);
    else
        hipLaunchKernelGGL((k_count_slow<K128, false, true>), dim3(grid), dim3(kCB), 0, s, items, nitems, segs,
                           (uint64_t *)nullptr, (uint64_t *)nullptr, n_out, ctl, (const uint32_t *)nullptr, guard,
                           d_nitems, false, false, status, fin_keys, fin_counts, fin_base);
}

}  // namespace okm
