// okm_count.hip — LDS counting of key-range partitions ("items").
//
// Replaces the DashMap RMW of count.rs:31-34 and the sort of count.rs:119 for
// one key range at a time.  One workgroup per item (items dealt to blocks by
// blockIdx stride; an LDS-broadcast dynamic queue deadlocked under hipcc's
// structuriser).
//
// The LDS table is ORDER-PRESERVING: an item is a contiguous key range, so a
// key's home slot is the next kHomeBits bits of the key below the item's
// common prefix (monotone in the key), collisions probe forward only and the
// table has a kCap-slot tail instead of wrapping.  Every key then sits in the
// maximal run of occupied slots ("cluster") that contains its home, and
// clusters appear in key order.  After inserting, a key's rank in the sorted
// output is
//     (ordinal of its slot among occupied slots) - (its offset in its cluster)
//   + (number of keys in its cluster that are smaller),
// which costs a few LDS reads per key at the table's load (<= 50 % of the
// home range): no sort network at all.
//
// An item whose distinct keys exceed one pass's capacity (kCap) is processed
// as 2, 4, ... sub-ranges of its remaining key bits, in key order, so any
// item size is correct; the host sizes items so that this is rare.
#include "okm_dev_common.h"

namespace okm {

constexpr int kCB = 512;                  // threads per workgroup
constexpr int kHomeBits = 11;
constexpr int kHomes = 1 << kHomeBits;    // home slots
constexpr int kCap = 2048;                // distinct keys per pass
constexpr int kSlots = kHomes + kCap;     // homes + forward-probe tail (never wraps)
constexpr int kSlotsPer = kSlots / kCB;   // table slots ranked per thread (8)
constexpr int kLoadU = 4;                 // independent key loads in flight per thread

uint32_t count_item_capacity() { return kCap; }

template <bool W>
struct CountType {
    typedef uint32_t T;
};
template <>
struct CountType<true> {
    typedef ull T;
};

// Monotone home slot: the kHomeBits key bits below the top `lg` bits of the
// item's `rem` remaining bits (fewer remaining bits are scaled up).
__device__ __forceinline__ uint32_t home_of(uint64_t key, uint32_t r) {
    if (r >= (uint32_t)kHomeBits) return (uint32_t)(key >> (r - kHomeBits)) & (kHomes - 1);
    return ((uint32_t)key & ((1u << r) - 1u)) << (kHomeBits - r);
}

template <bool W>
__global__ __launch_bounds__(kCB) void k_count_items(const DevItem *__restrict__ items, uint32_t nitems,
                                                     const DevSeg *__restrict__ segs,
                                                     uint64_t *__restrict__ out_keys,
                                                     uint64_t *__restrict__ out_counts,
                                                     ull *__restrict__ n_out, ull *__restrict__ ctl) {
    typedef typename CountType<W>::T CT;
    __shared__ ull tk[kSlots];
    __shared__ CT tc[kSlots];
    __shared__ ull wsum[kCB / 64];
    __shared__ uint32_t s_distinct, s_ovf;

    const uint32_t t = threadIdx.x;
    // Block-uniform values that steer loops containing barriers are kept
    // scalar (blockIdx, readfirstlane of LDS words): hipcc otherwise treats
    // LDS loads as divergent and structurises those loops with exec masks.
    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        const DevItem it = items[item];
        uint32_t lg = 0, sub = 0;  // current pass: sub-range `sub` of 2^lg
        ull written = 0;
        for (;;) {
            for (int j = t; j < kSlots; j += kCB) {
                tk[j] = kEmptyKey;
                tc[j] = 0;
            }
            if (t == 0) {
                s_distinct = 0;
                s_ovf = 0;
            }
            __syncthreads();
            const uint32_t r = it.rem_bits - lg;  // bits below the sub-range id
            const uint64_t smask = (1ull << lg) - 1ull;
            for (uint32_t sg = 0; sg < it.seg_count; ++sg) {
                const DevSeg s = segs[it.seg_begin + sg];
                for (uint64_t base = 0; base < s.len; base += (uint64_t)kCB * kLoadU) {
                    ull kk[kLoadU];
                    CT ww[kLoadU];
#pragma unroll
                    for (int u = 0; u < kLoadU; ++u) {
                        const uint64_t idx = base + (uint64_t)u * kCB + t;
                        kk[u] = idx < s.len ? s.keys[idx] : kEmptyKey;
                        ww[u] = 1;
                        if (W && idx < s.len && s.counts) ww[u] = (CT)s.counts[idx];
                    }
#pragma unroll
                    for (int u = 0; u < kLoadU; ++u) {
                        const ull key = kk[u];
                        if (key == kEmptyKey) continue;
                        if (lg && ((key >> r) & smask) != sub) continue;
                        if (s_ovf) continue;
                        // DashMap entry().or_insert().fetch_add() (count.rs:31-34)
                        for (uint32_t h = home_of(key, r); h < (uint32_t)kSlots; ++h) {
                            const ull old = atomicCAS(&tk[h], (ull)kEmptyKey, key);
                            if (old == kEmptyKey) {
                                if (atomicAdd(&s_distinct, 1u) >= (uint32_t)kCap) s_ovf = 1;
                                atomicAdd(&tc[h], ww[u]);
                                break;
                            }
                            if (old == key) {
                                atomicAdd(&tc[h], ww[u]);
                                break;
                            }
                            if (h == (uint32_t)kSlots - 1) s_ovf = 1;  // tail exhausted
                        }
                    }
                }
            }
            __syncthreads();
            const bool ovf = __builtin_amdgcn_readfirstlane(s_ovf) != 0;
            __syncthreads();
            if (ovf) {  // more than kCap distinct keys in this sub-range: halve it
                ++lg;
                sub <<= 1;
                if (lg > it.rem_bits || lg > 40) {  // cannot happen: 2^11 keys always fit
                    if (t == 0) atomicOr(reinterpret_cast<unsigned int *>(ctl), 2u);
                    break;
                }
                continue;
            }
            // ordinal of every occupied slot (table order)
            const uint32_t s0 = t * kSlotsPer;
            ull rk[kSlotsPer];
            uint32_t mine = 0;
#pragma unroll
            for (int j = 0; j < kSlotsPer; ++j) {
                rk[j] = tk[s0 + j];
                mine += rk[j] != kEmptyKey;
            }
            ull total;
            uint32_t ord = (uint32_t)block_excl_scan<kCB>(mine, wsum, &total);
            const uint32_t D = __builtin_amdgcn_readfirstlane((uint32_t)total);
            const uint64_t o = it.out_off + written;
#pragma unroll
            for (int j = 0; j < kSlotsPer; ++j) {
                const ull key = rk[j];
                if (key == kEmptyKey) continue;
                const uint32_t i = s0 + j;
                uint32_t a = i;
                while (a > 0 && tk[a - 1] != kEmptyKey) --a;  // cluster start
                uint32_t less = 0;
                for (uint32_t q = a; q < (uint32_t)kSlots; ++q) {
                    const ull x = tk[q];
                    if (x == kEmptyKey) break;
                    less += x < key;
                }
                const uint32_t rank = ord - (i - a) + less;  // count.rs:119 order
                out_keys[o + rank] = key;
                out_counts[o + rank] = (uint64_t)tc[i];
                ++ord;
            }
            written += D;
            ++sub;
            __syncthreads();
            if (sub >> lg) break;
        }
        if (t == 0) n_out[item] = written;
    }
}

void launch_count_items(void *stream, const DevItem *items, uint32_t nitems, const DevSeg *segs,
                        uint64_t *out_keys, uint64_t *out_counts, unsigned long long *n_out,
                        unsigned long long *ctl, bool weighted) {
    if (!nitems) return;
    const uint32_t grid = nitems < 2048u ? nitems : 2048u;
    if (weighted)
        hipLaunchKernelGGL(k_count_items<true>, dim3(grid), dim3(kCB), 0, (hipStream_t)stream, items, nitems,
                           segs, out_keys, out_counts, n_out, ctl);
    else
        hipLaunchKernelGGL(k_count_items<false>, dim3(grid), dim3(kCB), 0, (hipStream_t)stream, items, nitems,
                           segs, out_keys, out_counts, n_out, ctl);
}

}  // namespace okm
