// okm_merge.hip — k-way merge of SORTED (key, count) runs, reduced by key.
//
// Used when every run of a count is already a sorted unique table: the
// multi-GPU owner merging the per-rank slices it received,
// the union of several references' sets (compare.rs:51-66, db_types.rs:43-53)
// and the engine's folded batch tables (one table across all inputs,
// count.rs:52-89).  The work list is count_sorted's: every item is one key
// range, split out of each run by binary search (k_sorted_items), holding at
// most kMergeCap instances over at most kMergeMaxRuns runs.
//
// One workgroup per item, all in LDS (no hashing, no sort network):
//   1. load the item's R sub-runs into LDS, concatenated (keys; weights kept in
//      registers);
//   2. rank every element in the merged order by binary search in the other
//      R-1 sub-runs (ties ordered by run: count `<=` in earlier runs, `<` in
//      later ones, so equal keys of different runs get adjacent ranks);
//   3. scatter (key, weight) to its rank in LDS;
//   4. a block scan over "first of its key" flags gives each distinct key its
//      output slot; its count is the sum of the (at most R) equal neighbours.
// Two passes, so the table is written once, at its exact size, with no
// staging or compaction: COUNT mode computes each item's distinct keys
// (instances minus those whose key an earlier run also holds) into n_out;
// after an exclusive scan, WRITE mode merges again and stores the item's
// sorted distinct keys and summed u64 counts at out + dense_off[item].
// HBM: 8 B (count) + 8 (+8) B (write) read per instance, 16 B (24 for
// k > 32) written per distinct key.
#include <mutex>

#include "okm_dev_common.h"

namespace okm {

constexpr int kMB = 512;                     // threads per workgroup
constexpr int kMPer = 8;                     // instances per thread
constexpr int kMergeCap = kMB * kMPer;       // 4096 = count_item_capacity()
constexpr int kMergeMaxRuns = 64;

template <typename KT>
__device__ __forceinline__ uint32_t lds_lower(const KT *a, uint32_t lo, uint32_t hi, const KT &key) {
    while (lo < hi) {  // first j with a[j] >= key
        const uint32_t mid = (lo + hi) >> 1;
        if (KeyOps<KT>::lt(a[mid], key)) lo = mid + 1; else hi = mid;
    }
    return lo;
}

template <typename KT>
__device__ __forceinline__ uint32_t lds_upper(const KT *a, uint32_t lo, uint32_t hi, const KT &key) {
    while (lo < hi) {  // first j with a[j] > key
        const uint32_t mid = (lo + hi) >> 1;
        if (KeyOps<KT>::lt(key, a[mid])) hi = mid; else lo = mid + 1;
    }
    return lo;
}

template <typename KT, bool W, bool WRITE>
__global__ __launch_bounds__(kMB) void k_merge_items(const DevItem *__restrict__ items, uint32_t nitems,
                                                     const DevSeg *__restrict__ segs, ull *__restrict__ n_out,
                                                     const ull *__restrict__ dense_off, uint64_t *__restrict__ out_keys_raw,
                                                     uint64_t *__restrict__ out_counts, ull *__restrict__ ctl) {
    extern __shared__ __attribute__((aligned(16))) ull lds[];
    KT *K = reinterpret_cast<KT *>(lds);                          // [kMergeCap] keys (then merged keys)
    ull *MC = reinterpret_cast<ull *>(K + kMergeCap);             // [kMergeCap] merged weights (WRITE)
    uint16_t *OI = reinterpret_cast<uint16_t *>(MC + kMergeCap);  // [kMergeCap] output slot of a first-of-key
    __shared__ uint32_t soff[kMergeMaxRuns + 1];
    __shared__ const KT *skeys[kMergeMaxRuns];
    __shared__ const uint64_t *scnt[kMergeMaxRuns];
    __shared__ ull wsum[kMB / 64];
    KT *out_keys = reinterpret_cast<KT *>(out_keys_raw);
    const uint32_t t = threadIdx.x;

    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        const DevItem it = items[item];
        // block-uniform values steer loops with barriers: keep them scalar
        const uint32_t R = __builtin_amdgcn_readfirstlane(it.seg_count);
        const uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)min(it.total, (uint64_t)kMergeCap + 1));
        if (R > (uint32_t)kMergeMaxRuns || n > (uint32_t)kMergeCap) {
            if (t == 0) {
                atomicMax(ctl, 3ull);
                if (!WRITE) n_out[item] = 0;
            }
            continue;
        }
        if (t < R) {
            const DevSeg s = segs[it.seg_begin + t];
            skeys[t] = reinterpret_cast<const KT *>(s.keys);
            scnt[t] = s.counts;
            soff[t + 1] = (uint32_t)s.len;
        }
        __syncthreads();
        if (t == 0) {
            soff[0] = 0;
            for (uint32_t r = 0; r < R; ++r) soff[r + 1] += soff[r];
        }
        __syncthreads();
        // 1. load (strided: coalesced within each sub-run)
        KT key[kMPer];
        ull w[kMPer];
        uint32_t run[kMPer];
#pragma unroll
        for (int j = 0; j < kMPer; ++j) {
            const uint32_t e = t + (uint32_t)j * kMB;
            run[j] = 0;
            w[j] = 1;
            key[j] = KeyOps<KT>::empty();
            if (e < n) {
                uint32_t lo = 0, hi = R;  // run of e: last r with soff[r] <= e
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (soff[mid] <= e) lo = mid; else hi = mid;
                }
                const uint32_t p = e - soff[lo];
                run[j] = lo;
                key[j] = skeys[lo][p];
                if (WRITE && W && scnt[lo]) w[j] = scnt[lo][p];
                K[e] = key[j];
            }
        }
        __syncthreads();
        if (!WRITE) {
            // distinct = instances whose key no earlier run holds
            uint32_t mine = 0;
#pragma unroll
            for (int j = 0; j < kMPer; ++j) {
                const uint32_t e = t + (uint32_t)j * kMB;
                if (e >= n) continue;
                bool dup = false;
                for (uint32_t q = 0; q < run[j] && !dup; ++q) {
                    const uint32_t lo = soff[q], hi = soff[q + 1];
                    const uint32_t u = lds_upper(K, lo, hi, key[j]);
                    dup = u > lo && KeyOps<KT>::eq(K[u - 1], key[j]);
                }
                mine += !dup;
            }
            ull total;
            (void)block_excl_scan<kMB>(mine, wsum, &total);
            if (t == 0) n_out[item] = total;
            __syncthreads();  // LDS is reused by the next item
            continue;
        }
        // 2. merged rank (ties ordered by run)
        uint32_t rank[kMPer];
#pragma unroll
        for (int j = 0; j < kMPer; ++j) {
            const uint32_t e = t + (uint32_t)j * kMB;
            rank[j] = 0;
            if (e < n) {
                const uint32_t r = run[j];
                uint32_t rk = e - soff[r];
                for (uint32_t q = 0; q < R; ++q) {
                    if (q == r) continue;
                    const uint32_t lo = soff[q], hi = soff[q + 1];
                    rk += (q < r ? lds_upper(K, lo, hi, key[j]) : lds_lower(K, lo, hi, key[j])) - lo;
                }
                rank[j] = rk;
            }
        }
        __syncthreads();
        // 3. scatter to the merged order
#pragma unroll
        for (int j = 0; j < kMPer; ++j) {
            const uint32_t e = t + (uint32_t)j * kMB;
            if (e < n) {
                K[rank[j]] = key[j];
                MC[rank[j]] = w[j];
            }
        }
        __syncthreads();
        // 4. first-of-key flags over a contiguous chunk per thread, block scan
        const uint32_t c0 = t * kMPer;
        uint32_t firsts = 0, fmask = 0;
#pragma unroll
        for (int j = 0; j < kMPer; ++j) {
            const uint32_t i = c0 + j;
            if (i < n && (i == 0 || !KeyOps<KT>::eq(K[i - 1], K[i]))) {
                fmask |= 1u << j;
                ++firsts;
            }
        }
        ull total;
        uint32_t slot = (uint32_t)block_excl_scan<kMB>(firsts, wsum, &total);
#pragma unroll
        for (int j = 0; j < kMPer; ++j) {
            const uint32_t i = c0 + j;
            if (i < n) OI[i] = (fmask >> j) & 1u ? (uint16_t)slot++ : (uint16_t)0xFFFFu;
        }
        __syncthreads();
        // 5. emit (strided: consecutive lanes -> consecutive output slots)
        const uint64_t base = dense_off[item];
#pragma unroll
        for (int j = 0; j < kMPer; ++j) {
            const uint32_t i = t + (uint32_t)j * kMB;
            if (i < n && OI[i] != 0xFFFFu) {
                const KT kk = K[i];
                ull sum = MC[i];
                for (uint32_t q = i + 1; q < n && KeyOps<KT>::eq(K[q], kk); ++q) sum += MC[q];
                out_keys[base + OI[i]] = kk;
                out_counts[base + OI[i]] = sum;
            }
        }
        __syncthreads();  // LDS is reused by the next item
    }
}

uint32_t merge_item_capacity() { return kMergeCap; }
uint32_t merge_max_runs() { return kMergeMaxRuns; }

template <typename KT, bool W, bool WRITE>
static void merge_launch(hipStream_t s, uint32_t grid, size_t lds, const DevItem *items, uint32_t nitems,
                         const DevSeg *segs, ull *n_out, const ull *dense_off, uint64_t *out_keys, uint64_t *out_counts,
                         ull *ctl) {
    static std::once_flag once;  // > 64 KiB of dynamic LDS for the wide variants (gfx950: 160 KiB per workgroup)
    std::call_once(once, [] {
        int dev = 0, optin = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || optin <= 0)
            optin = 64 * 1024;
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_merge_items<KT, W, WRITE>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, optin);
        (void)hipGetLastError();  // an unsupported attribute must not poison later checks
    });
    hipLaunchKernelGGL((k_merge_items<KT, W, WRITE>), dim3(grid), dim3(kMB), lds, s, items, nitems, segs, n_out,
                       dense_off, out_keys, out_counts, ctl);
}

void launch_merge_items(void *stream, const DevItem *items, uint32_t nitems, const DevSeg *segs,
                        unsigned long long *n_out, const unsigned long long *dense_off, uint64_t *out_keys,
                        uint64_t *out_counts, unsigned long long *ctl, bool weighted, bool wide, bool write) {
    if (!nitems) return;
    const uint32_t grid = nitems < 8191u ? nitems : 8191u;
    hipStream_t s = (hipStream_t)stream;
    const size_t lds = (size_t)kMergeCap * ((wide ? 16 : 8) + (write ? 8 + 2 : 0));
#define OKM_MERGE_CASE(KT, W)                                                                                   \
    do {                                                                                                        \
        if (write)                                                                                              \
            merge_launch<KT, W, true>(s, grid, lds, items, nitems, segs, n_out, dense_off, out_keys, out_counts, \
                                      ctl);                                                                     \
        else                                                                                                    \
            merge_launch<KT, W, false>(s, grid, lds, items, nitems, segs, n_out, dense_off, out_keys,            \
                                       out_counts, ctl);                                                        \
    } while (0)
    if (wide && weighted)
        OKM_MERGE_CASE(K128, true);
    else if (wide)
        OKM_MERGE_CASE(K128, false);
    else if (weighted)
        OKM_MERGE_CASE(ull, true);
    else
        OKM_MERGE_CASE(ull, false);
#undef OKM_MERGE_CASE
}

}  // namespace okm
