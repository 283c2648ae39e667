// okm_partition.hip — key-range partition passes over key arrays.
//
// Splits every segment of a pass into 2^b sub-ranges of its keys (the next b
// key bits below the segment's common prefix):
//   part_hist    per chunk (64 Ki keys) and local bin: key count -> HC (exact
//                placement), or only the bin totals Hg of a sample (sampled);
//   (device)     exclusive scan of the totals / capacities -> bin starts;
//   part_scatter every LDS tile of a chunk is counting-sorted by local bin and
//                each bin's run leaves as one contiguous stretch of its slice
//                (claimed per chunk, or per tile against a sampled capacity),
//                so HBM sees long runs instead of 8-byte scattered stores
//                (which cost ~3.5x the bytes: partially written lines leave
//                the 4 MiB XCD L2 early).
// Instantiated for u64 keys (k <= 32) and K128 keys (k <= 64).
#include "okm_dev_common.h"

namespace okm {

constexpr int kPartBlock = 1024;  // threads per workgroup (scatter: LDS-limited to 1 block/CU)
constexpr int kHistU = 4;         // 16-B loads per thread in flight (histogram)

// Output bins one pass can split a part into.  u64 unweighted passes take up
// to 2048 (two bins per scatter thread, 15 Ki-key tiles), so a fold's L1 bin
// of ~8 M instances splits straight into ~4 Ki-key children -- one item each,
// with no fan-out pass (k_fan_split) after the partition.
uint32_t part_max_bins(bool weighted, bool wide) {
    // the tile scan gives each thread one bin (two in the 2048-bin variant)
    return weighted ? 512u : (!wide ? 2u * kPartBlock : (uint32_t)kPartBlock);
}

template <typename KT>
__device__ __forceinline__ uint32_t local_bin(const KT &key, const DevSeg &s) {
    // (key >> shift) - key_base, modulo 2^64: exact because the key lies in the
    // segment's range (the difference is < nlocal)
    const uint64_t b = (s.shift >= (uint32_t)KeyOps<KT>::kBits ? 0ull : KeyOps<KT>::shr(key, s.shift)) - s.key_base;
    return b < s.nlocal ? (uint32_t)b : s.nlocal - 1;  // clamp: never true for canonical keys
}

template <typename KT>
__device__ __forceinline__ void hist_key(const KT &key, const DevSeg &s, uint32_t *lh) {
    if (!KeyOps<KT>::is_empty(key)) atomicAdd(&lh[local_bin(key, s)], 1u);
}

template <typename KT>
__global__ __launch_bounds__(kPartBlock) void k_part_hist(const DevSeg *__restrict__ segs,
                                                          const DevChunk *__restrict__ chunks,
                                                          uint32_t nchunks, uint32_t max_local,
                                                          uint32_t *__restrict__ HC,
                                                          ull *__restrict__ Hg) {
    extern __shared__ uint32_t lh[];
    for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const DevChunk ch = chunks[c];
        const DevSeg s = segs[ch.seg];
        for (uint32_t b = threadIdx.x; b < s.nlocal; b += kPartBlock) lh[b] = 0;
        lds_sync();
        const KT *keys = reinterpret_cast<const KT *>(s.keys) + ch.begin;
        if (sizeof(KT) == 8 && (reinterpret_cast<uintptr_t>(keys) & 15u) == 0) {  // block-uniform: 2 keys / 16 B
            const uint4 *k4 = reinterpret_cast<const uint4 *>(keys);
            const uint64_t n2 = ch.len >> 1;
            for (uint64_t i = threadIdx.x; i < n2; i += (uint64_t)kPartBlock * kHistU) {
                uint4 v[kHistU];
#pragma unroll
                for (int u = 0; u < kHistU; ++u) {
                    const uint64_t q = i + (uint64_t)u * kPartBlock;
                    v[u] = q < n2 ? gload(k4 + q) : make_uint4(~0u, ~0u, ~0u, ~0u);
                }
#pragma unroll
                for (int u = 0; u < kHistU; ++u) {
                    const ull a = ((ull)v[u].y << 32) | v[u].x, b = ((ull)v[u].w << 32) | v[u].z;
                    hist_key(*reinterpret_cast<const KT *>(&a), s, lh);
                    hist_key(*reinterpret_cast<const KT *>(&b), s, lh);
                }
            }
            if ((ch.len & 1) && threadIdx.x == 0) hist_key(gload(keys + ch.len - 1), s, lh);
        } else {
            for (uint64_t i = threadIdx.x; i < ch.len; i += (uint64_t)kPartBlock * kHistU) {
                KT v[kHistU];
#pragma unroll
                for (int u = 0; u < kHistU; ++u) {
                    const uint64_t q = i + (uint64_t)u * kPartBlock;
                    v[u] = q < ch.len ? gload(keys + q) : KeyOps<KT>::empty();
                }
#pragma unroll
                for (int u = 0; u < kHistU; ++u) hist_key(v[u], s, lh);
            }
        }
        lds_sync();
        for (uint32_t b = threadIdx.x; b < s.nlocal; b += kPartBlock) {
            const uint32_t h = lh[b];
            if (HC) HC[(uint64_t)c * max_local + b] = h;
            if (h) atomicAdd(&Hg[s.out_base + b], (ull)h);
        }
        lds_sync();
    }
}

// Every 64-Ki-key chunk is processed in LDS tiles that are counting-sorted by
// local bin, and each bin's run leaves as one contiguous stretch of the
// chunk's slice (exact placement: no padding, no append rounds).
template <typename KT, bool W, bool BIG = false> struct Tile {
    // <= 128 KiB of staged keys (+ counts), + 16 KiB of per-bin state; BIG
    // (2048 bins: 32 KiB of per-bin state): 120 KiB of staged keys.  (18 Ki-key
    // tiles for <= 512 bins: 1.742 vs 1.738 ms, not kept; profiles/AB_LOG.md)
    static constexpr int kKeys = BIG ? 15 * kPartBlock
                                     : ((W && sizeof(KT) > 8) ? 4096 : ((W || sizeof(KT) > 8) ? 8192 : 16384));
    static constexpr int kPer = kKeys / kPartBlock;
};

template <typename KT, bool W, bool BIG = false>
__global__ __launch_bounds__(kPartBlock) __attribute__((amdgpu_waves_per_eu(1)))
void k_part_scatter_tile(
    const DevSeg *__restrict__ segs, const DevChunk *__restrict__ chunks, uint32_t nchunks,
    uint32_t max_local, const uint32_t *__restrict__ HC, ull *__restrict__ cursor,
    uint64_t *__restrict__ out_keys_raw, uint64_t *__restrict__ out_counts, const ull *__restrict__ cap_end,
    ull *__restrict__ ovf) {
    constexpr int T = Tile<KT, W, BIG>::kKeys, P = Tile<KT, W, BIG>::kPer;
    constexpr uint32_t BPT = BIG ? 2 : 1;  // bins per thread in the scan / claim phase
    extern __shared__ __attribute__((aligned(16))) ull lds[];
    KT *stage = reinterpret_cast<KT *>(lds);                              // [T]
    ull *cstage = reinterpret_cast<ull *>(stage + T);                     // [T] (W)
    ull *gcur = W ? cstage + T : cstage;                                  // [max_local]
    uint32_t *hist = reinterpret_cast<uint32_t *>(gcur + max_local);      // [max_local]
    uint32_t *lofs = hist + max_local;                                    // [max_local]
    __shared__ ull wsum[kPartBlock / 64];
    KT *out_keys = reinterpret_cast<KT *>(out_keys_raw);
    const uint32_t t = threadIdx.x;

    for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const DevChunk ch = chunks[c];
        const DevSeg s = segs[ch.seg];
        const uint32_t nl = s.nlocal;
        if (HC)  // exact: one claim per bin for the whole chunk
            for (uint32_t b = t; b < nl; b += kPartBlock) {
                const uint32_t h = HC[(uint64_t)c * max_local + b];
                gcur[b] = h ? atomicAdd(&cursor[s.out_base + b], (ull)h) : 0ull;
            }
        const KT *keys = reinterpret_cast<const KT *>(s.keys) + ch.begin;
        const uint64_t *cnts = s.counts ? s.counts + ch.begin : nullptr;
        for (uint64_t base = 0; base < ch.len; base += T) {
            for (uint32_t b = t; b < nl; b += kPartBlock) hist[b] = 0;
            lds_sync();
            KT kk[P];
            ull ww[P];
            uint32_t br[P];  // bin << 16 | rank; ~0 = empty
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const uint64_t idx = base + (uint64_t)u * kPartBlock + t;
                kk[u] = idx < ch.len ? gload(keys + idx) : KeyOps<KT>::empty();
                ww[u] = (W && idx < ch.len) ? (cnts ? gload(cnts + idx) : 1ull) : 1ull;
            }
#pragma unroll
            for (int u = 0; u < P; ++u) {
                br[u] = ~0u;
                if (!KeyOps<KT>::is_empty(kk[u])) {
                    const uint32_t b = local_bin(kk[u], s);
                    br[u] = (b << 16) | atomicAdd(&hist[b], 1u);
                }
            }
            lds_sync();
            // tile-local bin offsets (nl <= BPT * kPartBlock: thread t owns
            // bins BPT t .. BPT t + BPT - 1, so the scan runs in bin order)
            uint32_t my[BPT];
            uint32_t mine = 0;
#pragma unroll
            for (uint32_t q = 0; q < BPT; ++q) {
                const uint32_t b = BPT * t + q;
                my[q] = b < nl ? hist[b] : 0u;
                mine += my[q];
            }
            // sampled capacities: this tile's claim on its run of each bin is
            // issued now and consumed after the scan and the staging, so the
            // global atomic's round trip overlaps them
            ull claim[BPT];
#pragma unroll
            for (uint32_t q = 0; q < BPT; ++q) {
                claim[q] = 0;
                if (!HC && my[q]) claim[q] = atomicAdd(&cursor[s.out_base + BPT * t + q], (ull)my[q]);
            }
            ull tile_n;
            uint32_t off = (uint32_t)block_excl_scan<kPartBlock>(mine, wsum, &tile_n);
#pragma unroll
            for (uint32_t q = 0; q < BPT; ++q) {
                if (BPT * t + q < nl) lofs[BPT * t + q] = off;
                off += my[q];
            }
            lds_sync();
#pragma unroll
            for (int u = 0; u < P; ++u) {
                if (br[u] != ~0u) {
                    const uint32_t dst = lofs[br[u] >> 16] + (br[u] & 0xFFFFu);
                    stage[dst] = kk[u];
                    if (W) cstage[dst] = ww[u];
                }
            }
            if (!HC) {
#pragma unroll
                for (uint32_t q = 0; q < BPT; ++q) {
                    const uint32_t b = BPT * t + q;
                    if (b >= nl) continue;
                    ull g = ~0ull;
                    if (my[q]) {
                        if (claim[q] + my[q] <= cap_end[s.out_base + b])
                            g = claim[q];
                        else
                            atomicOr(ovf, 1ull);
                    }
                    gcur[b] = g;
                }
            }
            lds_sync();
            // each bin's run is contiguous in `stage` and in the output slice
            for (uint32_t j = t; j < (uint32_t)tile_n; j += kPartBlock) {
                const KT key = stage[j];
                const uint32_t b = local_bin(key, s);
                const ull g = gcur[b];
                if (g == ~0ull) continue;  // sampled mode: the bin overflowed
                const ull o = g + (j - lofs[b]);
                out_keys[o] = key;
                if (W) out_counts[o] = cstage[j];
            }
            lds_sync();
            if (HC)
                for (uint32_t b = t; b < nl; b += kPartBlock) gcur[b] += hist[b];
        }
        lds_sync();
    }
}

// Workgroups of the partition kernels (grids of 2048 / 8192 measured the same,
// profiles/AB_LOG.md round 4)
static uint32_t part_grid(uint32_t nchunks) { return nchunks < 4096u ? nchunks : 4096u; }

void launch_part_hist(void *stream, const DevSeg *segs, const DevChunk *chunks, uint32_t nchunks,
                      uint32_t max_local, uint32_t *HC, unsigned long long *Hg, bool wide) {
    if (!nchunks) return;
    const dim3 g(part_grid(nchunks)), b(kPartBlock);
    const size_t lds = max_local * sizeof(uint32_t);
    if (wide)
        hipLaunchKernelGGL(k_part_hist<K128>, g, b, lds, (hipStream_t)stream, segs, chunks, nchunks, max_local, HC, Hg);
    else
        hipLaunchKernelGGL(k_part_hist<ull>, g, b, lds, (hipStream_t)stream, segs, chunks, nchunks, max_local, HC, Hg);
}

template <typename KT, bool W>
static void scatter_launch(void *stream, const DevSeg *segs, const DevChunk *chunks, uint32_t nchunks,
                           uint32_t max_local, const uint32_t *HC, unsigned long long *cursor, uint64_t *out_keys,
                           uint64_t *out_counts, const ull *cap_end, ull *ovf) {
    static bool attr_done = false;  // allow > 64 KiB of dynamic LDS (gfx950: 160 KiB per workgroup)
    if (!attr_done) {
        int dev = 0, optin = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || optin <= 0)
            optin = 64 * 1024;
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_part_scatter_tile<KT, W>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, optin);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_part_scatter_tile<KT, W, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, optin);
        (void)hipGetLastError();  // an unsupported attribute must not poison later checks
        attr_done = true;
    }
    const size_t bin_state = (size_t)max_local * (sizeof(ull) + 2 * sizeof(uint32_t));
    if (max_local > (uint32_t)kPartBlock) {  // 2048 bins: u64 unweighted passes only (part_max_bins)
        constexpr int T = Tile<KT, W, true>::kKeys;
        const size_t lds = (size_t)T * (sizeof(KT) + (W ? sizeof(ull) : 0)) + bin_state;
        hipLaunchKernelGGL((k_part_scatter_tile<KT, W, true>), dim3(part_grid(nchunks)), dim3(kPartBlock), lds,
                           (hipStream_t)stream, segs, chunks, nchunks, max_local, HC, cursor, out_keys, out_counts,
                           cap_end, ovf);
        return;
    }
    constexpr int T = Tile<KT, W>::kKeys;
    const size_t lds = (size_t)T * (sizeof(KT) + (W ? sizeof(ull) : 0)) + bin_state;
    hipLaunchKernelGGL((k_part_scatter_tile<KT, W>), dim3(part_grid(nchunks)), dim3(kPartBlock), lds,
                       (hipStream_t)stream, segs, chunks, nchunks, max_local, HC, cursor, out_keys, out_counts, cap_end,
                       ovf);
}

void launch_part_scatter(void *stream, const DevSeg *segs, const DevChunk *chunks, uint32_t nchunks,
                         uint32_t max_local, const uint32_t *HC, unsigned long long *cursor, uint64_t *out_keys,
                         uint64_t *out_counts, bool wide, const ull *cap_end, ull *ovf) {
    if (!nchunks) return;
    if (wide) {
        if (out_counts)
            scatter_launch<K128, true>(stream, segs, chunks, nchunks, max_local, HC, cursor, out_keys, out_counts,
                                      cap_end, ovf);
        else
            scatter_launch<K128, false>(stream, segs, chunks, nchunks, max_local, HC, cursor, out_keys, out_counts,
                                       cap_end, ovf);
    } else {
        if (out_counts)
            scatter_launch<ull, true>(stream, segs, chunks, nchunks, max_local, HC, cursor, out_keys, out_counts,
                                    cap_end, ovf);
        else
            scatter_launch<ull, false>(stream, segs, chunks, nchunks, max_local, HC, cursor, out_keys, out_counts,
                                     cap_end, ovf);
    }
}

}  // namespace okm
