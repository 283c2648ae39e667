// okm_device.hip — gfx950 kernels of the k-mer engine.
//
// Pipeline:
//   L1   extract_hist / extract_scatter : batch bytes -> canonical k-mers ->
//        key-range partitions (top l1 bits of the 2k-bit key), exact placement.
//   Lx   part_hist / part_scatter       : re-partition keys by further bits.
//   cnt  count_items                    : one workgroup per partition, LDS
//        open-addressing table (64-bit CAS + add), then LDS bitonic sort of the
//        distinct entries -> sorted (key, count) runs.  Partitions are key
//        ranges in key order, so concatenating runs is globally sorted.
//   out  compact_items / filter_*       : dense result, min_count filter.
//
// Reference semantics restated on the device:
//   kmer.rs:12-20  dna_base_to_u64      -> base_code/base_valid (+U/u from
//                                          needletail normalize, count.rs:71)
//   kmer.rs:37-57  seq_to_u64           -> rolling forward word `fwd`
//   kmer.rs:79-94  reverse_complement   -> rolling `rc`
//   kmer.rs:99-106 canonical_u64        -> min(fwd, rc)
//   count.rs:23-38 window loop          -> scan_segment + valid-run counter
//   count.rs:31-34 DashMap fetch_add    -> LDS table in count_items
//   count.rs:106-119 filter + sort      -> count_items sort + filter kernels
#include <hip/hip_runtime.h>

#include "okm_internal.h"

namespace okm {

typedef unsigned long long ull;

// ---------------------------------------------------------------------------
// codec
// ---------------------------------------------------------------------------

// Valid bytes after needletail normalize(false) + dna_base_to_u64:
// A/a C/c G/g T/t U/u (kmer.rs:14-17; U->T is normalize's).  c & 0xDF folds
// case and has exactly {X, X|0x20} as preimages of an upper-case letter X.
__device__ __forceinline__ bool base_valid(uint32_t c) {
    const uint32_t u = c & 0xDFu;
    return (u == 'A') | (u == 'C') | (u == 'G') | (u == 'T') | (u == 'U');
}
// A=0 C=1 G=2 T=3 (and U=3) for either case: ((c>>1) ^ (c>>2)) & 3.
__device__ __forceinline__ uint32_t base_code(uint32_t c) { return ((c >> 1) ^ (c >> 2)) & 3u; }

__device__ __forceinline__ uint32_t bin_of(uint64_t key, uint32_t shift) {
    return shift >= 64 ? 0u : (uint32_t)(key >> shift);
}

constexpr int kSeg = 32;           // window starts per thread
constexpr int kLoad = kSeg + 32;   // bytes per thread: covers kSeg + k - 1 for k <= 32
constexpr int kExtractBlock = 256;
constexpr int kTile = kExtractBlock * kSeg;

// Walk the windows starting in [w0, w0 + kSeg) of a batch of n bytes.  Every
// window whose k bytes are all valid is canonicalised and handed to emit().
// Bytes at or beyond n read as 0 (invalid), so windows never run off the end;
// record separators are invalid bytes, so windows never cross records.
template <typename Emit>
__device__ __forceinline__ void scan_segment(const uint8_t *__restrict__ seq, uint64_t n,
                                             uint64_t w0, uint32_t k, Emit &&emit) {
    uint32_t w[kLoad / 4];
    if (w0 + kLoad <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(seq + w0);
#pragma unroll
        for (int q = 0; q < kLoad / 16; ++q) {
            const uint4 v = p[q];
            w[4 * q + 0] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < kLoad / 4; ++q) {
            uint32_t x = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint64_t idx = w0 + 4 * q + b;
                const uint32_t c = idx < n ? (uint32_t)seq[idx] : 0u;
                x |= c << (8 * b);
            }
            w[q] = x;
        }
    }
    const uint64_t kmask = (k >= 32) ? ~0ull : ((1ull << (2 * k)) - 1ull);
    const uint32_t rcs = 2 * k - 2;
    uint64_t fwd = 0, rc = 0;
    uint32_t run = 0;
#pragma unroll
    for (int i = 0; i < kLoad - 1; ++i) {
        const uint32_t c = (w[i >> 2] >> ((i & 3) * 8)) & 0xFFu;
        const uint32_t code = base_code(c);
        fwd = ((fwd << 2) | code) & kmask;                    // kmer.rs:51, rolled
        rc = (rc >> 2) | ((uint64_t)(code ^ 3u) << rcs);     // kmer.rs:87-91, rolled
        run = base_valid(c) ? run + 1 : 0;
        const int start = i - (int)k + 1;
        if (run >= k && start >= 0 && start < kSeg) emit(fwd < rc ? fwd : rc);  // kmer.rs:101
    }
}

// ---------------------------------------------------------------------------
// L1: extraction + histogram
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(kExtractBlock) void k_extract_hist(const uint8_t *__restrict__ seq,
                                                                ExtractGeom g,
                                                                uint32_t *__restrict__ HC,
                                                                ull *__restrict__ Hg) {
    extern __shared__ uint32_t lh[];
    for (uint32_t b = threadIdx.x; b < g.nbins; b += kExtractBlock) lh[b] = 0;
    __syncthreads();
    const uint64_t beg = (uint64_t)blockIdx.x * g.chunk;
    const uint64_t end = beg + g.chunk < g.n ? beg + g.chunk : g.n;
    const uint32_t shift = g.shift;
    for (uint64_t t0 = beg; t0 < end; t0 += kTile) {
        const uint64_t w0 = t0 + (uint64_t)threadIdx.x * kSeg;
        if (w0 < end)
            scan_segment(seq, g.n, w0, g.k, [&](uint64_t key) { atomicAdd(&lh[bin_of(key, shift)], 1u); });
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < g.nbins; b += kExtractBlock) {
        const uint32_t h = lh[b];
        HC[(uint64_t)blockIdx.x * g.nbins + b] = h;
        if (h) atomicAdd(&Hg[b], (ull)h);
    }
}

// Each block claims, per bin, a contiguous slice of the bin's region sized by
// its own histogram (one returning atomic per (block, bin)), then places every
// key at slice base + LDS rank: no per-key global atomics.
__global__ __launch_bounds__(kExtractBlock) void k_extract_scatter(const uint8_t *__restrict__ seq,
                                                                   ExtractGeom g,
                                                                   const uint32_t *__restrict__ HC,
                                                                   ull *__restrict__ cursor,
                                                                   uint64_t *__restrict__ out) {
    extern __shared__ ull ls[];
    ull *gbase = ls;
    uint32_t *rank = reinterpret_cast<uint32_t *>(ls + g.nbins);
    for (uint32_t b = threadIdx.x; b < g.nbins; b += kExtractBlock) {
        const uint32_t h = HC[(uint64_t)blockIdx.x * g.nbins + b];
        gbase[b] = h ? atomicAdd(&cursor[b], (ull)h) : 0ull;
        rank[b] = 0;
    }
    __syncthreads();
    const uint64_t beg = (uint64_t)blockIdx.x * g.chunk;
    const uint64_t end = beg + g.chunk < g.n ? beg + g.chunk : g.n;
    const uint32_t shift = g.shift;
    for (uint64_t t0 = beg; t0 < end; t0 += kTile) {
        const uint64_t w0 = t0 + (uint64_t)threadIdx.x * kSeg;
        if (w0 < end)
            scan_segment(seq, g.n, w0, g.k, [&](uint64_t key) {
                const uint32_t b = bin_of(key, shift);
                const uint32_t r = atomicAdd(&rank[b], 1u);
                out[gbase[b] + r] = key;
            });
    }
}

void launch_extract_hist(void *stream, const uint8_t *seq, const ExtractGeom &g, uint32_t *HC,
                         unsigned long long *Hg) {
    hipLaunchKernelGGL(k_extract_hist, dim3(g.nblocks), dim3(kExtractBlock),
                       g.nbins * sizeof(uint32_t), (hipStream_t)stream, seq, g, HC, Hg);
}

void launch_extract_scatter(void *stream, const uint8_t *seq, const ExtractGeom &g,
                            const uint32_t *HC, unsigned long long *cursor, uint64_t *out_keys) {
    hipLaunchKernelGGL(k_extract_scatter, dim3(g.nblocks), dim3(kExtractBlock),
                       g.nbins * (sizeof(ull) + sizeof(uint32_t)), (hipStream_t)stream, seq, g, HC,
                       cursor, out_keys);
}

// ---------------------------------------------------------------------------
// Generic partition pass over (segment, chunk) lists
// ---------------------------------------------------------------------------

constexpr int kPartBlock = 256;

__device__ __forceinline__ uint32_t local_bin(uint64_t key, const DevSeg &s) {
    const uint64_t b = (s.shift >= 64 ? 0ull : (key >> s.shift)) - s.key_base;
    return b < s.nlocal ? (uint32_t)b : s.nlocal - 1;  // clamp: never true for canonical keys
}

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
        __syncthreads();
        const uint64_t *keys = s.keys + ch.begin;
        for (uint64_t i = threadIdx.x; i < ch.len; i += kPartBlock)
            atomicAdd(&lh[local_bin(keys[i], s)], 1u);
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < s.nlocal; b += kPartBlock) {
            const uint32_t h = lh[b];
            HC[(uint64_t)c * max_local + b] = h;
            if (h) atomicAdd(&Hg[s.out_base + b], (ull)h);
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kPartBlock) void k_part_scatter(
    const DevSeg *__restrict__ segs, const DevChunk *__restrict__ chunks, uint32_t nchunks,
    uint32_t max_local, const uint32_t *__restrict__ HC, ull *__restrict__ cursor,
    uint64_t *__restrict__ out_keys, uint64_t *__restrict__ out_counts) {
    extern __shared__ ull ls[];
    ull *gbase = ls;
    uint32_t *rank = reinterpret_cast<uint32_t *>(ls + max_local);
    for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const DevChunk ch = chunks[c];
        const DevSeg s = segs[ch.seg];
        for (uint32_t b = threadIdx.x; b < s.nlocal; b += kPartBlock) {
            const uint32_t h = HC[(uint64_t)c * max_local + b];
            gbase[b] = h ? atomicAdd(&cursor[s.out_base + b], (ull)h) : 0ull;
            rank[b] = 0;
        }
        __syncthreads();
        const uint64_t *keys = s.keys + ch.begin;
        const uint64_t *cnts = s.counts ? s.counts + ch.begin : nullptr;
        for (uint64_t i = threadIdx.x; i < ch.len; i += kPartBlock) {
            const uint64_t key = keys[i];
            const uint32_t b = local_bin(key, s);
            const uint64_t dst = gbase[b] + atomicAdd(&rank[b], 1u);
            out_keys[dst] = key;
            if (out_counts) out_counts[dst] = cnts ? cnts[i] : 1ull;
        }
        __syncthreads();
    }
}

static uint32_t part_grid(uint32_t nchunks) { return nchunks < 4096u ? nchunks : 4096u; }

void launch_part_hist(void *stream, const DevSeg *segs, const DevChunk *chunks, uint32_t nchunks,
                      uint32_t max_local, uint32_t *HC, unsigned long long *Hg) {
    if (!nchunks) return;
    hipLaunchKernelGGL(k_part_hist, dim3(part_grid(nchunks)), dim3(kPartBlock),
                       max_local * sizeof(uint32_t), (hipStream_t)stream, segs, chunks, nchunks,
                       max_local, HC, Hg);
}

void launch_part_scatter(void *stream, const DevSeg *segs, const DevChunk *chunks,
                         uint32_t nchunks, uint32_t max_local, const uint32_t *HC,
                         unsigned long long *cursor, uint64_t *out_keys, uint64_t *out_counts) {
    if (!nchunks) return;
    hipLaunchKernelGGL(k_part_scatter, dim3(part_grid(nchunks)), dim3(kPartBlock),
                       max_local * (sizeof(ull) + sizeof(uint32_t)), (hipStream_t)stream, segs,
                       chunks, nchunks, max_local, HC, cursor, out_keys, out_counts);
}

uint32_t extract_tile() { return (uint32_t)kTile; }

// ---------------------------------------------------------------------------
// Exclusive scan (u64): per-block scan + recursive scan of block sums + add.
// ---------------------------------------------------------------------------

constexpr int kScanBlock = 256;
constexpr int kScanPer = 8;
constexpr uint64_t kScanTile = (uint64_t)kScanBlock * kScanPer;

__device__ __forceinline__ ull wave_incl_scan(ull v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const ull o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// Block-wide exclusive scan of one value per thread; returns the exclusive
// prefix and writes the block total to *total (all threads).
template <int BLOCK>
__device__ __forceinline__ ull block_excl_scan(ull v, ull *wsum, ull *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const ull inc = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    ull wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) {
        const ull s = wsum[w];
        if (w < wid) wbase += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wbase + inc - v;
}

__global__ __launch_bounds__(kScanBlock) void k_scan_block(const ull *__restrict__ in,
                                                           ull *__restrict__ out, uint64_t n,
                                                           ull *__restrict__ block_sums) {
    __shared__ ull wsum[kScanBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
    ull v[kScanPer];
    ull s = 0;
#pragma unroll
    for (int j = 0; j < kScanPer; ++j) {
        v[j] = base + j < n ? in[base + j] : 0ull;
        s += v[j];
    }
    ull total;
    ull run = block_excl_scan<kScanBlock>(s, wsum, &total);
#pragma unroll
    for (int j = 0; j < kScanPer; ++j) {
        if (base + j < n) out[base + j] = run;
        run += v[j];
    }
    if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanBlock) void k_scan_add(ull *__restrict__ out, uint64_t n,
                                                         const ull *__restrict__ block_offsets) {
    const ull add = block_offsets[blockIdx.x];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
    for (uint32_t j = threadIdx.x; j < kScanTile; j += kScanBlock)
        if (base + j < n) out[base + j] += add;
}

size_t scan_tmp_elems(uint64_t n) {
    size_t total = 0;
    uint64_t m = n;
    while (m > 1) {
        m = (m + kScanTile - 1) / kScanTile;
        total += m + 1;
    }
    return total + 2;
}

void launch_exclusive_scan(void *stream, const ull *in, ull *out, uint64_t n, ull *tmp) {
    if (n == 0) return;
    const uint64_t nb = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_block, dim3((uint32_t)nb), dim3(kScanBlock), 0, (hipStream_t)stream,
                       in, out, n, tmp);
    if (nb > 1) {
        launch_exclusive_scan(stream, tmp, tmp, nb, tmp + nb + 1);
        hipLaunchKernelGGL(k_scan_add, dim3((uint32_t)nb), dim3(kScanBlock), 0,
                           (hipStream_t)stream, out, n, tmp);
    }
}

// ---------------------------------------------------------------------------
// LDS counting of partitions
// ---------------------------------------------------------------------------

constexpr int kCountBlock = 256;
constexpr int kSlots = 4096;                 // table slots per workgroup
constexpr int kSlotBits = 12;
constexpr int kCapDistinct = 3072;           // max distinct keys per item (75 % load)
constexpr int kPerThread = kSlots / kCountBlock;

uint32_t count_item_capacity() { return kCapDistinct; }

__device__ __forceinline__ uint32_t slot_of(uint64_t key) {
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - kSlotBits));
}

__global__ __launch_bounds__(kCountBlock) void k_count_items(const DevItem *__restrict__ items,
                                                             uint32_t nitems,
                                                             const DevSeg *__restrict__ segs,
                                                             uint64_t *__restrict__ out_keys,
                                                             uint64_t *__restrict__ out_counts,
                                                             ull *__restrict__ n_out,
                                                             ull *__restrict__ overflow) {
    __shared__ ull tk[kSlots];
    __shared__ ull tc[kSlots];
    __shared__ ull wsum[kCountBlock / 64];
    __shared__ uint32_t s_distinct;

    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        for (int j = threadIdx.x; j < kSlots; j += kCountBlock) {
            tk[j] = kEmptyKey;
            tc[j] = 0;
        }
        if (threadIdx.x == 0) s_distinct = 0;
        __syncthreads();
        const DevItem it = items[item];
        // insert: the DashMap entry().or_insert().fetch_add() of count.rs:31-34
        for (uint32_t sg = 0; sg < it.seg_count; ++sg) {
          const DevSeg s = segs[it.seg_begin + sg];
          for (uint64_t i = threadIdx.x; i < s.len; i += kCountBlock) {
            const uint64_t key = s.keys[i];
            const uint64_t w = s.counts ? s.counts[i] : 1ull;
            uint32_t h = slot_of(key);
            uint32_t probes = 0;
            for (;;) {
                const ull old = atomicCAS(&tk[h], (ull)kEmptyKey, (ull)key);
                if (old == kEmptyKey || old == key) {
                    if (old == kEmptyKey) atomicAdd(&s_distinct, 1u);
                    atomicAdd(&tc[h], (ull)w);
                    break;
                }
                h = (h + 1) & (kSlots - 1);
                if (++probes >= (uint32_t)kSlots) {  // full table: impossible under host sizing
                    atomicOr((unsigned int *)overflow, 1u);
                    break;
                }
            }
          }
        }
        __syncthreads();
        if (s_distinct > (uint32_t)kCapDistinct) {
            if (threadIdx.x == 0) atomicOr((unsigned int *)overflow, 1u);
        }
        // compact occupied slots to the front (in place, via registers)
        ull rk[kPerThread], rc[kPerThread];
        uint32_t mine = 0;
#pragma unroll
        for (int j = 0; j < kPerThread; ++j) {
            rk[j] = tk[threadIdx.x * kPerThread + j];
            rc[j] = tc[threadIdx.x * kPerThread + j];
            mine += rk[j] != kEmptyKey;
        }
        ull total;
        ull pos = block_excl_scan<kCountBlock>(mine, wsum, &total);
        const uint32_t D = (uint32_t)total;
        uint32_t P2 = 1;
        while (P2 < D) P2 <<= 1;
#pragma unroll
        for (int j = 0; j < kPerThread; ++j) {
            if (rk[j] != kEmptyKey) {
                tk[pos] = rk[j];
                tc[pos] = rc[j];
                ++pos;
            }
        }
        __syncthreads();
        for (uint32_t j = D + threadIdx.x; j < P2; j += kCountBlock) tk[j] = kEmptyKey;
        __syncthreads();
        // bitonic sort of (tk, tc) on [0, P2): count.rs:119 sort_by_key
        for (uint32_t size = 2; size <= P2; size <<= 1) {
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                for (uint32_t t = threadIdx.x; t < P2 / 2; t += kCountBlock) {
                    const uint32_t i = 2 * t - (t & (stride - 1));
                    const uint32_t j = i + stride;
                    const bool asc = (i & size) == 0;
                    const ull a = tk[i], b = tk[j];
                    if ((a > b) == asc) {
                        tk[i] = b;
                        tk[j] = a;
                        const ull ca = tc[i];
                        tc[i] = tc[j];
                        tc[j] = ca;
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t j = threadIdx.x; j < D; j += kCountBlock) {
            out_keys[it.out_off + j] = tk[j];
            out_counts[it.out_off + j] = tc[j];
        }
        if (threadIdx.x == 0) n_out[item] = D;
        __syncthreads();
    }
}

void launch_count_items(void *stream, const DevItem *items, uint32_t nitems, const DevSeg *segs,
                        uint64_t *out_keys, uint64_t *out_counts, unsigned long long *n_out,
                        unsigned long long *overflow) {
    if (!nitems) return;
    const uint32_t grid = nitems < 2048u ? nitems : 2048u;
    hipLaunchKernelGGL(k_count_items, dim3(grid), dim3(kCountBlock), 0, (hipStream_t)stream, items,
                       nitems, segs, out_keys, out_counts, n_out, overflow);
}

// ---------------------------------------------------------------------------
// Result assembly
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_compact_items(const DevItem *__restrict__ items,
                                                       uint32_t nitems, const ull *__restrict__ n_out,
                                                       const ull *__restrict__ dense_off,
                                                       const uint64_t *__restrict__ sk,
                                                       const uint64_t *__restrict__ sc,
                                                       uint64_t *__restrict__ dk,
                                                       uint64_t *__restrict__ dc) {
    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        const uint64_t n = n_out[item], src = items[item].out_off, dst = dense_off[item];
        for (uint64_t j = threadIdx.x; j < n; j += 256) {
            dk[dst + j] = sk[src + j];
            dc[dst + j] = sc[src + j];
        }
    }
}

void launch_compact_items(void *stream, const DevItem *items, uint32_t nitems,
                          const unsigned long long *n_out, const unsigned long long *dense_off,
                          const uint64_t *src_keys, const uint64_t *src_counts, uint64_t *dst_keys,
                          uint64_t *dst_counts) {
    if (!nitems) return;
    const uint32_t grid = nitems < 8192u ? nitems : 8192u;
    hipLaunchKernelGGL(k_compact_items, dim3(grid), dim3(256), 0, (hipStream_t)stream, items,
                       nitems, n_out, dense_off, src_keys, src_counts, dst_keys, dst_counts);
}

constexpr int kFilterBlock = 256;
constexpr int kFilterPer = 16;
constexpr uint64_t kFilterTile = (uint64_t)kFilterBlock * kFilterPer;

uint32_t filter_blocks(uint64_t n) { return (uint32_t)((n + kFilterTile - 1) / kFilterTile); }

__global__ __launch_bounds__(kFilterBlock) void k_filter_count(const uint64_t *__restrict__ counts,
                                                               uint64_t n, uint64_t min_count,
                                                               ull *__restrict__ block_counts) {
    __shared__ ull wsum[kFilterBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kFilterTile + (uint64_t)threadIdx.x * kFilterPer;
    ull c = 0;
    for (int j = 0; j < kFilterPer; ++j)
        if (base + j < n && counts[base + j] >= min_count) ++c;
    ull total;
    block_excl_scan<kFilterBlock>(c, wsum, &total);
    if (threadIdx.x == 0) block_counts[blockIdx.x] = total;
}

__global__ __launch_bounds__(kFilterBlock) void k_filter_scatter(
    const uint64_t *__restrict__ keys, const uint64_t *__restrict__ counts, uint64_t n,
    uint64_t min_count, const ull *__restrict__ block_offsets, uint64_t *__restrict__ dk,
    uint64_t *__restrict__ dc) {
    __shared__ ull wsum[kFilterBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kFilterTile + (uint64_t)threadIdx.x * kFilterPer;
    ull c = 0;
    for (int j = 0; j < kFilterPer; ++j)
        if (base + j < n && counts[base + j] >= min_count) ++c;
    ull total;
    ull pos = block_excl_scan<kFilterBlock>(c, wsum, &total) + block_offsets[blockIdx.x];
    for (int j = 0; j < kFilterPer; ++j) {
        if (base + j < n && counts[base + j] >= min_count) {
            dk[pos] = keys[base + j];
            if (dc) dc[pos] = counts[base + j];
            ++pos;
        }
    }
}

void launch_filter_count(void *stream, const uint64_t *counts, uint64_t n, uint64_t min_count,
                         unsigned long long *block_counts, uint32_t) {
    const uint32_t nb = filter_blocks(n);
    if (!nb) return;
    hipLaunchKernelGGL(k_filter_count, dim3(nb), dim3(kFilterBlock), 0, (hipStream_t)stream, counts,
                       n, min_count, block_counts);
}

void launch_filter_scatter(void *stream, const uint64_t *keys, const uint64_t *counts, uint64_t n,
                           uint64_t min_count, const unsigned long long *block_offsets,
                           uint64_t *dst_keys, uint64_t *dst_counts) {
    const uint32_t nb = filter_blocks(n);
    if (!nb) return;
    hipLaunchKernelGGL(k_filter_scatter, dim3(nb), dim3(kFilterBlock), 0, (hipStream_t)stream, keys,
                       counts, n, min_count, block_offsets, dst_keys, dst_counts);
}

// ---------------------------------------------------------------------------
// |A ∩ B| for compare.rs:58
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_intersect_count(const uint64_t *__restrict__ a,
                                                         uint64_t na, const uint64_t *__restrict__ b,
                                                         uint64_t nb, ull *__restrict__ out) {
    __shared__ ull wsum[4];
    ull hits = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < na; i += (uint64_t)gridDim.x * 256) {
        const uint64_t x = a[i];
        uint64_t lo = 0, hi = nb;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (b[mid] < x) lo = mid + 1; else hi = mid;
        }
        hits += (lo < nb && b[lo] == x);
    }
    ull total;
    block_excl_scan<256>(hits, wsum, &total);
    if (threadIdx.x == 0 && total) atomicAdd(out, total);
}

void launch_intersect_count(void *stream, const uint64_t *a, uint64_t na, const uint64_t *b,
                            uint64_t nb, unsigned long long *out) {
    if (!na || !nb) return;
    uint64_t g = (na + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_intersect_count, dim3((uint32_t)g), dim3(256), 0, (hipStream_t)stream, a, na,
                       b, nb, out);
}

}  // namespace okm
