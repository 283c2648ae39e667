// okm_device.hip — utility kernels of the k-mer engine: exclusive scan,
// result compaction, min_count filter (count.rs:106-116) and |A ∩ B|
// (compare.rs:58).  The hot path lives in okm_extract.hip (L1 extraction),
// okm_partition.hip (key-range passes) and okm_count.hip (LDS counting).
#include "okm_dev_common.h"

namespace okm {

// ---------------------------------------------------------------------------
// Exclusive scan (u64): per-block scan + recursive scan of block sums + add.
// ---------------------------------------------------------------------------

constexpr int kScanBlock = 256;
constexpr int kScanPer = 8;
constexpr uint64_t kScanTile = (uint64_t)kScanBlock * kScanPer;

// Fan-out jobs of at most this many keys are "small" (the register / 512-thread
// variants of k_fan_split); k_make_items files them from the front of the job
// list and the larger ones from the back.
constexpr uint64_t kFanSmallJob = 16384;


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
// Work list of the LDS counting pass, built on the device
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_make_items(const ull *__restrict__ offs, const ull *__restrict__ ends,
                                                    uint32_t nout,
                                                    const DevParent *__restrict__ parents, uint32_t nparents,
                                                    const uint64_t *__restrict__ lk,
                                                    const uint64_t *__restrict__ lc, DevItem *__restrict__ items,
                                                    DevSeg *__restrict__ segs, uint64_t item_max,
                                                    uint32_t capbits, ull *__restrict__ flags, uint32_t kw,
                                                    FanOut fan, const ull *__restrict__ doff) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nout) return;
    // parent = last part whose first output bin is <= i
    uint32_t lo = 0, hi = nparents;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (parents[mid].out_base <= i) lo = mid; else hi = mid;
    }
    const uint32_t rem = parents[lo].rem;
    const ull o = offs[i], len = (ends ? ends[i] : offs[i + 1]) - o;
    const ull so = doff ? doff[i] : o;  // staged output slot: dense, or the level's own range
    const uint32_t F = 1u << fan.bits;  // item slots per child (in key order)
    uint32_t b = 0;                     // this child's own fan-out
    if (len > item_max && rem > capbits) {
        if (fan.bits && len <= fan.split_max) {
            b = 1;
            while (b < fan.bits && b < rem && (len >> b) > fan.target) ++b;
        } else {
            atomicAdd(&flags[0], 1ull);  // still too big: the host plans another round
        }
    }
    if (len >= (1ull << 32)) atomicOr(&flags[1], 2ull);  // u32 LDS counts could overflow: count weighted
    for (uint32_t j = 0; j < F; ++j) {
        if (b && j < (1u << b)) continue;  // written by k_fan_split
        DevSeg s;
        s.keys = lk + o * kw;
        s.counts = lc ? lc + o : nullptr;
        s.len = j == 0 ? len : 0;  // slots past the child's own are empty items
        s.key_base = 0;
        s.out_base = 0;
        s.shift = kSingleBin;
        s.nlocal = 1;
        s.pad = 0;
        segs[(uint64_t)i * F + j] = s;
        DevItem it;
        it.seg_begin = i * F + j;
        it.seg_count = 1;
        it.out_off = so;  // distinct <= instances: the child's own range is a safe output slot
        it.rem_bits = rem;
        it.pad = j == 0 ? 0u : kItemEmpty;
        it.total = s.len;
        it.keys0 = s.keys;
        it.counts0 = s.counts;
        items[(uint64_t)i * F + j] = it;
    }
    if (b) {
        // jobs of <= fan_split_small() keys from the front (flags[3] of them),
        // larger ones from the back (flags[4]): each fan-out kernel variant
        // walks only its own
        const ull jb = len <= kFanSmallJob ? atomicAdd(&flags[3], 1ull) : nout - 1 - atomicAdd(&flags[4], 1ull);
        fan.jobs[jb] = DevFanJob{o, len, i * F, b, rem, 0, so};
    } else {
        atomicMax(&flags[2], len);
    }
}

void launch_make_items(void *stream, const ull *offs, const ull *ends, uint32_t nout, const DevParent *parents,
                       uint32_t nparents, const uint64_t *lk, const uint64_t *lc, DevItem *items, DevSeg *segs,
                       uint64_t item_max, uint32_t capbits, ull *flags, uint32_t kw, const FanOut &fan,
                       const ull *doff) {
    if (!nout) return;
    hipLaunchKernelGGL(k_make_items, dim3((nout + 255) / 256), dim3(256), 0, (hipStream_t)stream, offs, ends, nout,
                       parents, nparents, lk, lc, items, segs, item_max, capbits, flags, kw, fan, doff);
}

__global__ __launch_bounds__(256) void k_child_lens(const ull *__restrict__ offs, const ull *__restrict__ ends,
                                                    uint32_t nout, ull *__restrict__ lens) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i <= nout) lens[i] = i < nout ? (ends ? ends[i] : offs[i + 1]) - offs[i] : 0ull;
}

void launch_child_offsets(void *stream, const ull *offs, const ull *ends, uint32_t nout, ull *doff, ull *tmp) {
    hipLaunchKernelGGL(k_child_lens, dim3(nout / 256 + 1), dim3(256), 0, (hipStream_t)stream, offs, ends, nout, doff);
    launch_exclusive_scan(stream, doff, doff, (uint64_t)nout + 1, tmp);
}

// Fan-out split of one oversized child per job: its keys (<= 64 Ki) are
// counting-sorted by the next `bits` (<= 4) key bits into the same index range
// of `dk` (order inside a sub-range is free: items are multisets), and each
// sub-range becomes the item slot item0 + j.  Ranks come from wave ballots (no
// LDS atomics on the few counters) and wait in LDS between the two passes; the
// keys are read twice (the second time from L2: a job is <= 1 MiB).  Jobs are
// latency-bound (a few rows each), so two variants run: 512-thread
// workgroups for jobs of <= 16 Ki keys (32 KiB of ranks: 4 workgroups per CU)
// and 1024-thread ones with 128 KiB of ranks for the larger jobs.
constexpr int kFanBins = 16;  // <= 4 bits per job
constexpr int kFanSmallBlock = 512, kFanSmallMax = 16384;
constexpr int kFanBigBlock = 1024, kFanBigMax = 65536;
uint64_t fan_split_max() { return (uint64_t)kFanBigMax; }
uint64_t fan_split_max_in_place() { return (uint64_t)kFanSmallJob; }
static_assert(kFanSmallMax == kFanSmallJob, "the job list's small/large cut is the small variants' capacity");

// Rank of a lane's key among the wave's valid keys in the same bin (lane
// order), and the bins' running counts: one ballot per bin bit (<= 4) instead
// of one per bin (16), so a row costs ~5 ballots and ~30 VALU instead of 16
// ballots and ~160.  runv: lane q < kFanBins holds bin q's running count
// (lanes q >= 2^bits hold nothing meaningful).
__device__ __forceinline__ uint32_t wave_bin_rank(bool v, uint32_t b, uint32_t bits, uint32_t &runv, uint32_t lane,
                                                  ull lt) {
    const ull vm = __ballot(v);
    ull miss = 0, qmiss = 0;  // lanes whose bin differs from mine / from bin `lane`
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        if (i < bits) {  // block-uniform
            const ull mi = __ballot(v && ((b >> i) & 1u));
            miss |= mi ^ (((b >> i) & 1u) ? ~0ull : 0ull);
            qmiss |= mi ^ (((lane >> i) & 1u) ? ~0ull : 0ull);
        }
    }
    const uint32_t base = (uint32_t)__shfl((int)runv, (int)b, 64);
    const uint32_t rank = base + (uint32_t)__popcll(vm & ~miss & lt);
    if (lane < (uint32_t)kFanBins) runv += (uint32_t)__popcll(vm & ~qmiss);
    return rank;
}

template <typename KT, bool W, int FB, int FMAX>
__global__ __launch_bounds__(FB) void k_fan_split(const DevFanJob *__restrict__ jobs, const ull *__restrict__ flags,
                                                  const KT *__restrict__ sk, const uint64_t *__restrict__ sc,
                                                  KT *__restrict__ dk, uint64_t *__restrict__ dc,
                                                  DevItem *__restrict__ items, DevSeg *__restrict__ segs,
                                                  uint64_t item_max, uint32_t capbits, ull *__restrict__ oflags,
                                                  uint32_t max_jobs) {
    constexpr int kWaves = FB / 64;
    static_assert(FMAX / FB * 64 <= 4096, "ranks fit 12 bits");
    // rows of a job held in registers between the passes (unweighted big jobs)
    // (12 rows of K128 keys: 128 VGPRs, no spills, once the rows' loads share
    // one lane offset; 16 rows spill 24 at the 128-VGPR cap)
    constexpr int kHold = (!W && FMAX > kFanSmallMax) ? 12 : 0;
    __shared__ uint16_t brs[FMAX];                // per key: bin << 12 | rank within (wave, bin)
    __shared__ uint32_t wtot[kWaves][kFanBins];   // per (wave, bin): count, then start in the job's range
    __shared__ uint32_t btot[kFanBins];
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    // the small jobs sit at the front of `jobs` (flags[3]), the large ones at
    // the back (flags[4])
    constexpr bool kBig = FMAX > kFanSmallMax;
    const uint32_t njobs = __builtin_amdgcn_readfirstlane((uint32_t)flags[kBig ? 4 : 3]);
    const uint32_t j0 = kBig ? max_jobs - njobs : 0u;
    for (uint32_t jx = blockIdx.x; jx < njobs; jx += gridDim.x) {
        const DevFanJob jb = jobs[j0 + jx];
        const uint32_t nb = 1u << jb.bits, shift = jb.rem - jb.bits;
        const uint32_t rows = (uint32_t)((jb.len + FB - 1) / FB);  // block-uniform
        const ull lt = (1ull << lane) - 1ull;
        // pass 1: bins and ranks
        uint32_t runv = 0;  // lane q: bin q's running count in this wave
        auto rank_row = [&](uint32_t u, const KT &key) {  // (every lane of the wave: ballots)
            const bool v = !KeyOps<KT>::is_empty(key);
            const uint32_t b = v ? (uint32_t)(KeyOps<KT>::shr(key, shift) & (nb - 1)) : 0u;
            const uint32_t rank = wave_bin_rank(v, b, jb.bits, runv, lane, lt);
            brs[u * FB + t] = (uint16_t)(v ? (b << 12) | rank : 0u);
        };
        // the job's first kHold rows stay in registers for pass 2, so only the
        // rest is read twice (big unweighted jobs: k = 63 children of 16-64 Ki
        // keys, a third of C4's keys)
        KT kk[kHold > 0 ? kHold : 1];
        if (kHold > 0) {
#pragma unroll
            for (int u = 0; u < kHold; ++u) {
                // (the row's start and its live lanes are block-uniform: one
                // lane offset serves every row, no per-row index registers)
                const int32_t left = __builtin_amdgcn_readfirstlane((int32_t)jb.len - u * FB);
                const KT *row = sk + jb.off + (uint64_t)u * FB;
                kk[u] = (int32_t)t < left ? row[t] : KeyOps<KT>::empty();
            }
#pragma unroll
            for (int u = 0; u < kHold; ++u) {
                if ((uint32_t)u < rows) rank_row((uint32_t)u, kk[u]);  // block-uniform
                __builtin_amdgcn_sched_barrier(0);  // one row's masks live at a time
            }
        }
        for (uint32_t u = kHold; u < rows; ++u) {
            const uint64_t idx = (uint64_t)u * FB + t;
            rank_row(u, idx < jb.len ? sk[jb.off + idx] : KeyOps<KT>::empty());
        }
        if (lane < (uint32_t)kFanBins) wtot[wv][lane] = lane < nb ? runv : 0u;
        __syncthreads();
        if (t < nb) {
            uint32_t s = 0;
            for (int w = 0; w < kWaves; ++w) s += wtot[w][t];
            btot[t] = s;
        }
        __syncthreads();
        if (t < nb) {  // thread q: bin q's item, and every wave's start in bin q
            uint32_t a = 0;
            for (uint32_t q = 0; q < t; ++q) a += btot[q];
            const ull o = jb.off + a, len = btot[t], so = jb.doff + a;
            uint32_t w0 = a;
            for (int w = 0; w < kWaves; ++w) {
                const uint32_t c = wtot[w][t];
                wtot[w][t] = w0;
                w0 += c;
            }
            DevSeg sg;
            sg.keys = reinterpret_cast<const uint64_t *>(dk + o);
            sg.counts = W ? dc + o : nullptr;
            sg.len = len;
            sg.key_base = 0;
            sg.out_base = 0;
            sg.shift = kSingleBin;
            sg.nlocal = 1;
            sg.pad = 0;
            segs[jb.item0 + t] = sg;
            DevItem it;
            it.seg_begin = jb.item0 + t;
            it.seg_count = 1;
            it.out_off = so;
            it.rem_bits = jb.rem - jb.bits;
            it.pad = len ? 0u : kItemEmpty;
            it.total = len;
            it.keys0 = sg.keys;
            it.counts0 = sg.counts;
            items[jb.item0 + t] = it;
            if (len > item_max && it.rem_bits > capbits) atomicAdd(&oflags[0], 1ull);
            atomicMax(&oflags[2], len);
        }
        __syncthreads();
        // pass 2: every key to its place (the held rows from registers, the
        // others read again)
        if (kHold > 0) {
#pragma unroll
            for (int u = 0; u < kHold; ++u) {
                if (KeyOps<KT>::is_empty(kk[u])) continue;  // (rows past the job's end were loaded empty)
                const uint32_t br = brs[u * FB + t];
                dk[jb.off + wtot[wv][br >> 12] + (br & 0xFFFu)] = kk[u];
            }
        }
        for (uint32_t u = kHold; u < rows; ++u) {
            const uint64_t idx = (uint64_t)u * FB + t;
            if (idx >= jb.len) continue;
            const KT key = sk[jb.off + idx];
            if (KeyOps<KT>::is_empty(key)) continue;
            const uint32_t br = brs[u * FB + t];
            const ull o = jb.off + wtot[wv][br >> 12] + (br & 0xFFFu);
            dk[o] = key;
            if (W) dc[o] = sc ? sc[jb.off + idx] : 1ull;
        }
        __syncthreads();  // brs / wtot reuse by the next job
    }
}

// Register variant for jobs of <= kFanRegMax keys (the common case: C3
// shards, k=63): one 1024-thread workgroup per job holds the job's keys in
// registers (16 rows), so they are read once — the LDS variants read them
// twice (ranks first, keys again for the scatter) — and only the per-(wave,
// bin) counters live in LDS.  (128 VGPRs, one workgroup per CU; 512-thread
// workgroups for the jobs of <= 8 Ki keys, two per CU, measured no faster.)
constexpr int kFanRegBlock = 1024, kFanRegRows = 16, kFanRegMax = kFanRegBlock * kFanRegRows;
static_assert(kFanRegMax == kFanSmallJob, "the register variant takes every small job");

template <typename KT>
__global__ __launch_bounds__(kFanRegBlock) void k_fan_split_reg(const DevFanJob *__restrict__ jobs,
                                                                const ull *__restrict__ flags,
                                                                const KT *__restrict__ sk, KT *__restrict__ dk,
                                                                DevItem *__restrict__ items,
                                                                DevSeg *__restrict__ segs, uint64_t item_max,
                                                                uint32_t capbits, ull *__restrict__ oflags) {
    constexpr int RB = kFanRegBlock;
    constexpr int kWaves = RB / 64;
    __shared__ uint32_t wtot[kWaves][kFanBins];
    __shared__ uint32_t btot[kFanBins];
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t njobs = __builtin_amdgcn_readfirstlane((uint32_t)flags[3]);  // the small jobs
    const ull lt = (1ull << lane) - 1ull;
    for (uint32_t jx = blockIdx.x; jx < njobs; jx += gridDim.x) {
        const DevFanJob jb = jobs[jx];
        const uint32_t nb = 1u << jb.bits, shift = jb.rem - jb.bits;
        const uint32_t len = (uint32_t)jb.len;
        KT kk[kFanRegRows];
        uint32_t br[kFanRegRows];  // bin << 16 | rank within (wave, bin); ~0: no key
#pragma unroll
        for (int u = 0; u < kFanRegRows; ++u) {
            // (each row's start and live-lane bound are block-uniform: one lane
            // offset serves every row, no per-row index registers)
            const int32_t left = __builtin_amdgcn_readfirstlane((int32_t)len - u * RB);
            const KT *row = sk + jb.off + (uint64_t)u * RB;
            kk[u] = (int32_t)t < left ? row[t] : KeyOps<KT>::empty();
        }
        uint32_t runv = 0;  // lane q: bin q's running count in this wave
#pragma unroll
        for (int u = 0; u < kFanRegRows; ++u) {
            br[u] = ~0u;
            if ((uint32_t)u * RB >= len) continue;  // block-uniform
            const bool v = !KeyOps<KT>::is_empty(kk[u]);
            const uint32_t b = v ? (uint32_t)(KeyOps<KT>::shr(kk[u], shift) & (nb - 1)) : 0u;
            const uint32_t rank = wave_bin_rank(v, b, jb.bits, runv, lane, lt);
            if (v) br[u] = (b << 16) | rank;
            __builtin_amdgcn_sched_barrier(0);  // one row's masks live at a time
        }
        if (lane < (uint32_t)kFanBins) wtot[wv][lane] = lane < nb ? runv : 0u;
        __syncthreads();
        if (t < nb) {
            uint32_t s = 0;
            for (int w = 0; w < kWaves; ++w) s += wtot[w][t];
            btot[t] = s;
        }
        __syncthreads();
        if (t < nb) {  // thread q: bin q's item, and every wave's start in bin q
            uint32_t a = 0;
            for (uint32_t q = 0; q < t; ++q) a += btot[q];
            const ull o = jb.off + a, n = btot[t], so = jb.doff + a;
            uint32_t w0 = a;
            for (int w = 0; w < kWaves; ++w) {
                const uint32_t c = wtot[w][t];
                wtot[w][t] = w0;
                w0 += c;
            }
            DevSeg sg;
            sg.keys = reinterpret_cast<const uint64_t *>(dk + o);
            sg.counts = nullptr;
            sg.len = n;
            sg.key_base = 0;
            sg.out_base = 0;
            sg.shift = kSingleBin;
            sg.nlocal = 1;
            sg.pad = 0;
            segs[jb.item0 + t] = sg;
            DevItem it;
            it.seg_begin = jb.item0 + t;
            it.seg_count = 1;
            it.out_off = so;
            it.rem_bits = jb.rem - jb.bits;
            it.pad = n ? 0u : kItemEmpty;
            it.total = n;
            it.keys0 = sg.keys;
            it.counts0 = nullptr;
            items[jb.item0 + t] = it;
            if (n > item_max && it.rem_bits > capbits) atomicAdd(&oflags[0], 1ull);
            atomicMax(&oflags[2], n);
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kFanRegRows; ++u)
            if (br[u] != ~0u) dk[jb.off + wtot[wv][br[u] >> 16] + (br[u] & 0xFFFFu)] = kk[u];
        __syncthreads();  // wtot reuse by the next job
    }
}

template <typename KT, bool W>
static void fan_launch(hipStream_t s, uint32_t max_jobs, const DevFanJob *jobs, const ull *flags, const KT *sk,
                       const uint64_t *sc, KT *dk, uint64_t *dc, DevItem *items, DevSeg *segs, uint64_t item_max,
                       uint32_t capbits, ull *oflags) {
    const dim3 gs(max_jobs < 4096u ? max_jobs : 4096u), gb(max_jobs < 2048u ? max_jobs : 2048u);
    if (!W) {  // unweighted jobs of <= 16 Ki keys: keys held in registers (read once)
        hipLaunchKernelGGL((k_fan_split_reg<KT>), gb, dim3(kFanRegBlock), 0, s, jobs, flags, sk, dk, items, segs,
                           item_max, capbits, oflags);
    } else {
        hipLaunchKernelGGL((k_fan_split<KT, W, kFanSmallBlock, kFanSmallMax>), gs, dim3(kFanSmallBlock), 0, s, jobs,
                           flags, sk, sc, dk, dc, items, segs, item_max, capbits, oflags, max_jobs);
    }
    // the large jobs are rare: a small grid walks them
    hipLaunchKernelGGL((k_fan_split<KT, W, kFanBigBlock, kFanBigMax>), dim3(max_jobs < 512u ? max_jobs : 512u),
                       dim3(kFanBigBlock), 0, s, jobs, flags, sk, sc, dk, dc, items, segs, item_max, capbits, oflags,
                       max_jobs);
}

void launch_fan_split(void *stream, const DevFanJob *jobs, uint32_t max_jobs, const ull *flags, const uint64_t *sk,
                      const uint64_t *sc, uint64_t *dk, uint64_t *dc, DevItem *items, DevSeg *segs,
                      uint64_t item_max, uint32_t capbits, ull *oflags, bool wide) {
    if (!max_jobs) return;
    hipStream_t s = (hipStream_t)stream;
    if (wide) {
        const K128 *a = reinterpret_cast<const K128 *>(sk);
        K128 *d = reinterpret_cast<K128 *>(dk);
        if (sc)
            fan_launch<K128, true>(s, max_jobs, jobs, flags, a, sc, d, dc, items, segs, item_max, capbits, oflags);
        else
            fan_launch<K128, false>(s, max_jobs, jobs, flags, a, sc, d, dc, items, segs, item_max, capbits, oflags);
    } else {
        const ull *a = reinterpret_cast<const ull *>(sk);
        ull *d = reinterpret_cast<ull *>(dk);
        if (sc)
            fan_launch<ull, true>(s, max_jobs, jobs, flags, a, sc, d, dc, items, segs, item_max, capbits, oflags);
        else
            fan_launch<ull, false>(s, max_jobs, jobs, flags, a, sc, d, dc, items, segs, item_max, capbits, oflags);
    }
}

// Sampled partition capacities: the slot of bin b gets scale * (sqrt(s) + 3)^2
// keys (s = H[b], the bin's sampled count; (sqrt(s) + 3)^2 = s + 6 sqrt(s) + 9
// bounds the Poisson mean that an observed s allows at ~6 sigma, also when s
// came out low), + 1% + 64, rounded up to 16 keys.
__global__ __launch_bounds__(256) void k_part_capacity(ull *__restrict__ H, uint32_t nout,
                                                       const DevCapParent *__restrict__ parents, uint32_t nparents,
                                                       double mul) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nout) return;
    uint32_t lo = 0, hi = nparents;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (parents[mid].out_base <= i) lo = mid; else hi = mid;
    }
    const double scale = parents[lo].scale, s = (double)H[i];
    const double r = sqrt(s) + 3.0;
    const double c = (r * r * scale * 1.01 + 64.0) * mul;
    H[i] = ((ull)c + 15) & ~15ull;
}

void launch_part_capacity(void *stream, ull *H, uint32_t nout, const DevCapParent *parents, uint32_t nparents,
                          double mul) {
    if (!nout) return;
    hipLaunchKernelGGL(k_part_capacity, dim3((nout + 255) / 256), dim3(256), 0, (hipStream_t)stream, H, nout,
                       parents, nparents, mul);
}

// ---------------------------------------------------------------------------
// Sorted runs (okm_add_sorted_pairs_device): key ranges by binary search
// ---------------------------------------------------------------------------

template <typename KT>
__device__ __forceinline__ uint64_t lower_bound_bin(const KT *keys, uint64_t lo, uint64_t hi, uint32_t shift,
                                                    uint64_t base, uint64_t target) {
    // first j in [lo, hi) with (key_j >> shift) - base >= target (keys sorted; modulo 2^64 is exact
    // because every key of the range lies in the part whose prefix `base` describes)
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const uint64_t x = (shift >= (uint32_t)KeyOps<KT>::kBits ? 0ull : KeyOps<KT>::shr(keys[mid], shift)) - base;
        if (x < target) lo = mid + 1; else hi = mid;
    }
    return lo;
}

template <typename KT>
__global__ void k_bin_bounds(const KT *__restrict__ keys, uint64_t n, uint32_t shift, uint32_t nbins,
                             ull *__restrict__ out) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nbins) return;
    out[b] = b == nbins ? n : lower_bound_bin(keys, 0, n, shift, 0, b);
}

void launch_bin_bounds(void *stream, const uint64_t *keys, uint64_t n, uint32_t shift, uint32_t nbins,
                       unsigned long long *out, bool wide) {
    const dim3 g((nbins + 1 + 255) / 256), b(256);
    if (wide)
        hipLaunchKernelGGL(k_bin_bounds<K128>, g, b, 0, (hipStream_t)stream, reinterpret_cast<const K128 *>(keys), n,
                           shift, nbins, out);
    else
        hipLaunchKernelGGL(k_bin_bounds<ull>, g, b, 0, (hipStream_t)stream, reinterpret_cast<const ull *>(keys), n,
                           shift, nbins, out);
}

// One thread per item: item i is child c of part parts[p] (split by `bits`);
// its segment in run r is the child's key range within rbins[p * nruns + r].
// The part of item i (parts sorted by item_base).
__device__ __forceinline__ uint32_t sorted_part_of(const DevSortedPart *__restrict__ parts, uint32_t nparts,
                                                   uint32_t i) {
    uint32_t lo = 0, hi = nparts;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (parts[mid].item_base <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// bounds[i * nruns + r] = where item i's key range starts in run r: one
// thread per (item, run), so the searches over the runs run side by side
// instead of 2 x nruns of them back to back in one thread per item.  Each
// search interpolates first: a part's keys are spread smoothly over its key
// range (canonical-key density varies linearly, not in steps), so two
// interpolation probes leave a window of ~sqrt(sqrt(n)) keys, where a plain
// binary search over a 200 K-key slice takes ~18 dependent loads.  After
// kInterp probes, or once the window is small, bisection finishes (exact
// whatever the distribution).
template <typename KT>
__device__ __forceinline__ uint64_t lower_bound_interp(const KT *keys, uint64_t n, uint32_t shift, uint64_t base,
                                                       uint64_t target) {
    constexpr int kInterp = 3;
    // f(j) = (key_j >> shift) - base >= target; v(j): the key's top bits as a
    // double (interpolation only: approximate is fine)
    // (only a guess: f decides, so a key whose top bits do not fit 64 bits
    // costs probes, never the answer)
    const uint32_t vs = shift > 20 ? shift - 20 : 0;  // 20 bits below the child index
    auto v = [&](const KT &k) -> double {
        return (double)(vs >= (uint32_t)KeyOps<KT>::kBits ? 0ull : KeyOps<KT>::shr(k, vs));
    };
    auto f = [&](const KT &k) -> bool {
        return (shift >= (uint32_t)KeyOps<KT>::kBits ? 0ull : KeyOps<KT>::shr(k, shift)) - base >= target;
    };
    uint64_t lo = 0, hi = n;  // answer in [lo, hi]
    if (n == 0) return 0;
    const KT k0 = keys[0], k1 = keys[n - 1];
    if (f(k0)) return 0;
    if (!f(k1)) return n;
    // invariants: f(lo) false, f(hi) true; answer in (lo, hi]
    hi = n - 1;
    double vlo = v(k0), vhi = v(k1);
    const double vt = (double)(base + target) * (double)(1ull << (shift - vs));
#pragma unroll 1
    for (int it = 0; it < kInterp && hi - lo > 64; ++it) {
        double fr = vhi > vlo ? (vt - vlo) / (vhi - vlo) : 0.5;
        fr = fr < 0.0 ? 0.0 : (fr > 1.0 ? 1.0 : fr);
        uint64_t m = lo + 1 + (uint64_t)(fr * (double)(hi - lo - 1));
        if (m >= hi) m = hi - 1;
        const KT km = keys[m];
        if (f(km)) { hi = m; vhi = v(km); } else { lo = m; vlo = v(km); }
    }
    ++lo;  // answer in [lo, hi]: first true
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (f(keys[mid])) hi = mid; else lo = mid + 1;
    }
    return lo;
}

template <typename KT>
__global__ void k_sorted_bounds(const DevSortedPart *__restrict__ parts, uint32_t nparts, uint32_t nitems,
                                const DevSeg *__restrict__ rbins, uint32_t nruns, uint32_t shift1,
                                ull *__restrict__ bounds) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= (uint64_t)nitems * nruns) return;
    const uint32_t i = (uint32_t)(x / nruns), r = (uint32_t)(x % nruns);
    const DevSortedPart P = parts[sorted_part_of(parts, nparts, i)];
    const uint32_t c = i - P.item_base;
    const DevSeg rb = rbins[(uint64_t)P.slot * nruns + r];
    bounds[x] = P.bits && c ? lower_bound_interp(reinterpret_cast<const KT *>(rb.keys), rb.len, shift1 - P.bits,
                                                 (uint64_t)P.bin << P.bits, c)
                            : 0;
}

template <typename KT>
__global__ void k_sorted_items(const DevSortedPart *__restrict__ parts, uint32_t nparts, uint32_t nitems,
                               const DevSeg *__restrict__ rbins, uint32_t nruns, uint32_t shift1, uint32_t kw,
                               DevItem *__restrict__ items, DevSeg *__restrict__ segs, ull *__restrict__ itemtot,
                               uint64_t item_max, uint32_t capbits, ull *__restrict__ flags,
                               const ull *__restrict__ bounds, ull *__restrict__ part_max) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    // no early exit: the wave reductions at the end need every lane
    const bool live = i < nitems;
    ull tot = 0;
    uint32_t slot = ~0u;
    if (live) {
        const DevSortedPart P = parts[sorted_part_of(parts, nparts, i)];
        slot = P.slot;
        const uint32_t c = i - P.item_base;
        const uint32_t shift = shift1 - P.bits;                 // child = next `bits` key bits
        const bool last = !P.bits || c + 1 == (1u << P.bits);  // the part's last child ends where its range does
        for (uint32_t r = 0; r < nruns; ++r) {
            const DevSeg rb = rbins[(uint64_t)P.slot * nruns + r];
            const uint64_t s0 = bounds[(uint64_t)i * nruns + r];
            const uint64_t s1 = last ? rb.len : bounds[(uint64_t)(i + 1) * nruns + r];
            DevSeg sg;
            sg.keys = rb.keys + s0 * kw;
            sg.counts = rb.counts ? rb.counts + s0 : nullptr;
            sg.len = s1 - s0;
            sg.key_base = 0;
            sg.out_base = 0;
            sg.shift = kSingleBin;
            sg.nlocal = 1;
            sg.pad = 0;
            segs[(uint64_t)i * nruns + r] = sg;
            tot += s1 - s0;
        }
        DevItem it;
        it.seg_begin = i * nruns;
        it.seg_count = nruns;
        it.out_off = 0;  // set from the scan of itemtot (k_set_out_off)
        it.rem_bits = shift;
        it.pad = 0;
        it.total = tot;
        it.keys0 = segs[(uint64_t)i * nruns].keys;
        it.counts0 = segs[(uint64_t)i * nruns].counts;
        items[i] = it;
        itemtot[i] = tot;
        if (tot > item_max && shift > capbits) atomicAdd(&flags[0], 1ull);
    }
    // the maxima: one atomic per wave (per part within it), not per item --
    // a part's thousand items on one address serialise in L2
    ull wmax = tot;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const ull o = __shfl_xor(wmax, d, 64);
        wmax = o > wmax ? o : wmax;
    }
    // items are consecutive lanes: a wave whose lane 0 has no item has none
    const uint32_t slot0 = __builtin_amdgcn_readfirstlane(slot);
    if (slot0 == ~0u) return;  // wave-uniform
    const bool one_part = __ballot(live && slot != slot0) == 0;  // wave-uniform
    if ((threadIdx.x & 63u) == 0) atomicMax(&flags[1], wmax);
    if (one_part) {
        if ((threadIdx.x & 63u) == 0) atomicMax(&part_max[slot0], wmax);
    } else if (live) {
        atomicMax(&part_max[slot], tot);
    }
}

__global__ void k_set_out_off(DevItem *__restrict__ items, uint32_t nitems, const ull *__restrict__ off) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nitems) items[i].out_off = off[i];
}

void launch_sorted_items(void *stream, const DevSortedPart *parts, uint32_t nparts, uint32_t nitems,
                         const DevSeg *rbins, uint32_t nruns, uint32_t shift1, DevItem *items, DevSeg *segs,
                         unsigned long long *itemtot, uint64_t item_max, uint32_t capbits, unsigned long long *flags,
                         bool wide, unsigned long long *bounds, unsigned long long *part_max) {
    if (!nitems) return;
    const dim3 g((nitems + 255) / 256), b(256);
    const dim3 gb((uint32_t)(((uint64_t)nitems * nruns + 255) / 256));
    hipStream_t s = (hipStream_t)stream;
    if (wide) {
        hipLaunchKernelGGL(k_sorted_bounds<K128>, gb, b, 0, s, parts, nparts, nitems, rbins, nruns, shift1, bounds);
        hipLaunchKernelGGL(k_sorted_items<K128>, g, b, 0, s, parts, nparts, nitems, rbins, nruns, shift1, 2u, items,
                           segs, itemtot, item_max, capbits, flags, (const ull *)bounds, part_max);
    } else {
        hipLaunchKernelGGL(k_sorted_bounds<ull>, gb, b, 0, s, parts, nparts, nitems, rbins, nruns, shift1, bounds);
        hipLaunchKernelGGL(k_sorted_items<ull>, g, b, 0, s, parts, nparts, nitems, rbins, nruns, shift1, 1u, items,
                           segs, itemtot, item_max, capbits, flags, (const ull *)bounds, part_max);
    }
}

void launch_set_out_off(void *stream, DevItem *items, uint32_t nitems, const unsigned long long *off) {
    if (!nitems) return;
    hipLaunchKernelGGL(k_set_out_off, dim3((nitems + 255) / 256), dim3(256), 0, (hipStream_t)stream, items, nitems,
                       off);
}

// ---------------------------------------------------------------------------
// Result assembly
// ---------------------------------------------------------------------------

template <typename KT, bool NARROW>
__global__ __launch_bounds__(256) void k_compact_items(const DevItem *__restrict__ items,
                                                       uint32_t nitems, const ull *__restrict__ n_out,
                                                       const ull *__restrict__ dense_off,
                                                       const KT *__restrict__ sk,
                                                       const uint64_t *__restrict__ sc,
                                                       KT *__restrict__ dk,
                                                       uint64_t *__restrict__ dc,
                                                       const ull *__restrict__ guard,
                                                       const ull *__restrict__ err,
                                                       const ull *__restrict__ d_nitems,
                                                       const ull *__restrict__ d_base) {
    if ((guard && (guard[0] | guard[1])) || (err && *err)) return;
    if (d_base) {  // the table's next free entry, known on the device only (pipelined key-range groups)
        const ull b = *d_base;
        if (b & kBasePoison) return;  // an earlier group was abandoned: it is counted again, and so is this one
        dk += b;
        dc += b;
    }
    if (d_nitems) nitems = __builtin_amdgcn_readfirstlane((uint32_t)min((ull)nitems, *d_nitems));
    // One wave per item (an item holds ~600 entries at C2: a 256-thread block
    // per item left most lanes idle behind three dependent descriptor loads);
    // the next item's descriptor is loaded during this item's copy, and every
    // lane keeps four entries in flight.
    // (an odd wave stride: fan-out slots, 2^bits per child, spread over waves)
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * 4u - 1u;
    uint32_t item = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (item >= nw) return;  // the last wave: its items belong to wave 0
    // sk == nullptr: the items' runs were staged in place (over their input,
    // okm_count.hip out_slot_keys), the counts at sc + out_off
    uint64_t n = 0, src = 0, dst = 0;
    const KT *kb = nullptr;
    if (item < nitems) {
        n = n_out[item];
        src = items[item].out_off;
        dst = dense_off[item];
        kb = sk ? sk + src : reinterpret_cast<const KT *>(items[item].keys0);
    }
    const uint32_t *sc32 = reinterpret_cast<const uint32_t *>(sc);
    for (; item < nitems; item += nw) {
        const uint32_t nxt = item + nw;
        uint64_t nn = 0, ns = 0, nd = 0;
        const KT *nkb = nullptr;
        if (nxt < nitems) {
            nn = n_out[nxt];
            ns = items[nxt].out_off;
            nd = dense_off[nxt];
            nkb = sk ? sk + ns : reinterpret_cast<const KT *>(items[nxt].keys0);
        }
        uint64_t j = lane;
        for (; j + 192 < n; j += 256) {
            KT k[4];
            uint64_t c[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                k[q] = kb[j + 64 * q];
                c[q] = NARROW ? (uint64_t)sc32[src + j + 64 * q] : sc[src + j + 64 * q];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                dk[dst + j + 64 * q] = k[q];
                dc[dst + j + 64 * q] = c[q];
            }
        }
        for (; j < n; j += 64) {
            dk[dst + j] = kb[j];
            dc[dst + j] = NARROW ? (uint64_t)sc32[src + j] : sc[src + j];
        }
        n = nn;
        src = ns;
        dst = nd;
        kb = nkb;
    }
}

// After a group's compaction: *d_base += the group's distinct keys (the
// exclusive scan's total).  An abandoned launch (guard / err) poisons the
// base instead, so no later group of the same pipelined pass writes into the
// table (the host counts them again from the first abandoned group, at the
// base without the poison bit: every group before it is in place).
__global__ void k_advance_base(ull *__restrict__ d_base, const ull *__restrict__ total, const ull *__restrict__ guard,
                               const ull *__restrict__ err) {
    const ull b = *d_base;
    if (b & kBasePoison) return;
    if ((guard && (guard[0] | guard[1])) || (err && *err)) {
        *d_base = b | kBasePoison;
        return;
    }
    *d_base = b + *total;
}

void launch_advance_base(void *stream, unsigned long long *d_base, const unsigned long long *total,
                         const unsigned long long *guard, const unsigned long long *err) {
    hipLaunchKernelGGL(k_advance_base, dim3(1), dim3(1), 0, (hipStream_t)stream, d_base, total, guard, err);
}

void launch_compact_items(void *stream, const DevItem *items, uint32_t nitems,
                          const unsigned long long *n_out, const unsigned long long *dense_off,
                          const uint64_t *src_keys, const uint64_t *src_counts, uint64_t *dst_keys,
                          uint64_t *dst_counts, bool wide, bool narrow, const unsigned long long *guard,
                          const unsigned long long *err, const unsigned long long *d_nitems,
                          const unsigned long long *d_base) {
    if (!nitems) return;
    constexpr uint32_t cap = 4096;  // grids of 2048 / 8192 measured the same (profiles/AB_LOG.md round 4)
    const dim3 g(nitems / 4u + 1u < cap ? nitems / 4u + 1u : cap), b(256);  // one wave per item
    hipStream_t s = (hipStream_t)stream;
    const K128 *sk2 = reinterpret_cast<const K128 *>(src_keys);
    K128 *dk2 = reinterpret_cast<K128 *>(dst_keys);
    const ull *sk1 = reinterpret_cast<const ull *>(src_keys);
    ull *dk1 = reinterpret_cast<ull *>(dst_keys);
    if (wide && narrow)
        hipLaunchKernelGGL((k_compact_items<K128, true>), g, b, 0, s, items, nitems, n_out, dense_off, sk2, src_counts,
                           dk2, dst_counts, guard, err, d_nitems, d_base);
    else if (wide)
        hipLaunchKernelGGL((k_compact_items<K128, false>), g, b, 0, s, items, nitems, n_out, dense_off, sk2,
                           src_counts, dk2, dst_counts, guard, err, d_nitems, d_base);
    else if (narrow)
        hipLaunchKernelGGL((k_compact_items<ull, true>), g, b, 0, s, items, nitems, n_out, dense_off, sk1, src_counts,
                           dk1, dst_counts, guard, err, d_nitems, d_base);
    else
        hipLaunchKernelGGL((k_compact_items<ull, false>), g, b, 0, s, items, nitems, n_out, dense_off, sk1,
                           src_counts, dk1, dst_counts, guard, err, d_nitems, d_base);
}

__global__ __launch_bounds__(256) void k_item_flags(const DevItem *__restrict__ items, uint32_t n,
                                                    ull *__restrict__ flags) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i <= n) flags[i] = i < n && items[i].pad != kItemEmpty ? 1ull : 0ull;
}

__global__ __launch_bounds__(256) void k_item_scatter(const DevItem *__restrict__ items, uint32_t n,
                                                      const ull *__restrict__ pos, DevItem *__restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n && pos[i + 1] != pos[i]) out[pos[i]] = items[i];
}

void launch_item_compact(void *stream, const DevItem *items, uint32_t nslots, DevItem *out, ull *flags, ull *pos,
                         ull *scan_tmp) {
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_item_flags, dim3(nslots / 256 + 1), dim3(256), 0, s, items, nslots, flags);
    launch_exclusive_scan(stream, flags, pos, (uint64_t)nslots + 1, scan_tmp);
    if (nslots) hipLaunchKernelGGL(k_item_scatter, dim3((nslots + 255) / 256), dim3(256), 0, s, items, nslots, pos, out);
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

template <typename KT>
__global__ __launch_bounds__(kFilterBlock) void k_filter_scatter(
    const KT *__restrict__ keys, const uint64_t *__restrict__ counts, uint64_t n,
    uint64_t min_count, const ull *__restrict__ block_offsets, KT *__restrict__ dk,
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
                           uint64_t *dst_keys, uint64_t *dst_counts, bool wide) {
    const uint32_t nb = filter_blocks(n);
    if (!nb) return;
    if (wide)
        hipLaunchKernelGGL(k_filter_scatter<K128>, dim3(nb), dim3(kFilterBlock), 0, (hipStream_t)stream,
                           reinterpret_cast<const K128 *>(keys), counts, n, min_count, block_offsets,
                           reinterpret_cast<K128 *>(dst_keys), dst_counts);
    else
        hipLaunchKernelGGL(k_filter_scatter<ull>, dim3(nb), dim3(kFilterBlock), 0, (hipStream_t)stream,
                           reinterpret_cast<const ull *>(keys), counts, n, min_count, block_offsets,
                           reinterpret_cast<ull *>(dst_keys), dst_counts);
}

// ---------------------------------------------------------------------------
// |A ∩ B| for compare.rs:58
// ---------------------------------------------------------------------------

template <typename KT>
__global__ __launch_bounds__(256) void k_intersect_count(const KT *__restrict__ a, uint64_t na,
                                                         const KT *__restrict__ b, uint64_t nb,
                                                         ull *__restrict__ out) {
    __shared__ ull wsum[4];
    ull hits = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < na; i += (uint64_t)gridDim.x * 256) {
        const KT x = a[i];
        uint64_t lo = 0, hi = nb;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (KeyOps<KT>::lt(b[mid], x)) lo = mid + 1; else hi = mid;
        }
        hits += (lo < nb && KeyOps<KT>::eq(b[lo], x));
    }
    ull total;
    block_excl_scan<256>(hits, wsum, &total);
    if (threadIdx.x == 0 && total) atomicAdd(out, total);
}

void launch_intersect_count(void *stream, const uint64_t *a, uint64_t na, const uint64_t *b,
                            uint64_t nb, unsigned long long *out, bool wide) {
    if (!na || !nb) return;
    uint64_t g = (na + 255) / 256;
    if (g > 8192) g = 8192;
    if (wide)
        hipLaunchKernelGGL(k_intersect_count<K128>, dim3((uint32_t)g), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const K128 *>(a), na, reinterpret_cast<const K128 *>(b), nb, out);
    else
        hipLaunchKernelGGL(k_intersect_count<ull>, dim3((uint32_t)g), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const ull *>(a), na, reinterpret_cast<const ull *>(b), nb, out);
}

}  // namespace okm
