// okm_extract.hip — L1 pass: batch bytes -> canonical k-mers -> key-range bins.
//
// Restates on the device:
//   kmer.rs:12-20   dna_base_to_u64      -> pack4: SWAR codes + invalid mask (+ U/u->T
//                                          of needletail normalize, count.rs:71)
//   kmer.rs:37-57   seq_to_u64           -> fwd_top64: a slice of the packed codes
//   kmer.rs:79-94   reverse_complement   -> rc_low64: a slice of the complemented codes
//   kmer.rs:99-106  canonical_u64        -> min(fwd, rc)
//   count.rs:23-38  window loop          -> scan_words (okm_scan.h), invalid-mask test
//
// Two kernels per batch.  extract_hist counts, per persistent block, the keys
// of each bin (top l1 bits of the 2k-bit key); the host turns the totals into
// bin offsets.  extract_scatter places every key exactly: each block owns one
// contiguous slice per bin (claimed with one returning atomic per (block,
// bin)), and every 16384-window tile (1024-thread workgroups, 128 KiB of staged keys; 8192
// windows: 1.62 vs 1.48 ms on C2) is counting-sorted by bin in LDS first so
// that each bin's keys leave the CU as one contiguous run (~256 B at 512 bins)
// instead of 8-byte scattered stores (which cost 3.5x the bytes in HBM
// writes).
//
// Windows are extracted directly (okm_scan.h: every window's key is a slice
// of SWAR-packed codes, no rolling state), so the window index is a
// compile-time constant for every k and extract_scatter keeps a thread's 16
// keys (and their within-bin ranks, returned by the histogram atomic) in
// registers, computing each k-mer once.  Kernels are instantiated for common
// k (template K: constant shifts) besides the runtime-k one.  Emits are
// branch-free: an invalid window counts into a dummy bin.
#include "okm_scan.h"

namespace okm {

__device__ __forceinline__ uint32_t bin_of(uint64_t key, uint32_t shift) {
    return shift >= 64 ? 0u : (uint32_t)(key >> shift);
}
// K >= 21 (compile time): shift = 2K - l1_bits lies in [32, 55] (l1_bits <= 10),
// so the bin is a 32-bit shift of the key's high word
template <int K>
__device__ __forceinline__ uint32_t bin_k(uint64_t key, uint32_t shift) {
    if (K >= 21) return (uint32_t)(key >> 32) >> (shift - 32u);
    return bin_of(key, shift);
}

constexpr int kExtractBlock = 256;  // histogram kernels
constexpr int kScatBlock = 1024;    // k <= 32 scatter: one workgroup per CU (128 KiB of staged keys)
constexpr int kScatWpe = 4;         // ... waves per SIMD its register budget must allow
constexpr int kSegS = 16;           // scatter: window starts per thread
constexpr int kTile = kScatBlock * kSegS;  // scatter tile: 16384 windows
static_assert(kSegS % 16 == 0, "scan_windows loads whole 16-B words");
constexpr int kSegH = 64;                      // hist: window starts per thread
constexpr int kHTile = kExtractBlock * kSegH;  // hist tile: 16384 windows
static_assert(kHTile % kTile == 0, "scatter tile must divide the hist tile");
// First-level key-range bins (2^bits <= the scatter block): 9 bits (8: extraction
// 1.51 vs 1.56 ms but partition 1.92 vs 1.74 ms on C2, C3 724 vs 696 ms); 10 for a
// context that folds (okm_engine.hip fold(): C3 414 vs 461 ms, C2 5.44 vs 5.23);
// k in 33..64: 9 (8: k=63 1 Gbases 39.3 vs 34.8 ms, C4 248 vs 237 ms)
constexpr int kL1Bits = 9, kL1BitsFold = 10, kL1BitsW = 9;
constexpr int kMaxL1Bins = 1 << kL1BitsFold;  // k <= 32 kernels
static_assert(2 * 21 - kL1BitsFold >= 32, "bin_k: the L1 shift of k >= 21 lies in the key's high word");
constexpr int kMaxL1BinsW = 1 << kL1BitsW;  // k in 33..64 kernels
static_assert(kMaxL1Bins <= kScatBlock, "one bin per scatter thread");

constexpr uint32_t gcd_u32(uint32_t a, uint32_t b) { return b ? gcd_u32(b, a % b) : a; }
constexpr uint32_t lcm_u32(uint32_t a, uint32_t b) { return a / gcd_u32(a, b) * b; }
uint32_t extract_max_bins(bool wide) { return (uint32_t)(wide ? kMaxL1BinsW : kMaxL1Bins); }
uint32_t extract_l1_bits(bool wide, bool folding) {
    return wide ? (uint32_t)kL1BitsW : (uint32_t)(folding ? kL1BitsFold : kL1Bits);
}

template <int K>
__global__ __launch_bounds__(kExtractBlock) void k_extract_hist(const uint8_t *__restrict__ seq, ExtractGeom g,
                                                                uint32_t *__restrict__ HC, ull *__restrict__ Hg) {
    __shared__ uint32_t lh[kMaxL1Bins + 1];  // + dummy bin for invalid windows
    for (uint32_t b = threadIdx.x; b <= g.nbins; b += kExtractBlock) lh[b] = 0;
    lds_sync();
    const uint64_t beg = (uint64_t)blockIdx.x * g.stride * g.chunk;  // stride > 1: a sample of the chunks
    const uint64_t end = beg + g.chunk < g.n ? beg + g.chunk : g.n;
    const uint32_t shift = g.shift, nb = g.nbins;
    for (uint64_t t0 = beg; t0 < end; t0 += kHTile) {
        const uint64_t w0 = t0 + (uint64_t)threadIdx.x * kSegH;
        if (w0 < end)
            scan_windows<kSegH, K>(seq, g.n, w0, g.k, [&](int, uint64_t key, bool valid) {
                atomicAdd(&lh[valid ? bin_k<K>(key, shift) : nb], 1u);
            });
    }
    lds_sync();
    for (uint32_t b = threadIdx.x; b < nb; b += kExtractBlock) {
        const uint32_t h = lh[b];
        if (HC) HC[(uint64_t)blockIdx.x * nb + b] = h;
        if (h) atomicAdd(&Hg[b], (ull)h);
    }
}

// Shared tail of the scatter tile: bin offsets within the tile.
template <int BLOCK>
__device__ __forceinline__ uint32_t tile_offsets(uint32_t t, uint32_t nb, uint32_t *hist, uint32_t *lofs,
                                                 uint32_t *lcur, ull *wsum) {
    ull tile_n;
    const uint32_t my = t < nb ? hist[t] : 0u;
    const uint32_t off = (uint32_t)block_excl_scan<BLOCK>(my, wsum, &tile_n);
    if (t < nb) {
        lofs[t] = off;
        lcur[t] = off;
    }
    return (uint32_t)tile_n;
}

// Sampled-capacity placement: this tile's run of bin t claims its slot.
__device__ __forceinline__ void claim_tile(uint32_t t, uint32_t nb, const uint32_t *hist, ull *cursor,
                                           const ull *cap_end, ull *ovf, ull *gcur) {
    if (t < nb) {
        const uint32_t h = hist[t];
        ull g = ~0ull;
        if (h) {
            const ull p = atomicAdd(&cursor[t * kL1CurStride], (ull)h);
            if (p + h <= cap_end[t])
                g = p;
            else
                atomicOr(ovf, 1ull);
        }
        gcur[t] = g;
    }
}

template <int K>
__global__ __launch_bounds__(kScatBlock) __attribute__((amdgpu_waves_per_eu(kScatWpe))) void k_extract_scatter(
    const uint8_t *__restrict__ seq, ExtractGeom g, const uint32_t *__restrict__ HC, ull *__restrict__ cursor,
    uint64_t *__restrict__ out, const ull *__restrict__ cap_end, ull *__restrict__ ovf) {
    __shared__ ull stage[kTile + 64];        // + one dummy slot per lane for invalid windows
    __shared__ ull gcur[kMaxL1Bins];         // this block's next output index per bin
    __shared__ uint32_t hist[kMaxL1Bins + 1];
    __shared__ uint32_t lofs[kMaxL1Bins];    // tile-local start of each bin in `stage`
    __shared__ ull wsum[kScatBlock / 64];
    const uint32_t t = threadIdx.x;
    const uint32_t nb = g.nbins;
    // HC: exact per-block counts (one claim per bin for the whole chunk);
    // HC == nullptr: sampled capacities, one claim per (tile, bin), checked
    // against cap_end (a run that would cross it is dropped and *ovf set)
    if (t < nb && HC) {
        const uint32_t h = HC[(uint64_t)blockIdx.x * nb + t];
        gcur[t] = h ? atomicAdd(&cursor[t], (ull)h) : 0ull;
    }
    const uint64_t beg = (uint64_t)blockIdx.x * g.chunk;
    const uint64_t end = beg + g.chunk < g.n ? beg + g.chunk : g.n;
    const uint32_t shift = g.shift;
    // this tile's bytes, loaded one tile ahead by branch-free clamped loads
    // (load_windows_clamped: bytes past the batch are marked invalid later)
    WinWords<kSegS> ww;
    load_windows_clamped<kSegS>(seq, g.n, beg + (uint64_t)t * kSegS, ww);
    const ull capb = (!HC && t < nb) ? cap_end[t] : 0ull;
    // five barriers per tile instead of seven: each thread clears its own bin's
    // counter once it has read it (the next tile's atomics are barriers away),
    // and the offsets scan needs no trailing barrier (its slots are next
    // written in the next tile)
    for (uint32_t b = t; b <= nb; b += kScatBlock) hist[b] = 0;
    lds_sync();
    for (uint64_t t0 = beg; t0 < end; t0 += kTile) {
        const uint64_t w0 = t0 + (uint64_t)t * kSegS;
        const bool live = w0 < end;
        uint32_t tile_n;
        uint32_t hmine;
        {  // one sweep: keys and their within-bin ranks stay in registers
            ull kk[kSegS];
            uint32_t rk[kSegS / 2];  // two within-bin ranks (< 2^15) per word; the bin is recomputed
            uint32_t vm = 0;         // valid windows
#pragma unroll
            for (int j = 0; j < kSegS / 2; ++j) rk[j] = 0;
            auto emit = [&](int j, uint64_t key, bool valid) {
                const uint32_t b = valid ? bin_k<K>(key, shift) : nb;
                kk[j] = key;
                rk[j >> 1] |= (atomicAdd(&hist[b], 1u) & 0xFFFFu) << (16 * (j & 1));
                vm |= valid ? 1u << j : 0u;
            };
            if (live) scan_words<kSegS, K>(ww, g.k, emit, g.n - w0);
            // next tile, in flight meanwhile; unconditional (a clamped load past the
            // end is harmless), so the loaded registers need no merge copies
            load_windows_clamped<kSegS>(seq, g.n, w0 + kTile, ww);
            lds_sync();
            hmine = t <= nb ? hist[t] : 0u;
            if (t <= nb) hist[t] = 0;
            {
                ull tn;
                const uint32_t off = (uint32_t)block_excl_scan_1b<kScatBlock>(t < nb ? hmine : 0u, wsum, &tn);
                if (t < nb) lofs[t] = off;
                tile_n = (uint32_t)tn;
            }
            // sampled capacities: issue this tile's claim now, consume it after the staging
            uint32_t ch = 0;
            ull cp;
            if (!HC && t < nb) {
                ch = hmine;
                cp = atomicAdd(&cursor[t * kL1CurStride], (ull)ch);  // + 0 when empty: no branch
            }
            lds_sync();
#pragma unroll
            for (int j = 0; j < kSegS; ++j) {
                const uint32_t rank = (rk[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                const uint32_t dst = (vm >> j) & 1u ? lofs[bin_k<K>(kk[j], shift)] + rank : (uint32_t)kTile + (t & 63u);
                stage[dst] = kk[j];
            }
            if (!HC && t < nb) {
                const bool fits = ch && cp + ch <= capb;
                if (ch && !fits) atomicOr(ovf, 1ull);
                gcur[t] = fits ? cp : ~0ull;
            }
        }
        lds_sync();
        // each bin's keys are contiguous in `stage` and go to a contiguous run
        for (uint32_t j = t; j < tile_n; j += kScatBlock) {
            const ull key = stage[j];
            const uint32_t b = bin_k<K>(key, shift);
            const ull gb = gcur[b];
            if (gb != ~0ull) out[gb + (j - lofs[b])] = key;
        }
        lds_sync();
        if (HC && t < nb) gcur[t] += hmine;
    }
}

__global__ __launch_bounds__(256) void k_fill_line_tails(const ull *__restrict__ end, uint32_t nbins,
                                                         uint64_t *__restrict__ keys, const ull *__restrict__ cap) {
    const uint32_t b = blockIdx.x * 16 + (threadIdx.x >> 4), j = threadIdx.x & 15;
    if (b >= nbins) return;
    const ull e = end[cap ? b * kL1CurStride : b];
    if (cap && e > cap[b]) return;  // an overflowed bin (the batch is redone)
    if (e + j < ((e + 15) & ~15ull)) keys[e + j] = kEmptyKey;
}

// ---------------------------------------------------------------------------
// k in 33..64: two-u64 keys (K128, MSB-first over 2k bits), runtime k
// ---------------------------------------------------------------------------

constexpr int kSegW = 16;                    // scatter windows per thread
constexpr int kScatBlockW = 512;             // wide scatter: threads per workgroup
constexpr int kTileW1 = kScatBlockW * kSegW;  // 8192 windows: 128 KiB of staged K128 keys (one workgroup per CU)
static_assert(kScatBlockW >= kMaxL1BinsW, "one L1 bin per wide scatter thread");
// chunks are multiples of every tile (the hist walks kHTile steps, the scatters kTile / kTileW1 steps)
uint32_t extract_tile() { return lcm_u32(lcm_u32((uint32_t)kHTile, (uint32_t)kTile), (uint32_t)kTileW1); }

// Windows [w0, w0 + SEG) with 2k-bit keys (direct extraction, okm_scan.h):
// the forward key is the 2k code bits from base j (MSB-first) and the reverse
// complement the 2k complemented bits from base j (LSB-first), over 128 bits.
template <int SEG, typename Emit>
__device__ __forceinline__ void scan_windows_wide(const uint8_t *__restrict__ seq, uint64_t n, uint64_t w0,
                                                  uint32_t k, Emit &&emit) {
    WinWords<SEG, 64> ww;
    load_windows<SEG, 64>(seq, n, w0, ww);
    constexpr int NP = WinWords<SEG, 64>::kLoad / 16;
    Codes<NP> c;
    make_codes<NP, false>(ww.w, c);
#pragma unroll
    for (int j = 0; j < SEG; ++j) {
        bool valid;
        const K128 key = window_key128(c, j, k, &valid);
        emit(j, key, valid);
    }
}

__device__ __forceinline__ uint32_t bin_of_wide(const K128 &key, uint32_t shift) {
    return shift >= 128 ? 0u : (uint32_t)KeyOps<K128>::shr(key, shift);
}

__global__ __launch_bounds__(kExtractBlock) void k_extract_hist_wide(const uint8_t *__restrict__ seq, ExtractGeom g,
                                                                     uint32_t *__restrict__ HC,
                                                                     ull *__restrict__ Hg) {
    __shared__ uint32_t lh[kMaxL1BinsW + 1];
    for (uint32_t b = threadIdx.x; b <= g.nbins; b += kExtractBlock) lh[b] = 0;
    lds_sync();
    const uint64_t beg = (uint64_t)blockIdx.x * g.stride * g.chunk;  // stride > 1: a sample of the chunks
    const uint64_t end = beg + g.chunk < g.n ? beg + g.chunk : g.n;
    const uint32_t shift = g.shift, nb = g.nbins;
    for (uint64_t t0 = beg; t0 < end; t0 += kHTile) {
        const uint64_t w0 = t0 + (uint64_t)threadIdx.x * kSegH;
        if (w0 < end)
            scan_windows_wide<kSegH>(seq, g.n, w0, g.k, [&](int, const K128 &key, bool valid) {
                atomicAdd(&lh[valid ? bin_of_wide(key, shift) : nb], 1u);
            });
    }
    lds_sync();
    for (uint32_t b = threadIdx.x; b < nb; b += kExtractBlock) {
        const uint32_t h = lh[b];
        if (HC) HC[(uint64_t)blockIdx.x * nb + b] = h;
        if (h) atomicAdd(&Hg[b], (ull)h);
    }
}

// Single sweep (512-thread workgroups, so an 8192-window tile: 128 KiB of
// staged keys, 512-B runs per bin; 256 threads measured 7.09 vs 6.29 ms at 1
// Gbases, k=63): the 16 keys of a thread and their within-bin ranks (returned
// by the histogram atomic) stay in registers, as in k_extract_scatter, so each
// window is extracted once; each thread codes only its own 16 bytes (the
// 64-byte halo's codes come from its next four neighbours' LDS slots); the
// next tile's bytes are loaded while this tile is staged and written.
// The 16 bytes at w0 as (MSB-first codes, LSB-first complemented codes,
// invalid-base bits, 0); bytes at or past n are invalid.
__device__ __forceinline__ uint4 slot_codes(const uint32_t (&w)[4], uint64_t n, uint64_t w0) {
    Codes<1> c;
    make_codes<1, false>(w, c);
    const uint64_t avail = w0 < n ? n - w0 : 0;
    if (avail < 16) mark_tail<1>(c, avail);
    return make_uint4(c.p[0], c.q[0], (uint32_t)c.bad[0] & 0xFFFFu, 0u);
}
__global__ __launch_bounds__(kScatBlockW) void k_extract_scatter_wide1(const uint8_t *__restrict__ seq,
                                                                         ExtractGeom g,
                                                                         const uint32_t *__restrict__ HC,
                                                                         ull *__restrict__ cursor,
                                                                         K128 *__restrict__ out,
                                                                         const ull *__restrict__ cap_end,
                                                                         ull *__restrict__ ovf) {
    __shared__ K128 stage[kTileW1 + 64];  // + one dummy slot per lane for invalid windows
    __shared__ ull gcur[kMaxL1BinsW];
    __shared__ uint32_t hist[kMaxL1BinsW + 1];
    __shared__ uint32_t lofs[kMaxL1BinsW];
    __shared__ uint32_t lcur[kMaxL1BinsW];
    __shared__ ull wsum[kScatBlockW / 64];
    // each thread codes only its own 16 bytes; the 64-byte halo's codes come
    // from its next four neighbours' slots ([kScatBlockW, +4): the 64 bytes
    // after the tile, coded by the last four threads)
    constexpr int kXS = 4;  // halo slots: 64 bytes
    __shared__ uint4 xcode[kScatBlockW + kXS];
    const uint32_t t = threadIdx.x;
    const uint32_t nb = g.nbins;
    if (t < nb && HC) {
        const uint32_t h = HC[(uint64_t)blockIdx.x * nb + t];
        gcur[t] = h ? atomicAdd(&cursor[t], (ull)h) : 0ull;
    }
    const uint64_t beg = (uint64_t)blockIdx.x * g.chunk;
    const uint64_t end = beg + g.chunk < g.n ? beg + g.chunk : g.n;
    const uint32_t shift = g.shift;
    constexpr int NP = WinWords<kSegW, 64>::kLoad / 16;
    static_assert(kSegW == 16 && NP == 1 + kXS, "one 16-byte slot per thread");
    WinWords<kSegW, 0> own, extra;  // this thread's 16 bytes; a halo slot after the tile (one tile ahead)
    auto extra_at = [&](uint64_t tt0) -> uint64_t {  // the last kXS threads: the bytes after the tile
        return t >= (uint32_t)(kScatBlockW - kXS) ? tt0 + kTileW1 + (uint64_t)kSegW * (t - (kScatBlockW - kXS))
                                                   : tt0 + (uint64_t)t * kSegW;
    };
    load_windows_clamped<kSegW, 0>(seq, g.n, beg + (uint64_t)t * kSegW, own);
    load_windows_clamped<kSegW, 0>(seq, g.n, extra_at(beg), extra);
    const ull capb = (!HC && t < nb) ? cap_end[t] : 0ull;
    for (uint64_t t0 = beg; t0 < end; t0 += kTileW1) {
        for (uint32_t b = t; b <= nb; b += blockDim.x) hist[b] = 0;  // + the dummy bin (nb may equal the block)
        const uint64_t w0 = t0 + (uint64_t)t * kSegW;
        xcode[t] = slot_codes(own.w, g.n, w0);
        if (t >= (uint32_t)(kScatBlockW - kXS)) xcode[t + kXS] = slot_codes(extra.w, g.n, extra_at(t0));
        lds_sync();
        const bool live = w0 < end;
        uint32_t tile_n;
        {
            K128 kk[kSegW];
            uint32_t rk[kSegW / 2];  // two within-bin ranks per word; the bin is recomputed
            uint32_t vm = 0;         // valid windows
#pragma unroll
            for (int j = 0; j < kSegW / 2; ++j) rk[j] = 0;
            if (live) {
                Codes<NP> c;
#pragma unroll
                for (int i = 0; i < (NP * 16 + 63) / 64 + 1; ++i) c.bad[i] = 0;
#pragma unroll
                for (int i = 0; i < NP; ++i) {
                    const uint4 x = xcode[t + i];
                    c.p[i] = x.x;
                    c.q[i] = x.y;
                    c.bad[i >> 2] |= (uint64_t)x.z << (16 * (i & 3));
                }
#pragma unroll
                for (int j = 0; j < kSegW; ++j) {
                    bool valid;
                    const K128 key = window_key128(c, j, g.k, &valid);
                    const uint32_t b = valid ? bin_of_wide(key, shift) : nb;
                    kk[j] = key;
                    rk[j >> 1] |= (atomicAdd(&hist[b], 1u) & 0xFFFFu) << (16 * (j & 1));
                    vm |= valid ? 1u << j : 0u;
                }
            }
            // next tile, in flight (harmless past the end)
            load_windows_clamped<kSegW, 0>(seq, g.n, w0 + kTileW1, own);
            load_windows_clamped<kSegW, 0>(seq, g.n, extra_at(t0 + kTileW1), extra);
            lds_sync();
            tile_n = tile_offsets<kScatBlockW>(t, nb, hist, lofs, lcur, wsum);
            uint32_t ch = 0;
            ull cp;
            if (!HC && t < nb) {
                ch = hist[t];
                cp = atomicAdd(&cursor[t * kL1CurStride], (ull)ch);  // + 0 when empty: no branch
            }
            lds_sync();
#pragma unroll
            for (int j = 0; j < kSegW; ++j) {
                const uint32_t rank = (rk[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                const uint32_t dst =
                    (vm >> j) & 1u ? lofs[bin_of_wide(kk[j], shift)] + rank : (uint32_t)kTileW1 + (t & 63u);
                stage[dst] = kk[j];
            }
            if (!HC && t < nb) {
                const bool fits = ch && cp + ch <= capb;
                if (ch && !fits) atomicOr(ovf, 1ull);
                gcur[t] = fits ? cp : ~0ull;
            }
        }
        lds_sync();
        for (uint32_t j = t; j < tile_n; j += kScatBlockW) {
            const K128 key = stage[j];
            const uint32_t b = bin_of_wide(key, shift);
            const ull gb = gcur[b];
            if (gb != ~0ull) out[gb + (j - lofs[b])] = key;
        }
        lds_sync();
        if (HC && t < nb) gcur[t] += hist[t];
    }
}

__global__ __launch_bounds__(256) void k_fill_line_tails_wide(const ull *__restrict__ end, uint32_t nbins,
                                                              K128 *__restrict__ keys, const ull *__restrict__ cap) {
    const uint32_t b = blockIdx.x * 32 + (threadIdx.x >> 3), j = threadIdx.x & 7;
    if (b >= nbins) return;
    const ull e = end[cap ? b * kL1CurStride : b];
    if (cap && e > cap[b]) return;
    if (e + j < ((e + 7) & ~7ull)) keys[e + j] = KeyOps<K128>::empty();
}

// k values with a specialised instantiation (others use the runtime-k kernel)
#define OKM_EXTRACT_KS(X) X(17) X(21) X(25) X(27) X(31) X(32)

void launch_extract_hist(void *stream, const uint8_t *seq, const ExtractGeom &g, uint32_t *HC,
                         unsigned long long *Hg) {
    hipStream_t s = (hipStream_t)stream;
    if (g.k > 32) {
        hipLaunchKernelGGL(k_extract_hist_wide, dim3(g.nblocks), dim3(kExtractBlock), 0, s, seq, g, HC, Hg);
        return;
    }
    switch (g.k) {
#define OKM_CASE(KV)                                                                                  \
    case KV:                                                                                          \
        hipLaunchKernelGGL(k_extract_hist<KV>, dim3(g.nblocks), dim3(kExtractBlock), 0, s, seq, g, HC, Hg); \
        return;
        OKM_EXTRACT_KS(OKM_CASE)
#undef OKM_CASE
    default:
        hipLaunchKernelGGL(k_extract_hist<0>, dim3(g.nblocks), dim3(kExtractBlock), 0, s, seq, g, HC, Hg);
    }
}

void launch_extract_scatter(void *stream, const uint8_t *seq, const ExtractGeom &g,
                            const uint32_t *HC, unsigned long long *cursor, uint64_t *out_keys,
                            const unsigned long long *cap_end, unsigned long long *ovf) {
    hipStream_t s = (hipStream_t)stream;
    if (g.k > 32) {
        hipLaunchKernelGGL(k_extract_scatter_wide1, dim3(g.nblocks), dim3(kScatBlockW), 0, s, seq, g, HC, cursor,
                           reinterpret_cast<K128 *>(out_keys), cap_end, ovf);
        return;
    }
    switch (g.k) {
#define OKM_CASE(KV)                                                                                      \
    case KV:                                                                                              \
        hipLaunchKernelGGL(k_extract_scatter<KV>, dim3(g.nblocks), dim3(kScatBlock), 0, s, seq, g, HC, \
                           cursor, out_keys, cap_end, ovf);                                               \
        return;
        OKM_EXTRACT_KS(OKM_CASE)
#undef OKM_CASE
    default:
        hipLaunchKernelGGL(k_extract_scatter<0>, dim3(g.nblocks), dim3(kScatBlock), 0, s, seq, g, HC, cursor,
                           out_keys, cap_end, ovf);
    }
}

void launch_fill_line_tails(void *stream, const unsigned long long *end, uint32_t nbins, uint64_t *keys, bool wide,
                            const unsigned long long *cap) {
    if (wide)
        hipLaunchKernelGGL(k_fill_line_tails_wide, dim3((nbins + 31) / 32), dim3(256), 0, (hipStream_t)stream, end,
                           nbins, reinterpret_cast<K128 *>(keys), cap);
    else
        hipLaunchKernelGGL(k_fill_line_tails, dim3((nbins + 15) / 16), dim3(256), 0, (hipStream_t)stream, end,
                           nbins, keys, cap);
}

// Sampled L1 capacities (one block, nb <= kMaxL1Bins): Hs holds the window
// counts of a sample of the tiles; bin b gets scale * (sqrt(s) + 3)^2 keys
// (s = Hs[b]; s + 6 sqrt(s) + 9 bounds the Poisson mean an observed s allows
// at ~6 sigma) + 1% + 256, rounded up to `align` keys.  Starts are exclusive sums (line
// aligned); l1cap = [cap_end(nb) | start(nb + 1) | overflow flag].
__global__ __launch_bounds__(256) void k_l1_capacity(const ull *__restrict__ Hs, uint32_t nb, double scale,
                                                     double mul, uint32_t align, ull limit, ull *__restrict__ cursor,
                                                     ull *__restrict__ l1cap) {
    __shared__ ull cap[kMaxL1Bins > kMaxL1BinsW ? kMaxL1Bins : kMaxL1BinsW];
    for (uint32_t t = threadIdx.x; t < nb; t += 256) {
        const double s = (double)Hs[t];
        const double r = sqrt(s) + 3.0;  // (sqrt(s) + 3)^2: the Poisson mean s allows at ~6 sigma
        const double c = (r * r * scale * 1.01 + 256.0) * mul;
        cap[t] = ((ull)c + align - 1) / align * align;
    }
    const uint32_t t = threadIdx.x;
    lds_sync();
    if (t == 0) {
        ull o = 0;
        for (uint32_t b = 0; b < nb; ++b) {
            const ull st = o < limit ? o : limit;
            o += cap[b];
            const ull en = o < limit ? o : limit;
            cursor[b * kL1CurStride] = st;
            l1cap[b] = en;
            l1cap[nb + b] = st;
        }
        l1cap[2 * nb] = o < limit ? o : limit;
        l1cap[2 * nb + 1] = 0;
    }
}

void launch_l1_capacity(void *stream, const unsigned long long *Hs, uint32_t nb, double scale, double mul,
                        uint32_t align, unsigned long long limit, unsigned long long *cursor,
                        unsigned long long *l1cap) {
    hipLaunchKernelGGL(k_l1_capacity, dim3(1), dim3(256), 0, (hipStream_t)stream, Hs, nb, scale, mul, align, limit,
                       cursor, l1cap);
}

}  // namespace okm
