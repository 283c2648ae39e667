// okm_partition.hip — key-range partition passes over key arrays.
//
// Splits every segment of a pass into 2^b sub-ranges of its keys (the next b
// key bits below the segment's common prefix) with exact placement:
//   part_hist    per chunk (64 Ki keys) and local bin: key count -> HC, and
//                the count rounded up to a 16-key line -> Hg (bin totals);
//   (host)       exclusive scan of Hg -> every output bin starts on a 128-B
//                line;
//   part_scatter each chunk claims a line-aligned slice per bin, appends keys
//                to per-bin 16-key LDS buffers and writes each full buffer as
//                ONE aligned 128-B line; the chunk's last partial line of a
//                bin is padded with kEmptyKey (skipped by every consumer).
// HBM therefore only sees whole-line writes (8-byte scattered stores cost
// ~3.5x the bytes: partially written lines leave the 4 MiB XCD L2 early).
#include "okm_dev_common.h"

namespace okm {

#ifndef OKM_PART_BLOCK
#define OKM_PART_BLOCK 1024
#endif
constexpr int kPartBlock = OKM_PART_BLOCK;  // scatter threads per workgroup (LDS-limited to 1 block/CU)
constexpr int kLine = 16;      // keys per 128-B line
constexpr int kLoadU = 8;      // keys per thread in flight per batch (4 x 16-B loads when aligned)
constexpr int kHistU = 4;      // 16-B loads per thread in flight (histogram)

uint32_t part_max_bins(bool weighted) { return weighted ? 512u : 1024u; }

__device__ __forceinline__ uint32_t local_bin(uint64_t key, const DevSeg &s) {
    const uint64_t b = (s.shift >= 64 ? 0ull : (key >> s.shift)) - s.key_base;
    return b < s.nlocal ? (uint32_t)b : s.nlocal - 1;  // clamp: never true for canonical keys
}

__device__ __forceinline__ ull pad_line(ull n) { return (n + kLine - 1) & ~(ull)(kLine - 1); }

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
        if ((reinterpret_cast<uintptr_t>(keys) & 15u) == 0) {  // block-uniform: 2 keys per 16-B load
            const uint4 *k4 = reinterpret_cast<const uint4 *>(keys);
            const uint64_t n2 = ch.len >> 1;
            for (uint64_t i = threadIdx.x; i < n2; i += (uint64_t)kPartBlock * kHistU) {
                uint4 v[kHistU];
#pragma unroll
                for (int u = 0; u < kHistU; ++u) {
                    const uint64_t q = i + (uint64_t)u * kPartBlock;
                    v[u] = q < n2 ? k4[q] : make_uint4(~0u, ~0u, ~0u, ~0u);
                }
#pragma unroll
                for (int u = 0; u < kHistU; ++u) {
                    const uint64_t a = ((uint64_t)v[u].y << 32) | v[u].x, b = ((uint64_t)v[u].w << 32) | v[u].z;
                    if (a != kEmptyKey) atomicAdd(&lh[local_bin(a, s)], 1u);
                    if (b != kEmptyKey) atomicAdd(&lh[local_bin(b, s)], 1u);
                }
            }
            if ((ch.len & 1) && threadIdx.x == 0) {
                const uint64_t key = keys[ch.len - 1];
                if (key != kEmptyKey) atomicAdd(&lh[local_bin(key, s)], 1u);
            }
        } else {
            for (uint64_t i = threadIdx.x; i < ch.len; i += kPartBlock) {
                const uint64_t key = keys[i];
                if (key != kEmptyKey) atomicAdd(&lh[local_bin(key, s)], 1u);
            }
        }
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < s.nlocal; b += kPartBlock) {
            const uint32_t h = lh[b];
            HC[(uint64_t)c * max_local + b] = h;
            if (h) atomicAdd(&Hg[s.out_base + b], pad_line(h));
        }
        __syncthreads();
    }
}

// Writes one full line (16 keys [+ 16 counts]) from LDS buffers to global.
template <bool W>
__device__ __forceinline__ void flush_line(const ull *bk, const ull *bc, uint64_t *ok, uint64_t *oc) {
    const uint4 *src = reinterpret_cast<const uint4 *>(bk);
    uint4 *dst = reinterpret_cast<uint4 *>(ok);
#pragma unroll
    for (int q = 0; q < kLine / 2; ++q) dst[q] = src[q];
    if (W) {
        const uint4 *cs = reinterpret_cast<const uint4 *>(bc);
        uint4 *cd = reinterpret_cast<uint4 *>(oc);
#pragma unroll
        for (int q = 0; q < kLine / 2; ++q) cd[q] = cs[q];
    }
}

template <bool W>
__global__ __launch_bounds__(kPartBlock) void k_part_scatter(
    const DevSeg *__restrict__ segs, const DevChunk *__restrict__ chunks, uint32_t nchunks,
    uint32_t max_local, const uint32_t *__restrict__ HC, ull *__restrict__ cursor,
    uint64_t *__restrict__ out_keys, uint64_t *__restrict__ out_counts) {
    extern __shared__ __attribute__((aligned(16))) ull lds[];
    ull *buf = lds;                                       // [max_local][kLine] keys
    ull *cbuf = buf + (size_t)max_local * kLine;          // [max_local][kLine] counts (W)
    ull *gcur = W ? cbuf + (size_t)max_local * kLine : cbuf;  // [max_local]
    uint32_t *fill = reinterpret_cast<uint32_t *>(gcur + max_local);  // [max_local]
    const uint32_t t = threadIdx.x;

    for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const DevChunk ch = chunks[c];
        const DevSeg s = segs[ch.seg];
        const uint32_t nl = s.nlocal;
        for (uint32_t b = t; b < nl; b += kPartBlock) {
            const uint32_t h = HC[(uint64_t)c * max_local + b];
            gcur[b] = h ? atomicAdd(&cursor[s.out_base + b], pad_line(h)) : 0ull;
            fill[b] = 0;
        }
        __syncthreads();
        const uint64_t *keys = s.keys + ch.begin;
        const uint64_t *cnts = s.counts ? s.counts + ch.begin : nullptr;
        // 16-B pair loads measured slower here than one key per lane (2.08 vs 1.97 ms
        // on C2); kept for reference, off.
        const bool aligned = false && ((reinterpret_cast<uintptr_t>(keys) | reinterpret_cast<uintptr_t>(cnts)) & 15u) == 0;
        for (uint64_t base = 0; base < ch.len; base += (uint64_t)kPartBlock * kLoadU) {
            ull kk[kLoadU];
            ull ww[kLoadU];
            uint32_t pend = 0;
            if (aligned) {  // block-uniform: pairs of keys (and counts) per 16-B load
#pragma unroll
                for (int u = 0; u < kLoadU / 2; ++u) {
                    const uint64_t idx = base + 2 * ((uint64_t)u * kPartBlock + t);
                    if (idx + 1 < ch.len) {
                        const uint4 v = *reinterpret_cast<const uint4 *>(keys + idx);
                        kk[2 * u] = ((uint64_t)v.y << 32) | v.x;
                        kk[2 * u + 1] = ((uint64_t)v.w << 32) | v.z;
                        if (W) {
                            if (cnts) {
                                const uint4 c = *reinterpret_cast<const uint4 *>(cnts + idx);
                                ww[2 * u] = ((uint64_t)c.y << 32) | c.x;
                                ww[2 * u + 1] = ((uint64_t)c.w << 32) | c.z;
                            } else {
                                ww[2 * u] = ww[2 * u + 1] = 1ull;
                            }
                        }
                    } else {
                        kk[2 * u] = idx < ch.len ? keys[idx] : kEmptyKey;
                        kk[2 * u + 1] = kEmptyKey;
                        ww[2 * u] = (W && idx < ch.len && cnts) ? cnts[idx] : 1ull;
                        ww[2 * u + 1] = 1ull;
                    }
                }
            } else {
#pragma unroll
                for (int u = 0; u < kLoadU; ++u) {
                    const uint64_t idx = base + (uint64_t)u * kPartBlock + t;
                    kk[u] = idx < ch.len ? keys[idx] : kEmptyKey;
                    ww[u] = (W && idx < ch.len) ? (cnts ? cnts[idx] : 1ull) : 1ull;
                }
            }
#pragma unroll
            for (int u = 0; u < kLoadU; ++u)
                if (kk[u] != kEmptyKey) pend |= 1u << u;
            // append rounds: a key whose bin buffer is full waits for the flush
            while (__syncthreads_or(pend != 0)) {
#pragma unroll
                for (int u = 0; u < kLoadU; ++u) {
                    if (pend & (1u << u)) {
                        const uint32_t b = local_bin(kk[u], s);
                        const uint32_t pos = atomicAdd(&fill[b], 1u);
                        if (pos < (uint32_t)kLine) {
                            buf[b * kLine + pos] = kk[u];
                            if (W) cbuf[b * kLine + pos] = ww[u];
                            pend &= ~(1u << u);
                        }
                    }
                }
                __syncthreads();
                for (uint32_t b = t; b < nl; b += kPartBlock) {
                    if (fill[b] >= (uint32_t)kLine) {
                        const ull g = gcur[b];
                        flush_line<W>(buf + b * kLine, cbuf + b * kLine, out_keys + g, W ? out_counts + g : nullptr);
                        gcur[b] = g + kLine;
                        fill[b] = 0;  // keys that overshot retry next round
                    }
                }
            }
        }
        __syncthreads();
        // last partial line per bin, padded
        for (uint32_t b = t; b < nl; b += kPartBlock) {
            const uint32_t f = fill[b];
            if (f) {
                for (uint32_t q = f; q < (uint32_t)kLine; ++q) {
                    buf[b * kLine + q] = kEmptyKey;
                    if (W) cbuf[b * kLine + q] = 0;
                }
                const ull g = gcur[b];
                flush_line<W>(buf + b * kLine, cbuf + b * kLine, out_keys + g, W ? out_counts + g : nullptr);
            }
        }
        __syncthreads();
    }
}

static uint32_t part_grid(uint32_t nchunks) { return nchunks < 4096u ? nchunks : 4096u; }

void launch_part_hist(void *stream, const DevSeg *segs, const DevChunk *chunks, uint32_t nchunks,
                      uint32_t max_local, uint32_t *HC, unsigned long long *Hg) {
    if (!nchunks) return;
    hipLaunchKernelGGL(k_part_hist, dim3(part_grid(nchunks)), dim3(kPartBlock), max_local * sizeof(uint32_t),
                       (hipStream_t)stream, segs, chunks, nchunks, max_local, HC, Hg);
}

void launch_part_scatter(void *stream, const DevSeg *segs, const DevChunk *chunks, uint32_t nchunks,
                         uint32_t max_local, const uint32_t *HC, unsigned long long *cursor, uint64_t *out_keys,
                         uint64_t *out_counts) {
    if (!nchunks) return;
    static bool attr_done = false;  // allow > 64 KiB of dynamic LDS (gfx950: 160 KiB per workgroup)
    if (!attr_done) {
        int dev = 0, optin = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || optin <= 0)
            optin = 64 * 1024;
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_part_scatter<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, optin);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_part_scatter<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, optin);
        (void)hipGetLastError();  // an unsupported attribute must not poison later checks
        attr_done = true;
    }
    const bool W = out_counts != nullptr;
    const size_t lds = (size_t)max_local * (kLine * sizeof(ull) * (W ? 2 : 1) + sizeof(ull) + sizeof(uint32_t));
    if (W)
        hipLaunchKernelGGL(k_part_scatter<true>, dim3(part_grid(nchunks)), dim3(kPartBlock), lds,
                           (hipStream_t)stream, segs, chunks, nchunks, max_local, HC, cursor, out_keys, out_counts);
    else
        hipLaunchKernelGGL(k_part_scatter<false>, dim3(part_grid(nchunks)), dim3(kPartBlock), lds,
                           (hipStream_t)stream, segs, chunks, nchunks, max_local, HC, cursor, out_keys, out_counts);
}

}  // namespace okm
