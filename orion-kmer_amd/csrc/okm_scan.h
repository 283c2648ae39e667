// okm_scan.h — byte-level window helpers shared by the extraction kernels
// (okm_extract.hip) and the probe kernels (okm_probe.hip).
#pragma once

#include "okm_dev_common.h"

namespace okm {

// Valid bytes after needletail normalize(false) + dna_base_to_u64:
// A/a C/c G/g T/t U/u (kmer.rs:14-17; U->T is normalize's).  c & 0xDF folds
// case and has exactly {X, X|0x20} as preimages of an upper-case letter X.
__device__ __forceinline__ bool base_valid(uint32_t c) {
    const uint32_t u = c & 0xDFu;
    return (u == 'A') | (u == 'C') | (u == 'G') | (u == 'T') | (u == 'U');
}
// A=0 C=1 G=2 T=3 (and U=3) for either case: ((c>>1) ^ (c>>2)) & 3.
__device__ __forceinline__ uint32_t base_code(uint32_t c) { return ((c >> 1) ^ (c >> 2)) & 3u; }

// Valid bytes of query.rs:86-88, which windows the RAW record.sequence()
// (no normalize): only A/a C/c G/g T/t (kmer.rs:14-17) — U is invalid there.
__device__ __forceinline__ bool base_valid_raw(uint32_t c) {
    const uint32_t u = c & 0xDFu;
    return (u == 'A') | (u == 'C') | (u == 'G') | (u == 'T');
}

// The bytes a thread needs for the windows starting in [w0, w0 + SEG): SEG
// plus a k - 1 <= 31 byte halo, rounded to whole 16-B loads.
template <int SEG> struct WinWords {
    static constexpr int kLoad = SEG + 32;  // bytes: covers SEG + k - 1 for k <= 32 (16-B multiple)
    uint32_t w[kLoad / 4];
};

// The bytes of windows [w0, w0 + SEG) (bytes at or beyond n read as 0).
template <int SEG>
__device__ __forceinline__ void load_windows(const uint8_t *__restrict__ seq, uint64_t n, uint64_t w0,
                                             WinWords<SEG> &ww) {
    constexpr int LOAD = WinWords<SEG>::kLoad;
    uint32_t *w = ww.w;
    if (w0 + LOAD <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(seq + w0);
#pragma unroll
        for (int q = 0; q < LOAD / 16; ++q) {
            const uint4 v = p[q];
            w[4 * q + 0] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < LOAD / 4; ++q) {
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
}

}  // namespace okm
