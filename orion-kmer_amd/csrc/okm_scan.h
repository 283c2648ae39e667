// okm_scan.h — byte-level window helpers shared by the extraction kernels
// (okm_extract.hip) and the probe kernels (okm_probe.hip).
#pragma once

#include "okm_dev_common.h"

namespace okm {

// The bytes a thread needs for the windows starting in [w0, w0 + SEG): SEG
// plus a k - 1 byte halo (HALO = 32: k <= 32; 64: k <= 64), whole 16-B loads.
template <int SEG, int HALO = 32> struct WinWords {
    static constexpr int kLoad = SEG + HALO;  // bytes: covers SEG + k - 1 (16-B multiple)
    static_assert(kLoad % 16 == 0, "whole 16-B loads");
    uint32_t w[kLoad / 4];
};

// The bytes of windows [w0, w0 + SEG) (bytes at or beyond n read as 0).
template <int SEG, int HALO>
__device__ __forceinline__ void load_windows(const uint8_t *__restrict__ seq, uint64_t n, uint64_t w0,
                                             WinWords<SEG, HALO> &ww) {
    constexpr int LOAD = WinWords<SEG, HALO>::kLoad;
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

// The same bytes without a data-dependent branch (the tail-safe byte loop of
// load_windows sits on a path the wait-count pass must join, and it then
// waits for every load in flight, the next tile's prefetch included): each
// 16-B granule is loaded from min(its address, the batch's last granule) --
// a 16-B aligned granule that starts inside the batch never leaves the
// allocation -- and bytes at or past n are marked invalid afterwards
// (mark_tail), so their contents never matter.  seq is 16-B aligned and
// w0 % 16 == 0; any w0 is safe (past the end: the last granule, again).
template <int SEG, int HALO>
__device__ __forceinline__ void load_windows_clamped(const uint8_t *__restrict__ seq, uint64_t n, uint64_t w0,
                                                     WinWords<SEG, HALO> &ww) {
    constexpr int LOAD = WinWords<SEG, HALO>::kLoad;
    const uint64_t lastg = (n - 1) >> 4, g0 = w0 >> 4;  // n >= 1
    const uint64_t g0c = g0 < lastg ? g0 : lastg;
    const uint64_t dd = lastg - g0c;  // granules after the first
    const uint32_t d = dd < (uint64_t)(LOAD / 16) ? (uint32_t)dd : (uint32_t)(LOAD / 16);
    const uint4 *p = reinterpret_cast<const uint4 *>(seq) + g0c;
#pragma unroll
    for (int q = 0; q < LOAD / 16; ++q) {
        const uint4 v = p[(uint32_t)q < d ? (uint32_t)q : d];
        ww.w[4 * q + 0] = v.x;
        ww.w[4 * q + 1] = v.y;
        ww.w[4 * q + 2] = v.z;
        ww.w[4 * q + 3] = v.w;
    }
}

// ---------------------------------------------------------------------------
// Direct window extraction.  Every 16 loaded bytes become three 32-bit words
// (SWAR, no per-byte loop): the 2-bit codes MSB-first (the forward k-mer of
// any window is then a shifted slice, kmer.rs:45-55), the complemented codes
// LSB-first (the reverse complement of any window is a slice too,
// kmer.rs:79-94), and a mask of invalid bytes (kmer.rs:12-20: a window is
// valid iff its k bits are clear).  No rolling state: windows are independent,
// the k - 1 halo costs nothing per window, and j is a compile-time constant in
// every caller's unrolled loop.
// ---------------------------------------------------------------------------

// 0x80 in every zero byte of x, exactly (no borrow propagation).
__host__ __device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}

// Per byte: "ACGT"[code] (upper case) for the 2-bit codes in the low bits of
// each byte of cb.
__host__ __device__ __forceinline__ uint32_t letters_of(uint32_t cb) {
#if defined(__HIP_DEVICE_COMPILE__)
    // v_perm_b32 byte select; the table sits in both halves, so the operand
    // order of the two sources does not matter
    return __builtin_amdgcn_perm(0x54474341u, 0x54474341u, cb);
#else
    uint32_t r = 0;
    for (int b = 0; b < 4; ++b) r |= (uint32_t)("ACGT"[(cb >> (8 * b)) & 3u]) << (8 * b);
    return r;
#endif
}

// Four bytes -> their codes packed MSB-first in 8 bits (byte 0 in bits 7:6);
// *bad4 = bit b set when byte b is not a valid base.  RAW: query.rs's
// validity (U invalid) instead of count.rs's (normalize maps U to T).
template <bool RAW>
__host__ __device__ __forceinline__ uint32_t pack4(uint32_t x, uint32_t *bad4) {
    const uint32_t cb = ((x >> 1) ^ (x >> 2)) & 0x03030303u;  // base_code per byte
    const uint32_t u = x & 0xDFDFDFDFu;                        // case fold
    uint32_t ok = zero_bytes(u ^ letters_of(cb));
    if (!RAW) ok |= zero_bytes(u ^ 0x55555555u);  // 'U'
    *bad4 = ((((~ok) >> 7) & 0x01010101u) * 0x00204081u) >> 21 & 0xFu;
    return ((cb << 6) | (cb >> 4) | (cb >> 14) | (cb >> 24)) & 0xFFu;
}

// Reverse the order of the 16 2-bit groups of x.
__host__ __device__ __forceinline__ uint32_t rev2(uint32_t x) {
    const uint32_t r = __builtin_bitreverse32(x);
    return ((r >> 1) & 0x55555555u) | ((r << 1) & 0xAAAAAAAAu);
}

template <int NP> struct Codes {
    uint32_t p[NP];                 // MSB-first codes: base 16i+b at bits 31-2b..30-2b of p[i]
    uint32_t q[NP];                 // LSB-first complemented codes: base 16i+b at bits 2b+1..2b of q[i]
    uint64_t bad[(NP * 16 + 63) / 64 + 1];  // bit m: base m invalid (zero past the load)
};

template <int NP, bool RAW>
__host__ __device__ __forceinline__ void make_codes(const uint32_t *w, Codes<NP> &c) {
#pragma unroll
    for (int i = 0; i < (NP * 16 + 63) / 64 + 1; ++i) c.bad[i] = 0;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        uint32_t b0, b1, b2, b3;
        const uint32_t p = (pack4<RAW>(w[4 * i], &b0) << 24) | (pack4<RAW>(w[4 * i + 1], &b1) << 16) |
                           (pack4<RAW>(w[4 * i + 2], &b2) << 8) | pack4<RAW>(w[4 * i + 3], &b3);
        c.p[i] = p;
        c.q[i] = ~rev2(p);
        c.bad[i >> 2] |= (uint64_t)(b0 | (b1 << 4) | (b2 << 8) | (b3 << 12)) << (16 * (i & 3));
    }
}

// Bases at or past `avail` (the bytes the batch still holds from the load's
// first byte) become invalid: load_windows_clamped read other bytes there.
template <int NP>
__host__ __device__ __forceinline__ void mark_tail(Codes<NP> &c, uint64_t avail) {
#pragma unroll
    for (int i = 0; i < (NP * 16 + 63) / 64; ++i) {
        const uint64_t pos = 64ull * i;
        const uint64_t m = avail <= pos ? ~0ull : (avail - pos >= 64 ? 0ull : ~0ull << (avail - pos));
        c.bad[i] |= m;
    }
}

// 64 code bits starting at base j, MSB-first (needs p[j/16 .. j/16 + 2]).
template <int NP>
__host__ __device__ __forceinline__ uint64_t fwd_top64(const Codes<NP> &c, int j) {
    const int w = j >> 4, o = (j & 15) * 2;
    const uint64_t a = ((uint64_t)c.p[w] << 32) | c.p[w + 1];
    if (o == 0) return a;
    return (a << o) | (c.p[w + 2] >> (32 - o));
}

// 64 complemented code bits starting at base j, LSB-first.
template <int NP>
__host__ __device__ __forceinline__ uint64_t rc_low64(const Codes<NP> &c, int j) {
    const int w = j >> 4, o = (j & 15) * 2;
    const uint64_t a = (uint64_t)c.q[w] | ((uint64_t)c.q[w + 1] << 32);
    if (o == 0) return a;
    return (a >> o) | ((uint64_t)c.q[w + 2] << (64 - o));
}

// 64 invalid-bits starting at base j.
template <int NP>
__host__ __device__ __forceinline__ uint64_t bad_low64(const Codes<NP> &c, int j) {
    const int w = j >> 6, o = j & 63;
    if (o == 0) return c.bad[w];
    return (c.bad[w] >> o) | (c.bad[w + 1] << (64 - o));
}

// Low 32 bits of (hi:lo) >> s, s in [0, 31]: one v_alignbit_b32.
__host__ __device__ __forceinline__ uint32_t funnel32(uint32_t hi, uint32_t lo, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}

// 32 MSB-first code bits from stream bit s = 2 * base (p[s/32 .. s/32 + 1]).
template <int NP>
__host__ __device__ __forceinline__ uint32_t fwd32(const Codes<NP> &c, int s) {
    const int w = s >> 5, r = s & 31;
    return r == 0 ? c.p[w] : funnel32(c.p[w], c.p[w + 1], 32u - (uint32_t)r);
}

// 32 LSB-first complemented code bits from stream bit s (q[s/32 .. s/32 + 1]).
template <int NP>
__host__ __device__ __forceinline__ uint32_t rc32(const Codes<NP> &c, int s) {
    return funnel32(c.q[(s >> 5) + 1], c.q[s >> 5], (uint32_t)(s & 31));
}

// Canonical k-mer (k <= 32) of window j, validity not checked.  With j and k
// compile-time constants every word is one funnel shift of two code words
// (v_alignbit_b32) and a shift or mask: 6 VALU for both strands, where 64-bit
// shifts of 64-bit slices (fwd_top64 / rc_low64) took ~3x that.
template <int NP>
__host__ __device__ __forceinline__ uint64_t window_key_nv(const Codes<NP> &c, int j, uint32_t k) {
    uint32_t fh = 0, fl, rh = 0, rl;
    if (2 * k > 32) {
        fl = fwd32(c, 2 * j + 2 * (int)k - 32);                   // kmer.rs:37-57: bases j+k-16 .. j+k-1
        fh = fwd32(c, 2 * j) >> (64u - 2 * k);                      // ... and j .. j+k-17
        rl = rc32(c, 2 * j);                                        // kmer.rs:79-94
        const uint32_t hb = 2 * k - 32;                             // 2..32 bits in the high word
        rh = rc32(c, 2 * j + 32) & (hb >= 32 ? ~0u : ((1u << hb) - 1u));
    } else {
        fl = fwd32(c, 2 * j) >> (32u - 2 * k);
        rl = rc32(c, 2 * j) & (2 * k >= 32 ? ~0u : ((1u << (2 * k)) - 1u));
    }
    const uint64_t f = ((uint64_t)fh << 32) | fl, r = ((uint64_t)rh << 32) | rl;
    return f < r ? f : r;  // kmer.rs:99-106
}

// Canonical k-mer (k <= 32) of window j and its validity.
template <int NP>
__host__ __device__ __forceinline__ uint64_t window_key(const Codes<NP> &c, int j, uint32_t k, bool *valid) {
    *valid = (bad_low64(c, j) & (k >= 64 ? ~0ull : ((1ull << k) - 1ull))) == 0;
    return window_key_nv(c, j, k);
}

// Invalid windows among j = 0 .. SEG-1 (bit j: a base of j .. j+k-1 is
// invalid), for SEG + k - 1 <= 64: an OR over runs of k bits of the
// per-base invalid bits, by doubling -- ~5 64-bit steps per thread instead of
// a 64-bit shift, mask and compare per window.
template <int SEG, int NP>
__host__ __device__ __forceinline__ uint32_t invalid_windows(const Codes<NP> &c, uint32_t k) {
    static_assert(SEG + 31 <= 64, "one 64-bit word of invalid bits");
    uint64_t x = c.bad[0];
    uint32_t len = 1;
    while (2 * len <= k) {  // x bit j: any invalid base in j .. j+len-1
        x |= x >> len;
        len *= 2;
    }
    x |= x >> (k - len);  // j .. j+k-1 (the two runs of len overlap)
    return (uint32_t)x & (SEG >= 32 ? ~0u : ((1u << SEG) - 1u));
}

// Canonical k-mer (k in 33..64, K128 {lo, hi} over 2k bits) of window j and
// its validity (needs p/q up to word j/16 + 4).
template <int NP>
__host__ __device__ __forceinline__ K128 window_key128(const Codes<NP> &c, int j, uint32_t k, bool *valid) {
    const uint32_t s = 128 - 2 * k;     // 0..62
    const uint32_t hbits = 2 * k - 64;  // key bits held in `hi`
    const uint64_t hmask = hbits >= 64 ? ~0ull : ((1ull << hbits) - 1ull);
    const uint64_t hi = fwd_top64(c, j), lo = fwd_top64(c, j + 32);
    K128 f, r;
    f.lo = s ? (lo >> s) | (hi << (64 - s)) : lo;  // kmer.rs:37-57 over 2k bits
    f.hi = hi >> s;
    r.lo = rc_low64(c, j);                          // kmer.rs:79-94 over 2k bits
    r.hi = rc_low64(c, j + 32) & hmask;
    *valid = (bad_low64(c, j) & (k >= 64 ? ~0ull : ((1ull << k) - 1ull))) == 0;
    return KeyOps<K128>::lt(f, r) ? f : r;          // kmer.rs:99-106
}

// Walk the windows starting in [w0, w0 + SEG) of a batch and call
// emit(j, key, valid) for each window start j = 0..SEG-1, in order, j a
// compile-time constant.  Bytes at or beyond n read as 0 (invalid), so windows
// never run off the end; record separators are invalid bytes, so windows never
// cross records.  K > 0: k known at compile time; K = 0: k_rt.
// avail: bytes of the batch from the load's first byte (~0: no tail marking,
// the words were loaded by load_windows).
template <int SEG, int K, bool RAW = false, typename Emit>
__device__ __forceinline__ void scan_words(const WinWords<SEG> &ww, uint32_t k_rt, Emit &&emit,
                                           uint64_t avail = ~0ull) {
    constexpr int NP = WinWords<SEG>::kLoad / 16;
    const uint32_t k = K ? (uint32_t)K : k_rt;
    Codes<NP> c;
    make_codes<NP, RAW>(ww.w, c);
    if (avail < (uint64_t)WinWords<SEG>::kLoad) mark_tail<NP>(c, avail);  // the batch's last bytes only
    if (SEG + 31 <= 64) {  // validity of all SEG windows at once
        const uint32_t inv = invalid_windows<(SEG + 31 <= 64 ? SEG : 32), NP>(c, k);
#pragma unroll
        for (int j = 0; j < SEG; ++j) emit(j, window_key_nv(c, j, k), ((inv >> j) & 1u) == 0);
        return;
    }
#pragma unroll
    for (int j = 0; j < SEG; ++j) {
        bool valid;
        const uint64_t key = window_key(c, j, k, &valid);
        emit(j, key, valid);
    }
}

template <int SEG, int K, bool RAW = false, typename Emit>
__device__ __forceinline__ void scan_windows(const uint8_t *__restrict__ seq, uint64_t n, uint64_t w0,
                                             uint32_t k_rt, Emit &&emit) {
    WinWords<SEG> ww;
    load_windows<SEG>(seq, n, w0, ww);
    scan_words<SEG, K, RAW>(ww, k_rt, emit);
}

}  // namespace okm
