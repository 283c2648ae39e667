// okm_codec.cpp — CPU k-mer codec: the parity surface of kmer.rs's pub fns.
//
// These are host-side conveniences for callers (the CLI decodes output keys
// with okm_u64_to_seq) and for tests; the device path rolls the same
// encodings in okm_device.hip (scan_segment).
#include <stdint.h>
#include <stddef.h>

#include "orion_kmer.h"

extern "C" {

// kmer.rs:12-20 dna_base_to_u64
static inline int base_code(uint8_t b) {
    switch (b) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return -1;
    }
}

// kmer.rs:37-57 seq_to_u64 (None -> 0, Some(v) -> 1 with *out = v)
int okm_seq_to_u64(const uint8_t *seq, size_t len, uint8_t k, uint64_t *out) {
    if (k == 0 || k > 32 || len != (size_t)k || !seq) return 0;
    uint64_t v = 0;
    for (size_t i = 0; i < len; ++i) {
        const int c = base_code(seq[i]);
        if (c < 0) return 0;
        v = (v << 2) | (uint64_t)c;  // first base ends in the top used bits
    }
    if (out) *out = v;
    return 1;
}

// kmer.rs:61-75 u64_to_seq (the reference panics for k outside 1..=32)
int okm_u64_to_seq(uint64_t v, uint8_t k, char *out) {
    if (k == 0 || k > 32 || !out) return 0;
    for (int i = k - 1; i >= 0; --i) {
        out[i] = "ACGT"[v & 3u];
        v >>= 2;
    }
    return 1;
}

// kmer.rs:79-94 reverse_complement_u64: complement = XOR 3, then reverse the
// 2-bit groups of the low 2k bits.
uint64_t okm_reverse_complement_u64(uint64_t v, uint8_t k) {
    if (k == 0 || k > 32) return 0;
    uint64_t x = ~v;
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    x = ((x >> 8) & 0x00FF00FF00FF00FFull) | ((x & 0x00FF00FF00FF00FFull) << 8);
    x = ((x >> 16) & 0x0000FFFF0000FFFFull) | ((x & 0x0000FFFF0000FFFFull) << 16);
    x = (x >> 32) | (x << 32);
    return x >> (64 - 2 * (unsigned)k);
}

// kmer.rs:99-106 canonical_u64
uint64_t okm_canonical_u64(uint64_t v, uint8_t k) {
    const uint64_t rc = okm_reverse_complement_u64(v, k);
    return v < rc ? v : rc;
}

// ---- k in 33..64: the same MSB-first encoding over 2k bits (restatement-defined)

typedef unsigned __int128 u128;
static inline u128 to128(okm_key128 v) { return ((u128)v.hi << 64) | v.lo; }
static inline okm_key128 from128(u128 x) { return okm_key128{(uint64_t)x, (uint64_t)(x >> 64)}; }

int okm_seq_to_u128(const uint8_t *seq, size_t len, uint8_t k, okm_key128 *out) {
    if (k == 0 || k > 64 || len != (size_t)k || !seq) return 0;
    u128 v = 0;
    for (size_t i = 0; i < len; ++i) {
        const int c = base_code(seq[i]);
        if (c < 0) return 0;
        v = (v << 2) | (u128)c;
    }
    if (out) *out = from128(v);
    return 1;
}

int okm_u128_to_seq(okm_key128 v, uint8_t k, char *out) {
    if (k == 0 || k > 64 || !out) return 0;
    u128 x = to128(v);
    for (int i = k - 1; i >= 0; --i) {
        out[i] = "ACGT"[(unsigned)(x & 3u)];
        x >>= 2;
    }
    return 1;
}

okm_key128 okm_reverse_complement_u128(okm_key128 v, uint8_t k) {
    if (k == 0 || k > 64) return okm_key128{0, 0};
    u128 x = to128(v), r = 0;
    for (int i = 0; i < k; ++i) {  // kmer.rs:83-92 over 2k bits
        r = (r << 2) | ((x & 3u) ^ 3u);
        x >>= 2;
    }
    return from128(r);
}

okm_key128 okm_canonical_u128(okm_key128 v, uint8_t k) {
    const okm_key128 rc = okm_reverse_complement_u128(v, k);
    return to128(v) < to128(rc) ? v : rc;
}

}  // extern "C"
