// okm_key.h — key types of the device engine.
//
// k <= 32: a canonical k-mer is one u64 (kmer.rs:37-57, MSB-first 2-bit codes,
// upper 64-2k bits zero).  k in 33..64 (the opt-in two-u64 extension, BASELINE
// configs[3]): the same MSB-first 2k-bit value in K128 {lo, hi}.  In both the
// all-ones value is never canonical (k < 32 / k < 64: high bits are zero;
// k = 32 / 64: all-T's canonical is all-A = 0), so it is the empty/padding key.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace okm {

struct __attribute__((aligned(16))) K128 {
    unsigned long long lo, hi;
};

template <typename KT> struct KeyOps;

template <> struct KeyOps<unsigned long long> {
    typedef unsigned long long T;
    static constexpr int kBits = 64;
    __host__ __device__ static __forceinline__ T empty() { return ~0ull; }
    __host__ __device__ static __forceinline__ bool is_empty(T a) { return a == ~0ull; }
    __host__ __device__ static __forceinline__ bool lt(T a, T b) { return a < b; }
    __host__ __device__ static __forceinline__ bool eq(T a, T b) { return a == b; }
    // low 64 bits of (a >> s), s < 64
    __host__ __device__ static __forceinline__ unsigned long long shr(T a, uint32_t s) { return a >> s; }
};

template <> struct KeyOps<K128> {
    typedef K128 T;
    static constexpr int kBits = 128;
    __host__ __device__ static __forceinline__ T empty() { return T{~0ull, ~0ull}; }
    __host__ __device__ static __forceinline__ bool is_empty(T a) { return (a.lo & a.hi) == ~0ull; }
    __host__ __device__ static __forceinline__ bool lt(T a, T b) {
        return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo);
    }
    __host__ __device__ static __forceinline__ bool eq(T a, T b) { return a.hi == b.hi && a.lo == b.lo; }
    // low 64 bits of (a >> s), s < 128
    __host__ __device__ static __forceinline__ unsigned long long shr(T a, uint32_t s) {
        if (s >= 64) return a.hi >> (s - 64);
        if (s == 0) return a.lo;
        return (a.lo >> s) | (a.hi << (64 - s));
    }
};

// Shift value meaning "the whole segment is one bin" (DevSeg::shift).
constexpr uint32_t kSingleBin = 255;

}  // namespace okm
