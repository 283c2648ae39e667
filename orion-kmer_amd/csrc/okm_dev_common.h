// okm_dev_common.h — device helpers shared by the engine's kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "okm_internal.h"
#include "okm_key.h"

namespace okm {

typedef unsigned long long ull;

// The streaming kernels' barriers: plain __syncthreads().  (A barrier that
// orders LDS only -- a workgroup fence on the local address space + s_barrier,
// so global loads and stores stay in flight across it -- measured the kernels
// within 1-2 % either way and the three-stream step 3 % slower, 5.69 vs 5.52
// ms on C2: profiles/AB_LOG.md.)
__device__ __forceinline__ void lds_sync() { __syncthreads(); }

// A load through a pointer the kernel read from a descriptor (DevSeg /
// DevItem keys and counts): the compiler cannot prove such a pointer global
// and emits FLAT loads, which also count against lgkmcnt -- so every LDS wait
// behind them (the count's tag CASes, the partition's histogram atomics)
// waits for the whole batch of key loads.  Every descriptor pointer is a
// device (global) allocation.
template <typename T>
__device__ __forceinline__ T gload(const T *p) {
    return *(const __attribute__((address_space(1))) T *)p;
}
// 16-B types: one global_load_dwordx4 through a plain vector type (class
// types such as K128 and uint4 cannot be copied out of address space 1)
__device__ __forceinline__ K128 gload(const K128 *p) {
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    const u64x2 v = *(const __attribute__((address_space(1))) u64x2 *)p;
    return K128{v.x, v.y};
}
__device__ __forceinline__ uint4 gload(const uint4 *p) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = *(const __attribute__((address_space(1))) u32x4 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ ull wave_incl_scan(ull v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const ull o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// Block-wide exclusive scan of one value per thread; *total = block sum.
// wsum: BLOCK/64 LDS words.  Contains two barriers (LDS only).
template <int BLOCK>
__device__ __forceinline__ ull block_excl_scan(ull v, ull *wsum, ull *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const ull inc = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = inc;
    lds_sync();
    ull wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) {
        const ull s = wsum[w];
        if (w < wid) wbase += s;
        tot += s;
    }
    lds_sync();
    *total = tot;
    return wbase + inc - v;
}

// block_excl_scan without the trailing barrier: for callers whose next
// write to wsum is separated from this scan's reads by a later barrier anyway.
template <int BLOCK>
__device__ __forceinline__ ull block_excl_scan_1b(ull v, ull *wsum, ull *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const ull inc = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = inc;
    lds_sync();
    ull wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) {
        const ull s = wsum[w];
        if (w < wid) wbase += s;
        tot += s;
    }
    *total = tot;
    return wbase + inc - v;
}

}  // namespace okm
