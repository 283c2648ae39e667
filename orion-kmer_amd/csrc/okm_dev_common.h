// okm_dev_common.h — device helpers shared by the engine's kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "okm_internal.h"
#include "okm_key.h"

namespace okm {

typedef unsigned long long ull;

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
// wsum: BLOCK/64 LDS words.  Contains two __syncthreads().
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

}  // namespace okm
