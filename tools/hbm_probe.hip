// hbm_probe.hip — what the partition pass's memory shape can reach on this
// GPU (tools/hbm_probe.sh builds and runs it):
//   copy4      grid-stride 16-B-per-lane copy (the guide's "float4 copy")
//   tilecopy   k_part_scatter_tile's shape without the sort: 1024-thread
//              workgroups, one per CU, 16 keys per thread loaded into
//              registers, staged through 128 KiB of LDS, written back
//   tilecopy2  the same with the stores going out as 16-key (128-B) runs to
//              1024 scattered destinations per tile (the partition's runs)
// Prints GB/s (bytes read + written per second) per kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned long long ull;

__global__ void copy4(const uint4 *__restrict__ a, uint4 *__restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

constexpr int kB = 1024, kP = 16, kT = kB * kP;

template <bool RUNS>
__global__ __launch_bounds__(kB) void tilecopy(const ull *__restrict__ a, ull *__restrict__ b, size_t ntiles,
                                               size_t nout) {
    extern __shared__ ull st[];
    const uint32_t t = threadIdx.x;
    for (size_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        ull kk[kP];
#pragma unroll
        for (int u = 0; u < kP; ++u) kk[u] = a[tile * kT + u * kB + t];
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kP; ++u) st[u * kB + t] = kk[u];
        __syncthreads();
        for (uint32_t j = t; j < (uint32_t)kT; j += kB) {
            size_t o;
            if (RUNS) {  // run r = j / 16 of this tile goes to a pseudo-random 128-B slot of the output
                const uint32_t r = j >> 4;
                const size_t slot = ((tile * 1024 + r) * 2654435761ull) % (nout / 16);
                o = slot * 16 + (j & 15);
            } else {
                o = tile * kT + j;
            }
            b[o] = st[j];
        }
    }
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : (size_t)3200 << 20;
    const size_t n = bytes / 8 / kT * kT;
    ull *a, *b;
    hipMalloc(&a, n * 8);
    hipMalloc(&b, n * 8);
    hipMemset(a, 1, n * 8);
    hipMemset(b, 0, n * 8);
    hipFuncSetAttribute((const void *)tilecopy<false>, hipFuncAttributeMaxDynamicSharedMemorySize, kT * 8);
    hipFuncSetAttribute((const void *)tilecopy<true>, hipFuncAttributeMaxDynamicSharedMemorySize, kT * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, auto launch) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int reps = 10;
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("%-10s %8.1f GB/s  (%.3f ms for %.2f GB read + write)\n", name, 2.0 * n * 8 / (ms * 1e-3) / 1e9, ms,
               n * 8 / 1e9);
    };
    run("copy4", [&] { copy4<<<4096, 256>>>((const uint4 *)a, (uint4 *)b, n / 2); });
    run("copy4_big", [&] { copy4<<<65536, 256>>>((const uint4 *)a, (uint4 *)b, n / 2); });
    const size_t ntiles = n / kT;
    run("tilecopy", [&] { tilecopy<false><<<256, kB, kT * 8>>>(a, b, ntiles, n); });
    run("tilecopy_runs", [&] { tilecopy<true><<<256, kB, kT * 8>>>(a, b, ntiles, n); });
    run("tilecopy_runs1k", [&] { tilecopy<true><<<1024, kB, kT * 8>>>(a, b, ntiles, n); });
    return 0;
}
