// probe_ceiling.hip — the random-probe ceiling that bounds k_query_hits and
// the classify probe (okm_probe.hip): every probe reads one 8-B slot at a
// hashed index of a u64 table, 16 independent probes per thread in flight (the
// query kernel's shape), hits summed per wave.  Run over table sizes from
// L2-resident to the query's 2 GiB open-addressing set, it gives the probes/s
// a one-line-per-probe design can reach on this GPU, i.e. what `query`'s
// roofline should be priced against (its streaming-byte fraction is not).
//   usage: probe_ceiling [probes_millions]      (tools/probe_ceiling.sh)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long ull;

__device__ __forceinline__ ull mix(ull x) {  // murmur3 fmix64, as slot_hash
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

constexpr int kP = 16;

__global__ __launch_bounds__(256) void gather(const ull *__restrict__ tab, uint32_t shift, ull nprobe, ull seed,
                                              ull *__restrict__ out) {
    const ull base = ((ull)blockIdx.x * 256 + threadIdx.x) * kP;
    if (base >= nprobe) return;
    ull s[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j) s[j] = tab[mix(seed + base + j) >> shift];
    ull hit = 0;
#pragma unroll
    for (int j = 0; j < kP; ++j) hit += s[j] == (base + j) ? 1u : 0u;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) hit += __shfl_xor(hit, d, 64);
    if ((threadIdx.x & 63) == 0 && hit) atomicAdd(out, hit);
}

int main(int argc, char **argv) {
    const ull nprobe = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 400ull) * 1000000ull / (256 * kP) * (256 * kP);
    ull *tab, *out;
    const int max_log2 = 28;  // 2 GiB of u64 slots: the query set's table at C2
    if (hipMalloc(&tab, (8ull << max_log2)) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
    hipMemset(tab, 0xff, 8ull << max_log2);
    hipMemset(out, 0, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const dim3 grid((uint32_t)(nprobe / (256 * kP)));
    printf("%llu probes per launch, %d in flight per lane\n", nprobe, kP);
    for (int lg = 20; lg <= max_log2; lg += 2) {
        const uint32_t shift = 64 - lg;
        gather<<<grid, 256>>>(tab, shift, nprobe, 1, out);
        hipDeviceSynchronize();
        const int reps = 5;
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) gather<<<grid, 256>>>(tab, shift, nprobe, 7 + r, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        const double gps = nprobe / (ms * 1e-3) / 1e9;
        printf("table %8.1f MiB  %7.3f ms  %7.2f G probes/s  (x64 B = %6.0f GB/s, x128 B = %6.0f GB/s of lines)\n",
               (8ull << lg) / 1048576.0, ms, gps, gps * 64, gps * 128);
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
