// rccl_big_p2p.hip — diagnostic for DESIGN §8's "a single 7.9 GB self
// send/recv arrived corrupted": one RCCL rank sends a patterned buffer to
// itself (grouped ncclSend/ncclRecv, as okm_merge_owned at one rank) for a
// list of message sizes and element types, and a kernel counts the received
// words that differ from the pattern.  Sizes straddle 2^31 and 2^32 bytes and
// 2^31 elements, so the failing boundary names the counter that overflows.
//
//   hipcc --offload-arch=gfx950 -O2 tools/rccl_big_p2p.hip -o tools/bin/rccl_big_p2p -lrccl
//   tools/bin/rccl_big_p2p u64:1073741824 u64:4294967296 u8:4294967296 ...
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                            \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)
#define NK(x)                                                                                  \
    do {                                                                                       \
        ncclResult_t r_ = (x);                                                                 \
        if (r_ != ncclSuccess) {                                                               \
            fprintf(stderr, "%s: %s\n", #x, ncclGetErrorString(r_));                           \
            exit(3);                                                                           \
        }                                                                                      \
    } while (0)

__device__ __forceinline__ unsigned long long pat(unsigned long long i) {
    unsigned long long z = i * 0x9E3779B97F4A7C15ull + 0x1234567ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    return z ^ (z >> 31);
}

__global__ void k_fill(unsigned long long *p, unsigned long long n) {
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x)
        p[i] = pat(i);
}

// out[0] = mismatching words, out[1] = first bad word index, out[2] = last bad
__global__ void k_check(const unsigned long long *p, unsigned long long n, unsigned long long *out) {
    unsigned long long bad = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x)
        if (p[i] != pat(i)) {
            ++bad;
            atomicMin(&out[1], i);
            atomicMax(&out[2], i);
        }
    if (bad) atomicAdd(&out[0], bad);
}

int main(int argc, char **argv) {
    ncclUniqueId id;
    NK(ncclGetUniqueId(&id));
    ncclComm_t comm;
    CK(hipSetDevice(0));
    NK(ncclCommInitRank(&comm, 1, id, 0));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    unsigned long long *res;
    CK(hipMalloc(&res, 3 * sizeof(unsigned long long)));
    for (int a = 1; a < argc; ++a) {
        std::string spec(argv[a]);
        const bool u8 = spec.rfind("u8:", 0) == 0;
        const unsigned long long bytes = strtoull(spec.substr(spec.find(':') + 1).c_str(), nullptr, 10) & ~7ull;
        const unsigned long long words = bytes / 8;
        unsigned long long *src, *dst;
        CK(hipMalloc(&src, bytes));
        CK(hipMalloc(&dst, bytes));
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, src, words);
        CK(hipMemsetAsync(dst, 0xA5, bytes, s));
        CK(hipStreamSynchronize(s));
        const size_t count = u8 ? bytes : words;
        const ncclDataType_t t = u8 ? ncclUint8 : ncclUint64;
        auto t0 = std::chrono::steady_clock::now();
        NK(ncclGroupStart());
        NK(ncclSend(src, count, t, 0, comm, s));
        NK(ncclRecv(dst, count, t, 0, comm, s));
        NK(ncclGroupEnd());
        CK(hipStreamSynchronize(s));
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        unsigned long long init[3] = {0, ~0ull, 0}, h[3];
        CK(hipMemcpy(res, init, sizeof(init), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, s, dst, words, res);
        CK(hipMemcpyAsync(h, res, sizeof(h), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        printf("{\"type\": \"%s\", \"bytes\": %llu, \"count\": %zu, \"ms\": %.2f, \"GBs\": %.1f, \"bad_words\": %llu, "
               "\"first_bad_byte\": %lld, \"last_bad_byte\": %lld}\n",
               u8 ? "u8" : "u64", bytes, count, ms, bytes / ms / 1e6, h[0], h[0] ? (long long)(h[1] * 8) : -1LL,
               h[0] ? (long long)(h[2] * 8) : -1LL);
        fflush(stdout);
        CK(hipFree(src));
        CK(hipFree(dst));
    }
    NK(ncclCommDestroy(comm));
    return 0;
}
