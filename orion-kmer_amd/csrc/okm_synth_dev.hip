// okm_synth_dev.hip — the seeded synthetic read generator of okm_synth.cpp
//  as a gfx950 kernel, so BASELINE configs[2]-sized inputs
// (C3: 167,772,160 reads = 25.4 GB in the batch layout) are made resident in
// HBM in well under a second instead of being generated on the host and
// copied.  Byte-identical to okm_synth_reads for the same arguments (a -m gpu
// test compares them): every read is a pure function of (seed, read index),
// and the genome is never stored — base x of the genome is 2 bits of
// splitmix64(genome_seed * C + x / 32), recomputed where a read needs it.
//
// Layout: one thread writes 16 consecutive bytes of the output (a 16-B vector
// store; reads of 150 bases + separator are 151 bytes, so a thread's bytes
// span at most two reads).
#include "okm_dev_common.h"
#include "okm_hip_try.h"

namespace okm {

__device__ __forceinline__ uint64_t d_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct SynthArgs {
    uint64_t genome_mix;   // genome_seed * 0xD1B54A32D192ED03
    uint64_t npos;         // genome_len - read_len + 1
    uint64_t seed, first_read, n_reads;
    uint64_t total;        // output bytes = n_reads * stride
    uint64_t t_sub, t_n;   // 32-bit thresholds (okm_synth.cpp)
    uint32_t read_len, stride;
};

constexpr int kSynthBlock = 256;

__global__ __launch_bounds__(kSynthBlock) void k_synth_reads(SynthArgs a, uint8_t *__restrict__ out) {
    const uint64_t p0 = ((uint64_t)blockIdx.x * kSynthBlock + threadIdx.x) * 16;
    if (p0 >= a.total) return;
    uint64_t r = p0 / a.stride;
    uint32_t j = (uint32_t)(p0 - r * a.stride);
    // per-read state
    auto read_state = [&](uint64_t rr, uint64_t &h, uint64_t &pos, bool &rev) {
        h = d_splitmix64(a.seed ^ d_splitmix64(a.first_read + rr));
        pos = h % a.npos;
        rev = (d_splitmix64(h) >> 63) != 0;
    };
    uint64_t h, pos;
    bool rev;
    read_state(r, h, pos, rev);
    uint64_t gw_idx = ~0ull, gw = 0;   // cached genome word
    uint64_t draw = 0;
    uint32_t draw_j = ~0u;
    uint8_t b[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        uint8_t ch = 0;
        if (p0 + i < a.total) {
            if (j == a.read_len) {
                ch = OKM_RECORD_SEPARATOR;
            } else {
                const uint64_t x = rev ? pos + a.read_len - 1 - j : pos + j;
                if ((x >> 5) != gw_idx) {
                    gw_idx = x >> 5;
                    gw = d_splitmix64(a.genome_mix + gw_idx);
                }
                uint32_t code = (uint32_t)(gw >> (2 * (x & 31))) & 3u;
                if (rev) code = 3u - code;
                const uint32_t je = j & ~1u;
                if (je != draw_j) {
                    draw_j = je;
                    draw = d_splitmix64(h + 0x632BE59BD9B4E019ull * (uint64_t)(je + 1));
                }
                const uint64_t u = (j & 1) ? (draw >> 32) : (draw & 0xFFFFFFFFull);
                if (u < a.t_sub) {
                    code = (code + 1 + (uint32_t)(u % 3)) & 3u;
                    ch = (uint8_t)"ACGT"[code];
                } else if (u < a.t_sub + a.t_n) {
                    ch = 'N';
                } else {
                    ch = (uint8_t)"ACGT"[code];
                }
            }
            if (++j == a.stride) {  // next read
                j = 0;
                ++r;
                if (r < a.n_reads) read_state(r, h, pos, rev);
                gw_idx = ~0ull;
                draw_j = ~0u;
            }
        }
        b[i] = ch;
    }
    if (p0 + 16 <= a.total && ((uintptr_t)(out + p0) & 15) == 0) {
        uint4 v;
        memcpy(&v, b, 16);
        *(uint4 *)(out + p0) = v;
    } else {
        for (int i = 0; i < 16 && p0 + i < a.total; ++i) out[p0 + i] = b[i];
    }
}

}  // namespace okm

using namespace okm;

extern "C" okm_status okm_synth_reads_device(uint64_t genome_seed, uint64_t genome_len, uint64_t seed,
                                             uint64_t first_read, uint64_t n_reads, uint32_t read_len,
                                             double sub_rate, double n_rate, uint8_t *d_out, int device) {
    if (!d_out || read_len == 0 || genome_len < read_len)
        return fail(OKM_E_ARG, "okm_synth_reads_device: bad arguments");
    if (n_reads == 0) return OKM_OK;
    HIP_TRY(hipSetDevice(device));
    SynthArgs a{};
    a.genome_mix = genome_seed * 0xD1B54A32D192ED03ull;
    a.npos = genome_len - read_len + 1;
    a.seed = seed;
    a.first_read = first_read;
    a.n_reads = n_reads;
    a.stride = read_len + 1;
    a.read_len = read_len;
    a.total = n_reads * (uint64_t)a.stride;
    a.t_sub = (uint64_t)(sub_rate * 4294967296.0);
    a.t_n = (uint64_t)(n_rate * 4294967296.0);
    const uint64_t threads = (a.total + 15) / 16;
    const uint64_t blocks = (threads + kSynthBlock - 1) / kSynthBlock;
    if (blocks > 0x7FFFFFFFull) return fail(OKM_E_ARG, "okm_synth_reads_device: output too large for one launch");
    hipLaunchKernelGGL(k_synth_reads, dim3((uint32_t)blocks), dim3(kSynthBlock), 0, nullptr, a, d_out);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    return OKM_OK;
}
