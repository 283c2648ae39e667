// okm_synth.cpp — seeded synthetic reads for the benchmark and the tests
// (reads sampled uniformly from a random genome, strand
// 50/50, substitution errors, N bases).  Counter-based: every read is a pure
// function of (seed, read index), so any thread count, any shard of read
// indices and any machine produce identical bytes.
#include <stdlib.h>
#include <string.h>

#include <cmath>

#include <algorithm>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "okm_internal.h"

namespace okm {

static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Genome {
    uint64_t seed = 0, len = 0;
    std::vector<uint8_t> codes;  // one 2-bit code per byte
};

// The last few genomes, shared: callers on several threads (one per sample,
// tools/bench_paths.py --loopback) may ask for different genomes at once, and
// a genome stays alive while any caller still reads it.
static std::mutex g_mu;
static std::vector<std::shared_ptr<const Genome>> g_genomes;  // most recent last
constexpr size_t kGenomesKept = 8;

static std::shared_ptr<const Genome> genome(uint64_t seed, uint64_t len) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (size_t i = 0; i < g_genomes.size(); ++i)
            if (g_genomes[i]->seed == seed && g_genomes[i]->len == len) {
                auto g = g_genomes[i];
                g_genomes.erase(g_genomes.begin() + i);
                g_genomes.push_back(g);
                return g;
            }
    }
    auto G = std::make_shared<Genome>();
    G->seed = seed;
    G->len = len;
    G->codes.resize(len);
    // 32 bases per splitmix64 draw
    for (uint64_t i = 0; i < len; i += 32) {
        uint64_t r = splitmix64(seed * 0xD1B54A32D192ED03ull + i / 32);
        const uint64_t m = std::min<uint64_t>(32, len - i);
        for (uint64_t j = 0; j < m; ++j) {
            G->codes[i + j] = (uint8_t)(r & 3);
            r >>= 2;
        }
    }
    std::lock_guard<std::mutex> lk(g_mu);
    g_genomes.push_back(G);
    if (g_genomes.size() > kGenomesKept) g_genomes.erase(g_genomes.begin());
    return G;
}

}  // namespace okm

using namespace okm;

extern "C" okm_status okm_synth_reads(uint64_t genome_seed, uint64_t genome_len, uint64_t seed, uint64_t first_read,
                                      uint64_t n_reads, uint32_t read_len, double sub_rate, double n_rate,
                                      uint8_t *out, int threads) {
    if (!out || read_len == 0 || genome_len < read_len) return fail(OKM_E_ARG, "okm_synth_reads: bad arguments");
    const std::shared_ptr<const Genome> G = genome(genome_seed, genome_len);
    const uint8_t *g = G->codes.data();
    const uint64_t npos = genome_len - read_len + 1;
    // per-base draw: 32-bit uniform u; u < t_sub => substitution, t_sub <= u < t_sub + t_n => N
    const uint64_t t_sub = (uint64_t)(sub_rate * 4294967296.0);
    const uint64_t t_n = (uint64_t)(n_rate * 4294967296.0);
    const size_t stride = (size_t)read_len + 1;
    auto work = [&](uint64_t a, uint64_t b) {
        for (uint64_t i = a; i < b; ++i) {
            const uint64_t r = first_read + i;
            const uint64_t h = splitmix64(seed ^ splitmix64(r));
            const uint64_t pos = h % npos;
            const bool rev = (splitmix64(h) >> 63) != 0;
            uint8_t *o = out + i * stride;
            uint64_t draw = 0;
            for (uint32_t j = 0; j < read_len; ++j) {
                if ((j & 1) == 0) draw = splitmix64(h + 0x632BE59BD9B4E019ull * (j + 1));
                const uint64_t u = (j & 1) ? (draw >> 32) : (draw & 0xFFFFFFFFull);
                uint32_t code = rev ? 3u - g[pos + read_len - 1 - j] : g[pos + j];
                uint8_t ch;
                if (u < t_sub) {
                    code = (code + 1 + (uint32_t)(u % 3)) & 3u;
                    ch = "ACGT"[code];
                } else if (u < t_sub + t_n) {
                    ch = 'N';
                } else {
                    ch = "ACGT"[code];
                }
                o[j] = ch;
            }
            o[read_len] = OKM_RECORD_SEPARATOR;
        }
    };
    int nt = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = (int)std::min<uint64_t>((uint64_t)nt, std::max<uint64_t>(1, n_reads / 4096));
    if (nt <= 1) {
        work(0, n_reads);
        return OKM_OK;
    }
    std::vector<std::thread> ts;
    const uint64_t per = (n_reads + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const uint64_t a = std::min<uint64_t>(n_reads, t * per), b = std::min<uint64_t>(n_reads, a + per);
        ts.emplace_back(work, a, b);
    }
    for (auto &t : ts) t.join();
    return OKM_OK;
}

// ---------------------------------------------------------------------------
// ONT-like long reads: lognormal lengths, either strand,
// substitutions, insertions and deletions.  Counter-based like the reads above.
// ---------------------------------------------------------------------------

namespace okm {

static inline double unit_open(uint64_t x) { return ((double)(x >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

// Read r's length: exp(ln(median) + sigma * z), z standard normal (Box-Muller
// over two splitmix64 draws), clipped to [min_len, max_len].
static uint32_t long_read_len(uint64_t seed, uint64_t r, double median, double sigma, uint32_t lo, uint32_t hi) {
    const uint64_t h = splitmix64(seed ^ splitmix64(r ^ 0x5851F42D4C957F2Dull));
    const double u1 = unit_open(h), u2 = unit_open(splitmix64(h));
    const double z = std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    const double L = std::exp(std::log(median) + sigma * z);
    return (uint32_t)std::min<double>(hi, std::max<double>(lo, std::floor(L)));
}

}  // namespace okm

extern "C" okm_status okm_synth_long_reads(uint64_t genome_seed, uint64_t genome_len, uint64_t seed,
                                           uint64_t first_read, uint64_t n_reads, double median_len, double sigma,
                                           uint32_t min_len, uint32_t max_len, double sub_rate, double ins_rate,
                                           double del_rate, uint8_t **out, uint64_t *n_bytes, uint32_t *lens,
                                           int threads) {
    if (!n_bytes || min_len == 0 || max_len < min_len || median_len <= 0 || sigma < 0 ||
        genome_len < 2ull * max_len + 1 || sub_rate < 0 || ins_rate < 0 || del_rate < 0 ||
        sub_rate + ins_rate + del_rate >= 1.0)
        return fail(OKM_E_ARG, "okm_synth_long_reads: bad arguments");
    if (out) *out = nullptr;
    std::vector<uint64_t> off(n_reads + 1, 0);
    for (uint64_t i = 0; i < n_reads; ++i) {
        const uint32_t L = long_read_len(seed, first_read + i, median_len, sigma, min_len, max_len);
        if (lens) lens[i] = L;
        off[i + 1] = off[i] + L + 1;
    }
    *n_bytes = off[n_reads];
    if (!out) return OKM_OK;  // lengths only
    uint8_t *buf = (uint8_t *)malloc(std::max<uint64_t>(off[n_reads], 1));
    if (!buf) return fail(OKM_E_NOMEM, "okm_synth_long_reads: host allocation");
    const std::shared_ptr<const Genome> G = genome(genome_seed, genome_len);
    const uint8_t *g = G->codes.data();
    const uint64_t npos = genome_len - 2ull * max_len;  // a read consumes < 2 L source bases
    // per-base draw u (32 bits): [0, t1) substitution, [t1, t2) insertion after
    // the base, [t2, t3) deletion of the base, else the base as it is
    const uint64_t t1 = (uint64_t)(sub_rate * 4294967296.0);
    const uint64_t t2 = t1 + (uint64_t)(ins_rate * 4294967296.0);
    const uint64_t t3 = t2 + (uint64_t)(del_rate * 4294967296.0);
    auto work = [&](uint64_t a, uint64_t b) {
        for (uint64_t i = a; i < b; ++i) {
            const uint64_t r = first_read + i;
            const uint64_t h = splitmix64(seed ^ splitmix64(r));
            const uint64_t pos = h % npos;
            const bool rev = (splitmix64(h) >> 63) != 0;
            uint8_t *o = buf + off[i];
            const uint64_t L = off[i + 1] - off[i] - 1;
            uint64_t j = 0, src = pos, d = 0;
            while (j < L) {
                const uint64_t draw = splitmix64(h + 0x632BE59BD9B4E019ull * (++d));
                const uint64_t u = draw & 0xFFFFFFFFull;
                // a run of deletions can consume more than 2 L source bases
                // (npos above assumes fewer): wrap instead of reading past the
                // genome, which leaves every read that stays inside unchanged
                const uint32_t code = g[src];
                src = src + 1 == genome_len ? 0 : src + 1;
                if (u < t1) {
                    o[j++] = (uint8_t)((code + 1 + (uint32_t)((draw >> 32) % 3)) & 3u);
                } else if (u < t2) {
                    o[j++] = (uint8_t)code;
                    if (j < L) o[j++] = (uint8_t)((draw >> 32) & 3u);
                } else if (u >= t3) {
                    o[j++] = (uint8_t)code;
                }  // else: deleted
            }
            if (rev) {  // the other strand: reverse complement of the read
                std::reverse(o, o + L);
                for (uint64_t q = 0; q < L; ++q) o[q] = (uint8_t)(3u - o[q]);
            }
            for (uint64_t q = 0; q < L; ++q) o[q] = (uint8_t)"ACGT"[o[q]];
            o[L] = OKM_RECORD_SEPARATOR;
        }
    };
    int nt = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = (int)std::min<uint64_t>((uint64_t)nt, std::max<uint64_t>(1, n_reads / 64));
    std::vector<std::thread> ts;
    const uint64_t per = (n_reads + nt - 1) / std::max(nt, 1);
    for (int t = 0; t < nt; ++t) {
        const uint64_t a = std::min<uint64_t>(n_reads, t * per), b = std::min<uint64_t>(n_reads, a + per);
        if (a < b) ts.emplace_back(work, a, b);
    }
    for (auto &t : ts) t.join();
    *out = buf;
    return OKM_OK;
}
