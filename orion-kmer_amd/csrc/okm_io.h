// okm_io.h — internal host I/O helpers (okm_io.cpp).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <functional>
#include <memory>
#include <utility>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "orion_kmer.h"

namespace okm {

// Byte buffers whose resize() does not zero-fill: the feed overwrites every
// byte it grows into, and leaving the first touch to the (parallel) writers
// keeps page faults off one thread.
template <typename T> struct DefaultInitAlloc : std::allocator<T> {
    template <typename U> struct rebind { using other = DefaultInitAlloc<U>; };
    DefaultInitAlloc() = default;
    template <typename U> DefaultInitAlloc(const DefaultInitAlloc<U> &) noexcept {}
    template <typename U> void construct(U *p) noexcept { ::new ((void *)p) U; }
    template <typename U, typename... A> void construct(U *p, A &&...a) {
        ::new ((void *)p) U(std::forward<A>(a)...);
    }
};
using Bytes = std::vector<uint8_t, DefaultInitAlloc<uint8_t>>;

// Host worker threads for the feed (parse, normalise, (de)compress, format):
// OKM_HOST_THREADS, else OMP_NUM_THREADS, else the hardware's, capped at 16.
int host_threads();
// OKM_PROFILE_HOST=1: host-phase wall times on stderr.
bool prof_host();

// Run f(i) for i in [0, n) on up to host_threads() threads (dynamic).
template <typename F> void parallel_for(size_t n, F &&f) {
    const size_t nt = std::min<size_t>(n, (size_t)host_threads());
    if (nt <= 1) {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> ts;
    ts.reserve(nt);
    for (size_t t = 0; t < nt; ++t)
        ts.emplace_back([&]() {
            for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
        });
    for (auto &th : ts) th.join();
}

// One gzip member (header at in[0]) inflated on the host threads
// (okm_inflate.cpp), appended to out; *used = the member's bytes.  *applied is
// false (and nothing done) when the member is too small to split or parallel
// inflate is off (OKM_GZ_PARALLEL=0); an error leaves out's new tail
// unspecified (the caller decodes the member serially instead).
okm_status gunzip_member_parallel(const uint8_t *in, size_t n, Bytes &out, size_t *used, bool *applied);

std::string lower_extension(const std::string &path);
okm_status read_whole_file(const std::string &path, Bytes &data);
// utils.rs:125-152: .gz/.xz/.zst/.zstd by lower-cased last extension.
okm_status decompress_by_extension(const std::string &path, Bytes &data);
// needletail 0.5.1 sniffing: gzip / bzip2 / xz magic bytes.
okm_status sniff_decompress(Bytes &data);
size_t format_counts_tsv(uint8_t k, const uint64_t *keys, const uint64_t *counts, size_t n, std::string &out);

// The count.rs:127-135 TSV of a table that arrives in chunks (e.g. copied off
// the device while the previous chunk is formatted): get(i, &keys, &counts,
// &n) hands over chunk i of nchunks (host memory, valid until get(i + 1) is
// called); lines with count < min_count are skipped.  Plain output is written
// in place with pwrite (no truncation of an existing file's pages until the
// end); .gz/.xz/.zst go through OutWriter in order.  *n_lines (optional)
// receives the lines written.
okm_status write_counts_tsv_chunks(const char *path, uint8_t k, uint64_t min_count, size_t nchunks,
                                   const std::function<okm_status(size_t, const uint64_t **, const uint64_t **,
                                                                  uint64_t *)> &get,
                                   uint64_t *n_lines);

// utils.rs:167-198 get_output_writer: compressor chosen by extension.
class OutWriter {
  public:
    OutWriter();
    ~OutWriter();
    okm_status open(const std::string &path);
    okm_status write(const void *data, size_t n);
    // Several blocks at once (.gz: compressed in parallel, one member each).
    okm_status write_blocks(const std::vector<std::pair<const uint8_t *, size_t>> &blocks);
    // .gz written as parallel-compressed members: true when gzip_member() /
    // write_raw() may be used (the caller compresses on its own threads).
    bool parallel_gzip() const;
    // One block as a complete gzip member (level OKM_GZ_LEVEL; `comp` is a
    // compressor from new_compressor()), into out.
    static okm_status gzip_member(void *comp, const uint8_t *data, size_t n, Bytes &out);
    static void *new_compressor();
    static void free_compressor(void *comp);
    // Bytes already in the output format (compressed members), appended.
    okm_status write_raw(const uint8_t *data, size_t n);
    okm_status close();

  private:
    struct Impl;
    Impl *p_;
};

}  // namespace okm
