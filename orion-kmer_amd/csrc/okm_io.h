// okm_io.h — internal host I/O helpers (okm_io.cpp).
#pragma once

#include <stdint.h>
#include <string>
#include <vector>

#include "orion_kmer.h"

namespace okm {

std::string lower_extension(const std::string &path);
okm_status read_whole_file(const std::string &path, std::vector<uint8_t> &data);
// utils.rs:125-152: .gz/.xz/.zst/.zstd by lower-cased last extension.
okm_status decompress_by_extension(const std::string &path, std::vector<uint8_t> &data);
// needletail 0.5.1 sniffing: gzip / bzip2 / xz magic bytes.
okm_status sniff_decompress(std::vector<uint8_t> &data);
size_t format_counts_tsv(uint8_t k, const uint64_t *keys, const uint64_t *counts, size_t n, std::string &out);

// utils.rs:167-198 get_output_writer: compressor chosen by extension.
class OutWriter {
  public:
    OutWriter();
    ~OutWriter();
    okm_status open(const std::string &path);
    okm_status write(const void *data, size_t n);
    okm_status close();

  private:
    struct Impl;
    Impl *p_;
};

}  // namespace okm
