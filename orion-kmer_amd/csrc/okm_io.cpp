// okm_io.cpp — extension-selected (de)compression and the TSV writer.
//
// Restates orion-kmer's I/O helpers:
//   utils.rs:125-152 get_decompressed_input_reader  (.gz MultiGz / .xz / .zst|.zstd by
//                                                    lower-cased last extension)
//   utils.rs:167-198 get_output_writer              (.gz default level, .xz level 6,
//                                                    .zst level 0 = zstd default)
//   count.rs:127-135 "{KMER}\t{count}\n" lines
// and needletail 0.5.1's compression sniffing (gzip/bzip2/xz magic; its
// Cargo features have no zstd, Cargo.lock:580-591).
//
// zlib is linked; liblzma, libzstd and libbz2 exist in the image only as
// runtime libraries (no headers), so they are bound with dlopen() and the few
// stable prototypes/structs of their public C APIs are declared here.
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "okm_io.h"
#include "okm_internal.h"

namespace okm {

// ---------------------------------------------------------------------------
// dlopen'ed codec libraries
// ---------------------------------------------------------------------------
struct LzmaStream {  // lzma_stream (liblzma 5.x public layout)
    const uint8_t *next_in;
    size_t avail_in;
    uint64_t total_in;
    uint8_t *next_out;
    size_t avail_out;
    uint64_t total_out;
    const void *allocator;
    void *internal;
    void *reserved_ptr1, *reserved_ptr2, *reserved_ptr3, *reserved_ptr4;
    uint64_t reserved_int1, reserved_int2;
    size_t reserved_int3, reserved_int4;
    int reserved_enum1, reserved_enum2;
};
struct ZstdInBuf { const void *src; size_t size; size_t pos; };
struct ZstdOutBuf { void *dst; size_t size; size_t pos; };
struct BzStream {  // bz_stream (libbz2 1.0 public layout)
    char *next_in;
    unsigned int avail_in, total_in_lo32, total_in_hi32;
    char *next_out;
    unsigned int avail_out, total_out_lo32, total_out_hi32;
    void *state;
    void *(*bzalloc)(void *, int, int);
    void (*bzfree)(void *, void *);
    void *opaque;
};

struct Lzma {
    void *h = nullptr;
    int (*stream_decoder)(LzmaStream *, uint64_t, uint32_t) = nullptr;
    int (*easy_encoder)(LzmaStream *, uint32_t, int) = nullptr;
    int (*code)(LzmaStream *, int) = nullptr;
    void (*end)(LzmaStream *) = nullptr;
};
struct Zstd {
    void *h = nullptr;
    void *(*createDStream)() = nullptr;
    size_t (*initDStream)(void *) = nullptr;
    size_t (*decompressStream)(void *, ZstdOutBuf *, ZstdInBuf *) = nullptr;
    size_t (*freeDStream)(void *) = nullptr;
    void *(*createCCtx)() = nullptr;
    size_t (*setParameter)(void *, int, int) = nullptr;
    size_t (*compressStream2)(void *, ZstdOutBuf *, ZstdInBuf *, int) = nullptr;
    size_t (*freeCCtx)(void *) = nullptr;
    unsigned (*isError)(size_t) = nullptr;
};
struct Bz2 {
    void *h = nullptr;
    int (*decompressInit)(BzStream *, int, int) = nullptr;
    int (*decompress)(BzStream *) = nullptr;
    int (*decompressEnd)(BzStream *) = nullptr;
};

template <typename F>
static bool bind(void *h, const char *name, F &f) {
    f = reinterpret_cast<F>(dlsym(h, name));
    return f != nullptr;
}

static Lzma *lzma_lib() {
    static Lzma L;
    static bool tried = false;
    if (!tried) {
        tried = true;
        L.h = dlopen("liblzma.so.5", RTLD_NOW | RTLD_LOCAL);
        if (L.h && !(bind(L.h, "lzma_stream_decoder", L.stream_decoder) &&
                     bind(L.h, "lzma_easy_encoder", L.easy_encoder) && bind(L.h, "lzma_code", L.code) &&
                     bind(L.h, "lzma_end", L.end)))
            L.h = nullptr;
    }
    return L.h ? &L : nullptr;
}

static Zstd *zstd_lib() {
    static Zstd Z;
    static bool tried = false;
    if (!tried) {
        tried = true;
        Z.h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
        if (Z.h && !(bind(Z.h, "ZSTD_createDStream", Z.createDStream) &&
                     bind(Z.h, "ZSTD_initDStream", Z.initDStream) &&
                     bind(Z.h, "ZSTD_decompressStream", Z.decompressStream) &&
                     bind(Z.h, "ZSTD_freeDStream", Z.freeDStream) && bind(Z.h, "ZSTD_createCCtx", Z.createCCtx) &&
                     bind(Z.h, "ZSTD_CCtx_setParameter", Z.setParameter) &&
                     bind(Z.h, "ZSTD_compressStream2", Z.compressStream2) &&
                     bind(Z.h, "ZSTD_freeCCtx", Z.freeCCtx) && bind(Z.h, "ZSTD_isError", Z.isError)))
            Z.h = nullptr;
    }
    return Z.h ? &Z : nullptr;
}

static Bz2 *bz2_lib() {
    static Bz2 B;
    static bool tried = false;
    if (!tried) {
        tried = true;
        B.h = dlopen("libbz2.so.1", RTLD_NOW | RTLD_LOCAL);
        if (B.h && !(bind(B.h, "BZ2_bzDecompressInit", B.decompressInit) &&
                     bind(B.h, "BZ2_bzDecompress", B.decompress) &&
                     bind(B.h, "BZ2_bzDecompressEnd", B.decompressEnd)))
            B.h = nullptr;
    }
    return B.h ? &B : nullptr;
}

// ---------------------------------------------------------------------------
// decoders (whole buffer -> whole buffer)
// ---------------------------------------------------------------------------
static okm_status gunzip(const uint8_t *in, size_t n, std::vector<uint8_t> &out) {
    // flate2::read::MultiGzDecoder: decode every concatenated gzip member
    out.clear();
    size_t pos = 0;
    std::vector<uint8_t> buf(1 << 20);
    while (pos < n) {
        z_stream z;
        memset(&z, 0, sizeof(z));
        if (inflateInit2(&z, 15 + 16) != Z_OK) return fail(OKM_E_IO, "zlib init failed");
        z.next_in = const_cast<Bytef *>(in + pos);
        z.avail_in = (uInt)std::min<size_t>(n - pos, 1u << 30);
        int rc;
        do {
            z.next_out = buf.data();
            z.avail_out = (uInt)buf.size();
            rc = inflate(&z, Z_NO_FLUSH);
            if (rc != Z_OK && rc != Z_STREAM_END && rc != Z_BUF_ERROR) {
                inflateEnd(&z);
                return fail(OKM_E_IO, "invalid gzip data");
            }
            out.insert(out.end(), buf.data(), buf.data() + (buf.size() - z.avail_out));
            if (rc == Z_BUF_ERROR && z.avail_in == 0) {
                inflateEnd(&z);
                return fail(OKM_E_IO, "truncated gzip data");
            }
        } while (rc != Z_STREAM_END);
        pos += z.total_in;
        inflateEnd(&z);
        // trailing zero padding after the last member is tolerated
        size_t p = pos;
        while (p < n && in[p] == 0) ++p;
        if (p == n) break;
    }
    return OKM_OK;
}

static okm_status unxz(const uint8_t *in, size_t n, std::vector<uint8_t> &out) {
    Lzma *L = lzma_lib();
    if (!L) return fail(OKM_E_IO, "liblzma.so.5 not available");
    LzmaStream s;
    memset(&s, 0, sizeof(s));
    if (L->stream_decoder(&s, UINT64_MAX, 0x08 /*LZMA_CONCATENATED*/) != 0)
        return fail(OKM_E_IO, "lzma decoder init failed");
    std::vector<uint8_t> buf(1 << 20);
    s.next_in = in;
    s.avail_in = n;
    out.clear();
    for (;;) {
        s.next_out = buf.data();
        s.avail_out = buf.size();
        const int rc = L->code(&s, 3 /*LZMA_FINISH*/);
        out.insert(out.end(), buf.data(), buf.data() + (buf.size() - s.avail_out));
        if (rc == 1 /*LZMA_STREAM_END*/) break;
        if (rc != 0) {
            L->end(&s);
            return fail(OKM_E_IO, "invalid xz data");
        }
    }
    L->end(&s);
    return OKM_OK;
}

static okm_status unzstd(const uint8_t *in, size_t n, std::vector<uint8_t> &out) {
    Zstd *Z = zstd_lib();
    if (!Z) return fail(OKM_E_IO, "libzstd.so.1 not available");
    void *ds = Z->createDStream();
    Z->initDStream(ds);
    ZstdInBuf ib{in, n, 0};
    std::vector<uint8_t> buf(1 << 20);
    out.clear();
    for (;;) {
        ZstdOutBuf ob{buf.data(), buf.size(), 0};
        const size_t r = Z->decompressStream(ds, &ob, &ib);
        if (Z->isError(r)) {
            Z->freeDStream(ds);
            return fail(OKM_E_IO, "invalid zstd data");
        }
        out.insert(out.end(), buf.data(), buf.data() + ob.pos);
        if (ib.pos == ib.size && ob.pos < ob.size) break;  // input consumed, output flushed
    }
    Z->freeDStream(ds);
    return OKM_OK;
}

static okm_status unbz2(const uint8_t *in, size_t n, std::vector<uint8_t> &out) {
    Bz2 *B = bz2_lib();
    if (!B) return fail(OKM_E_IO, "libbz2.so.1 not available");
    out.clear();
    size_t pos = 0;
    std::vector<uint8_t> buf(1 << 20);
    while (pos < n) {  // concatenated streams
        BzStream s;
        memset(&s, 0, sizeof(s));
        if (B->decompressInit(&s, 0, 0) != 0) return fail(OKM_E_IO, "bzip2 init failed");
        s.next_in = (char *)(in + pos);
        s.avail_in = (unsigned)std::min<size_t>(n - pos, 1u << 30);
        int rc;
        do {
            s.next_out = (char *)buf.data();
            s.avail_out = (unsigned)buf.size();
            rc = B->decompress(&s);
            if (rc != 0 && rc != 4) {
                B->decompressEnd(&s);
                return fail(OKM_E_IO, "invalid bzip2 data");
            }
            out.insert(out.end(), buf.data(), buf.data() + (buf.size() - s.avail_out));
            if (rc == 0 && s.avail_in == 0 && s.avail_out == buf.size()) {
                B->decompressEnd(&s);
                return fail(OKM_E_IO, "truncated bzip2 data");
            }
        } while (rc != 4 /*BZ_STREAM_END*/);
        pos += ((uint64_t)s.total_in_hi32 << 32) | s.total_in_lo32;
        B->decompressEnd(&s);
    }
    return OKM_OK;
}

std::string lower_extension(const std::string &path) {
    // Path::extension(): text after the last '.' of the file name, if the name
    // does not start with it.
    size_t slash = path.find_last_of('/');
    std::string name = slash == std::string::npos ? path : path.substr(slash + 1);
    size_t dot = name.find_last_of('.');
    if (dot == std::string::npos || dot == 0) return "";
    std::string e = name.substr(dot + 1);
    for (auto &ch : e) ch = (char)tolower((unsigned char)ch);
    return e;
}

okm_status read_whole_file(const std::string &path, std::vector<uint8_t> &data) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return fail(OKM_E_IO, "cannot open " + path);
    data.clear();
    std::vector<uint8_t> buf(1 << 22);
    size_t got;
    while ((got = fread(buf.data(), 1, buf.size(), f)) > 0) data.insert(data.end(), buf.data(), buf.data() + got);
    const bool err = ferror(f);
    fclose(f);
    if (err) return fail(OKM_E_IO, "read error on " + path);
    return OKM_OK;
}

okm_status decompress_by_extension(const std::string &path, std::vector<uint8_t> &data) {
    const std::string e = lower_extension(path);
    std::vector<uint8_t> out;
    if (e == "gz") {
        okm_status s = gunzip(data.data(), data.size(), out);
        if (s != OKM_OK) return s;
    } else if (e == "xz") {
        okm_status s = unxz(data.data(), data.size(), out);
        if (s != OKM_OK) return s;
    } else if (e == "zst" || e == "zstd") {
        okm_status s = unzstd(data.data(), data.size(), out);
        if (s != OKM_OK) return s;
    } else {
        return OKM_OK;
    }
    data.swap(out);
    return OKM_OK;
}

okm_status sniff_decompress(std::vector<uint8_t> &data) {
    std::vector<uint8_t> out;
    const size_t n = data.size();
    const uint8_t *d = data.data();
    okm_status s = OKM_OK;
    if (n >= 2 && d[0] == 0x1f && d[1] == 0x8b) s = gunzip(d, n, out);
    else if (n >= 3 && d[0] == 'B' && d[1] == 'Z' && d[2] == 'h') s = unbz2(d, n, out);
    else if (n >= 6 && d[0] == 0xFD && d[1] == '7' && d[2] == 'z' && d[3] == 'X' && d[4] == 'Z' && d[5] == 0)
        s = unxz(d, n, out);
    else return OKM_OK;
    if (s != OKM_OK) return s;
    data.swap(out);
    return OKM_OK;
}

// ---------------------------------------------------------------------------
// streaming writer selected by extension (utils.rs:167-198)
// ---------------------------------------------------------------------------
struct OutWriter::Impl {
    FILE *f = nullptr;
    int kind = 0;  // 0 plain 1 gz 2 xz 3 zst
    z_stream z;
    LzmaStream lz;
    void *zc = nullptr;
    std::vector<uint8_t> obuf;
    bool ok = true;
};

OutWriter::OutWriter() : p_(new Impl) {}
OutWriter::~OutWriter() {
    if (p_->f) fclose(p_->f);
    delete p_;
}

okm_status OutWriter::open(const std::string &path) {
    p_->f = fopen(path.c_str(), "wb");
    if (!p_->f) return fail(OKM_E_IO, "cannot create " + path);
    const std::string e = lower_extension(path);
    p_->obuf.resize(1 << 20);
    if (e == "gz") {
        p_->kind = 1;
        memset(&p_->z, 0, sizeof(p_->z));
        if (deflateInit2(&p_->z, 6 /*flate2 Compression::default()*/, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK)
            return fail(OKM_E_IO, "zlib deflate init failed");
    } else if (e == "xz") {
        Lzma *L = lzma_lib();
        if (!L) return fail(OKM_E_IO, "liblzma.so.5 not available");
        p_->kind = 2;
        memset(&p_->lz, 0, sizeof(p_->lz));
        if (L->easy_encoder(&p_->lz, 6, 10 /*LZMA_CHECK_CRC64*/) != 0) return fail(OKM_E_IO, "lzma encoder init failed");
    } else if (e == "zst" || e == "zstd") {
        Zstd *Z = zstd_lib();
        if (!Z) return fail(OKM_E_IO, "libzstd.so.1 not available");
        p_->kind = 3;
        p_->zc = Z->createCCtx();
        Z->setParameter(p_->zc, 100 /*ZSTD_c_compressionLevel*/, 3 /*level 0 => default 3*/);
    }
    return OKM_OK;
}

okm_status OutWriter::write(const void *data, size_t n) {
    Impl &I = *p_;
    if (!I.f) return fail(OKM_E_STATE, "writer not open");
    if (n == 0) return OKM_OK;
    switch (I.kind) {
    case 0:
        if (fwrite(data, 1, n, I.f) != n) return fail(OKM_E_IO, "write failed");
        return OKM_OK;
    case 1: {
        I.z.next_in = (Bytef *)data;
        I.z.avail_in = (uInt)n;
        while (I.z.avail_in) {
            I.z.next_out = I.obuf.data();
            I.z.avail_out = (uInt)I.obuf.size();
            if (deflate(&I.z, Z_NO_FLUSH) == Z_STREAM_ERROR) return fail(OKM_E_IO, "deflate failed");
            fwrite(I.obuf.data(), 1, I.obuf.size() - I.z.avail_out, I.f);
        }
        return OKM_OK;
    }
    case 2: {
        Lzma *L = lzma_lib();
        I.lz.next_in = (const uint8_t *)data;
        I.lz.avail_in = n;
        while (I.lz.avail_in) {
            I.lz.next_out = I.obuf.data();
            I.lz.avail_out = I.obuf.size();
            if (L->code(&I.lz, 0 /*LZMA_RUN*/) != 0) return fail(OKM_E_IO, "lzma encode failed");
            fwrite(I.obuf.data(), 1, I.obuf.size() - I.lz.avail_out, I.f);
        }
        return OKM_OK;
    }
    case 3: {
        Zstd *Z = zstd_lib();
        ZstdInBuf ib{data, n, 0};
        while (ib.pos < ib.size) {
            ZstdOutBuf ob{I.obuf.data(), I.obuf.size(), 0};
            size_t r = Z->compressStream2(I.zc, &ob, &ib, 0 /*ZSTD_e_continue*/);
            if (Z->isError(r)) return fail(OKM_E_IO, "zstd compress failed");
            fwrite(I.obuf.data(), 1, ob.pos, I.f);
        }
        return OKM_OK;
    }
    }
    return OKM_OK;
}

okm_status OutWriter::close() {
    Impl &I = *p_;
    if (!I.f) return OKM_OK;
    okm_status st = OKM_OK;
    if (I.kind == 1) {
        int rc;
        do {
            I.z.next_out = I.obuf.data();
            I.z.avail_out = (uInt)I.obuf.size();
            rc = deflate(&I.z, Z_FINISH);
            fwrite(I.obuf.data(), 1, I.obuf.size() - I.z.avail_out, I.f);
        } while (rc == Z_OK);
        deflateEnd(&I.z);
        if (rc != Z_STREAM_END) st = fail(OKM_E_IO, "deflate finish failed");
    } else if (I.kind == 2) {
        Lzma *L = lzma_lib();
        int rc;
        do {
            I.lz.next_out = I.obuf.data();
            I.lz.avail_out = I.obuf.size();
            rc = L->code(&I.lz, 3 /*LZMA_FINISH*/);
            fwrite(I.obuf.data(), 1, I.obuf.size() - I.lz.avail_out, I.f);
        } while (rc == 0);
        L->end(&I.lz);
        if (rc != 1) st = fail(OKM_E_IO, "lzma finish failed");
    } else if (I.kind == 3) {
        Zstd *Z = zstd_lib();
        size_t r;
        do {
            ZstdInBuf ib{nullptr, 0, 0};
            ZstdOutBuf ob{I.obuf.data(), I.obuf.size(), 0};
            r = Z->compressStream2(I.zc, &ob, &ib, 2 /*ZSTD_e_end*/);
            if (Z->isError(r)) {
                st = fail(OKM_E_IO, "zstd end failed");
                break;
            }
            fwrite(I.obuf.data(), 1, ob.pos, I.f);
        } while (r != 0);
        Z->freeCCtx(I.zc);
        I.zc = nullptr;
    }
    if (fclose(I.f) != 0 && st == OKM_OK) st = fail(OKM_E_IO, "close failed");
    I.f = nullptr;
    return st;
}

// 4 bases per byte -> 4 chars
static const char *base4_table() {
    static char t[256 * 4];
    static bool init = false;
    if (!init) {
        for (int b = 0; b < 256; ++b)
            for (int j = 0; j < 4; ++j) t[b * 4 + j] = "ACGT"[(b >> (6 - 2 * j)) & 3];
        init = true;
    }
    return t;
}

size_t format_counts_tsv(uint8_t k, const uint64_t *keys, const uint64_t *counts, size_t n, std::string &out) {
    const char *t = base4_table();
    out.clear();
    out.reserve(n * (k + 8));
    char line[112];
    for (size_t i = 0; i < n; ++i) {
        int pos = 0;
        if (k > 32) {  // two-u64 keys {lo, hi}: base i from bits 2(k-1-i) of hi:lo
            const uint64_t lo = keys[2 * i], hi = keys[2 * i + 1];
            for (int j = 0; j < k; ++j) {
                const unsigned b = 2 * (k - 1 - j);
                line[pos++] = "ACGT"[(b >= 64 ? (hi >> (b - 64)) : (lo >> b)) & 3];
            }
            line[pos++] = '\t';
            char num[24];
            int nd = 0;
            uint64_t c = counts[i];
            do {
                num[nd++] = (char)('0' + c % 10);
                c /= 10;
            } while (c);
            while (nd) line[pos++] = num[--nd];
            line[pos++] = '\n';
            out.append(line, pos);
            continue;
        }
        const uint64_t v = keys[i];
        // u64_to_seq (kmer.rs:61-75): base i from bits 2(k-1-i)
        int rem = k;
        while (rem >= 4) {
            const unsigned shift = 2 * (rem - 4);
            memcpy(line + pos, t + ((v >> shift) & 0xFF) * 4, 4);
            pos += 4;
            rem -= 4;
        }
        while (rem > 0) {
            line[pos++] = "ACGT"[(v >> (2 * (rem - 1))) & 3];
            --rem;
        }
        line[pos++] = '\t';
        // count as decimal
        char num[24];
        int nd = 0;
        uint64_t c = counts[i];
        do {
            num[nd++] = (char)('0' + c % 10);
            c /= 10;
        } while (c);
        while (nd) line[pos++] = num[--nd];
        line[pos++] = '\n';
        out.append(line, pos);
    }
    return out.size();
}

}  // namespace okm

using namespace okm;

extern "C" {

okm_status okm_write_counts_tsv(const char *path, uint8_t k, const uint64_t *keys, const uint64_t *counts,
                                uint64_t n) {
    if (!path) return fail(OKM_E_ARG, "null path");
    if (k == 0 || k > 64) return fail(OKM_E_INVALID_K, "Invalid K-mer size");
    OutWriter w;
    okm_status s = w.open(path);
    if (s != OKM_OK) return s;
    std::string buf;
    const uint64_t step = 1 << 20;
    for (uint64_t o = 0; o < n; o += step) {
        const uint64_t m = std::min(step, n - o);
        format_counts_tsv(k, keys + o * (k > 32 ? 2 : 1), counts + o, m, buf);
        s = w.write(buf.data(), buf.size());
        if (s != OKM_OK) return s;
    }
    return w.close();
}

okm_status okm_write_file(const char *path, const uint8_t *data, uint64_t n) {
    if (!path) return fail(OKM_E_ARG, "null path");
    OutWriter w;
    okm_status s = w.open(path);
    if (s != OKM_OK) return s;
    s = w.write(data, n);
    if (s != OKM_OK) return s;
    return w.close();
}

okm_status okm_read_file(const char *path, int decompress_by_ext, uint8_t **data, uint64_t *n) {
    if (!path || !data || !n) return fail(OKM_E_ARG, "null argument");
    std::vector<uint8_t> v;
    okm_status s = read_whole_file(path, v);
    if (s != OKM_OK) return s;
    if (decompress_by_ext) {
        s = decompress_by_extension(path, v);
        if (s != OKM_OK) return s;
    }
    *data = (uint8_t *)malloc(v.size() ? v.size() : 1);
    if (!*data) return fail(OKM_E_NOMEM, "host allocation");
    memcpy(*data, v.data(), v.size());
    *n = v.size();
    return OKM_OK;
}

}  // extern "C"
