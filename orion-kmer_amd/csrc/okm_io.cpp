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
// zlib is linked; liblzma, libzstd, libbz2 and libdeflate exist in the image
// only as runtime libraries (no headers), so they are bound with dlopen() and
// the few stable prototypes/structs of their public C APIs are declared here.
//
// Host feed: gzip input is inflated with libdeflate when present
// (BGZF members in parallel), .gz output is written as parallel-compressed
// gzip members (flate2's MultiGzDecoder and every gzip reader take them; the
// parity unit is the decompressed text), TSV lines are formatted in parallel
// chunks, and files are read with one sized read().
#include <dlfcn.h>
#include <fcntl.h>
#include <stdio.h>
#include <sys/stat.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <string>
#include <vector>

#include "okm_io.h"
#include "okm_internal.h"
#include "orion_kmer_testing.h"

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

struct Deflate {  // libdeflate 1.x
    void *h = nullptr;
    void *(*alloc_decompressor)() = nullptr;
    void (*free_decompressor)(void *) = nullptr;
    int (*gzip_decompress_ex)(void *, const void *, size_t, void *, size_t, size_t *, size_t *) = nullptr;
    int (*deflate_decompress)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;
    void *(*alloc_compressor)(int) = nullptr;
    void (*free_compressor)(void *) = nullptr;
    size_t (*gzip_compress)(void *, const void *, size_t, void *, size_t) = nullptr;
    size_t (*gzip_compress_bound)(void *, size_t) = nullptr;
};

static Deflate *deflate_lib() {
    static Deflate D;
    static bool tried = false;
    if (!tried) {
        tried = true;
        if (test_knob(OKM_TEST_NO_LIBDEFLATE) != 1) D.h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (D.h && !(bind(D.h, "libdeflate_alloc_decompressor", D.alloc_decompressor) &&
                     bind(D.h, "libdeflate_free_decompressor", D.free_decompressor) &&
                     bind(D.h, "libdeflate_gzip_decompress_ex", D.gzip_decompress_ex) &&
                     bind(D.h, "libdeflate_deflate_decompress", D.deflate_decompress) &&
                     bind(D.h, "libdeflate_alloc_compressor", D.alloc_compressor) &&
                     bind(D.h, "libdeflate_free_compressor", D.free_compressor) &&
                     bind(D.h, "libdeflate_gzip_compress", D.gzip_compress) &&
                     bind(D.h, "libdeflate_gzip_compress_bound", D.gzip_compress_bound)))
            D.h = nullptr;
    }
    return D.h ? &D : nullptr;
}

// ---------------------------------------------------------------------------
// decoders (whole buffer -> whole buffer)
// ---------------------------------------------------------------------------

// BGZF (blocked gzip: every member carries its size in a 'BC' extra field and
// its ISIZE in the trailer) -> member list, or false for plain gzip.
static bool bgzf_members(const uint8_t *in, size_t n, std::vector<size_t> &mb, std::vector<size_t> &ob) {
    mb.assign(1, 0);
    ob.assign(1, 0);
    size_t pos = 0;
    while (pos < n) {
        if (n - pos < 18 || in[pos] != 0x1f || in[pos + 1] != 0x8b || in[pos + 2] != 8 || !(in[pos + 3] & 4))
            return false;
        const size_t xlen = in[pos + 10] | ((size_t)in[pos + 11] << 8);
        size_t bsize = 0;
        for (size_t x = pos + 12; x + 4 <= pos + 12 + xlen && x + 4 <= n;) {
            const size_t slen = in[x + 2] | ((size_t)in[x + 3] << 8);
            if (in[x] == 'B' && in[x + 1] == 'C' && slen == 2 && x + 6 <= n) bsize = (in[x + 4] | ((size_t)in[x + 5] << 8)) + 1;
            x += 4 + slen;
        }
        if (!bsize || pos + bsize > n || bsize < 26) return false;
        const uint8_t *t = in + pos + bsize - 4;
        const size_t isize = t[0] | ((size_t)t[1] << 8) | ((size_t)t[2] << 16) | ((size_t)t[3] << 24);
        pos += bsize;
        mb.push_back(pos);
        ob.push_back(ob.back() + isize);
    }
    return mb.size() > 1;
}

// A member inflated on the host threads (okm_inflate.cpp): true when that
// path took it (pos advanced past it, or st set under OKM_TEST_GZ_STRICT, which
// makes a rejected member an error instead of a serial retry: tests).
static bool member_parallel(const uint8_t *in, size_t n, size_t &pos, Bytes &out, okm_status &st) {
    const size_t base = out.size();
    size_t used = 0;
    bool applied = false;
    const okm_status s = gunzip_member_parallel(in + pos, n - pos, out, &used, &applied);
    if (!applied) return false;
    if (s == OKM_OK) {
        pos += used;
        st = OKM_OK;
        return true;
    }
    out.resize(base);
    if (test_knob(OKM_TEST_GZ_STRICT) == 1) {
        st = s;
        return true;
    }
    return false;
}

static okm_status gunzip_libdeflate(Deflate *D, const uint8_t *in, size_t n, Bytes &out) {
    std::vector<size_t> mb, ob;
    if (bgzf_members(in, n, mb, ob)) {  // members are independent: inflate them in parallel
        out.resize(ob.back());
        std::atomic<int> bad{0};
        const size_t nm = mb.size() - 1, per = 64;
        parallel_for((nm + per - 1) / per, [&](size_t g) {
            void *d = D->alloc_decompressor();
            for (size_t m = g * per; m < std::min(nm, (g + 1) * per) && d; ++m) {
                size_t used = 0, got = 0;
                if (D->gzip_decompress_ex(d, in + mb[m], mb[m + 1] - mb[m], out.data() + ob[m], ob[m + 1] - ob[m],
                                          &used, &got) != 0 || got != ob[m + 1] - ob[m])
                    bad = 1;
            }
            if (d) D->free_decompressor(d);
            else bad = 1;
        });
        if (bad) return fail(OKM_E_IO, "invalid gzip data");
        return OKM_OK;
    }
    // flate2::read::MultiGzDecoder: every concatenated member, in order
    void *d = D->alloc_decompressor();
    if (!d) return fail(OKM_E_NOMEM, "libdeflate allocation");
    out.clear();
    size_t pos = 0;
    okm_status st = OKM_OK;
    // the parallel inflater cuts the rest of the FILE into chunks: once a member
    // ends within the first half of what was left (many concatenated members),
    // the remaining members are inflated one by one instead
    bool par = true;
    while (pos < n) {
        const size_t pos0 = pos;
        if (par && member_parallel(in, n, pos, out, st)) {
            if (st != OKM_OK) break;
            if (2 * (pos - pos0) < n - pos0) par = false;
            size_t p = pos;  // trailing zero padding after the last member is tolerated
            while (p < n && in[p] == 0) ++p;
            if (p == n) break;
            continue;
        }
        // a single-member file's ISIZE (mod 2^32) sizes the output exactly
        size_t cap = std::max<size_t>(n - pos, 1 << 16) * 4;
        const uint8_t *t = in + n - 4;
        const size_t isz = t[0] | ((size_t)t[1] << 8) | ((size_t)t[2] << 16) | ((size_t)t[3] << 24);
        if (pos == 0 && isz > cap) cap = isz + 1;
        for (;;) {
            const size_t base = out.size();
            out.resize(base + cap);
            size_t used = 0, got = 0;
            const int rc = D->gzip_decompress_ex(d, in + pos, n - pos, out.data() + base, cap, &used, &got);
            if (rc == 0) {
                out.resize(base + got);
                pos += used;
                break;
            }
            out.resize(base);
            if (rc != 3 /*LIBDEFLATE_INSUFFICIENT_SPACE*/ || cap > ((size_t)1 << 40)) {
                st = fail(OKM_E_IO, rc == 2 ? "truncated gzip data" : "invalid gzip data");
                break;
            }
            cap *= 2;
        }
        if (st != OKM_OK) break;
        size_t p = pos;  // trailing zero padding after the last member is tolerated
        while (p < n && in[p] == 0) ++p;
        if (p == n) break;
    }
    D->free_decompressor(d);
    return st;
}

static okm_status gunzip(const uint8_t *in, size_t n, Bytes &out) {
    if (Deflate *D = deflate_lib()) return gunzip_libdeflate(D, in, n, out);
    // flate2::read::MultiGzDecoder: decode every concatenated gzip member
    out.clear();
    size_t pos = 0;
    Bytes buf(1 << 20);
    while (pos < n) {
        okm_status pst = OKM_OK;
        if (member_parallel(in, n, pos, out, pst)) {
            if (pst != OKM_OK) return pst;
            size_t p = pos;  // trailing zero padding after the last member is tolerated
            while (p < n && in[p] == 0) ++p;
            if (p == n) break;
            continue;
        }
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

static okm_status unxz(const uint8_t *in, size_t n, Bytes &out) {
    Lzma *L = lzma_lib();
    if (!L) return fail(OKM_E_IO, "liblzma.so.5 not available");
    LzmaStream s;
    memset(&s, 0, sizeof(s));
    if (L->stream_decoder(&s, UINT64_MAX, 0x08 /*LZMA_CONCATENATED*/) != 0)
        return fail(OKM_E_IO, "lzma decoder init failed");
    Bytes buf(1 << 20);
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

static okm_status unzstd(const uint8_t *in, size_t n, Bytes &out) {
    Zstd *Z = zstd_lib();
    if (!Z) return fail(OKM_E_IO, "libzstd.so.1 not available");
    void *ds = Z->createDStream();
    Z->initDStream(ds);
    ZstdInBuf ib{in, n, 0};
    Bytes buf(1 << 20);
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

static okm_status unbz2(const uint8_t *in, size_t n, Bytes &out) {
    Bz2 *B = bz2_lib();
    if (!B) return fail(OKM_E_IO, "libbz2.so.1 not available");
    out.clear();
    size_t pos = 0;
    Bytes buf(1 << 20);
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

int host_threads() {
    static int n = 0;
    if (!n) {
        const char *e = getenv("OKM_HOST_THREADS");
        if (!e || !*e) e = getenv("OMP_NUM_THREADS");
        int v = e && *e ? atoi(e) : (int)std::thread::hardware_concurrency();
        n = std::max(1, std::min(v > 0 ? v : 1, 16));
    }
    return n;
}

bool prof_host() {
    static const bool on = [] {
        const char *e = getenv("OKM_PROFILE_HOST");
        return e && *e && *e != '0';
    }();
    return on;
}

okm_status read_whole_file(const std::string &path, Bytes &data) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return fail(OKM_E_IO, "cannot open " + path);
    struct stat st;
    data.clear();
    okm_status s = OKM_OK;
    if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {  // one sized buffer, parallel pread()s
        // (the destination pages are first touched by the reading threads)
        const size_t size = (size_t)st.st_size, chunk = (size_t)64 << 20;
        data.resize(size);
        const size_t nc = (size + chunk - 1) / chunk;
        std::vector<size_t> got(nc, 0);
        std::atomic<int> bad{0};
        parallel_for(nc, [&](size_t c) {
            const size_t b = c * chunk, e = std::min(size, b + chunk);
            size_t o = b;
            while (o < e) {
                const ssize_t r = ::pread(fd, data.data() + o, e - o, (off_t)o);
                if (r < 0) {
                    bad = 1;
                    break;
                }
                if (r == 0) break;
                o += (size_t)r;
            }
            got[c] = o - b;
        });
        size_t o = 0;  // a file that shrank while being read: keep the prefix that was read
        for (size_t c = 0; c < nc; ++c) {
            o += got[c];
            if (got[c] < std::min(chunk, size - c * chunk)) break;
        }
        if (bad) s = fail(OKM_E_IO, "read error on " + path);
        data.resize(o);
        if (s == OKM_OK && lseek(fd, (off_t)o, SEEK_SET) < 0) s = fail(OKM_E_IO, "read error on " + path);
    }
    if (s == OKM_OK) {  // anything the size did not cover (pipes, growing files)
        Bytes buf(1 << 22);
        ssize_t r;
        while ((r = ::read(fd, buf.data(), buf.size())) > 0) data.insert(data.end(), buf.data(), buf.data() + r);
        if (r < 0) s = fail(OKM_E_IO, "read error on " + path);
    }
    ::close(fd);
    return s;
}

okm_status decompress_by_extension(const std::string &path, Bytes &data) {
    const std::string e = lower_extension(path);
    Bytes out;
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

okm_status sniff_decompress(Bytes &data) {
    Bytes out;
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
    int kind = 0;  // 0 plain 1 gz (zlib stream) 2 xz 3 zst 4 gz (parallel libdeflate members)
    bool wrote = false;
    z_stream z;
    LzmaStream lz;
    void *zc = nullptr;
    Bytes obuf;
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
    if (e == "gz" && deflate_lib()) {
        p_->kind = 4;
    } else if (e == "gz") {
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
    case 4: {
        const size_t piece = (size_t)4 << 20;
        std::vector<std::pair<const uint8_t *, size_t>> blocks;
        for (size_t o = 0; o < n; o += piece) blocks.emplace_back((const uint8_t *)data + o, std::min(piece, n - o));
        return write_blocks(blocks);
    }
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

// Blocks in order.  Kind 4 compresses each block into its own gzip member on
// parallel threads and writes the members in order: the concatenation
// decompresses to the blocks' concatenation (MultiGzDecoder, gzip -d, zcat).
// Level: OKM_GZ_LEVEL, default 1.  flate2's default (6, utils.rs:172) makes
// a k-mer TSV 5 % smaller (0.274 vs 0.289 of the text) at 4.6x the CPU
// (libdeflate, one thread: 35.6 vs 163 MB/s), and it bound `count -o x.tsv.gz`:
// 3.9 of the C2 run's 4.6 s (profiles/r03_e2e_cli.txt).  Parity is on the
// decompressed bytes.
static int gz_level() {
    static const int lvl = [] {
        const char *e = getenv("OKM_GZ_LEVEL");
        const int v = e ? atoi(e) : 1;
        return v >= 1 && v <= 12 ? v : 1;
    }();
    return lvl;
}

bool OutWriter::parallel_gzip() const { return p_->f && p_->kind == 4; }
void *OutWriter::new_compressor() {
    Deflate *D = deflate_lib();
    return D ? D->alloc_compressor(gz_level()) : nullptr;
}
void OutWriter::free_compressor(void *comp) {
    if (comp) deflate_lib()->free_compressor(comp);
}
okm_status OutWriter::gzip_member(void *comp, const uint8_t *data, size_t n, Bytes &out) {
    Deflate *D = deflate_lib();
    if (!D || !comp) return fail(OKM_E_IO, "gzip compression failed");
    out.resize(D->gzip_compress_bound(comp, n));
    const size_t m = D->gzip_compress(comp, data, n, out.data(), out.size());
    if (!m) return fail(OKM_E_IO, "gzip compression failed");
    out.resize(m);
    return OKM_OK;
}
okm_status OutWriter::write_raw(const uint8_t *data, size_t n) {
    Impl &I = *p_;
    if (!I.f) return fail(OKM_E_STATE, "writer not open");
    if (!n) return OKM_OK;
    if (fwrite(data, 1, n, I.f) != n) return fail(OKM_E_IO, "write failed");
    I.wrote = true;
    return OKM_OK;
}

okm_status OutWriter::write_blocks(const std::vector<std::pair<const uint8_t *, size_t>> &blocks) {
    Impl &I = *p_;
    if (!I.f) return fail(OKM_E_STATE, "writer not open");
    if (I.kind != 4) {
        for (auto &b : blocks) {
            okm_status s = write(b.first, b.second);
            if (s != OKM_OK) return s;
        }
        return OKM_OK;
    }
    Deflate *D = deflate_lib();
    const size_t nb = blocks.size();
    std::vector<Bytes> out(nb);
    std::atomic<int> bad{0};
    const size_t nt = std::min<size_t>(nb, (size_t)host_threads());
    parallel_for(nt, [&](size_t t) {
        void *c = D->alloc_compressor(gz_level());
        if (!c) {
            bad = 1;
            return;
        }
        for (size_t i = t; i < nb; i += nt) {
            if (!blocks[i].second) continue;
            out[i].resize(D->gzip_compress_bound(c, blocks[i].second));
            const size_t m = D->gzip_compress(c, blocks[i].first, blocks[i].second, out[i].data(), out[i].size());
            if (!m) bad = 1;
            out[i].resize(m);
        }
        D->free_compressor(c);
    });
    if (bad) return fail(OKM_E_IO, "gzip compression failed");
    for (auto &o : out) {
        if (o.empty()) continue;
        if (fwrite(o.data(), 1, o.size(), I.f) != o.size()) return fail(OKM_E_IO, "write failed");
        I.wrote = true;
    }
    return OKM_OK;
}

okm_status OutWriter::close() {
    Impl &I = *p_;
    if (!I.f) return OKM_OK;
    okm_status st = OKM_OK;
    if (I.kind == 4 && !I.wrote) {  // an empty output is still one (empty) gzip member
        Deflate *D = deflate_lib();
        void *c = D->alloc_compressor(gz_level());
        Bytes o(c ? D->gzip_compress_bound(c, 0) : 0);
        const size_t m = c ? D->gzip_compress(c, "", 0, o.data(), o.size()) : 0;
        if (c) D->free_compressor(c);
        if (!m || fwrite(o.data(), 1, m, I.f) != m) st = fail(OKM_E_IO, "gzip compression failed");
    }
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

// Lines of keys[0, n) with count >= min_count, and their byte length.
static uint64_t tsv_block_bytes(uint8_t k, const uint64_t *counts, uint64_t n, uint64_t min_count, uint64_t *lines) {
    uint64_t bytes = 0, m = 0;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t c = counts[i];
        if (c < min_count) continue;
        int d = 1;
        while (c >= 10) {
            c /= 10;
            ++d;
        }
        bytes += (uint64_t)(k + 2) + d;  // k bases + tab + digits + newline
        ++m;
    }
    *lines = m;
    return bytes;
}

// format_counts_tsv over the entries with count >= min_count.
static void format_filtered(uint8_t k, const uint64_t *keys, const uint64_t *counts, uint64_t n, uint64_t min_count,
                            std::string &out, std::vector<uint64_t> &fk, std::vector<uint64_t> &fc) {
    if (min_count <= 1) {
        format_counts_tsv(k, keys, counts, n, out);
        return;
    }
    const int kw = k > 32 ? 2 : 1;
    fk.clear();
    fc.clear();
    for (uint64_t i = 0; i < n; ++i)
        if (counts[i] >= min_count) {
            fk.insert(fk.end(), keys + i * kw, keys + (i + 1) * kw);
            fc.push_back(counts[i]);
        }
    format_counts_tsv(k, fk.data(), fc.data(), fc.size(), out);
}

okm_status write_counts_tsv_chunks(const char *path, uint8_t k, uint64_t min_count, size_t nchunks,
                                   const std::function<okm_status(size_t, const uint64_t **, const uint64_t **,
                                                                  uint64_t *)> &get,
                                   uint64_t *n_lines) {
    if (!path) return fail(OKM_E_ARG, "null path");
    if (k == 0 || k > 64) return fail(OKM_E_INVALID_K, "Invalid K-mer size");
    const int kw = k > 32 ? 2 : 1;
    const std::string ext = lower_extension(path);
    bool plain = ext != "gz" && ext != "xz" && ext != "zst" && ext != "zstd";
    int fd = -1;
    OutWriter w;
    if (plain) {
        // A regular file is written in place by offset (pwrite) and cut to
        // length at the end: no O_TRUNC, so a rerun over an existing output
        // overwrites its page-cache pages instead of first truncating a
        // multi-GB file (~0.8 s).  Anything else (a pipe, FIFO, tty,
        // /dev/stdout) cannot seek: it takes the sequential writer below, like
        // the reference's File::create (utils.rs:168).
        struct stat st;
        if (::stat(path, &st) == 0 && !S_ISREG(st.st_mode)) {
            plain = false;
        } else {
            fd = ::open(path, O_WRONLY | O_CREAT, 0644);
            if (fd < 0) return fail(OKM_E_IO, std::string("cannot create ") + path);
            if (::fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
                ::close(fd);
                fd = -1;
                plain = false;
            }
        }
    }
    if (!plain) {
        okm_status s = w.open(path);
        if (s != OKM_OK) return s;
    }
    // on failure a plain output keeps only the complete chunks written so far
    // (never a new prefix over an old file's tail)
    auto abandon = [&](uint64_t keep) {
        if (fd >= 0) {
            if (::ftruncate(fd, (off_t)keep) != 0) (void)::unlink(path);
            ::close(fd);
            fd = -1;
        }
    };
    const uint64_t step = plain ? (1 << 16) : (1 << 17);
    uint64_t at_byte = 0, lines = 0;
    std::atomic<int> bad{0};
    for (size_t ci = 0; ci < nchunks && !bad; ++ci) {
        const uint64_t *keys = nullptr, *counts = nullptr;
        uint64_t n = 0;
        okm_status s = get(ci, &keys, &counts, &n);
        if (s != OKM_OK) {
            abandon(at_byte);
            return s;
        }
        if (!n) continue;
        const size_t nb = (size_t)((n + step - 1) / step);
        if (plain) {
            std::vector<uint64_t> off(nb + 1, 0), cnt(nb, 0);
            parallel_for(nb, [&](size_t b) {
                const uint64_t a = b * step, m = std::min<uint64_t>(step, n - a);
                off[b + 1] = tsv_block_bytes(k, counts + a, m, min_count, &cnt[b]);
            });
            for (size_t b = 0; b < nb; ++b) {
                off[b + 1] += off[b];
                lines += cnt[b];
            }
            const uint64_t chunk_start = at_byte;
            const size_t nt = std::min<size_t>(nb, (size_t)host_threads());
            parallel_for(nt, [&](size_t t) {
                std::string buf;
                std::vector<uint64_t> fk, fc;
                for (size_t b = t; b < nb && !bad; b += nt) {
                    const uint64_t a = b * step, m = std::min<uint64_t>(step, n - a);
                    format_filtered(k, keys + a * kw, counts + a, m, min_count, buf, fk, fc);
                    if (buf.size() != off[b + 1] - off[b]) {
                        bad = 2;
                        return;
                    }
                    for (size_t o = 0; o < buf.size();) {
                        const ssize_t wr = ::pwrite(fd, buf.data() + o, buf.size() - o, (off_t)(at_byte + off[b] + o));
                        if (wr <= 0) {
                            bad = 1;
                            return;
                        }
                        o += (size_t)wr;
                    }
                }
            });
            if (bad) {
                abandon(chunk_start);
                break;
            }
            at_byte += off[nb];
        } else if (w.parallel_gzip()) {
            // .gz: every block formatted and compressed into its own gzip member
            // by one thread while it is in cache, and the members appended in
            // order by a writer thread, so the file writes overlap the next
            // blocks' compression (the members decompress to the text in order)
            const size_t nt = std::min<size_t>(nb, (size_t)host_threads());
            std::vector<Bytes> mem(nb);
            std::vector<uint64_t> cnt(nb, 0);
            std::vector<std::atomic<int>> ready(nb);
            for (auto &r : ready) r = 0;
            std::atomic<int> cbad{0};
            std::thread writer([&]() {  // in order, as members complete
                for (size_t b = 0; b < nb; ++b) {
                    while (!ready[b].load(std::memory_order_acquire) && !cbad)
                        std::this_thread::sleep_for(std::chrono::microseconds(50));
                    if (cbad) return;
                    if (w.write_raw(mem[b].data(), mem[b].size()) != OKM_OK) {
                        cbad = 1;
                        return;
                    }
                    Bytes().swap(mem[b]);
                }
            });
            std::atomic<size_t> next{0};
            parallel_for(nt, [&](size_t) {
                void *comp = OutWriter::new_compressor();
                std::string buf;
                std::vector<uint64_t> fk, fc;
                for (size_t b; !cbad && (b = next.fetch_add(1)) < nb;) {  // blocks in order, so the writer never waits long
                    const uint64_t a = b * step, m = std::min<uint64_t>(step, n - a);
                    format_filtered(k, keys + a * kw, counts + a, m, min_count, buf, fk, fc);
                    cnt[b] = (uint64_t)std::count(buf.begin(), buf.end(), '\n');
                    // a block min_count filtered to nothing adds no member (as write_blocks);
                    // close() still writes the one empty member of an empty output
                    if (!buf.empty() &&
                        OutWriter::gzip_member(comp, (const uint8_t *)buf.data(), buf.size(), mem[b]) != OKM_OK) {
                        cbad = 1;
                        break;
                    }
                    ready[b].store(1, std::memory_order_release);
                }
                OutWriter::free_compressor(comp);
            });
            writer.join();
            if (cbad) return fail(OKM_E_IO, std::string("write failed: ") + path);
            for (size_t b = 0; b < nb; ++b) lines += cnt[b];
        } else {
            const size_t per_round = 2 * (size_t)host_threads();
            std::vector<std::string> buf(per_round);
            for (size_t b0 = 0; b0 < nb; b0 += per_round) {
                const size_t rb = std::min(per_round, nb - b0);
                std::vector<uint64_t> cnt(rb, 0);
                parallel_for(rb, [&](size_t j) {
                    std::vector<uint64_t> fk, fc;
                    const uint64_t a = (b0 + j) * step, m = std::min<uint64_t>(step, n - a);
                    format_filtered(k, keys + a * kw, counts + a, m, min_count, buf[j], fk, fc);
                    cnt[j] = (uint64_t)std::count(buf[j].begin(), buf[j].end(), '\n');
                });
                std::vector<std::pair<const uint8_t *, size_t>> blocks;
                for (size_t j = 0; j < rb; ++j) {
                    blocks.emplace_back((const uint8_t *)buf[j].data(), buf[j].size());
                    lines += cnt[j];
                }
                s = w.write_blocks(blocks);
                if (s != OKM_OK) return s;
            }
        }
    }
    if (n_lines) *n_lines = lines;
    if (plain) {
        if (bad == 2) return fail(OKM_E_IO, "TSV block length mismatch");
        if (bad) return fail(OKM_E_IO, std::string("write failed: ") + path);
        if (::ftruncate(fd, (off_t)at_byte) != 0) {
            abandon(0);
            return fail(OKM_E_IO, std::string("write failed: ") + path);
        }
        if (::close(fd) != 0) return fail(OKM_E_IO, std::string("write failed: ") + path);
        return OKM_OK;
    }
    return w.close();
}

}  // namespace okm

using namespace okm;

extern "C" {

// count.rs:127-135 over a host table: one chunk of write_counts_tsv_chunks
// (plain output: every line's length is known from its count's digits, so
// each block of lines gets its byte offset from a prefix sum and the threads
// format and pwrite() their blocks concurrently; compressed output: blocks
// formatted in parallel rounds, compressed and written in order).
okm_status okm_write_counts_tsv(const char *path, uint8_t k, const uint64_t *keys, const uint64_t *counts,
                                uint64_t n) {
    return write_counts_tsv_chunks(path, k, 1, 1,
                                   [&](size_t, const uint64_t **kp, const uint64_t **cp, uint64_t *np) {
                                       *kp = keys;
                                       *cp = counts;
                                       *np = n;
                                       return OKM_OK;
                                   },
                                   nullptr);
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
    Bytes v;
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
