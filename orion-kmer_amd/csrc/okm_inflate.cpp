// okm_inflate.cpp — one gzip member inflated on several host threads.
//
// Host feed (utils.rs:125-152: `.gz` input goes through
// flate2's MultiGzDecoder).  A plain `gzip` file is ONE deflate stream: every
// block may copy from the 32 KiB before it, so a serial decoder (libdeflate,
// zlib) is the only off-the-shelf way in, and it leaves the GPU idle for the
// ~1 s a 1 GiB FASTQ takes to inflate (CLI).  Here the member is
// cut into chunks of compressed bytes and each chunk is decoded on its own
// thread from the first dynamic-Huffman block header found at or after its
// cut, speculatively:
//
//   * a block start is a bit position whose 3-bit header says "dynamic
//     Huffman" and whose code-length, literal/length and distance codes are
//     complete prefix codes (RFC 1951 §3.2.7, zlib's acceptance rules), whose
//     first block then decodes without an invalid symbol or distance, and
//     whose next header is a legal block type;
//   * the chunk's output is 16-bit: a literal is its byte, a copy from before
//     the chunk's first byte is a MARKER naming the byte of the (unknown)
//     32 KiB window it copies (copies of markers stay markers);
//   * each chunk decodes until the first block boundary at or past the next
//     chunk's cut.  The chunks are then stitched in order: a chunk is used
//     when its start equals the previous chunk's stop (the true block
//     boundary); otherwise (a false start, or a region with no dynamic block)
//     that stretch is decoded again from the true boundary;
//   * markers are resolved against the output before the chunk: the last
//     32 KiB of each chunk in order, then all the rest in parallel; the
//     trailer's CRC-32 (combined from per-slice CRCs) and ISIZE are checked.
//
// The output is the deflate stream's by construction: every byte comes from
// decoding the true block sequence (the stitch accepts a chunk only at a true
// boundary) and every marker is the byte at its distance.  Data this decoder
// rejects (a corrupt stream, a trailer mismatch) falls back to the serial
// decoder, which produces the error the reference reports.
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <vector>

#include "okm_internal.h"
#include "okm_io.h"
#include "orion_kmer_testing.h"

namespace okm {

namespace {

constexpr uint32_t kWin = 32768;       // deflate window
constexpr uint16_t kMarker = 0x8000;  // u16 output: kMarker | window index

const uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                               31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                                193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
const uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// LSB-first bit reader over [p, p + nbytes); `pos` is an absolute bit index.
struct Bits {
    const uint8_t *p = nullptr;
    size_t nbytes = 0;
    size_t pos = 0;
    // >= 56 valid bits from pos (zeros past the end)
    uint64_t peek() const {
        const size_t b = pos >> 3;
        uint64_t v = 0;
        if (b + 8 <= nbytes) memcpy(&v, p + b, 8);
        else if (b < nbytes) memcpy(&v, p + b, nbytes - b);
        return v >> (pos & 7);
    }
    uint32_t get(int n) {
        const uint32_t v = (uint32_t)(peek() & ((1ull << n) - 1));
        pos += n;
        return v;
    }
    bool past_end() const { return pos > 8 * nbytes; }
};

// Canonical Huffman decode table: a 10-bit primary table and 5-bit
// subtables for longer codes.  Entry: code length in bits 0-4 (0 = no code),
// symbol in bits 16-31; a subtable link has bit 5 set and its offset in bits
// 16-31.
struct Huff {
    static constexpr int kPri = 10;
    uint32_t t[(1 << kPri) + 32 * 320];
    uint32_t used = 1 << kPri;

    static uint32_t rev(uint32_t c, int len) {
        uint32_t r = 0;
        for (int i = 0; i < len; ++i) r |= ((c >> i) & 1u) << (len - 1 - i);
        return r;
    }
    // kind 0: code-length code (must be complete); 1: literal/length or
    // distance (incomplete only as a single 1-bit code; none at all is
    // accepted and then any use of it fails, like zlib's inflate_table).
    bool build(const uint8_t *lens, int n, int kind) {
        int count[16] = {0};
        int maxl = 0;
        for (int s = 0; s < n; ++s) {
            count[lens[s]]++;
            maxl = std::max<int>(maxl, lens[s]);
        }
        count[0] = 0;
        used = 1 << kPri;
        int left = 1;
        for (int l = 1; l < 16; ++l) {
            left = (left << 1) - count[l];
            if (left < 0) return false;  // over-subscribed
        }
        if (maxl == 0) {
            if (kind != 1) return false;
            memset(t, 0, sizeof(uint32_t) << kPri);
            return true;
        }
        if (left > 0 && (kind == 0 || maxl != 1)) return false;  // incomplete
        // a complete code of <= 10-bit codes writes every primary entry
        if (left > 0 || maxl > kPri) memset(t, 0, sizeof(uint32_t) << kPri);
        uint32_t next[16];
        uint32_t code = 0;
        next[0] = 0;
        for (int l = 1; l < 16; ++l) {
            code = (code + count[l - 1]) << 1;
            next[l] = code;
        }
        for (int s = 0; s < n; ++s) {
            const int l = lens[s];
            if (!l) continue;
            const uint32_t r = rev(next[l]++, l);
            const uint32_t e = ((uint32_t)s << 16) | (uint32_t)l;
            if (l <= kPri) {
                for (uint32_t i = r; i < (1u << kPri); i += 1u << l) t[i] = e;
                continue;
            }
            const uint32_t pri = r & ((1u << kPri) - 1);
            if (!(t[pri] & 32)) {
                if (used + 32 > sizeof(t) / sizeof(t[0])) return false;
                t[pri] = (used << 16) | 32u;
                memset(t + used, 0, 32 * sizeof(uint32_t));
                used += 32;
            }
            uint32_t *sub = t + (t[pri] >> 16);
            for (uint32_t i = r >> kPri; i < 32; i += 1u << (l - kPri)) sub[i] = e;
        }
        return true;
    }
    // symbol, or -1 for a bit pattern that is no code
    inline int decode(uint64_t v, int *len) const {
        uint32_t e = t[v & ((1u << kPri) - 1)];
        if (e & 32) e = t[(e >> 16) + ((v >> kPri) & 31)];
        *len = (int)(e & 31);
        return *len ? (int)(e >> 16) : -1;
    }
};

struct Codes {
    Huff lit, dist;
};

const Codes &fixed_codes() {
    static const Codes *c = [] {
        Codes *f = new Codes;
        uint8_t l[288];
        for (int i = 0; i < 144; ++i) l[i] = 8;
        for (int i = 144; i < 256; ++i) l[i] = 9;
        for (int i = 256; i < 280; ++i) l[i] = 7;
        for (int i = 280; i < 288; ++i) l[i] = 8;
        f->lit.build(l, 288, 1);
        uint8_t d[32];  // codes 30 and 31 exist and are invalid (decode rejects them)
        for (int i = 0; i < 32; ++i) d[i] = 5;
        f->dist.build(d, 32, 1);
        return f;
    }();
    return *c;
}

// The dynamic block header after the 3 type bits (RFC 1951 §3.2.7).
bool read_dynamic(Bits &br, Codes &c) {
    const int hlit = (int)br.get(5) + 257, hdist = (int)br.get(5) + 1, hclen = (int)br.get(4) + 4;
    if (hlit > 286 || hdist > 30) return false;
    uint8_t cl[19] = {0};
    for (int i = 0; i < hclen; ++i) cl[kClOrder[i]] = (uint8_t)br.get(3);
    if (!c.lit.build(cl, 19, 0)) return false;  // the code-length code, parked in `lit`
    uint8_t lens[286 + 30];
    const int total = hlit + hdist;
    for (int i = 0; i < total;) {
        int len;
        const int sym = c.lit.decode(br.peek(), &len);
        if (sym < 0) return false;
        br.pos += len;
        if (sym < 16) {
            lens[i++] = (uint8_t)sym;
            continue;
        }
        int rep;
        uint8_t val = 0;
        if (sym == 16) {
            if (i == 0) return false;
            val = lens[i - 1];
            rep = 3 + (int)br.get(2);
        } else if (sym == 17) {
            rep = 3 + (int)br.get(3);
        } else {
            rep = 11 + (int)br.get(7);
        }
        if (i + rep > total) return false;
        memset(lens + i, val, rep);
        i += rep;
    }
    if (br.past_end() || lens[256] == 0) return false;
    return c.lit.build(lens, hlit, 1) && c.dist.build(lens + hlit, hdist, 1);
}

// u16 output of one chunk (literals, and markers for copies from before it).
struct Out16 {
    std::vector<uint16_t, DefaultInitAlloc<uint16_t>> v;
    size_t n = 0;
    void reserve_more(size_t k) {
        if (n + k > v.size()) v.resize(std::max(v.size() * 2, n + k + (1u << 16)));
    }
};

// Decode one block's data (after its header) with codes c.  Copies reaching
// before the chunk's first output become markers when `spec`, else fail.
bool decode_huff(Bits &br, const Codes &c, Out16 &o, bool spec) {
    const uint32_t wmin = spec ? kWin : 0;  // how far before the chunk a copy may reach
    // bits in a register: buf holds `left` (>= 56 after a refill) unread bits
    const uint8_t *const p = br.p;
    const size_t nb = br.nbytes;
    size_t ip = br.pos >> 3;  // next byte to load (may count past nb: those bits are zeros)
    uint64_t buf = 0;
    unsigned left = 0;
    auto refill = [&]() {
        if (ip + 8 <= nb) {
            uint64_t w;
            memcpy(&w, p + ip, 8);
            buf |= w << left;
            ip += (63 - left) >> 3;
            left |= 56;
        } else {
            while (left <= 56) {  // past the end: zero bits (ip keeps counting, so the overrun shows)
                buf |= (uint64_t)(ip < nb ? p[ip] : 0) << left;
                ++ip;
                left += 8;
            }
        }
    };
    refill();
    buf >>= br.pos & 7;
    left -= br.pos & 7;
    auto pos_now = [&]() { return ip * 8 - left; };
    const uint32_t *lt = c.lit.t, *dt = c.dist.t;
    auto look = [](const uint32_t *t, uint64_t v) {
        uint32_t e = t[v & ((1u << Huff::kPri) - 1)];
        if (e & 32) e = t[(e >> 16) + ((v >> Huff::kPri) & 31)];
        return e;
    };
    for (;;) {
        o.reserve_more(1 << 16);
        uint16_t *out = o.v.data();
        size_t n = o.n;
        const size_t room = o.v.size() - 258 - 16;  // a symbol writes <= 258 (+ 7 of copy overrun)
        while (n <= room) {
            refill();
            uint32_t e = look(lt, buf);
            uint32_t len = e & 31;
            if (!len) return false;
            uint32_t sym = e >> 16;
            if (sym < 256) {  // up to two more literals from the same refill (3 x 15 bits <= 56)
                buf >>= len;
                left -= len;
                out[n++] = (uint16_t)sym;
                e = look(lt, buf);
                len = e & 31;
                sym = e >> 16;
                if (!len) return false;
                if (sym >= 256) goto not_literal;
                buf >>= len;
                left -= len;
                out[n++] = (uint16_t)sym;
                e = look(lt, buf);
                len = e & 31;
                sym = e >> 16;
                if (!len) return false;
                if (sym >= 256) {
                    refill();
                    goto not_literal;
                }
                buf >>= len;
                left -= len;
                out[n++] = (uint16_t)sym;
                continue;
            }
        not_literal:
            if (sym == 256) {
                buf >>= len;
                left -= len;
                o.n = n;
                br.pos = pos_now();
                return !br.past_end();
            }
            {
                if (left < 48) refill();
                const uint32_t li = sym - 257;
                if (li >= 29) return false;
                buf >>= len;
                left -= len;
                const uint32_t xl = kLenExtra[li];
                const uint32_t L = kLenBase[li] + (uint32_t)(buf & ((1u << xl) - 1));
                buf >>= xl;
                left -= xl;
                const uint32_t de = look(dt, buf), dl = de & 31, ds = de >> 16;
                if (!dl || ds >= 30) return false;
                buf >>= dl;
                left -= dl;
                const uint32_t xd = kDistExtra[ds];
                const uint32_t D = kDistBase[ds] + (uint32_t)(buf & ((1u << xd) - 1));
                buf >>= xd;
                left -= xd;
                if (D > n + wmin) return false;
                uint16_t *dst = out + n;
                if (D <= n) {
                    const uint16_t *src = dst - D;
                    if (D >= 8) {
                        for (uint32_t i = 0; i < L; i += 8) memcpy(dst + i, src + i, 16);
                    } else {
                        for (uint32_t i = 0; i < L; ++i) dst[i] = src[i];
                    }
                } else {
                    // the first D - n bytes come from the window before the chunk
                    for (uint32_t i = 0; i < L; ++i) {
                        const size_t at = n + i;  // output index being written
                        out[at] = at >= D ? out[at - D] : (uint16_t)(kMarker | (uint16_t)(kWin + at - D));
                    }
                }
                n += L;
            }
        }
        o.n = n;
        if (ip > nb + 8) return false;  // ran far past the input
    }
}

// One block (header included) at br.pos.  *final: BFINAL.
bool decode_block(Bits &br, Codes &scratch, Out16 &o, bool spec, bool *final) {
    *final = br.get(1) != 0;
    const uint32_t type = br.get(2);
    if (type == 0) {  // stored
        br.pos = (br.pos + 7) & ~(size_t)7;
        const size_t b = br.pos >> 3;
        if (b + 4 > br.nbytes) return false;
        const uint32_t len = br.p[b] | (br.p[b + 1] << 8), nlen = br.p[b + 2] | (br.p[b + 3] << 8);
        if ((len ^ 0xFFFFu) != nlen || b + 4 + len > br.nbytes) return false;
        o.reserve_more(len);
        for (uint32_t i = 0; i < len; ++i) o.v[o.n + i] = br.p[b + 4 + i];
        o.n += len;
        br.pos += 8 * (4 + (size_t)len);
        return true;
    }
    if (type == 1) return decode_huff(br, fixed_codes(), o, spec);
    if (type == 2) return read_dynamic(br, scratch) && decode_huff(br, scratch, o, spec);
    return false;
}

struct Piece {
    size_t start = 0;  // bit position of its first block header
    size_t stop = 0;   // bit position after its last block (a block boundary)
    bool final = false;
    bool ok = false;
    Out16 out;
};

// Decode blocks from `start` until a block boundary >= stop_at (or the final
// block).  spec: the window before `start` is unknown (markers).
bool decode_run(const uint8_t *p, size_t nbytes, size_t start, size_t stop_at, bool spec, Codes &scratch,
                Piece &pc) {
    Bits br{p, nbytes, start};
    pc.start = start;
    pc.final = false;
    for (;;) {
        bool fin;
        if (!decode_block(br, scratch, pc.out, spec, &fin)) return false;
        if (fin) {
            pc.final = true;
            break;
        }
        if (br.pos >= stop_at) break;
    }
    pc.stop = br.pos;
    return true;
}

// The first position in [from, to) where a dynamic block starts whose block
// decodes and is followed by a legal header; its decode continues to stop_at.
bool find_and_decode(const uint8_t *p, size_t nbytes, size_t from, size_t to, size_t stop_at, Codes &scratch,
                     Piece &pc) {
    for (size_t s = from; s < to; ++s) {
        Bits br{p, nbytes, s};
        const uint64_t v = br.peek();
        if (((v >> 1) & 3) != 2) continue;  // not a dynamic block
        br.pos += 3;
        // cheap header screen before building anything
        if (((v >> 3) & 31) + 257 > 286 || ((v >> 8) & 31) + 1 > 30) continue;
        if (!read_dynamic(br, scratch)) continue;
        pc.out.n = 0;
        if (!decode_huff(br, scratch, pc.out, true)) continue;
        if (!(v & 1)) {  // not final: the next header must be a legal type
            const uint64_t nx = br.peek();
            if (((nx >> 1) & 3) == 3) continue;
        }
        // accepted: the rest of the run from here
        if (v & 1) {
            pc.start = s;
            pc.stop = br.pos;
            pc.final = true;
            return true;
        }
        if (br.pos >= stop_at) {
            pc.start = s;
            pc.stop = br.pos;
            pc.final = false;
            return true;
        }
        Piece rest;
        rest.out = std::move(pc.out);
        Bits b2 = br;
        bool fin = false;
        bool good = true;
        while (good) {
            if (!decode_block(b2, scratch, rest.out, true, &fin)) {
                good = false;
                break;
            }
            if (fin || b2.pos >= stop_at) break;
        }
        pc.out = std::move(rest.out);
        if (!good) continue;  // a false start that decoded one block by chance
        pc.start = s;
        pc.stop = b2.pos;
        pc.final = fin;
        return true;
    }
    return false;
}

// Transparent huge pages for a large buffer about to be written (fewer page
// faults on first touch: the output of a 1 GiB member is 262 K small pages).
void huge_pages(void *p, size_t bytes) {
    const uintptr_t a = ((uintptr_t)p + 4095) & ~(uintptr_t)4095;
    const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)4095;
    if (bytes >= (8u << 20) && e > a) (void)madvise((void *)a, e - a, MADV_HUGEPAGE);
}

size_t gzip_header_len(const uint8_t *in, size_t n) {
    if (n < 18 || in[0] != 0x1f || in[1] != 0x8b || in[2] != 8) return 0;
    const uint8_t flg = in[3];
    if (flg & 0xE0) return 0;
    size_t h = 10;
    if (flg & 4) {
        if (h + 2 > n) return 0;
        h += 2 + (in[h] | ((size_t)in[h + 1] << 8));
    }
    if (flg & 8) {
        while (h < n && in[h]) ++h;
        ++h;
    }
    if (flg & 16) {
        while (h < n && in[h]) ++h;
        ++h;
    }
    if (flg & 2) h += 2;
    return h < n ? h : 0;
}

}  // namespace

// Smallest member inflated in parallel (16 MiB) and compressed bytes per
// chunk (4 MiB); tests go lower (OKM_TEST_GZ_PAR_MIN_BYTES / _CHUNK_BYTES).
static size_t knob_or(int knob, size_t dflt) {
    const int64_t v = test_knob(knob);
    return v >= 0 ? (size_t)v : dflt;
}

okm_status gunzip_member_parallel(const uint8_t *in, size_t n, Bytes &out, size_t *used, bool *applied) {
    *applied = false;
    *used = 0;
    const int nt = host_threads();
    const char *off = getenv("OKM_GZ_PARALLEL");  // 0: serial inflate
    const bool forced = test_knob(OKM_TEST_GZ_STRICT) == 1;  // tests: also on one thread
    if ((off && *off == '0') || (nt < 2 && !forced) ||
        n < std::max<size_t>(knob_or(OKM_TEST_GZ_PAR_MIN_BYTES, 16u << 20), 1 << 12))
        return OKM_OK;
    const size_t h = gzip_header_len(in, n);
    if (!h) return OKM_OK;
    *applied = true;
    const uint8_t *p = in + h;
    const size_t nbytes = n - h;
    // chunk cuts in compressed bytes: ~4 MiB each, at least two per thread
    const size_t cb = std::max<size_t>(knob_or(OKM_TEST_GZ_CHUNK_BYTES, 4u << 20), 1 << 10);
    const size_t want = std::max<size_t>(2 * (size_t)nt, nbytes / cb);
    const size_t nch = std::max<size_t>(1, std::min<size_t>(want, nbytes / std::min<size_t>(cb, 1 << 16) + 1));
    std::vector<size_t> cut(nch + 1);
    for (size_t i = 0; i <= nch; ++i) cut[i] = 8 * (nbytes * i / nch);
    cut[nch] = SIZE_MAX;
    // rounds of R chunks: the 16-bit pieces of one round at a time (host memory
    // stays ~R x 4 MiB x 12 B whatever the member's size)
    const size_t R = std::max<size_t>(2, 2 * (size_t)nt);
    const bool prof = prof_host();
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t_dec = 0, t_res = 0, t_crc = 0;
    size_t rounds = 0, used_pieces = 0, dropped = 0;
    const size_t base = out.size();
    {
        const uint8_t *t4 = in + n - 4;  // a single member's ISIZE (mod 2^32) as a size hint
        const size_t isz = t4[0] | (t4[1] << 8) | (t4[2] << 16) | ((size_t)t4[3] << 24);
        const size_t need = base + std::max(isz, nbytes * 4);
        if (need > out.capacity()) {  // geometric: a file of many members is not copied once per member
            out.reserve(std::max(need, 2 * out.capacity()));
            huge_pages(out.data() + base, out.capacity() - base);
        }
    }
    std::vector<Piece> pool(R);  // 16-bit piece buffers, reused round to round (their pages stay faulted in)
    uLong crc = crc32(0L, Z_NULL, 0);
    size_t pos = 0;  // bit position of the next block header (a true boundary)
    bool fin = false;
    size_t misses = 0;  // consecutive rounds that used only their first chunk
    while (!fin) {
        size_t j0 = 0;  // the chunk whose region holds pos
        while (j0 + 1 < nch && cut[j0 + 1] <= pos) ++j0;
        // a stretch with no dynamic blocks to find (stored blocks: incompressible
        // input) is decoded one chunk at a time, with a parallel try every 8 rounds
        const size_t nr = std::min(misses >= 2 && (rounds & 7) ? 1 : R, nch - j0);
        std::vector<Piece> &pcs = pool;
        std::atomic<int> broken{0};
        double t0 = now();
        parallel_for(nr, [&](size_t q) {
            const size_t i = j0 + q;
            Codes *scratch = new Codes;
            Piece &pc = pcs[q];
            pc.ok = pc.final = false;
            pc.out.n = 0;
            const size_t want = std::max<size_t>(1 << 16, (size_t)(nbytes / nch) * 6);
            if (pc.out.v.size() < want) {
                pc.out.v.resize(want);
                huge_pages(pc.out.v.data(), pc.out.v.size() * sizeof(uint16_t));
            }
            if (q == 0) {  // from the true boundary; copies before it are markers (unless the stream starts here)
                pc.ok = decode_run(p, nbytes, pos, cut[i + 1], pos != 0, *scratch, pc);
                if (!pc.ok) broken = 1;
            } else {
                // a block start within the chunk's first MiB (dynamic blocks are
                // far smaller; a stored-block stretch without one is decoded from
                // the true boundary by a later round instead of searched bit by bit)
                const size_t to = std::min({cut[i + 1], 8 * nbytes, cut[i] + (size_t(8) << 20)});
                pc.ok = find_and_decode(p, nbytes, cut[i], to, cut[i + 1], *scratch, pc);
            }
            delete scratch;
        });
        t_dec += now() - t0;
        if (broken) return fail(OKM_E_IO, "invalid gzip data");
        // stitch: a chunk is used where it starts at the previous one's stop;
        // the round ends at the first that does not (the next round decodes
        // from that true boundary)
        size_t ns = 1;
        pos = pcs[0].stop;
        fin = pcs[0].final;
        while (!fin && ns < nr && pcs[ns].ok && pcs[ns].start == pos) {
            pos = pcs[ns].stop;
            fin = pcs[ns].final;
            ++ns;
        }
        dropped += nr - ns;
        if (nr > 1) misses = ns == 1 ? misses + 1 : 0;
        used_pieces += ns;
        ++rounds;
        // place and resolve: markers name bytes of the 32 KiB before their piece
        t0 = now();
        const size_t rbase = out.size();
        std::vector<size_t> at(ns + 1, rbase);
        for (size_t q = 0; q < ns; ++q) at[q + 1] = at[q] + pcs[q].out.n;
        out.resize(at[ns]);
        uint8_t *o = out.data();
        std::atomic<int> bad{0};
        auto resolve = [&](size_t q, size_t a, size_t b) {  // piece q's outputs [a, b)
            const uint16_t *sv = pcs[q].out.v.data();
            uint8_t *d = o + at[q];
            const int64_t wbase = (int64_t)(at[q] - base) - (int64_t)kWin;  // member offset of window byte 0
            for (size_t x = a; x < b; ++x) {
                if ((x & 31) == 0 && x + 32 <= b) {  // a run of 32 literals narrows in one vector pass
                    uint16_t any = 0;
                    for (int u = 0; u < 32; ++u) any |= sv[x + u];
                    if (!(any & 0xFF00)) {
                        for (int u = 0; u < 32; ++u) d[x + u] = (uint8_t)sv[x + u];
                        x += 31;
                        continue;
                    }
                }
                const uint16_t v = sv[x];
                if (v < 256) {
                    d[x] = (uint8_t)v;
                    continue;
                }
                const int64_t src = wbase + (int64_t)(v & (kWin - 1));
                if (src < 0) {
                    bad = 1;
                    return;
                }
                d[x] = o[base + src];
            }
        };
        // the tail (last 32 KiB) of every piece in order, then the rest in
        // parallel; each stretch's CRC-32 is taken right after it is resolved
        // (while it is in cache) and the CRCs are combined in output order
        const uLong crc0 = crc32(0L, Z_NULL, 0);
        std::vector<uLong> tail_crc(ns);
        for (size_t q = 0; q < ns; ++q) {
            const size_t len = pcs[q].out.n, head = len > kWin ? len - kWin : 0;
            resolve(q, head, len);
            if (bad) return fail(OKM_E_IO, "invalid gzip data");
            tail_crc[q] = crc32(crc0, o + at[q] + head, (uInt)(len - head));
        }
        constexpr size_t kSlice = 1 << 20;
        std::vector<std::pair<size_t, size_t>> jobs;
        for (size_t q = 0; q < ns; ++q) {
            const size_t len = pcs[q].out.n, head = len > kWin ? len - kWin : 0;
            for (size_t a = 0; a < head; a += kSlice) jobs.emplace_back(q, a);
        }
        std::vector<uLong> job_crc(jobs.size());
        parallel_for(jobs.size(), [&](size_t j) {
            const size_t q = jobs[j].first, a = jobs[j].second;
            const size_t len = pcs[q].out.n, head = len > kWin ? len - kWin : 0;
            const size_t b = std::min(head, a + kSlice);
            resolve(q, a, b);
            job_crc[j] = crc32(crc0, o + at[q] + a, (uInt)(b - a));
        });
        if (bad) return fail(OKM_E_IO, "invalid gzip data");
        t_res += now() - t0;
        t0 = now();
        for (size_t q = 0, j = 0; q < ns; ++q) {  // jobs are in piece order, then offset order
            const size_t len = pcs[q].out.n, head = len > kWin ? len - kWin : 0;
            for (; j < jobs.size() && jobs[j].first == q; ++j)
                crc = crc32_combine(crc, job_crc[j], (z_off_t)(std::min(head, jobs[j].second + kSlice) - jobs[j].second));
            crc = crc32_combine(crc, tail_crc[q], (z_off_t)(len - head));
        }
        t_crc += now() - t0;
        if (rounds > 4 * nch + 4) return fail(OKM_E_IO, "invalid gzip data");  // no progress (cannot happen)
    }
    // trailer: CRC-32 and ISIZE of this member
    const size_t tb = (pos + 7) >> 3;
    if (tb + 8 > nbytes) return fail(OKM_E_IO, "truncated gzip data");
    const uint8_t *t = p + tb;
    const uint32_t crc_want = t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24);
    const uint32_t isz = t[4] | (t[5] << 8) | (t[6] << 16) | ((uint32_t)t[7] << 24);
    const size_t total = out.size() - base;
    if ((uint32_t)total != isz || (uint32_t)crc != crc_want) return fail(OKM_E_IO, "invalid gzip data");
    *used = h + tb + 8;
    if (prof)
        fprintf(stderr,
                "[okm gz] %zu chunks in %zu rounds (%zu pieces used, %zu dropped), %.1f MB -> %.1f MB: decode %.1f ms, "
                "resolve %.1f, crc %.1f\n",
                nch, rounds, used_pieces, dropped, nbytes / 1e6, total / 1e6, t_dec * 1e3, t_res * 1e3, t_crc * 1e3);
    return OKM_OK;
}

}  // namespace okm
