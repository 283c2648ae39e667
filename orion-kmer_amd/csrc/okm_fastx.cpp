// okm_fastx.cpp — host record source replacing needletail 0.5.1's
// parse_fastx_reader + SequenceRecord::normalize(false) at count.rs:59-72,
// build.rs:38-48 (crate pinned at Cargo.lock:580-591, not vendored; its
// record semantics are restated in SURVEY.md Appendix A):
//
//  - format by first byte: '>' FASTA, '@' FASTQ, anything else (or an empty
//    input) is a parse error (count.rs:63-64 context "Failed to parse FASTA/Q
//    content from: …");
//  - FASTA: header line after '>', sequence = every following line up to the
//    next line starting with '>'; line breaks are dropped by normalize, so
//    multi-line records are joined; header-only records have an empty
//    sequence;
//  - FASTQ: 4-line records (@id / seq / + / qual), seq and qual lengths must
//    match, otherwise a record error (count.rs:69-70 "Error reading record
//    from …");
//  - normalize(false): A C G T kept, a c g t upper-cased, U/u -> T,
//    '.', '~' -> '-', space/tab/CR/LF removed, every other byte -> 'N'.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

#include <string>
#include <vector>

#include "okm_internal.h"
#include "okm_io.h"

namespace okm {

static const uint8_t *norm_table() {
    static uint8_t t[256];
    static bool init = false;
    if (!init) {
        for (int c = 0; c < 256; ++c) t[c] = 'N';
        t['A'] = 'A'; t['C'] = 'C'; t['G'] = 'G'; t['T'] = 'T';
        t['a'] = 'A'; t['c'] = 'C'; t['g'] = 'G'; t['t'] = 'T';
        t['U'] = 'T'; t['u'] = 'T';
        t['-'] = '-'; t['.'] = '-'; t['~'] = '-';
        t[' '] = 0; t['\t'] = 0; t['\r'] = 0; t['\n'] = 0;  // removed
        init = true;
    }
    return t;
}

struct Parser {
    Bytes data;
    size_t pos = 0;
    bool fastq = false;
    bool raw = false;   // query.rs:66: record.sequence() as is (no normalize)
    bool want_ids = false;
    uint64_t records = 0;
    Bytes ids;     // ids of the records read by the current batch
    std::vector<uint64_t> id_off;

    void add_id(size_t b, size_t e) {  // needletail id(): header after the marker, CR trimmed
        e = rstrip_cr(data, b, e);
        ids.insert(ids.end(), data.begin() + b, data.begin() + e);
        id_off.push_back(ids.size());
    }

    // Append the sequences of records spans[i] = [b, e) to seq / off: raw
    // bytes (record.sequence(): multi-line FASTA keeps its interior '\n'; the
    // record's final line terminator and one trailing CR dropped) or their
    // normalize(false).  Groups of records are normalised on parallel threads
    // straight into seq, each group at the offset its raw byte count bounds;
    // groups that shrank (removed whitespace) are then slid down in order.
    void emit(const std::vector<std::pair<size_t, size_t>> &spans, Bytes &seq,
              std::vector<uint64_t> &off) {
        const size_t n = spans.size();
        if (!n) return;
        size_t total = 0;
        for (auto &sp : spans) total += sp.second - sp.first;
        const size_t ng = total < (4u << 20) ? 1 : std::min<size_t>(4 * (size_t)host_threads(), n);
        std::vector<size_t> gb(ng + 1), ub(ng + 1, seq.size()), got(ng);
        for (size_t g = 0; g <= ng; ++g) gb[g] = n * g / ng;
        for (size_t g = 0; g < ng; ++g) {
            size_t want = 0;
            for (size_t i = gb[g]; i < gb[g + 1]; ++i) want += spans[i].second - spans[i].first;
            ub[g + 1] = ub[g] + want;
        }
        seq.resize(ub[ng]);
        const size_t rec0 = off.size();
        off.resize(rec0 + n);
        const uint8_t *t = norm_table();
        parallel_for(ng, [&](size_t g) {
            uint8_t *d = seq.data() + ub[g];
            size_t o = 0;
            for (size_t i = gb[g]; i < gb[g + 1]; ++i) {
                const uint8_t *src = data.data() + spans[i].first;
                const size_t len = spans[i].second - spans[i].first;
                if (raw) {
                    memcpy(d + o, src, len);
                    o += len;
                } else {
                    for (size_t j = 0; j < len; ++j) {
                        const uint8_t v = t[src[j]];
                        d[o] = v;
                        o += v != 0;
                    }
                }
                off[rec0 + i] = o;  // group-relative end, rebased below
            }
            got[g] = o;
        });
        size_t at = ub[0];
        for (size_t g = 0; g < ng; ++g) {
            if (at != ub[g]) memmove(seq.data() + at, seq.data() + ub[g], got[g]);
            for (size_t i = gb[g]; i < gb[g + 1]; ++i) off[rec0 + i] += at;
            at += got[g];
        }
        seq.resize(at);
    }

    okm_status init() {
        okm_status s = sniff_decompress(data);
        if (s != OKM_OK) return fail(OKM_E_PARSE, std::string("decompression failed: ") + okm_last_error());
        if (data.empty()) return fail(OKM_E_PARSE, "empty input");
        if (data[0] == '>') fastq = false;
        else if (data[0] == '@') fastq = true;
        else return fail(OKM_E_PARSE, "expected '>' or '@' at the start of the input");
        pos = 0;
        index_lines();
        return OKM_OK;
    }

    // Positions of every '\n' (context-free, so found by parallel threads over
    // chunks); the record walk then costs O(1) per line.
    std::vector<uint64_t> nl;
    size_t li = 0;  // index of the first newline at or after pos

    void index_lines() {
        const size_t n = data.size(), chunk = (size_t)16 << 20;
        const size_t nc = (n + chunk - 1) / chunk;
        std::vector<std::vector<uint64_t>> part(nc);
        parallel_for(nc, [&](size_t c) {
            const uint8_t *d = data.data();
            const size_t b = c * chunk, e = std::min(n, b + chunk);
            auto &v = part[c];
            v.reserve((e - b) / 64);
            for (const uint8_t *q = d + b; q < d + e;) {
                const uint8_t *f = (const uint8_t *)memchr(q, '\n', (size_t)(d + e - q));
                if (!f) break;
                v.push_back((uint64_t)(f - d));
                q = f + 1;
            }
        });
        size_t tot = 0;
        for (auto &v : part) tot += v.size();
        nl.clear();
        nl.reserve(tot);
        for (auto &v : part) nl.insert(nl.end(), v.begin(), v.end());
        li = 0;
    }

    // line [pos, eol) ; returns false at end of data
    bool line(size_t &b, size_t &e) {
        if (pos >= data.size()) return false;
        b = pos;
        if (li < nl.size()) {
            e = nl[li++];
            pos = e + 1;
        } else {
            e = pos = data.size();
        }
        return true;
    }

    static size_t rstrip_cr(const Bytes &d, size_t b, size_t e) {
        while (e > b && d[e - 1] == '\r') --e;
        return e;
    }

    // Next record: its sequence bytes are data[*sb, *se) (raw; normalize()
    // applies to them unless `raw`).  *got=false at end.
    okm_status next_span(size_t *osb, size_t *ose, bool *got) {
        *got = false;
        if (!fastq) {
            if (pos >= data.size()) return OKM_OK;
            if (data[pos] != '>') return fail(OKM_E_RECORD, "expected '>' at the start of a FASTA record");
            size_t b, e;
            line(b, e);  // header
            if (want_ids) add_id(b + 1, e);
            const size_t s0 = pos;
            // the sequence runs to the next "\n>" (a line starting with '>')
            size_t end = data.size();
            size_t p = s0;  // every p below is a line start
            while (p < data.size()) {
                if (data[p] == '>') {
                    end = p;
                    break;
                }
                if (li >= nl.size()) break;
                p = nl[li++] + 1;
            }
            size_t se = end;
            if (raw) {
                if (se > s0 && data[se - 1] == '\n') --se;  // the record's last line terminator
                if (se > s0 && data[se - 1] == '\r') --se;
            }
            *osb = s0;
            *ose = se;
            pos = end;
            ++records;
            *got = true;
            return OKM_OK;
        }
        // FASTQ: skip blank lines at the very end
        size_t q = pos;
        while (q < data.size() && (data[q] == '\n' || data[q] == '\r')) ++q;
        if (q >= data.size()) {
            pos = data.size();
            li = nl.size();
            return OKM_OK;
        }
        size_t hb, he, sb, se, pb, pe, qb, qe;
        if (!line(hb, he) || data[hb] != '@') return fail(OKM_E_RECORD, "expected '@' at the start of a FASTQ record");
        if (!line(sb, se) || !line(pb, pe) || !line(qb, qe))
            return fail(OKM_E_RECORD, "truncated FASTQ record");
        if (data[pb] != '+') return fail(OKM_E_RECORD, "expected '+' separator line in FASTQ record");
        se = rstrip_cr(data, sb, se);
        qe = rstrip_cr(data, qb, qe);
        if (se - sb != qe - qb) return fail(OKM_E_RECORD, "sequence and quality lengths differ");
        if (want_ids) add_id(hb + 1, he);
        *osb = sb;
        *ose = se;
        ++records;
        *got = true;
        return OKM_OK;
    }
};

}  // namespace okm

using namespace okm;

struct okm_reader {
    Parser p;
    Bytes seq;
    std::vector<uint64_t> off;
};

extern "C" {

okm_status okm_reader_open(okm_reader **out, const char *path, int decompress_by_ext) {
    return okm_reader_open2(out, path, decompress_by_ext, 0);
}

okm_status okm_reader_open2(okm_reader **out, const char *path, int decompress_by_ext, int flags) {
    if (!out || !path) return fail(OKM_E_ARG, "null argument");
    *out = nullptr;
    okm_reader *r = new okm_reader();
    okm_status s = read_whole_file(path, r->p.data);
    if (s != OKM_OK) {  // utils.rs:126-127: the file cannot be opened
        delete r;
        return fail(OKM_E_IO, std::string(okm_last_error()));
    }
    if (decompress_by_ext && decompress_by_extension(path, r->p.data) != OKM_OK) {
        delete r;  // a corrupt stream surfaces when needletail first reads it
        return fail(OKM_E_PARSE, std::string(okm_last_error()));
    }
    s = r->p.init();
    if (s != OKM_OK) {
        delete r;
        return s;
    }
    r->p.raw = (flags & OKM_READ_RAW) != 0;
    r->p.want_ids = (flags & OKM_READ_IDS) != 0;
    *out = r;
    return OKM_OK;
}

okm_status okm_reader_next(okm_reader *r, uint64_t max_bytes, const uint8_t **seq, const uint64_t **offsets,
                           uint64_t *n_records) {
    if (!r || !seq || !offsets || !n_records) return fail(OKM_E_ARG, "null argument");
    r->seq.clear();
    r->off.assign(1, 0);
    r->p.ids.clear();
    r->p.id_off.assign(1, 0);
    std::vector<std::pair<size_t, size_t>> spans;
    uint64_t bytes = 0;
    auto T0 = std::chrono::steady_clock::now();
    for (;;) {
        bool got = false;
        size_t b = 0, e = 0;
        okm_status s = r->p.next_span(&b, &e, &got);
        if (s != OKM_OK) return s;
        if (!got) break;
        spans.emplace_back(b, e);
        bytes += e - b;
        if (bytes >= max_bytes) break;
    }
    auto T1 = std::chrono::steady_clock::now();
    r->p.emit(spans, r->seq, r->off);
    auto T2 = std::chrono::steady_clock::now();
    if (prof_host())
        fprintf(stderr, "reader: spans %.3f ms emit %.3f ms (%zu records)\n",
                std::chrono::duration<double, std::milli>(T1 - T0).count(),
                std::chrono::duration<double, std::milli>(T2 - T1).count(), spans.size());
    *seq = r->seq.data();
    *offsets = r->off.data();
    *n_records = r->off.size() - 1;
    return OKM_OK;
}

okm_status okm_reader_ids(const okm_reader *r, const uint8_t **ids, const uint64_t **id_offsets) {
    if (!r || !ids || !id_offsets) return fail(OKM_E_ARG, "null argument");
    if (!r->p.want_ids) return fail(OKM_E_STATE, "reader opened without OKM_READ_IDS");
    *ids = r->p.ids.data();
    *id_offsets = r->p.id_off.data();
    return OKM_OK;
}

uint64_t okm_reader_records(const okm_reader *r) { return r ? r->p.records : 0; }

void okm_reader_close(okm_reader *r) { delete r; }

okm_status okm_parse_buffer(const uint8_t *data, uint64_t n, uint8_t **seq, uint64_t **offsets,
                            uint64_t *n_records) {
    if (!seq || !offsets || !n_records || (!data && n)) return fail(OKM_E_ARG, "null argument");
    Parser p;
    p.data.assign(data, data + n);
    okm_status s = p.init();
    if (s != OKM_OK) return s;
    Bytes sq;
    std::vector<uint64_t> off(1, 0);
    std::vector<std::pair<size_t, size_t>> spans;
    for (;;) {
        bool got = false;
        size_t b = 0, e = 0;
        s = p.next_span(&b, &e, &got);
        if (s != OKM_OK) return s;
        if (!got) break;
        spans.emplace_back(b, e);
    }
    p.emit(spans, sq, off);
    *seq = (uint8_t *)malloc(sq.size() ? sq.size() : 1);
    *offsets = (uint64_t *)malloc(off.size() * sizeof(uint64_t));
    if (!*seq || !*offsets) return fail(OKM_E_NOMEM, "host allocation");
    memcpy(*seq, sq.data(), sq.size());
    memcpy(*offsets, off.data(), off.size() * sizeof(uint64_t));
    *n_records = off.size() - 1;
    return OKM_OK;
}

}  // extern "C"
