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
#include <string.h>

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

// Append normalize(src[0..n)) to out.
static void normalize_append(const uint8_t *src, size_t n, std::vector<uint8_t> &out) {
    const uint8_t *t = norm_table();
    const size_t base = out.size();
    out.resize(base + n);
    uint8_t *d = out.data() + base;
    size_t o = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t v = t[src[i]];
        d[o] = v;
        o += v != 0;
    }
    out.resize(base + o);
}

struct Parser {
    std::vector<uint8_t> data;
    size_t pos = 0;
    bool fastq = false;
    bool raw = false;   // query.rs:66: record.sequence() as is (no normalize)
    bool want_ids = false;
    uint64_t records = 0;
    std::vector<uint8_t> ids;     // ids of the records read by the current batch
    std::vector<uint64_t> id_off;

    void add_id(size_t b, size_t e) {  // needletail id(): header after the marker, CR trimmed
        e = rstrip_cr(data, b, e);
        ids.insert(ids.end(), data.begin() + b, data.begin() + e);
        id_off.push_back(ids.size());
    }

    // raw_seq: the sequence bytes with their line breaks (multi-line FASTA
    // keeps its interior '\n'; the record's final line terminator and one
    // trailing CR dropped).
    void append_seq(size_t b, size_t e, std::vector<uint8_t> &seq) {
        if (!raw) {
            normalize_append(data.data() + b, e - b, seq);
            return;
        }
        seq.insert(seq.end(), data.begin() + b, data.begin() + e);
    }

    okm_status init() {
        okm_status s = sniff_decompress(data);
        if (s != OKM_OK) return fail(OKM_E_PARSE, std::string("decompression failed: ") + okm_last_error());
        if (data.empty()) return fail(OKM_E_PARSE, "empty input");
        if (data[0] == '>') fastq = false;
        else if (data[0] == '@') fastq = true;
        else return fail(OKM_E_PARSE, "expected '>' or '@' at the start of the input");
        pos = 0;
        return OKM_OK;
    }

    // line [pos, eol) ; returns false at end of data
    bool line(size_t &b, size_t &e) {
        if (pos >= data.size()) return false;
        b = pos;
        const uint8_t *nl = (const uint8_t *)memchr(data.data() + pos, '\n', data.size() - pos);
        e = nl ? (size_t)(nl - data.data()) : data.size();
        pos = nl ? e + 1 : data.size();
        return true;
    }

    static size_t rstrip_cr(const std::vector<uint8_t> &d, size_t b, size_t e) {
        while (e > b && d[e - 1] == '\r') --e;
        return e;
    }

    // Next record: appends its normalised sequence to seq. *got=false at end.
    okm_status next(std::vector<uint8_t> &seq, bool *got) {
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
            size_t p = s0;
            while (p < data.size()) {
                if (data[p] == '>' && (p == s0 || data[p - 1] == '\n')) {
                    end = p;
                    break;
                }
                const uint8_t *nl = (const uint8_t *)memchr(data.data() + p, '\n', data.size() - p);
                if (!nl) break;
                p = (size_t)(nl - data.data()) + 1;
            }
            if (raw) {
                size_t se = end;
                if (se > s0 && data[se - 1] == '\n') --se;  // the record's last line terminator
                if (se > s0 && data[se - 1] == '\r') --se;
                append_seq(s0, se, seq);
            } else {
                append_seq(s0, end, seq);
            }
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
        append_seq(sb, se, seq);
        ++records;
        *got = true;
        return OKM_OK;
    }
};

}  // namespace okm

using namespace okm;

struct okm_reader {
    Parser p;
    std::vector<uint8_t> seq;
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
    for (;;) {
        bool got = false;
        okm_status s = r->p.next(r->seq, &got);
        if (s != OKM_OK) return s;
        if (!got) break;
        r->off.push_back(r->seq.size());
        if (r->seq.size() >= max_bytes) break;
    }
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
    std::vector<uint8_t> sq;
    std::vector<uint64_t> off(1, 0);
    for (;;) {
        bool got = false;
        s = p.next(sq, &got);
        if (s != OKM_OK) return s;
        if (!got) break;
        off.push_back(sq.size());
    }
    *seq = (uint8_t *)malloc(sq.size() ? sq.size() : 1);
    *offsets = (uint64_t *)malloc(off.size() * sizeof(uint64_t));
    if (!*seq || !*offsets) return fail(OKM_E_NOMEM, "host allocation");
    memcpy(*seq, sq.data(), sq.size());
    memcpy(*offsets, off.data(), off.size() * sizeof(uint64_t));
    *n_records = off.size() - 1;
    return OKM_OK;
}

}  // extern "C"
