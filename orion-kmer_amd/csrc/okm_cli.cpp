// okm_cli.cpp — `orion-kmer` command line, a drop-in for the reference's
// count / build / compare subcommands (cli.rs:4-189, main.rs:7-16,
// commands/mod.rs:10-33), driving the MI355X engine through the C ABI only.
//
// Same flags (clap-derived names, cli.rs:38-95), same outputs (count.rs:127-135
// TSV, build.rs:141-146 KmerDbV2, compare.rs:15-25,85-89 pretty JSON) and the
// same outermost error contexts, printed as env_logger would print
// `error!("Error: {}", e)` (main.rs:10-13), exit status 1; usage errors exit 2.
// Opt-in extension: --device <N> selects the GPU.
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <string>
#include <vector>

#include "orion_kmer.h"

static int g_verbose = 0;
static int g_device = 0;

static std::string timestamp() {
    char buf[64];
    time_t t = time(nullptr);
    struct tm tm;
    gmtime_r(&t, &tm);
    strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%SZ", &tm);
    return buf;
}

static void log_line(const char *level, const char *module, const std::string &msg) {
    fprintf(stderr, "[%s %-5s %s] %s\n", timestamp().c_str(), level, module, msg.c_str());
}

static void info(const char *module, const std::string &msg) {
    if (g_verbose >= 1) log_line("INFO", module, msg);
}

// main.rs:10-13: error!("Error: {}", e); exit(1)
static int die(const std::string &msg) {
    log_line("ERROR", "orion_kmer", "Error: " + msg);
    return 1;
}

static int usage_error(const std::string &msg) {
    fprintf(stderr, "error: %s\n\nFor more information, try '--help'.\n", msg.c_str());
    return 2;
}

// Rust `{:?}` of a PathBuf: quoted, with \" and \\ escaped.
static std::string dbg_path(const std::string &p) {
    std::string o = "\"";
    for (char ch : p) {
        if (ch == '"' || ch == '\\') o += '\\';
        o += ch;
    }
    return o + "\"";
}

static std::string basename_of(const std::string &p) {
    size_t s = p.find_last_of('/');
    std::string b = s == std::string::npos ? p : p.substr(s + 1);
    return b.empty() ? p : b;
}

// ---------------------------------------------------------------------------
// argument parsing (clap-like)
// ---------------------------------------------------------------------------
struct Args {
    std::string cmd;
    std::vector<std::string> pos;
    std::vector<std::pair<std::string, std::string>> opts;  // canonical long name -> value
    bool help = false, version = false;
};

struct OptSpec {
    const char *lng;
    char shrt;
    bool takes_value;
    bool multi;  // num_args = 1..
};

static const OptSpec *find_opt(const std::vector<OptSpec> &spec, const std::string &tok) {
    for (auto &o : spec) {
        if (tok == std::string("--") + o.lng) return &o;
        if (o.shrt && tok.size() == 2 && tok[0] == '-' && tok[1] == o.shrt) return &o;
    }
    return nullptr;
}

static int parse(int argc, char **argv, const std::vector<OptSpec> &spec, int start, Args &a) {
    for (int i = start; i < argc; ++i) {
        std::string tok = argv[i];
        if (tok == "-h" || tok == "--help") {
            a.help = true;
            continue;
        }
        if (tok == "-V" || tok == "--version") {
            a.version = true;
            continue;
        }
        std::string val;
        bool has_eq = false;
        if (tok.rfind("--", 0) == 0) {
            size_t eq = tok.find('=');
            if (eq != std::string::npos) {
                val = tok.substr(eq + 1);
                tok = tok.substr(0, eq);
                has_eq = true;
            }
        }
        // -vvv
        if (tok.size() > 2 && tok[0] == '-' && tok[1] != '-' && tok.find_first_not_of('v', 1) == std::string::npos) {
            g_verbose += (int)tok.size() - 1;
            continue;
        }
        const OptSpec *o = find_opt(spec, tok);
        if (!o && tok.size() > 2 && tok[0] == '-' && tok[1] != '-') {
            // -k5 style
            std::string t2 = tok.substr(0, 2);
            o = find_opt(spec, t2);
            if (o && o->takes_value) {
                val = tok.substr(2);
                has_eq = true;
                tok = t2;
            } else {
                o = nullptr;
            }
        }
        if (!o) {
            if (!tok.empty() && tok[0] == '-' && tok != "-") return usage_error("unexpected argument '" + tok + "' found");
            a.pos.push_back(tok);
            continue;
        }
        if (!o->takes_value) {
            if (std::string(o->lng) == "verbose")
                g_verbose++;
            else
                a.opts.emplace_back(o->lng, "1");
            continue;
        }
        if (!has_eq) {
            if (i + 1 >= argc) return usage_error(std::string("a value is required for '--") + o->lng + "' but none was supplied");
            val = argv[++i];
        }
        a.opts.emplace_back(o->lng, val);
        if (o->multi) {
            while (i + 1 < argc && argv[i + 1][0] != '-') a.opts.emplace_back(o->lng, argv[++i]);
        }
    }
    return 0;
}

static std::vector<std::string> get_all(const Args &a, const char *name) {
    std::vector<std::string> v;
    for (auto &kv : a.opts)
        if (kv.first == name) v.push_back(kv.second);
    return v;
}

static bool get_one(const Args &a, const char *name, std::string &out) {
    auto v = get_all(a, name);
    if (v.empty()) return false;
    out = v.back();
    return true;
}

static bool parse_u64(const std::string &s, uint64_t &v) {
    if (s.empty()) return false;
    char *end = nullptr;
    errno = 0;
    unsigned long long x = strtoull(s.c_str(), &end, 10);
    if (*end || errno || s[0] == '-') return false;
    v = x;
    return true;
}

static bool parse_k(const Args &a, uint8_t &k, int &rc) {
    std::string s;
    if (!get_one(a, "kmer-size", s)) {
        rc = usage_error("the following required arguments were not provided:\n  --kmer-size <KMER_SIZE>");
        return false;
    }
    uint64_t v;
    if (!parse_u64(s, v) || v > 255) {
        rc = usage_error("invalid value '" + s + "' for '--kmer-size <KMER_SIZE>': invalid digit found in string");
        return false;
    }
    k = (uint8_t)v;
    return true;
}

static const char *kVersion = "orion-kmer 0.1.0";

static void print_help(const std::string &cmd) {
    if (cmd == "count")
        printf("Count k-mers in FASTA/FASTQ files\n\nUsage: orion-kmer count [OPTIONS] --kmer-size <KMER_SIZE> --input-files <INPUT_FILES>... --output-file <OUTPUT_FILE>\n\nOptions:\n  -k, --kmer-size <KMER_SIZE>      The length of the k-mer\n  -i, --input-files <INPUT_FILES>...  One or more input FASTA/FASTQ files. Supports .gz, .xz, .zst compression.\n  -o, --output-file <OUTPUT_FILE>  Output file for k-mer counts (kmer<TAB>count)\n  -m, --min-count <MIN_COUNT>      Minimum count to report a k-mer [default: 1]\n      --wide                       Allow k up to 64 (two-u64 keys; extension, not in the reference)\n  -t, --threads <THREADS>          Number of threads to use (0 for all logical cores) [default: 0]\n  -v, --verbose...                 Verbosity level (e.g., -v, -vv)\n      --device <DEVICE>            GPU ordinal (MI355X engine) [default: 0]\n  -h, --help                       Print help\n  -V, --version                    Print version\n");
    else if (cmd == "build")
        printf("Build a unique k-mer database from genome assemblies\n\nUsage: orion-kmer build [OPTIONS] --kmer-size <KMER_SIZE> --genomes <GENOME_FILES>... --output-file <OUTPUT_FILE>\n");
    else if (cmd == "compare")
        printf("Compare two k-mer databases\n\nUsage: orion-kmer compare [OPTIONS] --db1 <DB1> --db2 <DB2> --output-file <OUTPUT_FILE>\n");
    else
        printf("Usage: orion-kmer [OPTIONS] <COMMAND>\n\nCommands:\n  count     Count k-mers in FASTA/FASTQ files\n  build     Build a unique k-mer database from genome assemblies\n  compare   Compare two k-mer databases\n  query     Query short reads against a k-mer database\n  classify  Classify sequences against k-mer databases and report coverage statistics\n  help      Print this message or the help of the given subcommand(s)\n\nOptions:\n  -t, --threads <THREADS>  Number of threads to use (0 for all logical cores) [default: 0]\n  -v, --verbose...         Verbosity level (e.g., -v, -vv)\n      --device <DEVICE>    GPU ordinal (MI355X engine) [default: 0]\n  -h, --help               Print help\n  -V, --version            Print version\n");
}

static std::string err_detail() { return std::string(okm_last_error()); }

// Feed every record of `path` into ctx (count.rs:59-79 / build.rs:38-70).
static int feed_file(okm_ctx *ctx, const std::string &path, bool decompress_by_ext, const char *open_ctx) {
    okm_reader *r = nullptr;
    okm_status s = okm_reader_open(&r, path.c_str(), decompress_by_ext ? 1 : 0);
    if (s == OKM_E_IO) return die(std::string(open_ctx) + path);
    if (s != OKM_OK) return die("Failed to parse FASTA/Q content from: " + path);
    info("orion_kmer::commands", "Processing records from " + path + "...");
    for (;;) {
        const uint8_t *seq;
        const uint64_t *off;
        uint64_t n;
        s = okm_reader_next(r, 256ull << 20, &seq, &off, &n);
        if (s != OKM_OK) {
            okm_reader_close(r);
            return die("Error reading record from " + path);
        }
        if (n == 0) break;
        s = okm_add_batch(ctx, seq, off, n, 1);
        if (s != OKM_OK) {
            okm_reader_close(r);
            return die("GPU engine failure on " + path + ": " + err_detail());
        }
    }
    info("orion_kmer::commands", "Finished processing " + std::to_string(okm_reader_records(r)) + " records from " + path);
    okm_reader_close(r);
    return 0;
}

static int open_engine(okm_ctx **ctx, uint8_t k, okm_mode mode) {
    okm_status s = okm_create(ctx, k, mode, g_device, 0);
    if (s == OKM_E_INVALID_K) return die(err_detail());  // errors.rs:6 text (or its k<=64 form with --wide)
    if (s != OKM_OK) return die("MI355X engine unavailable: " + err_detail());
    return 0;
}

// count.rs:40-141
static int run_count(const Args &a) {
    uint8_t k;
    int rc = 0;
    if (!parse_k(a, k, rc)) return rc;
    auto inputs = get_all(a, "input-files");
    std::string out, ms;
    if (inputs.empty()) return usage_error("the following required arguments were not provided:\n  --input-files <INPUT_FILES>...");
    if (!get_one(a, "output-file", out)) return usage_error("the following required arguments were not provided:\n  --output-file <OUTPUT_FILE>");
    uint64_t min_count = 1;
    if (get_one(a, "min-count", ms) && !parse_u64(ms, min_count))
        return usage_error("invalid value '" + ms + "' for '--min-count <MIN_COUNT>'");
    // --wide: opt-in two-u64 keys for k in 33..64 (not in the reference, whose
    // error for k > 32 is kept byte-identical without it)
    std::string wflag;
    const bool wide = get_one(a, "wide", wflag);
    if (k == 0 || k > (wide ? 64 : 32))
        return die("Invalid K-mer size: " + std::to_string(k) + ". Must be between 1 and " + (wide ? "64." : "32."));
    okm_ctx *ctx = nullptr;
    if ((rc = open_engine(&ctx, k, (okm_mode)(OKM_MODE_COUNT | (wide ? OKM_MODE_WIDE : 0))))) return rc;
    for (auto &p : inputs) {
        info("orion_kmer::commands::count", "Processing file: " + p);
        if ((rc = feed_file(ctx, p, true, "Failed to get input reader for file: "))) {
            okm_destroy(ctx);
            return rc;
        }
    }
    uint64_t *keys = nullptr, *counts = nullptr, n = 0, nd = 0;
    if (okm_count(ctx, &nd) != OKM_OK || okm_finish_counts(ctx, min_count, &keys, &counts, &n) != OKM_OK) {
        std::string d = err_detail();
        okm_destroy(ctx);
        return die("GPU engine failure while counting: " + d);
    }
    info("orion_kmer::commands::count", "Finished processing all input files. Found " + std::to_string(nd) + " unique canonical k-mers.");
    okm_destroy(ctx);
    okm_status s = okm_write_counts_tsv(out.c_str(), k, keys, counts, n);
    okm_free_result(keys);
    okm_free_result(counts);
    if (s != OKM_OK) return die("Failed to get output writer for counts file: " + dbg_path(out));
    info("orion_kmer::commands::count", "Successfully wrote k-mer counts to " + dbg_path(out));
    return 0;
}

// build.rs:80-160
static int run_build(const Args &a) {
    uint8_t k;
    int rc = 0;
    if (!parse_k(a, k, rc)) return rc;
    auto genomes = get_all(a, "genomes");
    std::string out;
    if (genomes.empty()) return usage_error("the following required arguments were not provided:\n  --genomes <GENOME_FILES>...");
    if (!get_one(a, "output-file", out)) return usage_error("the following required arguments were not provided:\n  --output-file <OUTPUT_FILE>");
    if (k == 0 || k > 32) return die("Invalid K-mer size: " + std::to_string(k) + ". Must be between 1 and 32.");
    okm_ctx *ctx = nullptr;
    if ((rc = open_engine(&ctx, k, OKM_MODE_SET))) return rc;
    okm_db *db = nullptr;
    okm_db_new(&db, k);
    for (auto &p : genomes) {
        okm_reset(ctx);  // a fresh DashSet per file (build.rs:95)
        if ((rc = feed_file(ctx, p, false, "Failed to get buffered file reader for file: "))) {
            okm_destroy(ctx);
            okm_db_free(db);
            return rc;
        }
        uint64_t *keys = nullptr, n = 0;
        if (okm_finish_set(ctx, &keys, &n) != OKM_OK) {
            std::string d = err_detail();
            okm_destroy(ctx);
            okm_db_free(db);
            return die("GPU engine failure while building: " + d);
        }
        const std::string name = basename_of(p);  // build.rs:106-109
        info("orion_kmer::commands::build", "Adding " + std::to_string(n) + " unique k-mers from reference '" + name + "' to the database.");
        okm_db_add_reference(db, name.c_str(), keys, n);
        okm_free_result(keys);
    }
    okm_destroy(ctx);
    okm_status s = okm_db_write(db, out.c_str());
    okm_db_free(db);
    if (s == OKM_E_IO && std::string(okm_last_error()).rfind("cannot create", 0) == 0)
        return die("Failed to get output writer for database file: " + dbg_path(out));
    if (s != OKM_OK) return die("Failed to serialize k-mer database (KmerDbV2) to " + dbg_path(out));
    return 0;
}

// serde_json's f64 output (ryu shortest round-trip, its decimal/exponent layout)
static std::string fmt_f64(double x) {
    if (x == 0) return std::signbit(x) ? "-0.0" : "0.0";
    char buf[64];
    int p = 1;
    for (; p <= 17; ++p) {
        snprintf(buf, sizeof(buf), "%.*e", p - 1, x);
        if (strtod(buf, nullptr) == x) break;
    }
    std::string s = buf;
    bool neg = s[0] == '-';
    if (neg) s = s.substr(1);
    size_t e = s.find('e');
    int exp10 = atoi(s.c_str() + e + 1);
    std::string digits;
    for (size_t i = 0; i < e; ++i)
        if (s[i] != '.') digits += s[i];
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    const int len = (int)digits.size();
    const int kk = exp10 + 1;            // 10^(kk-1) <= |x| < 10^kk
    const int kexp = kk - len;           // x = digits * 10^kexp
    std::string o;
    if (kexp >= 0 && kk <= 16) {
        o = digits + std::string(kexp, '0') + ".0";
    } else if (kk > 0 && kk <= 16) {
        o = digits.substr(0, kk) + "." + digits.substr(kk);
    } else if (kk > -5 && kk <= 0) {
        o = "0." + std::string(-kk, '0') + digits;
    } else if (len == 1) {
        o = digits + "e" + std::to_string(kk - 1);
    } else {
        o = digits.substr(0, 1) + "." + digits.substr(1) + "e" + std::to_string(kk - 1);
    }
    return neg ? "-" + o : o;
}

static std::string json_str(const std::string &s) {
    std::string o = "\"";
    for (unsigned char ch : s) {
        switch (ch) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        case 0x08: o += "\\b"; break;
        case 0x0C: o += "\\f"; break;
        default:
            if (ch < 0x20) {
                char b[8];
                snprintf(b, sizeof(b), "\\u%04x", ch);
                o += b;
            } else {
                o += (char)ch;
            }
        }
    }
    return o + "\"";
}

// db_types.rs:43-48 get_all_kmers_unified, on the GPU: every reference's keys
// into one SET context, sorted unique out.
static int unify(const okm_db *db, std::vector<uint64_t> &out) {
    out.clear();
    const uint8_t k = okm_db_k(db);
    uint64_t total = 0;
    for (uint64_t i = 0; i < okm_db_num_references(db); ++i) {
        uint64_t n;
        okm_db_reference(db, i, nullptr, nullptr, &n);
        total += n;
    }
    if (total == 0) return 0;
    okm_ctx *ctx = nullptr;
    int rc;
    if ((rc = open_engine(&ctx, k, OKM_MODE_SET))) return rc;
    for (uint64_t i = 0; i < okm_db_num_references(db); ++i) {
        const uint64_t *keys;
        uint64_t n;
        okm_db_reference(db, i, nullptr, &keys, &n);
        if (n && okm_add_pairs(ctx, keys, nullptr, n) != OKM_OK) {
            std::string d = err_detail();
            okm_destroy(ctx);
            return die("GPU engine failure while comparing: " + d);
        }
    }
    uint64_t *keys = nullptr, n = 0;
    if (okm_finish_set(ctx, &keys, &n) != OKM_OK) {
        std::string d = err_detail();
        okm_destroy(ctx);
        return die("GPU engine failure while comparing: " + d);
    }
    out.assign(keys, keys + n);
    okm_free_result(keys);
    okm_destroy(ctx);
    return 0;
}

// compare.rs:29-97
static int run_compare(const Args &a) {
    std::string p1, p2, out;
    if (!get_one(a, "db1", p1)) return usage_error("the following required arguments were not provided:\n  --db1 <DB1>");
    if (!get_one(a, "db2", p2)) return usage_error("the following required arguments were not provided:\n  --db2 <DB2>");
    if (!get_one(a, "output-file", out)) return usage_error("the following required arguments were not provided:\n  --output-file <OUTPUT_FILE>");
    okm_db *d1 = nullptr, *d2 = nullptr;
    okm_status s = okm_db_read(&d1, p1.c_str());
    if (s == OKM_E_IO) return die("Failed to get input reader for k-mer database: " + dbg_path(p1));
    if (s != OKM_OK) return die("Failed to deserialize KmerDbV2 from " + dbg_path(p1));
    s = okm_db_read(&d2, p2.c_str());
    if (s == OKM_E_IO) {
        okm_db_free(d1);
        return die("Failed to get input reader for k-mer database: " + dbg_path(p2));
    }
    if (s != OKM_OK) {
        okm_db_free(d1);
        return die("Failed to deserialize KmerDbV2 from " + dbg_path(p2));
    }
    const uint8_t k1 = okm_db_k(d1), k2 = okm_db_k(d2);
    if (k1 != k2) {
        okm_db_free(d1);
        okm_db_free(d2);
        return die("K-mer databases have incompatible k-mer sizes (overall comparison): " + std::to_string(k1) + " vs " + std::to_string(k2));
    }
    std::vector<uint64_t> A, B;
    int rc;
    if ((rc = unify(d1, A)) || (rc = unify(d2, B))) {
        okm_db_free(d1);
        okm_db_free(d2);
        return rc;
    }
    okm_db_free(d1);
    okm_db_free(d2);
    uint64_t inter = 0;
    if (!A.empty() && !B.empty() &&
        okm_set_intersection_size(A.data(), A.size(), B.data(), B.size(), g_device, &inter) != OKM_OK)
        return die("GPU engine failure while comparing: " + err_detail());
    const uint64_t uni = A.size() + B.size() - inter;  // compare.rs:60
    const double j = uni == 0 ? 0.0 : (double)inter / (double)uni;  // compare.rs:62-66
    std::string js = "{\n";
    js += "  \"db1_path\": " + json_str(p1) + ",\n";
    js += "  \"db2_path\": " + json_str(p2) + ",\n";
    js += "  \"kmer_size\": " + std::to_string(k1) + ",\n";
    js += "  \"db1_total_unique_kmers_across_references\": " + std::to_string(A.size()) + ",\n";
    js += "  \"db2_total_unique_kmers_across_references\": " + std::to_string(B.size()) + ",\n";
    js += "  \"intersection_size\": " + std::to_string(inter) + ",\n";
    js += "  \"union_size\": " + std::to_string(uni) + ",\n";
    js += "  \"jaccard_index\": " + fmt_f64(j) + "\n}";
    FILE *f = fopen(out.c_str(), "wb");  // compare.rs:85: File::create, never compressed
    if (!f) return die("Failed to create output JSON file: " + dbg_path(out));
    const bool ok = fwrite(js.data(), 1, js.size(), f) == js.size();
    if (fclose(f) != 0 || !ok) return die("Failed to write comparison JSON to " + dbg_path(out));
    return 0;
}

int main(int argc, char **argv) {
    static const std::vector<OptSpec> global = {
        {"threads", 't', true, false}, {"verbose", 'v', false, false}, {"device", 0, true, false}};
    // locate the subcommand (first non-option token, skipping global option values)
    int ci = 1;
    for (; ci < argc; ++ci) {
        std::string t = argv[ci];
        if (t == "-t" || t == "--threads" || t == "--device") {
            ++ci;
            continue;
        }
        if (t.empty() || t[0] != '-') break;
        if (t == "-h" || t == "--help") {
            print_help("");
            return 0;
        }
        if (t == "-V" || t == "--version") {
            printf("%s\n", kVersion);
            return 0;
        }
    }
    if (ci >= argc) {
        print_help("");
        return 2;
    }
    const std::string cmd = argv[ci];
    std::vector<OptSpec> spec = global;
    if (cmd == "count") {
        spec.push_back({"kmer-size", 'k', true, false});
        spec.push_back({"input-files", 'i', true, true});
        spec.push_back({"output-file", 'o', true, false});
        spec.push_back({"min-count", 'm', true, false});
        spec.push_back({"wide", 0, false, false});
    } else if (cmd == "build") {
        spec.push_back({"kmer-size", 'k', true, false});
        spec.push_back({"genomes", 'g', true, true});
        spec.push_back({"output-file", 'o', true, false});
    } else if (cmd == "compare") {
        spec.push_back({"db1", 0, true, false});
        spec.push_back({"db2", 0, true, false});
        spec.push_back({"output-file", 'o', true, false});
    } else if (cmd == "help") {
        print_help(ci + 1 < argc ? argv[ci + 1] : "");
        return 0;
    } else if (cmd == "query" || cmd == "classify") {
        return die("the '" + cmd + "' subcommand is outside this engine's scope (see DESIGN.md)");
    } else {
        return usage_error("unrecognized subcommand '" + cmd + "'");
    }
    Args a;
    a.cmd = cmd;
    // global options before the subcommand
    Args pre;
    int rc = parse(ci, argv, global, 1, pre);
    if (rc) return rc;
    rc = parse(argc, argv, spec, ci + 1, a);
    if (rc) return rc;
    if (a.help) {
        print_help(cmd);
        return 0;
    }
    if (a.version) {
        printf("%s\n", kVersion);
        return 0;
    }
    if (!a.pos.empty()) return usage_error("unexpected argument '" + a.pos[0] + "' found");
    std::string dev;
    if (get_one(pre, "device", dev) || get_one(a, "device", dev)) g_device = atoi(dev.c_str());
    if (cmd == "count") return run_count(a);
    if (cmd == "build") return run_build(a);
    return run_compare(a);
}
