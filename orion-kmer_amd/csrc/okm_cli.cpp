// okm_cli.cpp — `orion-kmer` command line, a drop-in for the reference's
// count / build / compare / query / classify subcommands (cli.rs:4-189, main.rs:7-16,
// commands/mod.rs:10-33), driving the MI355X engine through the C ABI only.
//
// Same flags (clap-derived names, cli.rs:38-95), same outputs (count.rs:127-135
// TSV, build.rs:141-146 KmerDbV2, compare.rs:15-25,85-89 pretty JSON) and the
// same outermost error contexts, printed as env_logger would print
// `error!("Error: {}", e)` (main.rs:10-13), exit status 1; usage errors exit 2.
// Opt-in extensions: --device <N> selects the GPU; count --gpus <N> counts on
// N GPUs of this node (okm_group: one table over RCCL key-range owners).
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>
#include <algorithm>

#include "orion_kmer.h"

static int g_verbose = 0;

// OKM_PROFILE_HOST=1: wall time of each phase of a run on stderr (tools/e2e_cli.sh)
static void phase(const char *what) {
    static const bool on = [] {
        const char *e = getenv("OKM_PROFILE_HOST");
        return e && *e && *e != '0';
    }();
    if (!on) return;
    static struct timespec t0 = [] {
        struct timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        return t;
    }();
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    fprintf(stderr, "[okm cli] %-14s %8.1f ms\n", what, (t.tv_sec - t0.tv_sec) * 1e3 + (t.tv_nsec - t0.tv_nsec) / 1e6);
}
static int g_device = 0;
static int g_gpus = 1;

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
        printf("Count k-mers in FASTA/FASTQ files\n\nUsage: orion-kmer count [OPTIONS] --kmer-size <KMER_SIZE> --input-files <INPUT_FILES>... --output-file <OUTPUT_FILE>\n\nOptions:\n  -k, --kmer-size <KMER_SIZE>      The length of the k-mer\n  -i, --input-files <INPUT_FILES>...  One or more input FASTA/FASTQ files. Supports .gz, .xz, .zst compression.\n  -o, --output-file <OUTPUT_FILE>  Output file for k-mer counts (kmer<TAB>count)\n  -m, --min-count <MIN_COUNT>      Minimum count to report a k-mer [default: 1]\n      --wide                       Allow k up to 64 (two-u64 keys; extension, not in the reference)\n  -t, --threads <THREADS>          Number of threads to use (0 for all logical cores) [default: 0]\n  -v, --verbose...                 Verbosity level (e.g., -v, -vv)\n      --device <DEVICE>            GPU ordinal (MI355X engine) [default: 0]\n      --gpus <GPUS>                Count on this many GPUs of the node, one table over RCCL (0: all) [default: 1]\n  -h, --help                       Print help\n  -V, --version                    Print version\n");
    else if (cmd == "build")
        printf("Build a unique k-mer database from genome assemblies\n\nUsage: orion-kmer build [OPTIONS] --kmer-size <KMER_SIZE> --genomes <GENOME_FILES>... --output-file <OUTPUT_FILE>\n");
    else if (cmd == "compare")
        printf("Compare two k-mer databases\n\nUsage: orion-kmer compare [OPTIONS] --db1 <DB1> --db2 <DB2> --output-file <OUTPUT_FILE>\n");
    else if (cmd == "query")
        printf("Query short reads against a k-mer database\n\nUsage: orion-kmer query [OPTIONS] --database <DATABASE_FILE> --reads <READS_FILE> --output-file <OUTPUT_FILE>\n\nOptions:\n  -d, --database <DATABASE_FILE>  K-mer database to query against. Supports .gz, .xz, .zst compression.\n  -r, --reads <READS_FILE>        Short-read file (FASTQ). Supports .gz, .xz, .zst compression.\n  -o, --output-file <OUTPUT_FILE>  Output file for the IDs of matching reads. Supports .gz, .xz, .zst compression based on extension.\n  -c, --min-hits <MIN_HITS>       Minimum number of k-mer hits to report a read [default: 1]\n  -h, --help                      Print help\n");
    else if (cmd == "classify")
        printf("Classify sequences against k-mer databases and report coverage statistics\n\nUsage: orion-kmer classify [OPTIONS] --input-file <INPUT_FILE> --databases <DATABASE_FILES>... --output-file <OUTPUT_FILE>\n\nOptions:\n  -i, --input-file <INPUT_FILE>  Input genome (FASTA) or reads (FASTQ) file.\n  -d, --databases <DATABASE_FILES>...  One or more k-mer database files (.db).\n  -o, --output-file <OUTPUT_FILE>  Output file for classification results (JSON format).\n  -k, --kmer-size <KMER_SIZE>    Optional: K-mer size to validate against databases.\n      --min-kmer-frequency <MIN_KMER_FREQUENCY>  [default: 1]\n      --min-coverage <MIN_COVERAGE>  [default: 0]\n      --output-tsv <OUTPUT_TSV>  Optional: Output file path for a TSV summary.\n  -h, --help                     Print help\n");
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

// The count engine, brought up on a thread of its own (HIP runtime start-up
// and device contexts take ~150-200 ms) while the reader parses the first
// batch; get() waits for it.
struct AsyncGroup {
    okm_group *g = nullptr;
    okm_status st = OKM_OK;
    std::string err;
    std::thread th;
    bool joined = false;
    void start(uint8_t k, okm_mode mode) {
        th = std::thread([this, k, mode] {
            // --device is the first ordinal: --gpus N counts on devices D .. D+N-1
            std::vector<int> devs;
            for (int i = 0; i < std::max(g_gpus, 1); ++i) devs.push_back(g_device + i);
            st = okm_group_create(&g, k, mode, g_gpus, g_gpus >= 1 ? devs.data() : nullptr, 0);
            if (st != OKM_OK) err = okm_last_error();
        });
    }
    okm_group *get() {
        if (!joined) {
            th.join();
            joined = true;
        }
        return st == OKM_OK ? g : nullptr;
    }
    ~AsyncGroup() {
        get();
        okm_group_destroy(g);
    }
};

// The output is complete and closed: leave without tearing down the GPU
// contexts and the HIP runtime one by one (~150 ms for a C2-sized table; the
// driver reclaims the device memory at exit).  Not under a profiler, whose
// atexit handlers must run (rocprofv3 preloads its tool library), or with
// OKM_CLI_NO_FAST_EXIT set.
static void fast_exit() {
    const char *pre = getenv("LD_PRELOAD");
    if (getenv("OKM_CLI_NO_FAST_EXIT") || (pre && strstr(pre, "rocprof"))) return;
    fflush(stdout);
    fflush(stderr);
    _exit(0);
}

static int engine_error(const AsyncGroup &ag) {
    if (ag.st == OKM_E_INVALID_K) return die(ag.err);  // errors.rs:6 text (or its k<=64 form with --wide)
    return die("MI355X engine unavailable: " + ag.err);
}

// Feed every record of `path` into a GPU group (count.rs:59-79): the group
// copies each batch and counts it on a worker thread, so the reader parses the
// next batch meanwhile.
static int feed_file_group(AsyncGroup &ag, const std::string &path, const char *open_ctx) {
    okm_reader *r = nullptr;
    okm_status s = okm_reader_open(&r, path.c_str(), 1);
    if (s == OKM_E_IO) return die(std::string(open_ctx) + path);
    if (s != OKM_OK) return die("Failed to parse FASTA/Q content from: " + path);
    info("orion_kmer::commands", "Processing records from " + path + "...");
    for (;;) {
        const uint8_t *seq;
        const uint64_t *off;
        uint64_t n;
        s = okm_reader_next(r, 128ull << 20, &seq, &off, &n);
        if (s != OKM_OK) {
            okm_reader_close(r);
            return die("Error reading record from " + path);
        }
        if (n == 0) break;
        okm_group *g = ag.get();
        if (!g) {
            okm_reader_close(r);
            return engine_error(ag);
        }
        s = okm_group_add_batch(g, seq, off, n, 1);
        if (s != OKM_OK) {
            okm_reader_close(r);
            return die("GPU engine failure on " + path + ": " + err_detail());
        }
    }
    info("orion_kmer::commands", "Finished processing " + std::to_string(okm_reader_records(r)) + " records from " + path);
    okm_reader_close(r);
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
    // one table across all inputs (count.rs:48), on g_gpus GPUs (default 1),
    // started while the first input is parsed
    phase("start");
    AsyncGroup ag;
    ag.start(k, (okm_mode)(OKM_MODE_COUNT | (wide ? OKM_MODE_WIDE : 0)));
    for (auto &p : inputs) {
        info("orion_kmer::commands::count", "Processing file: " + p);
        if ((rc = feed_file_group(ag, p, "Failed to get input reader for file: "))) return rc;
    }
    phase("input parsed");
    okm_group *grp = ag.get();
    if (!grp) return engine_error(ag);
    uint64_t nd = 0;
    if (okm_group_count(grp, &nd) != OKM_OK) return die("GPU engine failure while counting: " + err_detail());
    info("orion_kmer::commands::count", "Finished processing all input files. Found " + std::to_string(nd) + " unique canonical k-mers.");
    // count.rs:106-137: filter, sort (the table already is) and write, streamed
    // off the GPU while the previous chunk is formatted
    phase("counted");
    okm_status s = okm_group_write_counts_tsv(grp, out.c_str(), min_count, nullptr);
    phase("written");
    if (s != OKM_OK) return die("Failed to get output writer for counts file: " + dbg_path(out));
    info("orion_kmer::commands::count", "Successfully wrote k-mer counts to " + dbg_path(out));
    fast_exit();
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

// query.rs:24-134: reads whose canonical k-mer hits in the database's unified
// set reach min_hits, ids written in input order.
static int run_query(const Args &a) {
    std::string dbp, reads, out, mh;
    if (!get_one(a, "database", dbp)) return usage_error("the following required arguments were not provided:\n  --database <DATABASE_FILE>");
    if (!get_one(a, "reads", reads)) return usage_error("the following required arguments were not provided:\n  --reads <READS_FILE>");
    if (!get_one(a, "output-file", out)) return usage_error("the following required arguments were not provided:\n  --output-file <OUTPUT_FILE>");
    uint64_t min_hits = 1;
    if (get_one(a, "min-hits", mh) && !parse_u64(mh, min_hits))
        return usage_error("invalid value '" + mh + "' for '--min-hits <MIN_HITS>'");
    okm_db *db = nullptr;
    okm_status s = okm_db_read(&db, dbp.c_str());  // query.rs:28 (utils.rs:37-55)
    if (s == OKM_E_IO) return die("Failed to get input reader for k-mer database: " + dbg_path(dbp));
    if (s != OKM_OK) return die("Failed to deserialize KmerDbV2 from " + dbg_path(dbp));
    const uint8_t k = okm_db_k(db);
    if (k == 0 || k > 32) {  // query.rs:30-32
        okm_db_free(db);
        return die("Invalid K-mer size: " + std::to_string(k) + ". Must be between 1 and 32.");
    }
    // query.rs:36 get_all_kmers_unified -> a device set
    uint64_t total = 0;
    for (uint64_t i = 0; i < okm_db_num_references(db); ++i) {
        uint64_t n;
        okm_db_reference(db, i, nullptr, nullptr, &n);
        total += n;
    }
    okm_kset *set = nullptr;
    s = okm_kset_create(&set, k, g_device, total);
    if (s != OKM_OK) {
        okm_db_free(db);
        return die("MI355X engine unavailable: " + err_detail());
    }
    for (uint64_t i = 0; i < okm_db_num_references(db); ++i) {
        const uint64_t *keys;
        uint64_t n;
        okm_db_reference(db, i, nullptr, &keys, &n);
        if (n && okm_kset_insert(set, keys, n, 0, nullptr) != OKM_OK) {
            std::string d = err_detail();
            okm_kset_destroy(set);
            okm_db_free(db);
            return die("GPU engine failure while querying: " + d);
        }
    }
    okm_db_free(db);
    uint64_t nset = 0;
    okm_kset_size(set, &nset);
    info("orion_kmer::commands::query", "Querying reads from " + dbg_path(reads) + " against database with k=" + std::to_string(k) + " (" + std::to_string(nset) + " unique k-mers in DB)");
    okm_reader *r = nullptr;
    s = okm_reader_open2(&r, reads.c_str(), 1, OKM_READ_RAW | OKM_READ_IDS);  // query.rs:45-52
    if (s == OKM_E_IO) {
        okm_kset_destroy(set);
        return die("Failed to get input reader for reads file: " + dbg_path(reads));
    }
    if (s != OKM_OK) {
        okm_kset_destroy(set);
        return die("Failed to parse FASTQ content from: " + dbg_path(reads));
    }
    {  // query.rs:55-61: the output writer is created before any record is read
        FILE *f = fopen(out.c_str(), "wb");
        if (!f) {
            okm_reader_close(r);
            okm_kset_destroy(set);
            return die("Failed to get output writer for matching reads: " + dbg_path(out));
        }
        fclose(f);
    }
    std::string ids_out;
    std::vector<uint32_t> hits;
    uint64_t n_match = 0;
    for (;;) {
        const uint8_t *seq, *ids;
        const uint64_t *off, *ioff;
        uint64_t n;
        s = okm_reader_next(r, 256ull << 20, &seq, &off, &n);
        if (s != OKM_OK) {
            okm_reader_close(r);
            okm_kset_destroy(set);
            return die("Error reading record from " + dbg_path(reads));  // query.rs:69-70
        }
        if (n == 0) break;
        okm_reader_ids(r, &ids, &ioff);
        hits.resize(n);
        if (okm_query_hits(set, seq, off, n, hits.data()) != OKM_OK) {
            std::string d = err_detail();
            okm_reader_close(r);
            okm_kset_destroy(set);
            return die("GPU engine failure while querying: " + d);
        }
        for (uint64_t i = 0; i < n; ++i) {
            if (off[i + 1] - off[i] < k) continue;  // query.rs:83-85
            if (hits[i] < min_hits) continue;       // query.rs:97
            ids_out.append((const char *)ids + ioff[i], ioff[i + 1] - ioff[i]);
            ids_out += '\n';
            ++n_match;
        }
    }
    okm_reader_close(r);
    okm_kset_destroy(set);
    info("orion_kmer::commands::query", "Found " + std::to_string(n_match) + " reads matching criteria (min_hits: " + std::to_string(min_hits) + "). Writing to output...");
    if (okm_write_file(out.c_str(), (const uint8_t *)ids_out.data(), ids_out.size()) != OKM_OK)
        return die("Failed to get output writer for matching reads: " + dbg_path(out));
    return 0;
}

// csv crate (QuoteStyle::Necessary, '\t' delimiter): quote a field holding the
// delimiter, a quote or a line break.
static std::string tsv_field(const std::string &f) {
    if (f.find_first_of("\t\"\r\n") == std::string::npos) return f;
    std::string o = "\"";
    for (char ch : f) {
        if (ch == '"') o += '"';
        o += ch;
    }
    return o + "\"";
}

static std::string fmt4(double x) {  // Rust format!("{:.4}", x)
    char b[64];
    snprintf(b, sizeof(b), "%.4f", x);
    return b;
}

static double ratio(uint64_t a, uint64_t b) { return b > 0 ? (double)a / (double)b : 0.0; }

// classify.rs:58-385
static int run_classify(const Args &a) {
    std::string input, out, ks, mf, mc, tsv;
    if (!get_one(a, "input-file", input)) return usage_error("the following required arguments were not provided:\n  --input-file <INPUT_FILE>");
    auto dbs = get_all(a, "databases");
    if (dbs.empty()) return usage_error("the following required arguments were not provided:\n  --databases <DATABASE_FILES>...");
    if (!get_one(a, "output-file", out)) return usage_error("the following required arguments were not provided:\n  --output-file <OUTPUT_FILE>");
    const bool have_user_k = get_one(a, "kmer-size", ks);
    uint64_t user_k = 0, min_freq = 1;
    if (have_user_k && (!parse_u64(ks, user_k) || user_k > 255))
        return usage_error("invalid value '" + ks + "' for '--kmer-size <KMER_SIZE>': invalid digit found in string");
    if (get_one(a, "min-kmer-frequency", mf) && !parse_u64(mf, min_freq))
        return usage_error("invalid value '" + mf + "' for '--min-kmer-frequency <MIN_KMER_FREQUENCY>'");
    double min_cov = 0.0;
    if (get_one(a, "min-coverage", mc)) {
        char *end = nullptr;
        min_cov = strtod(mc.c_str(), &end);
        if (mc.empty() || *end) return usage_error("invalid value '" + mc + "' for '--min-coverage <MIN_COVERAGE>'");
    }
    const bool want_tsv = get_one(a, "output-tsv", tsv);
    // classify.rs:59-64 (unconditional eprintln)
    fprintf(stderr, "DEBUG: Entered run_classify. Input file: %s, Num DBs: %zu, Output: %s\n", dbg_path(input).c_str(),
            dbs.size(), dbg_path(out).c_str());
    // --- 1. databases and k (classify.rs:67-132)
    int final_k = -1;
    if (have_user_k) {
        if (user_k == 0 || user_k > 32) return die("Invalid K-mer size: " + std::to_string(user_k) + ". Must be between 1 and 32.");
        final_k = (int)user_k;
    }
    std::vector<okm_db *> loaded;
    auto free_dbs = [&]() {
        for (auto *d : loaded) okm_db_free(d);
        loaded.clear();
    };
    for (auto &p : dbs) {
        okm_db *d = nullptr;
        if (okm_db_read(&d, p.c_str()) != OKM_OK) {
            free_dbs();
            return die("Failed to load database: " + dbg_path(p));
        }
        const int dk = okm_db_k(d);
        if (final_k >= 0) {
            if (dk != final_k) {
                okm_db_free(d);
                free_dbs();
                if (have_user_k)
                    return die("User-provided k-mer size " + std::to_string(final_k) + " does not match k-mer size " + std::to_string(dk) + " from database: " + dbg_path(p));
                return die("Effective k-mer size " + std::to_string(final_k) + " (from first database) does not match k-mer size " + std::to_string(dk) + " from database: " + dbg_path(p));
            }
        } else {
            if (dk == 0 || dk > 32) {
                okm_db_free(d);
                free_dbs();
                return die("Invalid K-mer size: " + std::to_string(dk) + ". Must be between 1 and 32.");
            }
            final_k = dk;
        }
        loaded.push_back(d);
    }
    const uint8_t k = (uint8_t)final_k;
    // --- 2. input k-mer counts (classify.rs:135-199), on the device
    okm_ctx *ctx = nullptr;
    int rc;
    if ((rc = open_engine(&ctx, k, OKM_MODE_COUNT))) {
        free_dbs();
        return rc;
    }
    {
        okm_reader *r = nullptr;
        okm_status s = okm_reader_open(&r, input.c_str(), 0);  // utils.rs:157-161: no extension decompression
        if (s == OKM_E_IO) {
            okm_destroy(ctx);
            free_dbs();
            return die("Failed to get buffered file reader for file: " + dbg_path(input));
        }
        if (s != OKM_OK) {
            okm_destroy(ctx);
            free_dbs();
            return die("Failed to parse FASTA/Q content from: " + dbg_path(input));
        }
        for (;;) {
            const uint8_t *seq;
            const uint64_t *off;
            uint64_t n;
            s = okm_reader_next(r, 256ull << 20, &seq, &off, &n);
            if (s != OKM_OK) {
                okm_reader_close(r);
                okm_destroy(ctx);
                free_dbs();
                return die("Error reading record from input file: " + dbg_path(input));
            }
            if (n == 0) break;
            if (okm_add_batch(ctx, seq, off, n, 1) != OKM_OK) {
                std::string d = err_detail();
                okm_reader_close(r);
                okm_destroy(ctx);
                free_dbs();
                return die("GPU engine failure on " + input + ": " + d);
            }
        }
        okm_reader_close(r);
    }
    okm_classifier *cls = nullptr;
    uint64_t n_input = 0;
    if (okm_classifier_create(&cls, ctx, min_freq, &n_input) != OKM_OK) {
        std::string d = err_detail();
        okm_destroy(ctx);
        free_dbs();
        return die("GPU engine failure while classifying: " + d);
    }
    okm_destroy(ctx);
    info("orion_kmer::commands::classify", "After applying min_kmer_frequency filter (>= " + std::to_string(min_freq) + "), " + std::to_string(n_input) + " unique k-mers remain in input.");
    // --- 3. per database (classify.rs:206-308)
    std::string js = "{\n";
    js += "  \"input_file_path\": " + json_str(input) + ",\n";
    js += "  \"total_unique_kmers_in_input\": " + std::to_string(n_input) + ",\n";
    js += "  \"min_kmer_frequency_filter\": " + std::to_string(min_freq) + ",\n";
    js += "  \"databases_analyzed\": [";
    std::string tsv_out = "InputFile\tDatabase\tReference\tTotalKmersInReference\tInputKmersHittingReference\tSumDepthMatchedKmers\tAvgDepthMatchedKmers\tProportionInputKmersHittingReference\tReferenceBreadthOfCoverage\n";
    for (size_t di = 0; di < loaded.size(); ++di) {
        okm_db *d = loaded[di];
        const uint64_t nref = okm_db_num_references(d);
        std::vector<uint64_t> off(1, 0), keys;
        std::vector<std::string> names;
        for (uint64_t i = 0; i < nref; ++i) {
            const char *nm;
            const uint64_t *kk;
            uint64_t n;
            okm_db_reference(d, i, &nm, &kk, &n);
            names.emplace_back(nm);
            keys.insert(keys.end(), kk, kk + n);
            off.push_back(keys.size());
        }
        std::vector<uint64_t> rm(nref), rs(nref);
        uint64_t du = 0, dm = 0, ds = 0;
        if (okm_classifier_probe_db(cls, keys.data(), off.data(), nref, rm.data(), rs.data(), &du, &dm, &ds) != OKM_OK) {
            std::string e = err_detail();
            okm_classifier_destroy(cls);
            free_dbs();
            return die("GPU engine failure while classifying: " + e);
        }
        std::string refs;
        size_t nref_out = 0;
        for (uint64_t i = 0; i < nref; ++i) {
            const uint64_t tot = off[i + 1] - off[i];
            const double breadth = ratio(rm[i], tot);
            if (!(breadth >= min_cov)) continue;  // classify.rs:240
            const double avg = ratio(rs[i], rm[i]), prop = ratio(rm[i], n_input);
            refs += std::string(nref_out ? ",\n" : "\n") + "        {\n";
            refs += "          \"reference_name\": " + json_str(names[i]) + ",\n";
            refs += "          \"total_kmers_in_reference\": " + std::to_string(tot) + ",\n";
            refs += "          \"input_kmers_hitting_reference\": " + std::to_string(rm[i]) + ",\n";
            refs += "          \"sum_depth_of_matched_kmers_in_input\": " + std::to_string(rs[i]) + ",\n";
            refs += "          \"avg_depth_of_matched_kmers_in_input\": " + fmt_f64(avg) + ",\n";
            refs += "          \"proportion_input_kmers_hitting_reference\": " + fmt_f64(prop) + ",\n";
            refs += "          \"reference_breadth_of_coverage\": " + fmt_f64(breadth) + "\n";
            refs += "        }";
            ++nref_out;
            tsv_out += tsv_field(input) + "\t" + tsv_field(dbs[di]) + "\t" + tsv_field(names[i]) + "\t" +
                       std::to_string(tot) + "\t" + std::to_string(rm[i]) + "\t" + std::to_string(rs[i]) + "\t" +
                       fmt4(avg) + "\t" + fmt4(prop) + "\t" + fmt4(breadth) + "\n";
        }
        js += std::string(di ? ",\n" : "\n") + "    {\n";
        js += "      \"database_path\": " + json_str(dbs[di]) + ",\n";
        js += "      \"database_kmer_size\": " + std::to_string((int)okm_db_k(d)) + ",\n";
        js += "      \"total_unique_kmers_in_db_across_references\": " + std::to_string(du) + ",\n";
        js += "      \"overall_input_kmers_matched_in_db\": " + std::to_string(dm) + ",\n";
        js += "      \"overall_sum_depth_of_matched_kmers_in_input\": " + std::to_string(ds) + ",\n";
        js += "      \"overall_avg_depth_of_matched_kmers_in_input\": " + fmt_f64(ratio(ds, dm)) + ",\n";
        js += "      \"proportion_input_kmers_in_db_overall\": " + fmt_f64(ratio(dm, n_input)) + ",\n";
        js += "      \"proportion_db_kmers_covered_overall\": " + fmt_f64(ratio(dm, du)) + ",\n";
        js += "      \"references\": [" + refs + (nref_out ? "\n      ]" : "]") + "\n    }";
    }
    js += loaded.empty() ? "]\n}" : "\n  ]\n}";
    okm_classifier_destroy(cls);
    free_dbs();
    // --- 4./5. outputs (classify.rs:320-381)
    if (okm_write_file(out.c_str(), (const uint8_t *)js.data(), js.size()) != OKM_OK)
        return die("Failed to get output writer for JSON file: " + dbg_path(out));
    if (want_tsv && okm_write_file(tsv.c_str(), (const uint8_t *)tsv_out.data(), tsv_out.size()) != OKM_OK)
        return die("Failed to get output writer for TSV file: " + dbg_path(tsv));
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
        spec.push_back({"gpus", 0, true, false});
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
    } else if (cmd == "query") {
        spec.push_back({"database", 'd', true, false});
        spec.push_back({"reads", 'r', true, false});
        spec.push_back({"output-file", 'o', true, false});
        spec.push_back({"min-hits", 'c', true, false});
    } else if (cmd == "classify") {
        spec.push_back({"input-file", 'i', true, false});
        spec.push_back({"databases", 'd', true, true});
        spec.push_back({"output-file", 'o', true, false});
        spec.push_back({"kmer-size", 'k', true, false});
        spec.push_back({"min-kmer-frequency", 0, true, false});
        spec.push_back({"min-coverage", 0, true, false});
        spec.push_back({"output-tsv", 0, true, false});
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
    std::string gp;
    if (get_one(a, "gpus", gp)) {
        uint64_t v;
        if (!parse_u64(gp, v) || v > 64) return usage_error("invalid value '" + gp + "' for '--gpus <GPUS>'");
        g_gpus = (int)v;
        if (g_gpus == 0 && g_device != 0)
            return usage_error("the argument '--device <DEVICE>' cannot be used with '--gpus 0' (every visible GPU)");
    }
    if (cmd == "count") return run_count(a);
    if (cmd == "build") return run_build(a);
    if (cmd == "query") return run_query(a);
    if (cmd == "classify") return run_classify(a);
    return run_compare(a);
}
