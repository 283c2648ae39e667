/*
 * orion_kmer.h — C ABI of the MI355X-native k-mer engine (liborion_kmer.so).
 *
 * This is the drop-in boundary for orion-kmer's data-parallel hot path
 * (reference: motroy/orion-kmer, Rust crate `orion-kmer/`).  Everything is
 * `extern "C"`, plain pointers and sizes; no C++ types, exceptions or torch
 * types cross it.  Each entry point names the reference interface it
 * replaces (paths relative to the reference's `orion-kmer/` directory).
 *
 * The reference has no FFI of its own: its seam is the private
 *   fn process_sequence_chunk(seq: &[u8], k: u8, map: &DashMap<u64, AtomicUsize>)
 * (src/commands/count.rs:23), driven record by record from run_count's
 * `while let Some(record) = reader.next()` loop (count.rs:68-72), plus the
 * DashMap's drain/filter/sort at count.rs:106-119.  A Rust maintainer binds
 * this header with `extern "C"` declarations.
 *
 * Conventions
 *  - Every fallible call returns okm_status; nothing aborts across the ABI.
 *  - Caller owns inputs; results returned through `**` out-pointers are
 *    library-allocated host memory released with okm_free_result().
 *  - A context is used by one host thread at a time (the reference's `count`
 *    is single-threaded, count.rs:6,68-79).  Internally it owns one HIP
 *    stream on one device; results are complete when a call returns.
 *  - k in 1..=32 (u64 keys, kmer.rs:37-43).  Anything else is
 *    OKM_E_INVALID_K, which the CLI prints as the reference's
 *    "Invalid K-mer size: {k}. Must be between 1 and 32." (errors.rs:6).
 *  - The library has NO CPU fallback: without a usable gfx950 device every
 *    compute entry point fails with OKM_E_DEVICE.
 */
#ifndef ORION_KMER_H
#define ORION_KMER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OKM_ABI_VERSION 2

/* Byte that separates records in the device batch layout: any byte that is
 * not A/C/G/T/U (either case) kills every window containing it, so windows
 * never cross records (count.rs:23-38 is per record). */
#define OKM_RECORD_SEPARATOR ((uint8_t)'\n')

typedef struct okm_ctx okm_ctx;
typedef struct okm_reader okm_reader;

typedef enum okm_status {
    OKM_OK = 0,
    OKM_E_INVALID_K = 1,   /* errors.rs:6 InvalidKmerSize */
    OKM_E_NOMEM = 2,       /* host or device allocation failed */
    OKM_E_DEVICE = 3,      /* no usable GPU / HIP runtime error */
    OKM_E_COMM = 4,        /* multi-GPU exchange: RCCL missing or failed */
    OKM_E_ARG = 5,         /* bad argument (null pointer, bad length ...) */
    OKM_E_OVERFLOW = 6,    /* capacity exceeded (caller buffer too small) */
    OKM_E_IO = 7,          /* file open/read/write failed */
    OKM_E_PARSE = 8,       /* not FASTA/FASTQ (first byte), empty file */
    OKM_E_RECORD = 9,      /* malformed record */
    OKM_E_STATE = 10,      /* call out of order (e.g. fetch before count) */
    OKM_E_FORMAT = 11      /* bad KmerDbV2 bytes */
} okm_status;

typedef enum okm_mode {
    OKM_MODE_COUNT = 0,    /* count.rs: DashMap<u64, AtomicUsize> */
    OKM_MODE_SET = 1,      /* build.rs:50-58: DashSet<u64> */
    /* Flag, OR-ed into the mode: opt into k in 33..64 (two-u64 keys, SURVEY
     * §8 a3-a5 extension, BASELINE configs[3]).  Without it k > 32 fails with
     * OKM_E_INVALID_K exactly like the reference (count.rs:43-45). */
    OKM_MODE_WIDE = 0x100
} okm_mode;

/* A k-mer for k in 33..64: the same MSB-first 2-bit encoding as kmer.rs:37-57
 * over 2k bits, value = hi * 2^64 + lo.  In a context created with k > 32
 * every `keys` array of the calls below holds one okm_key128, i.e. two u64, per
 * entry instead of one u64: okm_add_pairs[_device], okm_fetch_counts,
 * okm_finish_counts / okm_finish_set, okm_result_device; so does
 * okm_write_counts_tsv for k > 32. */
typedef struct okm_key128 {
    uint64_t lo, hi;
} okm_key128;

/* ------------------------------------------------------------------------
 * Library / device
 * ---------------------------------------------------------------------- */

int okm_abi_version(void);
const char *okm_status_string(okm_status s);
/* Number of visible HIP devices (0 when none; never an error). */
int okm_device_count(void);
/* Name of the device's ISA ("gfx950"), or "" when unavailable. */
const char *okm_device_arch(int device);
/* Thread-local message of the last failing call on this thread. */
const char *okm_last_error(void);

/* ------------------------------------------------------------------------
 * Counting context — replaces DashMap::new() (count.rs:48) / DashSet::new()
 * (build.rs:95) and everything process_sequence_chunk (count.rs:23-38) does
 * to it.
 * ---------------------------------------------------------------------- */

/* device: HIP ordinal.  distinct_hint: expected distinct k-mers (0 = unknown);
 * sizing only, never correctness (>= 2^30: the context starts with the
 * folding geometry it would otherwise take at its first fold). */
okm_status okm_create(okm_ctx **out, uint8_t k, okm_mode mode, int device, uint64_t distinct_hint);
void okm_destroy(okm_ctx *ctx);
/* Forget all input and results; keep device allocations for reuse. */
okm_status okm_reset(okm_ctx *ctx);
/* Give the context's cached (unused) device blocks back to the HIP runtime;
 * what the input and the result hold stays.  For processes that keep several
 * contexts on one device and use them in turn (another context's planner
 * sees only the device's free memory). */
okm_status okm_trim(okm_ctx *ctx);

/* Append one batch of records held in HOST memory.  Record r is
 * seq[offsets[r] .. offsets[r+1]) (offsets has n_records+1 entries).
 * normalized=0: the bytes are raw sequence bytes and the library applies
 * needletail normalize(false) semantics (case fold, U->T, whitespace and
 * line breaks removed, anything else kills the window) — the call at
 * count.rs:71.  normalized=1: caller already normalised (whitespace-free).
 * Replaces the record loop count.rs:68-72. */
okm_status okm_add_batch(okm_ctx *ctx, const uint8_t *seq, const uint64_t *offsets,
                         uint64_t n_records, int normalized);

/* Append a batch already resident in DEVICE memory in the batch layout:
 * whitespace-free records joined by OKM_RECORD_SEPARATOR.  The bytes are
 * consumed (k-mers extracted) before the call returns; the caller may reuse
 * the buffer afterwards.  This is the zero-copy hot path. */
okm_status okm_add_batch_device(okm_ctx *ctx, const uint8_t *d_seq, uint64_t n_bytes);

/* Append (canonical key, count) pairs in DEVICE memory, e.g. partial tables
 * received from other GPUs.  Counts add (the AtomicUsize fetch_add of
 * count.rs:31-34 generalised to a weight). */
okm_status okm_add_pairs_device(okm_ctx *ctx, const uint64_t *d_keys, const uint64_t *d_counts,
                                uint64_t n);
/* Same, from HOST memory. */
okm_status okm_add_pairs(okm_ctx *ctx, const uint64_t *keys, const uint64_t *counts, uint64_t n);
/* (key, count) pairs in DEVICE memory whose keys are strictly ascending — e.g.
 * a slice of another context's okm_result_device table, as received by the
 * owner of a key range in the multi-GPU merge.  No copy: the buffers are
 * borrowed and must stay alive and unchanged until okm_count returns.  When
 * every input is sorted, counting splits them by binary search instead of
 * partitioning them (counts add, as in okm_add_pairs_device). */
okm_status okm_add_sorted_pairs_device(okm_ctx *ctx, const uint64_t *d_keys, const uint64_t *d_counts,
                                       uint64_t n);

/* Run the counting over everything added so far; *n_distinct receives the
 * number of distinct canonical k-mers (DashMap::len()).  Idempotent until the
 * next add. */
okm_status okm_count(okm_ctx *ctx, uint64_t *n_distinct);

/* Copy the counted table, filtered to count >= min_count and sorted
 * ascending by key (count.rs:106-119), into caller buffers of capacity
 * `cap` entries.  dst_on_device!=0: keys/counts are device pointers (counts
 * may be NULL).  *n receives the number of entries written. */
okm_status okm_fetch_counts(okm_ctx *ctx, uint64_t min_count, uint64_t *keys, uint64_t *counts,
                            uint64_t cap, uint64_t *n, int dst_on_device);
/* Number of entries okm_fetch_counts would return for min_count. */
okm_status okm_result_size(okm_ctx *ctx, uint64_t min_count, uint64_t *n);

/* count + fetch into library-allocated host arrays (free with okm_free_result). */
okm_status okm_finish_counts(okm_ctx *ctx, uint64_t min_count, uint64_t **keys, uint64_t **counts,
                             uint64_t *n);
/* Set mode result (build.rs:104): sorted unique canonical k-mers. */
okm_status okm_finish_set(okm_ctx *ctx, uint64_t **keys, uint64_t *n);
void okm_free_result(void *p);

/* Device pointers to the counted, sorted, unfiltered table (valid until the
 * next add/reset/destroy). */
okm_status okm_result_device(okm_ctx *ctx, const uint64_t **d_keys, const uint64_t **d_counts,
                             uint64_t *n);

/* |A ∩ B| of two sorted unique key arrays in host memory, computed on the
 * device (compare.rs:58 HashSet::intersection().count()). */
okm_status okm_set_intersection_size(const uint64_t *a, uint64_t na, const uint64_t *b,
                                     uint64_t nb, int device, uint64_t *out);
/* The same over device-resident arrays (e.g. two okm_result_device tables). */
okm_status okm_set_intersection_size_device(const uint64_t *d_a, uint64_t na, const uint64_t *d_b,
                                            uint64_t nb, int device, uint64_t *out);

/* ------------------------------------------------------------------------
 * Device k-mer sets — the read-only callers of the counting path.
 *
 * okm_kset replaces the unified HashSet<u64> of a database
 * (db_types.rs:43-48 get_all_kmers_unified, built at query.rs:36) and its
 * HashSet::contains probes (query.rs:88): an open-addressing table in HBM
 * (load <= 1/2, grows by rehash).  k in 1..=32 as the reference (query.rs:30-32).
 * ---------------------------------------------------------------------- */
typedef struct okm_kset okm_kset;
/* capacity_hint: expected distinct keys (sizing only). */
okm_status okm_kset_create(okm_kset **out, uint8_t k, int device, uint64_t capacity_hint);
void okm_kset_destroy(okm_kset *s);
/* HashSet::extend of a reference's keys (db_types.rs:46).  keys_on_device!=0:
 * `keys` is a device pointer.  *n_new (optional) = keys not present before. */
okm_status okm_kset_insert(okm_kset *s, const uint64_t *keys, uint64_t n, int keys_on_device,
                           uint64_t *n_new);
/* HashSet::len() (db_types.rs:50-53 total_unique_kmers). */
okm_status okm_kset_size(const okm_kset *s, uint64_t *n);
/* out[i] = 1 if keys[i] is in the set (host buffers). */
okm_status okm_kset_contains(okm_kset *s, const uint64_t *keys, uint64_t n, uint8_t *out);

/* query.rs:81-99, per record: hits[r] = number of k-windows of the RAW record
 * bytes (record.sequence(), no normalize: only A/C/G/T in either case are
 * valid, so U/u, N and line breaks of multi-line FASTA kill windows) whose
 * canonical k-mer is in the set.  Record r is seq[offsets[r]..offsets[r+1])
 * (host memory); hits has n_records entries.  The caller applies the
 * reference's `len < k -> no output` and `hits >= min_hits` tests. */
okm_status okm_query_hits(okm_kset *s, const uint8_t *seq, const uint64_t *offsets, uint64_t n_records,
                          uint32_t *hits);
/* Same over a DEVICE batch: records joined by OKM_RECORD_SEPARATOR (a
 * separator after the last record is optional; no other '\n' may occur),
 * n_records = number of records, d_hits a device array of n_records u32. */
okm_status okm_query_hits_device(okm_kset *s, const uint8_t *d_seq, uint64_t n_bytes, uint64_t n_records,
                                 uint32_t *d_hits);

/* classify.rs:176-308 on the device.  okm_classifier_create takes a COUNT
 * context holding the input's k-mers (classify.rs:135-181, counted with
 * okm_add_batch + okm_count), keeps the entries with count >=
 * min_kmer_frequency (classify.rs:195-199) in a device map, and returns
 * their number (total_unique_kmers_in_input) in *n_input_kmers.  The context
 * may be destroyed afterwards. */
typedef struct okm_classifier okm_classifier;
okm_status okm_classifier_create(okm_classifier **out, okm_ctx *input, uint64_t min_kmer_frequency,
                                 uint64_t *n_input_kmers);
void okm_classifier_destroy(okm_classifier *c);
/* One database (classify.rs:215-308): reference r owns
 * keys[ref_offsets[r] .. ref_offsets[r+1]) (a HashSet: no duplicates).
 * ref_matched[r] / ref_sum_depth[r] = input k-mers in reference r and the sum
 * of their counts (classify.rs:228-236); *db_union = |union of references|
 * (db_types.rs:50-53); *db_matched / *db_sum_depth = the same two numbers over
 * the union (classify.rs:237,268-272).  Host buffers. */
okm_status okm_classifier_probe_db(okm_classifier *c, const uint64_t *keys, const uint64_t *ref_offsets,
                                   uint64_t n_refs, uint64_t *ref_matched, uint64_t *ref_sum_depth,
                                   uint64_t *db_union, uint64_t *db_matched, uint64_t *db_sum_depth);
/* Same with the database keys in DEVICE memory (d_keys[ref_offsets[0] ..
 * ref_offsets[n_refs])); ref_offsets and the outputs stay on the host. */
okm_status okm_classifier_probe_db_device(okm_classifier *c, const uint64_t *d_keys, const uint64_t *ref_offsets,
                                          uint64_t n_refs, uint64_t *ref_matched, uint64_t *ref_sum_depth,
                                          uint64_t *db_union, uint64_t *db_matched, uint64_t *db_sum_depth);

/* ------------------------------------------------------------------------
 * Multi-GPU — replaces nothing in the reference (its count
 * is one process on one map, count.rs:48); it is how ONE table spans several
 * GPUs: reads shard by record, every rank counts its shard into its own
 * context, and okm_merge_owned turns the P local tables into the global one
 * over RCCL (xGMI).  Value-range ownership: rank r ends up holding a
 * contiguous key range, so ranks 0..P-1 concatenated are the sorted global
 * table of count.rs:106-119 with no final merge.
 * ---------------------------------------------------------------------- */
typedef struct okm_comm okm_comm;
#define OKM_COMM_ID_BYTES 128
/* A new communicator id (ncclGetUniqueId) for okm_comm_init_rank; rank 0
 * creates it and the caller hands the bytes to every rank (MPI, a file,
 * torch.distributed ...). */
okm_status okm_comm_unique_id(uint8_t *id /* OKM_COMM_ID_BYTES */);
/* One rank per process, on HIP device `device` (ncclCommInitRank). */
okm_status okm_comm_init_rank(okm_comm **out, int nranks, int rank, const uint8_t *id, int device);
/* Every rank in this process, rank i on devices[i] (NULL: device i)
 * (ncclCommInitAll); out has n entries.  Each rank's calls then run on a host
 * thread of its own. */
okm_status okm_comm_init_all(okm_comm **out, int n, const int *devices);
/* n virtual ranks in THIS process on ONE device, without RCCL: the same owner
 * plan, pack / widen / escape kernels, message pieces and owner merge as an
 * RCCL communicator, with every collective done by device copies between the
 * ranks' buffers (host threads meet at a barrier; a rank missing for 300 s
 * aborts it).  RCCL refuses two
 * ranks on one GPU: this is how the P > 1 merge runs on one device (tests,
 * rehearsals).  out has n entries; each rank's okm_merge_owned runs on a host
 * thread of its own. */
okm_status okm_comm_init_loopback(okm_comm **out, int n, int device);
void okm_comm_destroy(okm_comm *comm);
int okm_comm_rank(const okm_comm *comm);
int okm_comm_size(const okm_comm *comm);
/* What a communicator is, for audit lines (bench.py's N>1 `comm` object): the
 * ranks / rank / device it was created with, what the transport itself
 * reports (RCCL: ncclCommCount, ncclCommUserRank, ncclCommCuDevice; the
 * loopback transport: its virtual ranks, device -1), and the PCI bus id of
 * the device (hipDeviceGetPCIBusId), so N ranks can be shown to be N GPUs. */
typedef struct okm_comm_info {
    int size, rank, device;
    int transport_ranks, transport_rank, transport_device;  /* -1: not reported */
    char transport[16];                                     /* "rccl" | "loopback" */
    char pci_bus_id[32];                                    /* "0000:05:00.0"; empty when unknown */
} okm_comm_info;
okm_status okm_comm_get_info(const okm_comm *comm, okm_comm_info *info);
/* Collective over every rank of `comm`: `local` (counted or not) holds this
 * rank's shard; afterwards `owner` (reset first) holds this rank's key range
 * of the union of all ranks' tables, counted and sorted, and *n_owned its
 * distinct keys.  local, owner and comm share one device and k; k > 32
 * contexts (OKM_MODE_WIDE) move their K128 keys as u64 word pairs (never as
 * 5-byte deltas); owner may be local itself (its table is only read until
 * the exchange completes).
 * Set-mode contexts exchange keys only (build.rs / compare.rs sets).  The
 * owner keeps no pointer into local or the communicator afterwards: it may
 * take more input, and local may be reset.  A rank that fails between the
 * collectives (e.g. out of memory) reports it to its peers, so every rank
 * returns an error; a failure inside a send/recv aborts the communicator
 * (later calls: OKM_E_COMM).  At one rank (comm size 1, owner != local) the
 * owner's range is the whole table: it takes local's table as it stands (no
 * exchange, no copy: the two contexts swap their device memory) and local is
 * left reset. */
okm_status okm_merge_owned(okm_ctx *local, okm_comm *comm, okm_ctx *owner, uint64_t *n_owned);
/* okm_merge_owned for n tables under ONE owner split (balanced over the sum of
 * their histograms), so equal keys of different tables meet on one rank: the
 * distributed compare (compare.rs:51-66) intersects owners[0] and owners[1]
 * per rank and sums with okm_comm_allreduce_u64.  n_owned has n entries. */
okm_status okm_merge_owned_n(okm_ctx *const *locals, okm_comm *comm, okm_ctx *const *owners, int n,
                             uint64_t *n_owned);
/* Collective sum of n u64 (host memory; out may equal in). */
okm_status okm_comm_allreduce_u64(okm_comm *comm, const uint64_t *in, uint64_t *out, uint32_t n);
/* Host wall ms of the last okm_merge_owned: [0] plan (histogram, all-reduce,
 * sizes), [1] exchange (pack + send/recv + unpack), [2] reserved, [3] owner merge. */
okm_status okm_comm_last_times(const okm_comm *comm, double *ms4);
/* Bytes this rank sent to / received from OTHER ranks in the last
 * okm_merge_owned (keys, count bytes and escapes; the self slice excluded). */
okm_status okm_comm_last_bytes(const okm_comm *comm, uint64_t *sent, uint64_t *received);
/* The owner split (host, no device): bounds[0] = 0 <= ... <= bounds[world] =
 * nbins, rank r owns histogram bins [bounds[r], bounds[r+1]), cut where the
 * running total first reaches r/world of the whole. */
okm_status okm_owner_bounds(const uint64_t *hist, uint32_t nbins, int world, uint32_t *bounds);

/* One counting context per GPU in this process (`orion-kmer count --gpus N`),
 * behind the same add / count / finish calls as a context: host batches go to
 * the GPUs in turn and are counted on one worker thread per GPU while the
 * caller parses the next batch (okm_group_add_batch copies the batch and
 * returns); okm_group_count merges the GPUs' tables by key-range owner
 * (okm_merge_owned over okm_comm_init_all communicators).  n_gpus <= 0: every
 * visible device; 1: no RCCL at all.  devices: the n_gpus ordinals (NULL:
 * 0..n_gpus-1).  k > 32 (OKM_MODE_WIDE) too: its K128 keys cross as word pairs. */
typedef struct okm_group okm_group;
okm_status okm_group_create(okm_group **out, uint8_t k, okm_mode mode, int n_gpus, const int *devices,
                            uint64_t distinct_hint);
void okm_group_destroy(okm_group *g);
int okm_group_size(const okm_group *g);
okm_status okm_group_add_batch(okm_group *g, const uint8_t *seq, const uint64_t *offsets, uint64_t n_records,
                               int normalized);
okm_status okm_group_count(okm_group *g, uint64_t *n_distinct);
/* Rank r's context after okm_group_count: its owned key range (okm_result_size,
 * okm_fetch_counts, okm_result_device ...); ranges in rank order are the
 * sorted global table. */
okm_ctx *okm_group_owner(okm_group *g, int rank);
/* okm_finish_counts over the group: the concatenated ranges, filtered. */
okm_status okm_group_finish_counts(okm_group *g, uint64_t min_count, uint64_t **keys, uint64_t **counts,
                                   uint64_t *n);
/* count.rs:106-137 in one call: the group's table, filtered to count >=
 * min_count, written as "KMER\tCOUNT\n" lines to `path` (.gz/.xz/.zst by
 * extension, utils.rs:167-198), streamed off the GPUs in chunks while the host
 * formats the previous one.  *n_lines (optional) = lines written. */
okm_status okm_group_write_counts_tsv(okm_group *g, const char *path, uint64_t min_count, uint64_t *n_lines);

/* ------------------------------------------------------------------------
 * Instrumentation (bench.py measures kernels with HIP events on the
 * context's own stream).
 * ---------------------------------------------------------------------- */
okm_status okm_synchronize(okm_ctx *ctx);
okm_status okm_set_timing(okm_ctx *ctx, int enable);
/* Per-kernel stats accumulated since okm_set_timing(ctx,1): fills up to
 * `cap` entries; *n receives the number of kernels.  name[i] points into
 * library storage. */
typedef struct okm_kernel_stat {
    const char *name;
    uint64_t launches;
    double total_ms;        /* sum of HIP-event durations */
    double alg_bytes;       /* algorithmic HBM bytes moved */
} okm_kernel_stat;
okm_status okm_kernel_stats(okm_ctx *ctx, okm_kernel_stat *stats, int cap, int *n);
/* Engine counters of the last okm_count (partition levels, max partition,...) */
typedef struct okm_engine_info {
    uint64_t kmers;          /* valid windows (sum of counts) */
    uint64_t distinct;
    uint32_t l1_bits;        /* first-level key-range partition bits */
    uint32_t l2_bits;        /* second-level bits (0 = not needed) */
    uint32_t levels;         /* partition passes over keys */
    uint32_t work_items;     /* partitions counted in LDS */
    uint64_t max_partition;  /* largest partition (instances) */
    uint64_t device_bytes;   /* device memory held (mapped, including idle cached chunks) */
    uint32_t groups;         /* key-range groups counted one after the other (0/1 = one) */
    uint32_t folds;          /* times the uncounted batches were folded into a sorted table */
    uint64_t device_peak_bytes;  /* high-water mark of live device allocations since okm_create / okm_reset */
    uint64_t host_bytes;     /* sorted tables this context keeps in host memory (moved off a full device) */
    uint32_t spills;         /* tables moved to host memory since okm_create / okm_reset */
    uint32_t pad;
} okm_engine_info;
okm_status okm_engine_info_get(okm_ctx *ctx, okm_engine_info *info);

/* Device memory helpers (so a host program without a GPU framework can stage
 * device-resident batches). */
okm_status okm_device_alloc(int device, uint64_t bytes, void **d_ptr);
okm_status okm_device_free(void *d_ptr);
okm_status okm_memcpy_h2d(void *d_dst, const void *src, uint64_t bytes);
okm_status okm_memcpy_d2h(void *dst, const void *d_src, uint64_t bytes);

/* ------------------------------------------------------------------------
 * k-mer codec parity surface — kmer.rs pub fns (CPU; for tests and hosts).
 * ---------------------------------------------------------------------- */
/* kmer.rs:37-57 seq_to_u64: returns 1 and writes *out for Some, 0 for None. */
int okm_seq_to_u64(const uint8_t *seq, size_t len, uint8_t k, uint64_t *out);
/* kmer.rs:61-75 u64_to_seq: writes k bytes; returns 0 (reference panics) for bad k. */
int okm_u64_to_seq(uint64_t v, uint8_t k, char *out);
/* kmer.rs:79-94; returns 0 (reference panics) for bad k. */
uint64_t okm_reverse_complement_u64(uint64_t v, uint8_t k);
/* kmer.rs:99-106 */
uint64_t okm_canonical_u64(uint64_t v, uint8_t k);
/* The k in 33..64 extension of the four (no reference: restatement-defined). */
int okm_seq_to_u128(const uint8_t *seq, size_t len, uint8_t k, okm_key128 *out);
int okm_u128_to_seq(okm_key128 v, uint8_t k, char *out);
okm_key128 okm_reverse_complement_u128(okm_key128 v, uint8_t k);
okm_key128 okm_canonical_u128(okm_key128 v, uint8_t k);

/* ------------------------------------------------------------------------
 * Host record source — replaces needletail parse_fastx_reader + record
 * normalize (count.rs:59-72) and the extension-based decompression of
 * utils.rs:125-152.  Produces normalised batches in the layout okm_add_batch
 * takes.
 * ---------------------------------------------------------------------- */
/* decompress_by_extension=1: count/query behaviour (utils.rs:125-152:
 * .gz/.xz/.zst/.zstd by lower-cased extension); 0: build/classify behaviour
 * (utils.rs:157-161, raw bytes).  needletail's own gzip/bzip2/xz magic
 * sniffing is applied after that in both cases. */
okm_status okm_reader_open(okm_reader **out, const char *path, int decompress_by_extension);
/* okm_reader_open with flags: OKM_READ_RAW = record.sequence() bytes as they
 * are in the file, no normalize (query.rs:66; multi-line FASTA keeps its
 * interior line breaks), OKM_READ_IDS = also keep each record's id()
 * (query.rs:70: the header line after '>'/'@', CR trimmed). */
#define OKM_READ_RAW 1
#define OKM_READ_IDS 2
okm_status okm_reader_open2(okm_reader **out, const char *path, int decompress_by_extension, int flags);
/* Ids of the records of the last okm_reader_next batch: record r's id is
 * ids[id_offsets[r] .. id_offsets[r+1]).  Valid until the next call. */
okm_status okm_reader_ids(const okm_reader *r, const uint8_t **ids, const uint64_t **id_offsets);
/* Next batch of at most ~max_bytes sequence bytes (at least one record).
 * Pointers stay valid until the next call.  *n_records == 0 at end. */
okm_status okm_reader_next(okm_reader *r, uint64_t max_bytes, const uint8_t **seq,
                           const uint64_t **offsets, uint64_t *n_records);
uint64_t okm_reader_records(const okm_reader *r);
void okm_reader_close(okm_reader *r);
/* Parse a whole in-memory FASTA/FASTQ buffer (after sniffing compression). */
okm_status okm_parse_buffer(const uint8_t *data, uint64_t n, uint8_t **seq, uint64_t **offsets,
                            uint64_t *n_records);

/* ------------------------------------------------------------------------
 * Output codecs — utils.rs:167-198 get_output_writer (.gz/.xz/.zst by
 * extension, else plain) and the TSV of count.rs:127-135.
 * ---------------------------------------------------------------------- */
/* Writes "KMER\tCOUNT\n" lines for sorted (keys, counts); k in 1..64 (keys
 * are okm_key128 pairs for k > 32). */
okm_status okm_write_counts_tsv(const char *path, uint8_t k, const uint64_t *keys,
                                const uint64_t *counts, uint64_t n);
/* Writes `n` raw bytes through the extension-selected compressor. */
okm_status okm_write_file(const char *path, const uint8_t *data, uint64_t n);
/* Reads a whole file, decompressing by extension (utils.rs:125-152). */
okm_status okm_read_file(const char *path, int decompress_by_extension, uint8_t **data, uint64_t *n);

/* ------------------------------------------------------------------------
 * KmerDbV2 (db_types.rs:7-14) bincode 1.3 codec — build.rs:141-146 writer,
 * utils.rs:37-55 reader.  Layout: u8 k; u64 n_refs; per ref: u64 len, name
 * bytes, u64 n_keys, n_keys × u64 (all little-endian).
 * ---------------------------------------------------------------------- */
typedef struct okm_db okm_db;
okm_status okm_db_new(okm_db **out, uint8_t k);
/* db_types.rs:38-40 add_reference: a duplicate name overwrites. `keys` are
 * copied. */
okm_status okm_db_add_reference(okm_db *db, const char *name, const uint64_t *keys, uint64_t n);
okm_status okm_db_write(const okm_db *db, const char *path);
okm_status okm_db_read(okm_db **out, const char *path);
uint8_t okm_db_k(const okm_db *db);
uint64_t okm_db_num_references(const okm_db *db);
/* Reference i: name (NUL-terminated, library storage), keys (library storage). */
okm_status okm_db_reference(const okm_db *db, uint64_t i, const char **name, const uint64_t **keys,
                            uint64_t *n);
void okm_db_free(okm_db *db);

/* ------------------------------------------------------------------------
 * Seeded synthetic reads (bench / tests; SURVEY.md §8(d) generator).
 * Reads of `read_len` bases sampled from a random genome of `genome_len`
 * bases (genome drawn from genome_seed), strand 50/50, substitution rate
 * sub_rate, N rate n_rate, per-read draws keyed by (seed, read index).
 * Output: n_reads records in the device batch layout, each followed by
 * OKM_RECORD_SEPARATOR: out must hold n_reads*(read_len+1) bytes.
 * ---------------------------------------------------------------------- */
okm_status okm_synth_reads(uint64_t genome_seed, uint64_t genome_len, uint64_t seed,
                           uint64_t first_read, uint64_t n_reads, uint32_t read_len,
                           double sub_rate, double n_rate, uint8_t *out, int threads);
/* The same bytes generated on the device into d_out (n_reads*(read_len+1)
 * bytes of device memory on `device`), without a host copy: BASELINE
 * configs[2] (C3) shards are made resident this way.  Synchronous. */
okm_status okm_synth_reads_device(uint64_t genome_seed, uint64_t genome_len, uint64_t seed,
                                  uint64_t first_read, uint64_t n_reads, uint32_t read_len,
                                  double sub_rate, double n_rate, uint8_t *d_out, int device);
/* ONT-like long reads (BASELINE configs[3] shape): read
 * r's length is lognormal (median_len, sigma) clipped to [min_len, max_len];
 * its bases come from the genome (genome_seed, genome_len >= 2 max_len + 1)
 * with per-base errors: substitution (sub_rate), insertion of a random base
 * after the source base (ins_rate), deletion of the source base (del_rate);
 * strand 50/50 (reverse complement).  Reads [first_read, first_read +
 * n_reads), each followed by OKM_RECORD_SEPARATOR, into library-allocated
 * *out (okm_free_result); *n_bytes = bytes; lens (optional, n_reads entries) =
 * read lengths.  out == NULL: lengths and *n_bytes only. */
okm_status okm_synth_long_reads(uint64_t genome_seed, uint64_t genome_len, uint64_t seed, uint64_t first_read,
                                uint64_t n_reads, double median_len, double sigma, uint32_t min_len,
                                uint32_t max_len, double sub_rate, double ins_rate, double del_rate,
                                uint8_t **out, uint64_t *n_bytes, uint32_t *lens, int threads);

#ifdef __cplusplus
}
#endif
#endif /* ORION_KMER_H */
