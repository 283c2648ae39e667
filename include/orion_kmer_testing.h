/*
 * orion_kmer_testing.h — test hooks of liborion_kmer.so.  NOT for production
 * use: every knob forces a rare path of the engine (an overflowed sampled
 * capacity, a key-range group split, a message cut into tiny pieces, a rank
 * that fails mid-merge ...) so that the test suite can check it against the
 * oracle at small sizes.  The defaults (every knob unset) are what the
 * product runs; the run-time settings a user may touch are environment
 * variables listed in DESIGN.md's appendix.
 *
 * Knobs are process-wide (an atomic word each) and are read when the path
 * they steer runs, so a test sets one, makes its calls and unsets it.
 */
#ifndef ORION_KMER_TESTING_H
#define ORION_KMER_TESTING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum okm_test_knob {
    /* sampled placement: every capacity times value / 1000, so that a batch
     * overflows it and the pass is redone exactly (okm_engine.hip l1_sampled,
     * split_launch_sampled) */
    OKM_TEST_L1_CAP_PERMILLE = 0,
    OKM_TEST_PART_CAP_PERMILLE = 1,
    /* at most this many key bits per partition pass (fan-out and host rounds) */
    OKM_TEST_PART_MAX_BITS = 2,
    /* memory-bounded counting: key-range groups of about this many instances,
     * with (OKM_TEST_GROUP_EXACT = 0) one instance-bound table or (1) exact
     * per-group tables joined at the end */
    OKM_TEST_GROUP_KEYS = 3,
    OKM_TEST_GROUP_EXACT = 4,
    /* counts of sorted runs: 1 = the k-way merge kernel, 2 = the count kernels
     * in two passes (both otherwise taken only near the memory limit) */
    OKM_TEST_SORTED_PATH = 5,
    /* okm_merge_owned: 0 / 1 force u64 keys / 5-byte deltas on the wire; the
     * byte size of a message piece; the rank that fails while sizing its
     * receive buffers (after the size exchange, before any send) */
    OKM_TEST_WIRE_DELTAS = 6,
    OKM_TEST_PIECE_BYTES = 7,
    OKM_TEST_FAIL_RANK = 8,
    /* loopback communicator: ms a rank waits for its peers before aborting */
    OKM_TEST_LOOPBACK_TIMEOUT_MS = 9,
    /* okm_group_write_counts_tsv: entries per chunk copied off the GPUs */
    OKM_TEST_TSV_CHUNK = 10,
    /* parallel gzip inflate: smallest member (bytes), compressed bytes per
     * chunk, and 1 = a member the parallel path rejects is an error (instead
     * of a serial retry), also on one host thread */
    OKM_TEST_GZ_PAR_MIN_BYTES = 11,
    OKM_TEST_GZ_CHUNK_BYTES = 12,
    OKM_TEST_GZ_STRICT = 13,
    /* 1: never load libdeflate (zlib's inflate / deflate only); read when the
     * codec is first used in the process */
    OKM_TEST_NO_LIBDEFLATE = 14,
    /* device memory budget of the process's contexts in bytes (as OKM_HBM_CAP)
     * — a small GPU, for the out-of-memory paths */
    OKM_TEST_HBM_BUDGET_BYTES = 15,
    /* key-range groups of one batch write the table's keys over the batch's
     * own L1 run when memory-bounded counting splits them (the default);
     * 1 also with group_keys' forced groups, 0 never */
    OKM_TEST_GROUP_OVER = 16,
    OKM_TEST_KNOBS = 17
} okm_test_knob;

/* value < 0 unsets the knob (the product default). */
void okm_test_set(okm_test_knob knob, int64_t value);
/* The knob's value, -1 when unset. */
int64_t okm_test_get(okm_test_knob knob);

#ifdef __cplusplus
}
#endif
#endif /* ORION_KMER_TESTING_H */
