// okm_internal.h — internal declarations shared by the library's translation
// units (not part of the C ABI).
#pragma once

#include <stdint.h>
#include <stddef.h>
#include <string>
#include <vector>

#include "orion_kmer.h"

namespace okm {

// thread-local last error (okm_last_error)
void set_error(const std::string &msg);
okm_status fail(okm_status s, const std::string &msg);

constexpr uint64_t kEmptyKey = ~0ull;

// Page-locked host memory (hipHostMalloc) for the host translation units
// (okm_group.cpp's device-to-file stream); nullptr on failure.
void *host_pinned_alloc(size_t bytes);
void host_pinned_free(void *p);
// Device-to-host copy issued on `device` (this thread's current device is set
// to it first, so the copy does not queue behind device 0's null stream).
okm_status memcpy_d2h_on(int device, void *dst, const void *src, size_t bytes);
// Test hook value (orion_kmer_testing.h okm_test_knob), -1 when unset.
int64_t test_knob(int knob);

// Give back the idle device memory every context's pool on `device` caches
// (a hipMalloc outside the pools, e.g. a communicator buffer, retries after it).
void trim_device_pools(int device);
// Device bytes held outside the arenas (communicator buffers) count against
// the per-device budget too: +bytes when allocated, -bytes when freed.
void device_bytes_add(int device, int64_t delta);
// Would `bytes` more device memory pass the per-device budget (OKM_HBM_CAP)?
bool device_over_budget(int device, size_t bytes);

// The counted table where it lies: device memory, or (*on_host) page-locked
// host memory when count_spilled left it there (okm_group_write_counts_tsv
// streams either without moving it).
okm_status result_view(okm_ctx *c, const uint64_t **keys, const uint64_t **counts, uint64_t *n, bool *on_host);
// okm_merge_owned at one rank: the owner takes the local context's table
// without a copy (the two swap device pools); the local is left reset.
okm_status adopt_result(okm_ctx *owner, okm_ctx *local, bool *adopted);

// Context accessors for the other translation units (okm_probe.hip).
int ctx_device(const okm_ctx *c);
bool ctx_is_wide(const okm_ctx *c);  // never a canonical key
uint32_t ctx_k(const okm_ctx *c);
// Key density of the next count's sorted runs (okm_merge_owned's owner): pairs
// per top-`fine_bits` key bin over the whole key space (zero outside the
// owner's range).  count_sorted_plan sizes each L1 part's split from the
// densest of its fine bins, so the first plan fits; okm_reset / the count
// clear it.  fine == nullptr clears.
void set_sorted_hint(okm_ctx *c, const unsigned long long *fine, uint32_t fine_bits);
bool ctx_is_set(const okm_ctx *c);

// ----------------------------------------------------------------------------
// Device-side launchers (okm_device.hip).  All take a hipStream_t as void*.
// ----------------------------------------------------------------------------

// A run of keys in device memory (optionally weighted).
struct DevSeg {
    const uint64_t *keys;
    const uint64_t *counts;  // nullptr => every key weighs 1
    uint64_t len;
    uint64_t key_base;       // (key >> shift) - key_base = local bin in [0, nlocal)
    uint32_t out_base;       // first output bin of this segment (compact numbering)
    uint32_t shift;          // kSingleBin (255) => a single bin
    uint32_t nlocal;         // bins this segment splits into (<= pass maximum)
    uint32_t pad;
};

// One unit of partition-pass work: a slice of a segment.
struct DevChunk {
    uint32_t seg;
    uint32_t pad;
    uint64_t begin;
    uint64_t len;
};

// One partition to count in LDS: segs[seg_begin, seg_begin + seg_count).
constexpr uint32_t kItemEmpty = 1;

struct DevItem {
    uint32_t seg_begin;
    uint32_t seg_count;
    uint64_t out_off;        // where its sorted distinct entries go (scratch)
    uint32_t rem_bits;       // key bits below the item's common prefix
    uint32_t pad;            // kItemEmpty: an empty fan-out slot (no segment read)
    uint64_t total;          // instances over all its segments
    const uint64_t *keys0;   // seg_count == 1: its segment's keys / counts (no
    const uint64_t *counts0; //   dependent segment load in the count kernels)
};

// Sampled L1 placement: bin b's claim cursor lives at cursor[b * kL1CurStride]
// (a stride > 1, every cursor on its own 128-B line, measured no faster).
constexpr uint32_t kL1CurStride = 1;

struct ExtractGeom {
    uint64_t n;        // bytes in the batch
    uint32_t k;
    uint32_t shift;    // bin = key >> shift (64 => single bin)
    uint32_t nbins;    // 1 << l1 bits
    uint32_t nblocks;  // persistent blocks (chunks)
    uint64_t chunk;    // window starts per block (multiple of the tile)
    uint32_t stride;   // block b covers chunk b * stride (> 1: a sample of the batch)
};

// L1: k-mer extraction from a batch, histogram by top key bits.
void launch_extract_hist(void *stream, const uint8_t *seq, const ExtractGeom &g, uint32_t *HC,
                         unsigned long long *Hg);
// L1: k-mer extraction + scatter into key-range partitions.  HC != null:
// exact placement from launch_extract_hist's per-block counts.  HC == null:
// sampled capacities (launch_l1_capacity), one claim per (tile, bin); a run
// crossing cap_end[bin] is dropped and *ovf set (the caller redoes the batch).
void launch_extract_scatter(void *stream, const uint8_t *seq, const ExtractGeom &g,
                            const uint32_t *HC, unsigned long long *cursor, uint64_t *out_keys,
                            const unsigned long long *cap_end, unsigned long long *ovf);
void launch_l1_capacity(void *stream, const unsigned long long *Hs, uint32_t nb, double scale, double mul,
                        uint32_t align, unsigned long long limit, unsigned long long *cursor,
                        unsigned long long *l1cap);

// Generic key-range partition pass over a chunk list.  max_local bounds every
// segment's nlocal; HC is nchunks x max_local (null: only Hg, e.g. a sample).
// wide: keys are K128 (two u64 each; pointers stay uint64_t*, lengths count keys).
void launch_part_hist(void *stream, const DevSeg *segs, const DevChunk *chunks, uint32_t nchunks,
                      uint32_t max_local, uint32_t *HC, unsigned long long *Hg, bool wide);
// HC null (tile mode only): sampled capacities, bin b's slot ends at
// cap_end[b]; one claim per (tile, bin), a crossing run is dropped and *ovf set.
void launch_part_scatter(void *stream, const DevSeg *segs, const DevChunk *chunks,
                         uint32_t nchunks, uint32_t max_local, const uint32_t *HC,
                         unsigned long long *cursor, uint64_t *out_keys, uint64_t *out_counts, bool wide,
                         const unsigned long long *cap_end = nullptr, unsigned long long *ovf = nullptr);
// Sampled partition capacities: H[b] (sampled count of output bin b) becomes
// the bin's capacity (in place); parents sorted by out_base.
struct DevCapParent {
    uint32_t out_base;
    uint32_t pad;
    double scale;            // parent keys / sampled parent keys
};
void launch_part_capacity(void *stream, unsigned long long *H, uint32_t nout, const DevCapParent *parents,
                          uint32_t nparents, double mul);
// Pads [end[b], roundup(end[b], line)) of every bin with the empty key (bins
// start on 128-B lines: 16 u64 / 8 K128 keys; end = the cursor after the scatter).
// cap (optional): skip bins whose end passed cap[b] (an overflowed sampled placement).
void launch_fill_line_tails(void *stream, const unsigned long long *end, uint32_t nbins, uint64_t *keys, bool wide,
                            const unsigned long long *cap = nullptr);
uint32_t extract_tile();
uint32_t extract_max_bins(bool wide);  // L1 bins: k <= 32 kernels vs k in 33..64
// L1 key bits a context extracts with: wide keys, or k <= 32 counting batch by
// batch (9) vs folding many batches into one table (10)
uint32_t extract_l1_bits(bool wide, bool folding);
uint32_t part_max_bins(bool weighted, bool wide);

// Exclusive scan of n u64 values (in -> out, out may equal in); tmp >= scan_tmp_elems(n).
size_t scan_tmp_elems(uint64_t n);
void launch_exclusive_scan(void *stream, const unsigned long long *in, unsigned long long *out,
                           uint64_t n, unsigned long long *tmp);

// LDS counting of partitions (okm_count.hip); writes sorted distinct
// (key,count) at out_off and n_out[item] (counts u32 unless weighted).  ctl[0] = error word, ctl[1] =
// deferred-item count (both zeroed before the launch).  An item holds at most count_item_capacity() instances unless
// its rem_bits <= count_dense_bits() (direct-address counting, any size).
uint32_t count_item_capacity();
uint32_t count_dense_bits();
// ctl[1] counts deferred items (list `defer`, nitems entries) for the second
// kernel of the launch.
void launch_count_items(void *stream, const DevItem *items, uint32_t nitems, const DevSeg *segs,
                        uint64_t *out_keys, uint64_t *out_counts, unsigned long long *n_out,
                        unsigned long long *ctl, uint32_t *defer, bool weighted, bool wide,
                        const unsigned long long *guard = nullptr, const unsigned long long *d_nitems = nullptr,
                        bool nowrite = false,  // nowrite: n_out only (weighted or wide launches)
                        bool narrow = false);
// Wide keys straight into a caller's table (okm_count.hip: items by ticket,
// each run at its look-back prefix; no staging, no compaction).  status:
// nitems words and ctl[0..1] zeroed by the caller; fin_keys / fin_counts at
// the table's next entry, or at its start when fin_base (device) holds it.
void launch_count_direct(void *stream, const DevItem *items, uint32_t nitems, const DevSeg *segs,
                         unsigned long long *n_out, unsigned long long *ctl, bool weighted,
                         const unsigned long long *guard, const unsigned long long *d_nitems,
                         unsigned long long *status, uint64_t *fin_keys, uint64_t *fin_counts,
                         const unsigned long long *fin_base);  // weighted: u32 staged counts (ctl[0] |= 8 when one does not fit)

// k-way merge of sorted runs (okm_merge.hip): items as built by
// launch_sorted_items (each segment of an item a sorted unique run of keys),
// at most merge_item_capacity() instances and merge_max_runs() segments per
// item (else ctl[0] = 3).  write=0: n_out[item] = the item's distinct keys;
// write=1: its sorted distinct keys and summed u64 counts at
// out_keys/out_counts + dense_off[item] (the exclusive scan of n_out).
uint32_t merge_item_capacity();
uint32_t merge_max_runs();
void launch_merge_items(void *stream, const DevItem *items, uint32_t nitems, const DevSeg *segs,
                        unsigned long long *n_out, const unsigned long long *dense_off, uint64_t *out_keys,
                        uint64_t *out_counts, unsigned long long *ctl, bool weighted, bool wide, bool write);

// A part that took part in a device-side split round: its children are the
// output bins [out_base, out_base + nlocal) of the round.
struct DevParent {
    uint32_t out_base;
    uint32_t rem;            // key bits below the children's common prefix
};

// Fan-out of a round's children (k_fan_split): a child larger than one item
// (but <= split_max) is split in place by its next 1..bits key bits (the
// fewest that bring it to <= target); every child owns 2^bits item slots in
// key order, slots past its own sub-ranges are empty items.
struct DevFanJob {
    uint64_t off, len;
    uint32_t item0, bits, rem, pad;
    uint64_t doff;  // the child's first staged output slot (dense: the scan of child lengths)
};
struct FanOut {
    uint32_t bits = 0;          // 0: one item per child (no fan-out)
    uint32_t pad = 0;
    uint64_t target = 0;        // sub-range size aimed at
    uint64_t split_max = 0;     // largest child one job takes (fan_split_max())
    DevFanJob *jobs = nullptr;  // [nout]; job count in flags[3]
};
uint64_t fan_split_max();
// Unweighted jobs of at most this many keys are split in place (dk == sk):
// the register variant reads a job's keys before it writes any.
uint64_t fan_split_max_in_place();

// d_nitems (count kernels, compaction): when given, the item count is
// min(nitems, *d_nitems) -- a count known only on the device.

// One item (and one segment) per output bin of a split round, straight from
// the device offsets (nout + 1 entries; bin b ends at ends[b], or at
// offs[b + 1] when ends is null).  flags[0] += children that are still too
// big for one item; flags[1] |= 2 when a child needs 64-bit counting;
// flags[2] = max child length; flags[3] / flags[4] = fan-out jobs of <= / >
// 16 Ki keys (filed from the front / the back of fan.jobs[nout]).  Count and compact
// kernels given `guard` (= flags) return at once when guard[0] or guard[1] is
// set.  With fan.bits, item/segment slot i * 2^bits + j belongs to child i.
// doff (optional): every child's first staged output slot, the exclusive scan
// of the child lengths (launch_child_offsets) -- items then stage their
// (key, count) runs densely (L.total slots) instead of at their level offsets
// (the level's padded size).
void launch_make_items(void *stream, const unsigned long long *offs, const unsigned long long *ends, uint32_t nout,
                       const DevParent *parents, uint32_t nparents, const uint64_t *lk, const uint64_t *lc,
                       DevItem *items, DevSeg *segs, uint64_t item_max, uint32_t capbits,
                       unsigned long long *flags, uint32_t kw, const FanOut &fan,
                       const unsigned long long *doff = nullptr);
// doff[b] = sum of the lengths of children < b (b = 0..nout); tmp >= scan_tmp_elems(nout + 1).
void launch_child_offsets(void *stream, const unsigned long long *offs, const unsigned long long *ends, uint32_t nout,
                          unsigned long long *doff, unsigned long long *tmp);
// The fan-out jobs (flags[3] of them, <= max_jobs): keys of [off, off + len)
// of sk/sc are split into the same range of dk/dc and their sub-items written;
// oflags[0] += sub-ranges still too big, oflags[2] = max sub-range.
void launch_fan_split(void *stream, const DevFanJob *jobs, uint32_t max_jobs, const unsigned long long *flags,
                      const uint64_t *sk, const uint64_t *sc, uint64_t *dk, uint64_t *dc, DevItem *items,
                      DevSeg *segs, uint64_t item_max, uint32_t capbits, unsigned long long *oflags, bool wide);

// Sorted runs (okm_add_sorted_pairs_device).  out[b] = first index whose
// (key >> shift) >= b, b = 0..nbins (out[nbins] = n).
void launch_bin_bounds(void *stream, const uint64_t *keys, uint64_t n, uint32_t shift, uint32_t nbins,
                       unsigned long long *out, bool wide);
struct DevSortedPart {
    uint32_t bin;        // L1 bin of the part
    uint32_t bits;       // split into 2^bits children (0: one item)
    uint32_t item_base;  // first item of its children
    uint32_t slot;       // row of the part in the rbins table
};
// One multi-segment item per child (bounds: nitems * nruns words of scratch):
// segs[i * nruns + r] = the child's key range
// in run r (rbins[slot * nruns + r] = the part's range in run r); itemtot[i]
// = its instances; flags[0] += children still too big, flags[1] = max;
// part_max[slot] = the part's largest child (per-part replanning).
void launch_sorted_items(void *stream, const DevSortedPart *parts, uint32_t nparts, uint32_t nitems,
                         const DevSeg *rbins, uint32_t nruns, uint32_t shift1, DevItem *items, DevSeg *segs,
                         unsigned long long *itemtot, uint64_t item_max, uint32_t capbits, unsigned long long *flags,
                         bool wide, unsigned long long *bounds, unsigned long long *part_max);
void launch_set_out_off(void *stream, DevItem *items, uint32_t nitems, const unsigned long long *off);

// Gather the per-item results into dense arrays given exclusive offsets
// (nothing when a guard word or *err is set).  narrow: the per-item counts
// are u32 (unweighted count launches), widened to u64 here.
void launch_compact_items(void *stream, const DevItem *items, uint32_t nitems,
                          const unsigned long long *n_out, const unsigned long long *dense_off,
                          const uint64_t *src_keys, const uint64_t *src_counts,
                          uint64_t *dst_keys, uint64_t *dst_counts, bool wide, bool narrow,
                          const unsigned long long *guard = nullptr, const unsigned long long *err = nullptr,
                          const unsigned long long *d_nitems = nullptr, const unsigned long long *d_base = nullptr);
// Pipelined key-range groups: bit 63 of the device-side table base marks a
// pass in which a group was abandoned; no later group writes then.
constexpr unsigned long long kBasePoison = 1ull << 63;
// d_base (pipelined key-range groups): the compaction writes at dst + *d_base,
// and launch_advance_base then adds the group's distinct keys (*total) to it
// -- nothing of either when a guard word or *err is set.
void launch_advance_base(void *stream, unsigned long long *d_base, const unsigned long long *total,
                         const unsigned long long *guard, const unsigned long long *err);
// Drop the empty fan-out slots of items[0, nslots) (order kept) into out;
// *d_nitems (= pos[nslots]) receives the number kept.  flags/pos: nslots + 1
// words each, scan_tmp: scan_tmp_elems(nslots + 1).
void launch_item_compact(void *stream, const DevItem *items, uint32_t nslots, DevItem *out,
                         unsigned long long *flags, unsigned long long *pos, unsigned long long *scan_tmp);

// Filter (count >= min) with order preserved; flags/scan in tmp.
void launch_filter_count(void *stream, const uint64_t *counts, uint64_t n, uint64_t min_count,
                         unsigned long long *block_counts, uint32_t nblocks_hint);
void launch_filter_scatter(void *stream, const uint64_t *keys, const uint64_t *counts, uint64_t n,
                           uint64_t min_count, const unsigned long long *block_offsets,
                           uint64_t *dst_keys, uint64_t *dst_counts, bool wide);
uint32_t filter_blocks(uint64_t n);

// |A ∩ B| of sorted unique arrays (merge-path style binary search per element).
void launch_intersect_count(void *stream, const uint64_t *a, uint64_t na, const uint64_t *b,
                            uint64_t nb, unsigned long long *out, bool wide);

}  // namespace okm
