"""ctypes binding of the C restatement (oracle/okm_oracle.c).

TEST INFRASTRUCTURE ONLY — the checker for tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  Builds oracle/build/liboracle.so on demand with
gcc (oracle/Makefile).
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import c_uint32, POINTER, c_char_p, c_int, c_size_t, c_uint8, c_uint64, c_void_p
from typing import Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "okm_oracle.c")):
        build()
    lib = ctypes.CDLL(LIB)
    lib.oracle_seq_to_u64.restype = c_int
    lib.oracle_seq_to_u64.argtypes = [c_char_p, c_size_t, c_uint8, POINTER(c_uint64)]
    lib.oracle_reverse_complement_u64.restype = c_uint64
    lib.oracle_reverse_complement_u64.argtypes = [c_uint64, c_uint8]
    lib.oracle_canonical_u64.restype = c_uint64
    lib.oracle_canonical_u64.argtypes = [c_uint64, c_uint8]
    lib.oracle_u64_to_seq.restype = c_int
    lib.oracle_u64_to_seq.argtypes = [c_uint64, c_uint8, c_char_p]
    lib.oracle_normalize.restype = c_size_t
    lib.oracle_normalize.argtypes = [c_char_p, c_size_t, c_char_p]
    lib.oracle_counter_new.restype = c_void_p
    lib.oracle_counter_new.argtypes = [c_uint8]
    lib.oracle_counter_free.argtypes = [c_void_p]
    lib.oracle_counter_add_record.argtypes = [c_void_p, c_char_p, c_size_t, c_int]
    lib.oracle_counter_add_batch.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_int]
    lib.oracle_counter_add_pairs.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64]
    lib.oracle_counter_distinct.restype = c_uint64
    lib.oracle_counter_distinct.argtypes = [c_void_p]
    lib.oracle_counter_windows.restype = c_uint64
    lib.oracle_counter_windows.argtypes = [c_void_p]
    lib.oracle_counter_result.restype = c_uint64
    lib.oracle_counter_result.argtypes = [c_void_p, c_uint64, c_void_p, c_void_p, c_uint64]
    lib.oracle_seq_to_u128.restype = c_int
    lib.oracle_seq_to_u128.argtypes = [c_char_p, c_size_t, c_uint8, c_void_p]
    lib.oracle_counter_wide_new.restype = c_void_p
    lib.oracle_counter_wide_new.argtypes = [c_uint8]
    lib.oracle_counter_wide_free.argtypes = [c_void_p]
    lib.oracle_counter_wide_add_record.argtypes = [c_void_p, c_char_p, c_size_t, c_int]
    lib.oracle_counter_wide_add_batch.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_int]
    lib.oracle_counter_wide_add_pairs.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64]
    lib.oracle_counter_wide_add_separated_range.argtypes = [c_void_p, c_void_p, c_uint64, c_uint8, c_uint32,
                                                            c_uint64, c_uint64]
    lib.oracle_counter_wide_distinct.restype = c_uint64
    lib.oracle_counter_wide_distinct.argtypes = [c_void_p]
    lib.oracle_counter_wide_windows.restype = c_uint64
    lib.oracle_counter_wide_windows.argtypes = [c_void_p]
    lib.oracle_counter_wide_result.restype = c_uint64
    lib.oracle_counter_wide_result.argtypes = [c_void_p, c_uint64, c_void_p, c_void_p, c_uint64]
    lib.oracle_counter_add_separated_ranges.argtypes = [c_void_p, c_void_p, c_uint64, c_uint8, c_void_p, c_void_p,
                                                         c_uint32]
    lib.oracle_query_hits.argtypes = [c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_uint8, c_void_p]
    _lib = lib
    return lib


def query_hits(seqs: Sequence[bytes], set_keys: np.ndarray, k: int) -> np.ndarray:
    """query.rs:81-99 restated in C: per-record hit counts over RAW bytes
    against a sorted unique key array."""
    lib = load()
    data = np.frombuffer(b"".join(seqs), dtype=np.uint8) if seqs else np.zeros(0, np.uint8)
    offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
    np.cumsum([len(s) for s in seqs], out=offs[1:])
    keys = np.ascontiguousarray(set_keys, dtype=np.uint64)
    hits = np.zeros(len(seqs), dtype=np.uint32)
    lib.oracle_query_hits(data.ctypes.data, offs.ctypes.data, len(seqs), keys.ctypes.data, len(keys), k,
                          hits.ctypes.data)
    return hits


class OracleCounter:
    """count.rs:23-38 + :106-119 restated in C (O(k) per window, one core)."""

    def __init__(self, k: int):
        self.k = k
        self.h = load().oracle_counter_new(k)
        if not self.h:
            raise ValueError(f"Invalid K-mer size: {k}. Must be between 1 and 32.")

    def __del__(self):
        if getattr(self, "h", None):
            load().oracle_counter_free(self.h)
            self.h = None

    def add_records(self, seqs: Sequence[bytes], normalized: bool = False) -> None:
        for s in seqs:
            load().oracle_counter_add_record(self.h, s, len(s), 1 if normalized else 0)

    def add_batch(self, data: np.ndarray, offsets: np.ndarray, normalized: bool = False) -> None:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        load().oracle_counter_add_batch(self.h, data.ctypes.data, offsets.ctypes.data, len(offsets) - 1,
                                        1 if normalized else 0)

    def add_separated(self, data: np.ndarray, sep: int = ord("\n")) -> None:
        """A batch in the device layout (records joined by `sep`)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        cut = np.flatnonzero(data == sep)
        starts = np.concatenate([[0], cut + 1]).astype(np.uint64)
        ends = np.concatenate([cut, [len(data)]]).astype(np.uint64)
        keep = ends > starts
        # records are [start, end); express them as an offsets array over a
        # separator-free copy
        lens = (ends - starts)[keep]
        body = np.delete(data, cut) if len(cut) else data
        offs = np.zeros(len(lens) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum(lens)
        self.add_batch(body, offs, normalized=False)

    def add_separated_ranges(self, data: np.ndarray, ranges, sep: int = ord("\n")) -> None:
        """Restatement-MT helper (oracle_counter_add_separated_ranges): count
        only canonical keys inside one of the [lo, hi) `ranges` (rolling
        encode; every valid window still counts in `windows`)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        lo = np.ascontiguousarray([r[0] for r in ranges], dtype=np.uint64)
        hi = np.ascontiguousarray([r[1] for r in ranges], dtype=np.uint64)
        load().oracle_counter_add_separated_ranges(self.h, data.ctypes.data, len(data), sep, lo.ctypes.data,
                                                   hi.ctypes.data, len(lo))

    def add_pairs(self, keys: np.ndarray, counts: np.ndarray) -> None:
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        counts = np.ascontiguousarray(counts, dtype=np.uint64)
        load().oracle_counter_add_pairs(self.h, keys.ctypes.data, counts.ctypes.data, len(keys))

    @property
    def distinct(self) -> int:
        return int(load().oracle_counter_distinct(self.h))

    @property
    def windows(self) -> int:
        return int(load().oracle_counter_windows(self.h))

    def result(self, min_count: int = 1) -> Tuple[np.ndarray, np.ndarray]:
        n = self.distinct
        keys = np.empty(max(n, 1), dtype=np.uint64)
        counts = np.empty(max(n, 1), dtype=np.uint64)
        m = load().oracle_counter_result(self.h, min_count, keys.ctypes.data, counts.ctypes.data, n)
        return keys[:m].copy(), counts[:m].copy()


class OracleCounterWide(OracleCounter):
    """k in 33..64 (restatement-defined two-u64 extension): keys are (n, 2)
    uint64 arrays of [lo, hi] words, value = hi * 2**64 + lo."""

    def __init__(self, k: int):
        self.k = k
        self.h = load().oracle_counter_wide_new(k)
        if not self.h:
            raise ValueError(f"Invalid K-mer size: {k}. Must be between 1 and 64.")

    def __del__(self):
        if getattr(self, "h", None):
            load().oracle_counter_wide_free(self.h)
            self.h = None

    def add_records(self, seqs: Sequence[bytes], normalized: bool = False) -> None:
        for s in seqs:
            load().oracle_counter_wide_add_record(self.h, s, len(s), 1 if normalized else 0)

    def add_batch(self, data: np.ndarray, offsets: np.ndarray, normalized: bool = False) -> None:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        load().oracle_counter_wide_add_batch(self.h, data.ctypes.data, offsets.ctypes.data, len(offsets) - 1,
                                             1 if normalized else 0)

    def add_pairs(self, keys: np.ndarray, counts: np.ndarray) -> None:
        keys = np.ascontiguousarray(keys, dtype=np.uint64).reshape(-1, 2)
        counts = np.ascontiguousarray(counts, dtype=np.uint64)
        load().oracle_counter_wide_add_pairs(self.h, keys.ctypes.data, counts.ctypes.data, len(counts))

    def add_separated_range(self, data: np.ndarray, bits: int, lo: int, hi: int, sep: int = ord("\n")) -> None:
        """Normalised records joined by `sep`; only keys whose top `bits` bits
        lie in [lo, hi) are counted (rolling encode; range shards for large
        tests, see okm_oracle.c)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        load().oracle_counter_wide_add_separated_range(self.h, data.ctypes.data, len(data), sep, bits, lo, hi)

    @property
    def distinct(self) -> int:
        return int(load().oracle_counter_wide_distinct(self.h))

    @property
    def windows(self) -> int:
        return int(load().oracle_counter_wide_windows(self.h))

    def result(self, min_count: int = 1) -> Tuple[np.ndarray, np.ndarray]:
        n = self.distinct
        keys = np.empty((max(n, 1), 2), dtype=np.uint64)
        counts = np.empty(max(n, 1), dtype=np.uint64)
        m = load().oracle_counter_wide_result(self.h, min_count, keys.ctypes.data, counts.ctypes.data, n)
        return keys[:m].copy(), counts[:m].copy()


def count_separated_mt(data: np.ndarray, k: int, threads: int, sep: int = ord("\n")) -> Tuple[np.ndarray, np.ndarray]:
    """Restatement-MT (SURVEY.md §8(d) "cpu_ref --threads"): NOT the
    reference's behaviour — count.rs:68-79 is single-threaded — but the same
    per-window work split over host cores, as a labelled second CPU number.
    The batch (records joined by `sep`) is cut at record boundaries into
    `threads` shards, each counted by its own C counter on its own thread
    (ctypes drops the GIL), and the sorted per-shard tables are merged by key
    range, again one range per thread (numpy's sort drops the GIL too).
    Returns the sorted (keys, counts) of the whole batch, min_count 1."""
    import threading

    load()  # built / loaded once, before the threads
    data = np.ascontiguousarray(data, dtype=np.uint8)
    threads = max(1, int(threads))
    cut = np.flatnonzero(data == sep)
    # shard ends: the separator nearest each 1/threads point (a record never splits)
    ends = [0]
    for t in range(1, threads):
        i = int(np.searchsorted(cut, len(data) * t // threads))
        ends.append(int(cut[i]) + 1 if i < len(cut) else len(data))
    ends.append(len(data))
    tables = [None] * threads

    def count_shard(t: int) -> None:
        oc = OracleCounter(k)
        oc.add_separated(data[ends[t]:ends[t + 1]], sep)
        tables[t] = oc.result(1)

    ths = [threading.Thread(target=count_shard, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    # key-range merge: range r = keys in [b_r, b_{r+1}) of every shard's table
    bounds = np.linspace(0, float(1 << (2 * k)) if k < 32 else float(2 ** 64), threads + 1)
    bk = [np.uint64(min(int(b), 2 ** 64 - 1)) for b in bounds]
    parts = [None] * threads

    def merge_range(r: int) -> None:
        ks, cs = [], []
        for tk, tc in tables:
            lo = np.searchsorted(tk, bk[r], side="left") if r else 0
            hi = np.searchsorted(tk, bk[r + 1], side="left") if r + 1 < threads else len(tk)
            ks.append(tk[lo:hi])
            cs.append(tc[lo:hi])
        kk = np.concatenate(ks)
        cc = np.concatenate(cs)
        order = np.argsort(kk, kind="stable")
        kk, cc = kk[order], cc[order]
        if len(kk) == 0:
            parts[r] = (kk, cc)
            return
        first = np.concatenate([[True], kk[1:] != kk[:-1]])
        starts = np.flatnonzero(first)
        parts[r] = (kk[starts], np.add.reduceat(cc, starts).astype(np.uint64))

    ths = [threading.Thread(target=merge_range, args=(r,)) for r in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return (np.concatenate([p[0] for p in parts]).astype(np.uint64),
            np.concatenate([p[1] for p in parts]).astype(np.uint64))


def count_separated_wide_ranges(data: np.ndarray, k: int, threads: int, bits: int = 8, sep: int = ord("\n"),
                                shards: int = 0, on_range=None, bins=None):
    """k in 33..64 restatement sharded by key range for large tests (not
    reference behaviour: a labelled restatement-MT helper).  Every shard scans
    all of `data` (normalised records joined by `sep`) and counts only the
    canonical keys whose top `bits` bits fall in its contiguous bin range; the
    ranges are cut where the canonical-key density (min of a key and its
    reverse complement: f(x) = 2(1 - x) over the key range) gives each shard
    an equal share, and the per-range sorted tables concatenate in order.
    `threads` workers run `shards` (default: threads) shards; with `on_range`,
    on_range(lo, hi, keys, counts) gets each shard's table instead (nothing is
    kept); `bins`: explicit [(lo, hi), ...] ranges instead of the cover.
    Returns (keys (n, 2) [lo, hi] | None, counts | None, valid windows)."""
    from concurrent.futures import ThreadPoolExecutor
    nb = 1 << bits
    ns = shards or threads
    if bins is None:
        cuts = [0] + [min(nb, int(round(nb * (1.0 - (1.0 - t / ns) ** 0.5)))) for t in range(1, ns)] + [nb]
        cuts = sorted(set(cuts))
        bins = list(zip(cuts[:-1], cuts[1:]))
    data = np.ascontiguousarray(data, dtype=np.uint8)

    def shard(r):
        oc = OracleCounterWide(k)
        oc.add_separated_range(data, bits, r[0], r[1], sep)
        keys, counts = oc.result(1)
        w = oc.windows
        del oc
        if on_range is not None:
            on_range(r[0], r[1], keys, counts)
            return None, None, w
        return keys, counts, w

    with ThreadPoolExecutor(max_workers=max(1, min(threads, len(bins)))) as ex:
        parts = list(ex.map(shard, bins))
    w = parts[0][2] if parts else 0
    if on_range is not None:
        return None, None, w
    keys = np.concatenate([p[0] for p in parts]) if parts else np.zeros((0, 2), np.uint64)
    counts = np.concatenate([p[1] for p in parts]) if parts else np.zeros(0, np.uint64)
    return keys, counts, w


def count_separated_ranges_mt(chunks, k: int, ranges, threads: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """Restatement-MT helper for full-size parity (not reference behaviour: a
    labelled helper): the canonical keys inside `ranges` ([lo, hi) pairs) of
    every window of the batch chunks yielded by `chunks` (device layout,
    records joined by '\n', each chunk ending at a record boundary), each
    chunk split at record boundaries over `threads` counters.  Returns the
    sorted (keys, counts) restricted to the ranges, and the valid windows of
    all chunks."""
    import threading

    load()
    threads = max(1, int(threads))
    ctrs = [OracleCounter(k) for _ in range(threads)]
    for data in chunks:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        cut = np.flatnonzero(data == ord("\n"))
        ends = [0]
        for t in range(1, threads):
            i = int(np.searchsorted(cut, len(data) * t // threads))
            ends.append(int(cut[i]) + 1 if i < len(cut) else len(data))
        ends.append(len(data))
        ths = [threading.Thread(target=ctrs[t].add_separated_ranges, args=(data[ends[t]:ends[t + 1]], ranges))
               for t in range(threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    parts = [c.result(1) for c in ctrs]
    windows = sum(c.windows for c in ctrs)
    kk = np.concatenate([p[0] for p in parts])
    cc = np.concatenate([p[1] for p in parts])
    if len(kk) == 0:
        return kk.astype(np.uint64), cc.astype(np.uint64), windows
    order = np.argsort(kk, kind="stable")
    kk, cc = kk[order], cc[order]
    first = np.concatenate([[True], kk[1:] != kk[:-1]])
    starts = np.flatnonzero(first)
    return kk[starts].astype(np.uint64), np.add.reduceat(cc, starts).astype(np.uint64), windows
