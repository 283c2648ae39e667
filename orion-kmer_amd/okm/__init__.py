"""okm — Python host layer over the MI355X k-mer engine (liborion_kmer.so).

Mirrors the reference's library surface (``orion_kmer::kmer`` pub fns,
``kmer.rs:37-106``) and its ``count``/``build``/``compare``/``query``/``classify``
drivers (``commands/count.rs:40-141``, ``build.rs:80-160``, ``compare.rs:29-97``,
``query.rs:24-134``, ``classify.rs:58-385``) so
tests read like the reference's own.  All compute goes through the C ABI; the
engine itself is HIP on gfx950 and has no CPU fallback.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, byref, c_char_p, c_int, c_uint64, c_void_p
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import (OKM_E_DEVICE, OKM_E_INVALID_K, OKM_E_IO, OKM_E_PARSE, OKM_E_RECORD,
                   OKM_MODE_COUNT, OKM_MODE_SET, OKM_MODE_WIDE, OKM_OK, RECORD_SEPARATOR, OkmError, check)

__all__ = [
    "seq_to_u64", "u64_to_seq", "reverse_complement_u64", "canonical_u64",
    "KmerCounter", "DeviceBuffer", "device_count", "device_arch", "pack_records",
    "parse_fastx", "read_fastx_file", "write_counts_tsv", "synth_reads", "synth_reads_device", "synth_long_reads",
    "run_count", "run_build", "run_compare", "KmerDb", "OkmError",
    "KmerSet", "Classifier", "run_query", "run_classify", "read_fastx_records",
    "Comm", "comm_unique_id", "owner_bounds", "synth_reads_device", "distributed_compare",
]


def lib():
    return _lib.load()


# ---------------------------------------------------------------------------
# kmer.rs pub fns (CPU parity surface)
# ---------------------------------------------------------------------------

def seq_to_u64(seq: bytes, k: int) -> Optional[int]:
    """kmer.rs:37-57."""
    out = c_uint64(0)
    if k < 0 or k > 255:
        return None
    ok = lib().okm_seq_to_u64(bytes(seq), len(seq), k, byref(out))
    return out.value if ok else None


def u64_to_seq(v: int, k: int) -> bytes:
    """kmer.rs:61-75 (raises ValueError where the reference panics)."""
    if k <= 0 or k > 32:
        raise ValueError(f"Invalid k-mer length for decoding: {k}")
    buf = ctypes.create_string_buffer(k)
    lib().okm_u64_to_seq(v, k, buf)
    return buf.raw


def reverse_complement_u64(v: int, k: int) -> int:
    """kmer.rs:79-94 (raises ValueError where the reference panics)."""
    if k <= 0 or k > 32:
        raise ValueError(f"Invalid k-mer length for reverse complement: {k}")
    return int(lib().okm_reverse_complement_u64(v, k))


def canonical_u64(v: int, k: int) -> int:
    """kmer.rs:99-106."""
    if k <= 0 or k > 32:
        raise ValueError(f"Invalid k-mer length for reverse complement: {k}")
    return int(lib().okm_canonical_u64(v, k))


def _k128(v: int) -> "_lib.Key128":
    return _lib.Key128(v & 0xFFFFFFFFFFFFFFFF, v >> 64)


def seq_to_u128(seq: bytes, k: int) -> Optional[int]:
    """k in 1..64 extension of seq_to_u64 (restatement-defined for k > 32)."""
    out = _lib.Key128(0, 0)
    if k < 0 or k > 255:
        return None
    ok = lib().okm_seq_to_u128(bytes(seq), len(seq), k, byref(out))
    return (out.hi << 64 | out.lo) if ok else None


def u128_to_seq(v: int, k: int) -> bytes:
    if k <= 0 or k > 64:
        raise ValueError(f"Invalid k-mer length for decoding: {k}")
    buf = ctypes.create_string_buffer(k)
    lib().okm_u128_to_seq(_k128(v), k, buf)
    return buf.raw


def reverse_complement_u128(v: int, k: int) -> int:
    if k <= 0 or k > 64:
        raise ValueError(f"Invalid k-mer length for reverse complement: {k}")
    r = lib().okm_reverse_complement_u128(_k128(v), k)
    return r.hi << 64 | r.lo


def canonical_u128(v: int, k: int) -> int:
    if k <= 0 or k > 64:
        raise ValueError(f"Invalid k-mer length for reverse complement: {k}")
    r = lib().okm_canonical_u128(_k128(v), k)
    return r.hi << 64 | r.lo


def keys128_to_int(keys: np.ndarray) -> List[int]:
    """(n, 2) [lo, hi] uint64 key arrays -> Python ints."""
    keys = np.asarray(keys, dtype=np.uint64).reshape(-1, 2)
    return [(int(h) << 64) | int(l) for l, h in keys]


# ---------------------------------------------------------------------------
# device
# ---------------------------------------------------------------------------

def device_count() -> int:
    return int(lib().okm_device_count())


def device_arch(device: int = 0) -> str:
    return (lib().okm_device_arch(device) or b"").decode()


class DeviceBuffer:
    """Raw device allocation owned by Python (for device-resident batches)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.ptr = c_void_p()
        self.nbytes = int(nbytes)
        check(lib().okm_device_alloc(device, self.nbytes, byref(self.ptr)), "okm_device_alloc")

    def upload(self, host: np.ndarray) -> None:
        host = np.ascontiguousarray(host)
        assert host.nbytes <= self.nbytes
        check(lib().okm_memcpy_h2d(self.ptr, host.ctypes.data, host.nbytes), "okm_memcpy_h2d")

    def download(self, host: np.ndarray) -> None:
        assert host.flags.c_contiguous and host.nbytes <= self.nbytes
        check(lib().okm_memcpy_d2h(host.ctypes.data, self.ptr, host.nbytes), "okm_memcpy_d2h")

    @property
    def address(self) -> int:
        return int(self.ptr.value or 0)

    def free(self) -> None:
        if self.ptr:
            lib().okm_device_free(self.ptr)
            self.ptr = c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# record batches
# ---------------------------------------------------------------------------

def pack_records(seqs: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """(bytes, offsets[n+1]) for okm_add_batch."""
    offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
    if seqs:
        offs[1:] = np.cumsum([len(s) for s in seqs], dtype=np.uint64)
    data = np.frombuffer(b"".join(seqs), dtype=np.uint8) if seqs else np.zeros(0, np.uint8)
    return data.copy(), offs


def parse_fastx(data: bytes) -> List[bytes]:
    """Normalised sequences of a FASTA/FASTQ buffer (needletail semantics)."""
    seq = c_void_p()
    off = c_void_p()
    n = c_uint64()
    check(lib().okm_parse_buffer(data, len(data), byref(seq), byref(off), byref(n)), "okm_parse_buffer")
    try:
        offs = np.ctypeslib.as_array(ctypes.cast(off, POINTER(c_uint64)), shape=(n.value + 1,)).copy()
        total = int(offs[-1])
        raw = ctypes.string_at(seq, total) if total else b""
        return [raw[int(offs[i]):int(offs[i + 1])] for i in range(n.value)]
    finally:
        lib().okm_free_result(seq)
        lib().okm_free_result(off)


def read_fastx_file(path: str, decompress_by_extension: bool = True) -> List[bytes]:
    """All normalised records of a file via the C reader (count: True, build: False)."""
    r = c_void_p()
    check(lib().okm_reader_open(byref(r), path.encode(), 1 if decompress_by_extension else 0),
          f"okm_reader_open({path})")
    out: List[bytes] = []
    try:
        while True:
            seq = c_void_p()
            off = c_void_p()
            n = c_uint64()
            check(lib().okm_reader_next(r, 64 << 20, byref(seq), byref(off), byref(n)), "okm_reader_next")
            if n.value == 0:
                break
            offs = np.ctypeslib.as_array(ctypes.cast(off, POINTER(c_uint64)), shape=(n.value + 1,)).copy()
            raw = ctypes.string_at(seq, int(offs[-1])) if int(offs[-1]) else b""
            out.extend(raw[int(offs[i]):int(offs[i + 1])] for i in range(n.value))
    finally:
        lib().okm_reader_close(r)
    return out


def read_file(path: str, decompress_by_extension: bool = True) -> bytes:
    """A whole file through the library's reader (okm_read_file: .gz / .xz /
    .zst by extension, utils.rs:125-152; single-member gzip inflated on the
    host threads, okm_inflate.cpp)."""
    data = c_void_p()
    n = c_uint64()
    check(lib().okm_read_file(path.encode(), 1 if decompress_by_extension else 0, byref(data), byref(n)),
          f"okm_read_file({path})")
    try:
        return ctypes.string_at(data, n.value) if n.value else b""
    finally:
        lib().okm_free_result(data)


def write_counts_tsv(path: str, k: int, keys: np.ndarray, counts: np.ndarray) -> None:
    """keys: uint64 (k <= 32) or (n, 2) [lo, hi] (k in 33..64)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    counts = np.ascontiguousarray(counts, dtype=np.uint64)
    check(lib().okm_write_counts_tsv(path.encode(), k, keys.ctypes.data, counts.ctypes.data, len(counts)),
          "okm_write_counts_tsv")


def synth_reads(n_reads: int, read_len: int = 150, genome_len: int = 100_000_000, genome_seed: int = 2,
                seed: int = 2, first_read: int = 0, sub_rate: float = 0.001, n_rate: float = 0.0001,
                threads: int = 0) -> np.ndarray:
    """Seeded reads in the device batch layout (each read + '\\n')."""
    out = np.empty(n_reads * (read_len + 1), dtype=np.uint8)
    check(lib().okm_synth_reads(genome_seed, genome_len, seed, first_read, n_reads, read_len, sub_rate,
                                n_rate, out.ctypes.data, threads), "okm_synth_reads")
    return out


def synth_reads_device(d_out: int, n_reads: int, read_len: int = 150, genome_len: int = 100_000_000,
                       genome_seed: int = 2, seed: int = 2, first_read: int = 0, sub_rate: float = 0.001,
                       n_rate: float = 0.0001, device: int = 0) -> int:
    """synth_reads' bytes generated straight into device memory at d_out
    (n_reads * (read_len + 1) bytes); returns that byte count."""
    check(lib().okm_synth_reads_device(genome_seed, genome_len, seed, first_read, n_reads, read_len, sub_rate,
                                       n_rate, c_void_p(d_out), device), "okm_synth_reads_device")
    return n_reads * (read_len + 1)


def synth_long_reads(gbases: float, genome_len: int, genome_seed: int = 4, seed: int = 4,
                     median_len: float = 2891.0, sigma: float = 1.085, min_len: int = 200, max_len: int = 100_000,
                     sub_rate: float = 0.025, ins_rate: float = 0.0125, del_rate: float = 0.0125,
                     threads: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """ONT-like reads of at least `gbases` bases in the device batch layout
    (okm_synth_long_reads; BASELINE configs[3] / SURVEY §8(d) C4: lognormal
    lengths, median 2,891, sigma 1.085, 200..100k; 5 % errors split into
    substitutions 2.5 %, insertions 1.25 %, deletions 1.25 %).  Returns
    (batch, read lengths)."""
    target = int(gbases * 1e9)
    n_guess = max(16, int(target / (median_len * np.exp(sigma * sigma / 2))) + 1)
    while True:  # enough reads for the target (lengths only, cheap)
        lens = np.zeros(n_guess, np.uint32)
        nb = c_uint64()
        check(lib().okm_synth_long_reads(genome_seed, genome_len, seed, 0, n_guess, median_len, sigma, min_len,
                                         max_len, sub_rate, ins_rate, del_rate, None, byref(nb),
                                         lens.ctypes.data, threads), "okm_synth_long_reads")
        csum = np.cumsum(lens, dtype=np.uint64)
        if int(csum[-1]) >= target:
            n = int(np.searchsorted(csum, target)) + 1
            break
        n_guess *= 2
    ptr = c_void_p()
    nb = c_uint64()
    check(lib().okm_synth_long_reads(genome_seed, genome_len, seed, 0, n, median_len, sigma, min_len, max_len,
                                     sub_rate, ins_rate, del_rate, byref(ptr), byref(nb), None, threads),
          "okm_synth_long_reads")
    try:
        out = np.ctypeslib.as_array(ctypes.cast(ptr, POINTER(ctypes.c_uint8)), shape=(nb.value,)).copy()
    finally:
        lib().okm_free_result(ptr)
    return out, lens[:n].astype(np.int64)


# ---------------------------------------------------------------------------
# counting context
# ---------------------------------------------------------------------------

class KmerCounter:
    """The GPU replacement of ``DashMap<u64, AtomicUsize>`` (count.rs:48) and
    of process_sequence_chunk (count.rs:23-38).  mode='set' mirrors build.rs's
    DashSet.  k in 33..64 needs wide=True (the opt-in two-u64 extension; the
    reference rejects k > 32): keys are then (n, 2) uint64 arrays [lo, hi]."""

    def __init__(self, k: int, mode: str = "count", device: int = 0, distinct_hint: int = 0,
                 wide: bool = False):
        self.k = k
        self.device = device
        self.wide = bool(wide) and k > 32
        self.ctx = c_void_p()
        m = OKM_MODE_SET if mode == "set" else OKM_MODE_COUNT
        if wide:
            m |= OKM_MODE_WIDE
        check(lib().okm_create(byref(self.ctx), k, m, device, distinct_hint), "okm_create")

    def close(self) -> None:
        if self.ctx:
            lib().okm_destroy(self.ctx)
            self.ctx = c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self) -> None:
        check(lib().okm_reset(self.ctx), "okm_reset")

    def trim(self) -> None:
        """Return the context's cached device blocks (okm_trim)."""
        check(lib().okm_trim(self.ctx), "okm_trim")

    def add_records(self, seqs: Sequence[bytes], normalized: bool = False) -> None:
        data, offs = pack_records(list(seqs))
        self.add_batch(data, offs, normalized)

    def add_batch(self, data: np.ndarray, offsets: np.ndarray, normalized: bool = False) -> None:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(offsets) - 1
        if n <= 0:
            return
        check(lib().okm_add_batch(self.ctx, data.ctypes.data, offsets.ctypes.data, n, 1 if normalized else 0),
              "okm_add_batch")

    def add_device_batch(self, d_ptr: int, nbytes: int) -> None:
        check(lib().okm_add_batch_device(self.ctx, c_void_p(d_ptr), nbytes), "okm_add_batch_device")

    def add_pairs(self, keys: np.ndarray, counts: Optional[np.ndarray] = None) -> None:
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        n = keys.shape[0] if not self.wide else keys.size // 2
        if counts is not None:
            counts = np.ascontiguousarray(counts, dtype=np.uint64)
        check(lib().okm_add_pairs(self.ctx, keys.ctypes.data,
                                  counts.ctypes.data if counts is not None else None, n),
              "okm_add_pairs")

    def add_pairs_device(self, d_keys: int, d_counts: Optional[int], n: int) -> None:
        check(lib().okm_add_pairs_device(self.ctx, c_void_p(d_keys), c_void_p(d_counts) if d_counts else None, n),
              "okm_add_pairs_device")

    def add_sorted_pairs_device(self, d_keys: int, d_counts: Optional[int], n: int) -> None:
        """Strictly ascending keys in device memory, borrowed until count()."""
        check(lib().okm_add_sorted_pairs_device(self.ctx, c_void_p(d_keys), c_void_p(d_counts) if d_counts else None,
                                                n), "okm_add_sorted_pairs_device")

    def count(self) -> int:
        n = c_uint64()
        check(lib().okm_count(self.ctx, byref(n)), "okm_count")
        return n.value

    def result(self, min_count: int = 1) -> Tuple[np.ndarray, np.ndarray]:
        """Sorted (keys, counts) with count >= min_count (count.rs:106-119)."""
        n = c_uint64()
        check(lib().okm_result_size(self.ctx, min_count, byref(n)), "okm_result_size")
        keys = np.empty((n.value, 2) if self.wide else n.value, dtype=np.uint64)
        counts = np.empty(n.value, dtype=np.uint64)
        got = c_uint64()
        check(lib().okm_fetch_counts(self.ctx, min_count, keys.ctypes.data, counts.ctypes.data, n.value,
                                     byref(got), 0), "okm_fetch_counts")
        return keys[:got.value], counts[:got.value]

    def result_device(self) -> Tuple[int, int, int]:
        k = c_void_p()
        c = c_void_p()
        n = c_uint64()
        check(lib().okm_result_device(self.ctx, byref(k), byref(c), byref(n)), "okm_result_device")
        return int(k.value or 0), int(c.value or 0), n.value

    def fetch_into_device(self, d_keys: int, d_counts: int, cap: int, min_count: int = 1) -> int:
        got = c_uint64()
        check(lib().okm_fetch_counts(self.ctx, min_count, c_void_p(d_keys), c_void_p(d_counts), cap, byref(got), 1),
              "okm_fetch_counts(device)")
        return got.value

    def synchronize(self) -> None:
        check(lib().okm_synchronize(self.ctx), "okm_synchronize")

    def set_timing(self, on: bool) -> None:
        check(lib().okm_set_timing(self.ctx, 1 if on else 0), "okm_set_timing")

    def kernel_stats(self) -> Dict[str, Dict[str, float]]:
        arr = (_lib.KernelStat * 64)()
        n = c_int()
        check(lib().okm_kernel_stats(self.ctx, arr, 64, byref(n)), "okm_kernel_stats")
        out = {}
        for i in range(min(n.value, 64)):
            s = arr[i]
            out[s.name.decode()] = {"launches": int(s.launches), "total_ms": float(s.total_ms),
                                    "alg_bytes": float(s.alg_bytes)}
        return out

    def engine_info(self) -> Dict[str, int]:
        info = _lib.EngineInfo()
        check(lib().okm_engine_info_get(self.ctx, byref(info)), "okm_engine_info_get")
        return {f: int(getattr(info, f)) for f, _ in _lib.EngineInfo._fields_}


# ---------------------------------------------------------------------------
# multi-GPU: key-range owners over RCCL (okm_dist.hip)
# ---------------------------------------------------------------------------

def owner_bounds(hist: np.ndarray, world: int) -> List[int]:
    """okm_owner_bounds: histogram bins [b_r, b_{r+1}) owned by rank r (host code)."""
    hist = np.ascontiguousarray(hist, dtype=np.uint64)
    out = np.zeros(world + 1, dtype=np.uint32)
    check(lib().okm_owner_bounds(hist.ctypes.data if len(hist) else None, len(hist), world, out.ctypes.data),
          "okm_owner_bounds")
    return [int(x) for x in out]


def comm_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(_lib.OKM_COMM_ID_BYTES)
    check(lib().okm_comm_unique_id(buf), "okm_comm_unique_id")
    return buf.raw


class Comm:
    """One rank of an RCCL communicator owned by the library (okm_comm)."""

    def __init__(self, nranks: int, rank: int, unique_id: bytes, device: int = 0, _handle=None):
        self.h = c_void_p()
        if _handle is not None:
            self.h = _handle
            return
        idb = ctypes.create_string_buffer(bytes(unique_id), _lib.OKM_COMM_ID_BYTES)
        check(lib().okm_comm_init_rank(byref(self.h), nranks, rank, idb, device), "okm_comm_init_rank")

    @classmethod
    def init_all(cls, devices: Sequence[int]) -> List["Comm"]:
        n = len(devices)
        arr = (c_void_p * n)()
        devs = (c_int * n)(*devices)
        check(lib().okm_comm_init_all(arr, n, devs), "okm_comm_init_all")
        return [cls(n, i, b"", devices[i], _handle=c_void_p(arr[i])) for i in range(n)]

    @classmethod
    def init_loopback(cls, n: int, device: int = 0) -> List["Comm"]:
        """n virtual ranks on one device (okm_comm_init_loopback): the P > 1
        merge without RCCL; drive each rank's merge_owned from its own thread."""
        arr = (c_void_p * n)()
        check(lib().okm_comm_init_loopback(arr, n, device), "okm_comm_init_loopback")
        return [cls(n, i, b"", device, _handle=c_void_p(arr[i])) for i in range(n)]

    @property
    def rank(self) -> int:
        return int(lib().okm_comm_rank(self.h))

    @property
    def size(self) -> int:
        return int(lib().okm_comm_size(self.h))

    def info(self) -> Dict[str, object]:
        """What this rank's communicator is (okm_comm_get_info): the ranks /
        rank / device it was created with, what the transport itself reports
        (RCCL: ncclCommCount, ncclCommUserRank, ncclCommCuDevice) and the
        device's PCI bus id."""
        ci = _lib.CommInfo()
        check(lib().okm_comm_get_info(self.h, byref(ci)), "okm_comm_get_info")
        return {"size": ci.size, "rank": ci.rank, "device": ci.device, "transport": ci.transport.decode(),
                "transport_ranks": ci.transport_ranks, "transport_rank": ci.transport_rank,
                "transport_device": ci.transport_device, "pci_bus_id": ci.pci_bus_id.decode()}

    def merge_owned(self, local: "KmerCounter", owner: "KmerCounter") -> int:
        """Collective: owner <- this rank's key range of all ranks' tables."""
        n = c_uint64()
        check(lib().okm_merge_owned(local.ctx, self.h, owner.ctx, byref(n)), "okm_merge_owned")
        return n.value

    def merge_owned_n(self, locals_: Sequence["KmerCounter"], owners: Sequence["KmerCounter"]) -> List[int]:
        """Collective: owners[i] <- this rank's key range of every rank's
        locals_[i], all tables under one owner split (okm_merge_owned_n)."""
        n = len(locals_)
        la = (c_void_p * n)(*[c.ctx for c in locals_])
        oa = (c_void_p * n)(*[c.ctx for c in owners])
        out = (c_uint64 * n)()
        check(lib().okm_merge_owned_n(la, self.h, oa, n, out), "okm_merge_owned_n")
        return [int(x) for x in out]

    def allreduce(self, values: Sequence[int]) -> List[int]:
        """Collective sum of u64 values (okm_comm_allreduce_u64)."""
        n = len(values)
        a = (c_uint64 * n)(*[int(v) for v in values])
        out = (c_uint64 * n)()
        check(lib().okm_comm_allreduce_u64(self.h, a, out, n), "okm_comm_allreduce_u64")
        return [int(x) for x in out]

    def last_times(self) -> Dict[str, float]:
        v = (ctypes.c_double * 4)()
        check(lib().okm_comm_last_times(self.h, v), "okm_comm_last_times")
        return {"plan_ms": v[0], "exchange_ms": v[1], "merge_ms": v[3]}

    def last_bytes(self) -> Tuple[int, int]:
        """(sent, received) bytes to / from other ranks in the last merge_owned."""
        a, b = c_uint64(), c_uint64()
        check(lib().okm_comm_last_bytes(self.h, byref(a), byref(b)), "okm_comm_last_bytes")
        return a.value, b.value

    def close(self) -> None:
        if self.h:
            lib().okm_comm_destroy(self.h)
            self.h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def distributed_compare(comm: "Comm", a: "KmerCounter", b: "KmerCounter", owner_a: "KmerCounter",
                        owner_b: "KmerCounter") -> Tuple[int, int, int]:
    """compare.rs:51-66 over the ranks of `comm` (collective): a / b hold this
    rank's share of DB1's / DB2's k-mers (set contexts).  Both go to key-range
    owners under ONE split (okm_merge_owned_n), so a key of A and the same key
    of B meet on one rank; each owner intersects its two ranges on its GPU
    (compare.rs:58) and |A|, |B|, |A ∩ B| are summed over the ranks.  Every
    rank returns the global (|A|, |B|, |A ∩ B|); union and Jaccard follow on
    the host (compare.rs:60-66)."""
    if any(c.wide for c in (a, b, owner_a, owner_b)):
        # okm_set_intersection_size_device reads plain u64 keys; compare.rs:37-39
        # only ever sees k <= 32 databases (KmerDbV2 stores u64 keys)
        raise OkmError(_lib.OKM_E_ARG, "distributed_compare: k > 32 (two-u64) sets are not supported")
    na, nb = comm.merge_owned_n([a, b], [owner_a, owner_b])
    inter = 0
    if na and nb:
        pa, _, _ = owner_a.result_device()
        pb, _, _ = owner_b.result_device()
        inter = set_intersection_size_device(pa, na, pb, nb, owner_a.device)
    ta, tb, ti = comm.allreduce([na, nb, inter])
    return ta, tb, ti


def set_intersection_size(a: np.ndarray, b: np.ndarray, device: int = 0) -> int:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    out = c_uint64()
    check(lib().okm_set_intersection_size(a.ctypes.data, len(a), b.ctypes.data, len(b), device, byref(out)),
          "okm_set_intersection_size")
    return out.value


def set_intersection_size_device(d_a: int, na: int, d_b: int, nb: int, device: int = 0) -> int:
    """|A ∩ B| of two sorted unique u64 arrays in device memory (compare.rs:58)."""
    out = c_uint64()
    check(lib().okm_set_intersection_size_device(c_void_p(d_a), na, c_void_p(d_b), nb, device, byref(out)),
          "okm_set_intersection_size_device")
    return out.value


# ---------------------------------------------------------------------------
# KmerDbV2 (db_types.rs:7-14)
# ---------------------------------------------------------------------------

class KmerDb:
    def __init__(self, k: int, references: Optional[Dict[str, np.ndarray]] = None):
        self.k = k
        self.references: Dict[str, np.ndarray] = dict(references or {})

    def add_reference(self, name: str, keys: np.ndarray) -> None:
        self.references[name] = np.asarray(keys, dtype=np.uint64)

    def write(self, path: str) -> None:
        db = c_void_p()
        check(lib().okm_db_new(byref(db), self.k), "okm_db_new")
        try:
            for name, keys in self.references.items():
                keys = np.ascontiguousarray(keys, dtype=np.uint64)
                check(lib().okm_db_add_reference(db, name.encode(), keys.ctypes.data, len(keys)),
                      "okm_db_add_reference")
            check(lib().okm_db_write(db, path.encode()), "okm_db_write")
        finally:
            lib().okm_db_free(db)

    @classmethod
    def read(cls, path: str) -> "KmerDb":
        db = c_void_p()
        check(lib().okm_db_read(byref(db), path.encode()), "okm_db_read")
        try:
            out = cls(int(lib().okm_db_k(db)))
            for i in range(int(lib().okm_db_num_references(db))):
                name = c_char_p()
                keys = c_void_p()
                n = c_uint64()
                check(lib().okm_db_reference(db, i, byref(name), byref(keys), byref(n)), "okm_db_reference")
                arr = np.ctypeslib.as_array(ctypes.cast(keys, POINTER(c_uint64)), shape=(n.value,)).copy() \
                    if n.value else np.zeros(0, np.uint64)
                out.references[name.value.decode()] = arr
            return out
        finally:
            lib().okm_db_free(db)

    def get_all_kmers_unified(self) -> set:
        s: set = set()
        for v in self.references.values():
            s.update(int(x) for x in v)
        return s


# ---------------------------------------------------------------------------
# drivers (the reference's commands, through the engine)
# ---------------------------------------------------------------------------

def run_count(k: int, input_files: Iterable[str], output_file: Optional[str] = None, min_count: int = 1,
              device: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """count.rs:40-141: every file in order into one table, filter, sort, TSV."""
    if k == 0 or k > 32:
        raise OkmError(OKM_E_INVALID_K, f"Invalid K-mer size: {k}. Must be between 1 and 32.")
    with KmerCounter(k, "count", device) as c:
        for p in input_files:
            c.add_records(read_fastx_file(p, True), normalized=True)
        keys, counts = c.result(min_count)
    if output_file:
        write_counts_tsv(output_file, k, keys, counts)
    return keys, counts


def run_build(k: int, genome_files: Iterable[str], output_file: Optional[str] = None,
              device: int = 0) -> KmerDb:
    """build.rs:80-160: per-file canonical k-mer sets under the basename."""
    if k == 0 or k > 32:
        raise OkmError(OKM_E_INVALID_K, f"Invalid K-mer size: {k}. Must be between 1 and 32.")
    db = KmerDb(k)
    with KmerCounter(k, "set", device) as c:
        for p in genome_files:
            c.reset()
            c.add_records(read_fastx_file(p, False), normalized=True)
            keys, _ = c.result(1)
            db.add_reference(os.path.basename(p) or p, keys)
    if output_file:
        db.write(output_file)
    return db


def run_compare(db1: KmerDb, db2: KmerDb, device: int = 0) -> Dict[str, object]:
    """compare.rs:29-97 on the device (union per DB, |A∩B|, Jaccard)."""
    if db1.k != db2.k:
        raise OkmError(OKM_E_INVALID_K, "K-mer databases have incompatible k-mer sizes (overall comparison): "
                                        f"{db1.k} vs {db2.k}")

    def unified(db: KmerDb) -> np.ndarray:
        arrs = [v for v in db.references.values() if len(v)]
        if not arrs:
            return np.zeros(0, np.uint64)
        with KmerCounter(db.k, "set", device) as c:
            for v in arrs:
                c.add_pairs(v)
            return c.result(1)[0]

    a, b = unified(db1), unified(db2)
    inter = set_intersection_size(a, b, device) if len(a) and len(b) else 0
    union = len(a) + len(b) - inter
    return {"kmer_size": db1.k, "db1_total_unique_kmers_across_references": len(a),
            "db2_total_unique_kmers_across_references": len(b), "intersection_size": inter,
            "union_size": union, "jaccard_index": 0.0 if union == 0 else inter / union}


# ---------------------------------------------------------------------------
# query / classify (query.rs, classify.rs) — device sets and probes
# ---------------------------------------------------------------------------

def read_fastx_records(path: str, decompress_by_extension: bool = True, raw: bool = False
                       ) -> List[Tuple[bytes, bytes]]:
    """(id, sequence) of every record; raw=True keeps record.sequence() as in
    the file (query.rs:66), otherwise normalize(false) is applied."""
    r = c_void_p()
    flags = _lib.OKM_READ_IDS | (_lib.OKM_READ_RAW if raw else 0)
    check(lib().okm_reader_open2(byref(r), path.encode(), 1 if decompress_by_extension else 0, flags),
          "okm_reader_open2")
    out: List[Tuple[bytes, bytes]] = []
    try:
        while True:
            seq, offs, n = c_void_p(), c_void_p(), c_uint64()
            check(lib().okm_reader_next(r, 256 << 20, byref(seq), byref(offs), byref(n)), "okm_reader_next")
            if n.value == 0:
                break
            ids, ioff = c_void_p(), c_void_p()
            check(lib().okm_reader_ids(r, byref(ids), byref(ioff)), "okm_reader_ids")
            o = np.ctypeslib.as_array(ctypes.cast(offs, POINTER(c_uint64)), shape=(n.value + 1,))
            io = np.ctypeslib.as_array(ctypes.cast(ioff, POINTER(c_uint64)), shape=(n.value + 1,))
            sb = ctypes.string_at(seq, int(o[-1])) if o[-1] else b""
            ib = ctypes.string_at(ids, int(io[-1])) if io[-1] else b""
            for i in range(n.value):
                out.append((ib[io[i]:io[i + 1]], sb[o[i]:o[i + 1]]))
    finally:
        lib().okm_reader_close(r)
    return out


class KmerSet:
    """Device hash set of canonical k-mers: the unified ``HashSet<u64>`` of a
    database (db_types.rs:43-48) and its ``contains`` probes (query.rs:88)."""

    def __init__(self, k: int, device: int = 0, capacity_hint: int = 0):
        self.k = k
        self.h = c_void_p()
        check(lib().okm_kset_create(byref(self.h), k, device, capacity_hint), "okm_kset_create")

    def close(self) -> None:
        if self.h:
            lib().okm_kset_destroy(self.h)
            self.h = c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def insert(self, keys: np.ndarray) -> int:
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        n_new = c_uint64()
        check(lib().okm_kset_insert(self.h, keys.ctypes.data, len(keys), 0, byref(n_new)), "okm_kset_insert")
        return n_new.value

    def insert_device(self, d_keys: int, n: int) -> int:
        n_new = c_uint64()
        check(lib().okm_kset_insert(self.h, c_void_p(d_keys), n, 1, byref(n_new)), "okm_kset_insert")
        return n_new.value

    def __len__(self) -> int:
        n = c_uint64()
        check(lib().okm_kset_size(self.h, byref(n)), "okm_kset_size")
        return n.value

    def contains(self, keys: np.ndarray) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros(len(keys), dtype=np.uint8)
        check(lib().okm_kset_contains(self.h, keys.ctypes.data, len(keys), out.ctypes.data), "okm_kset_contains")
        return out.astype(bool)

    def query_hits(self, seqs: Sequence[bytes]) -> np.ndarray:
        """query.rs:86-93 per record over RAW bytes."""
        data, offs = pack_records(list(seqs))
        hits = np.zeros(len(seqs), dtype=np.uint32)
        if len(seqs):
            check(lib().okm_query_hits(self.h, data.ctypes.data, offs.ctypes.data, len(seqs), hits.ctypes.data),
                  "okm_query_hits")
        return hits

    def query_hits_device(self, d_seq: int, nbytes: int, n_records: int, d_hits: int) -> None:
        check(lib().okm_query_hits_device(self.h, c_void_p(d_seq), nbytes, n_records, c_void_p(d_hits)),
              "okm_query_hits_device")


class Classifier:
    """classify.rs:176-308: the filtered input counts as a device map, probed
    by every reference key of a database."""

    def __init__(self, counter: KmerCounter, min_kmer_frequency: int = 1):
        self.h = c_void_p()
        n = c_uint64()
        check(lib().okm_classifier_create(byref(self.h), counter.ctx, min_kmer_frequency, byref(n)),
              "okm_classifier_create")
        self.n_input = n.value

    def close(self) -> None:
        if self.h:
            lib().okm_classifier_destroy(self.h)
            self.h = c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def pack_db(refs: Sequence[np.ndarray]):
        """(keys, ref_offsets): the references' keys back to back, as
        okm_classifier_probe_db[_device] take them."""
        offs = np.zeros(len(refs) + 1, dtype=np.uint64)
        if refs:
            offs[1:] = np.cumsum([len(r) for r in refs])
        keys = np.concatenate([np.asarray(r, dtype=np.uint64) for r in refs]) if refs else np.zeros(0, np.uint64)
        return np.ascontiguousarray(keys), offs

    def probe_db(self, refs: Sequence[np.ndarray] = None, packed=None, d_keys: int = None) -> Dict[str, object]:
        """refs: one key array per reference; or packed = pack_db(refs) (keys
        on the host), or d_keys = a device address holding pack_db's keys with
        packed = (None, ref_offsets) (okm_classifier_probe_db_device)."""
        keys, offs = packed if packed is not None else self.pack_db(refs)
        nrefs = len(offs) - 1
        rm = np.zeros(nrefs, dtype=np.uint64)
        rs = np.zeros(nrefs, dtype=np.uint64)
        du, dm, ds = c_uint64(), c_uint64(), c_uint64()
        if d_keys is not None:
            check(lib().okm_classifier_probe_db_device(self.h, c_void_p(d_keys), offs.ctypes.data, nrefs,
                                                       rm.ctypes.data, rs.ctypes.data, byref(du), byref(dm),
                                                       byref(ds)),
                  "okm_classifier_probe_db_device")
        else:
            check(lib().okm_classifier_probe_db(self.h, keys.ctypes.data, offs.ctypes.data, nrefs, rm.ctypes.data,
                                                rs.ctypes.data, byref(du), byref(dm), byref(ds)),
                  "okm_classifier_probe_db")
        return {"ref_matched": rm, "ref_sum_depth": rs, "union": du.value, "matched": dm.value,
                "sum_depth": ds.value}


def run_query(db: KmerDb, reads_file: str, min_hits: int = 1, device: int = 0) -> List[bytes]:
    """query.rs:24-134: ids of reads (input order) with >= min_hits windows in
    the DB's unified set; reads shorter than k never match."""
    k = db.k
    if k == 0 or k > 32:
        raise OkmError(OKM_E_INVALID_K, f"Invalid K-mer size: {k}. Must be between 1 and 32.")
    recs = read_fastx_records(reads_file, True, raw=True)
    total = sum(len(v) for v in db.references.values())
    with KmerSet(k, device, total) as s:
        for v in db.references.values():
            if len(v):
                s.insert(v)
        hits = s.query_hits([q for _i, q in recs])
    return [rid for (rid, q), h in zip(recs, hits) if len(q) >= k and h >= min_hits]


def run_classify(input_file: str, dbs: Sequence[KmerDb], min_kmer_frequency: int = 1,
                 device: int = 0) -> Dict[str, object]:
    """classify.rs:135-308 statistics (numbers only; the CLI writes the JSON)."""
    k = dbs[0].k
    with KmerCounter(k, "count", device) as c:
        c.add_records([q for _i, q in read_fastx_records(input_file, False)], normalized=True)
        with Classifier(c, min_kmer_frequency) as cl:
            per_db = [dict(cl.probe_db(list(db.references.values())), names=list(db.references))
                      for db in dbs]
            return {"total_unique_kmers_in_input": cl.n_input, "databases": per_db}
