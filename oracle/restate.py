"""Pure-Python restatement of orion-kmer's count/build/compare hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the HIP library, the
CLI, ``okm``) may import this module; only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg use it, and only as the checker.

It restates, function by function, the reference Rust code at
``/root/reference/orion-kmer`` (cited as ``file:line``) plus the record
semantics of the third-party crate ``needletail 0.5.1`` (pinned in
``orion-kmer/Cargo.lock:580-591``, not vendored), whose published behaviour is
restated in SURVEY.md Appendix A.  It is deliberately naive (O(k) work per
window, exactly as the reference) and meant for inputs of a few KB; the C
restatement in ``oracle/okm_oracle.c`` is the one used at MB scale.

Pinning: ``tests/test_oracle_golden.py`` checks this module against every
known-answer value in ``kmer.rs:108-341`` and every expected output of the
reference's content-string tests that the reference code can actually produce
(SURVEY.md §4.3 "PASS" rows).  The compressed-fixture expectations in
``count_tests.rs:369,410,463`` / ``build_tests.rs:335,342`` contradict the
reference code and are replaced by regenerated values.
"""

from __future__ import annotations

import bz2
import gzip
import json
import lzma
import os
from typing import Dict, Iterable, List, Optional, Tuple

BITS_PER_BASE = 2  # kmer.rs:3


class OracleError(Exception):
    """Mirrors the outermost anyhow context the reference prints (main.rs:10-13)."""


# --------------------------------------------------------------------------
# k-mer codec — kmer.rs
# --------------------------------------------------------------------------

def dna_base_to_u64(base: int) -> Optional[int]:
    """kmer.rs:12-20 — A/a=0, C/c=1, G/g=2, T/t=3, anything else None."""
    return {65: 0, 97: 0, 67: 1, 99: 1, 71: 2, 103: 2, 84: 3, 116: 3}.get(base)


def u64_to_dna_base(val: int) -> int:
    """kmer.rs:24-32 — panics (here: ValueError) outside 0..=3."""
    if val not in (0, 1, 2, 3):
        raise ValueError("Invalid 2-bit value for DNA base")
    return b"ACGT"[val]


def seq_to_u64(seq: bytes, k: int) -> Optional[int]:
    """kmer.rs:37-57 — MSB-first 2-bit packing; None on bad k, len!=k or non-ACGT."""
    if k == 0 or k > 32:
        return None
    if len(seq) != k:
        return None
    v = 0
    for i, b in enumerate(seq):
        code = dna_base_to_u64(b)
        if code is None:
            return None
        v |= code << (BITS_PER_BASE * (k - 1 - i))
    return v


def u64_to_seq(v: int, k: int) -> bytes:
    """kmer.rs:61-75 — panics (ValueError) for k outside 1..=32."""
    if k == 0 or k > 32:
        raise ValueError(f"Invalid k-mer length for decoding: {k}")
    return bytes(u64_to_dna_base((v >> (BITS_PER_BASE * (k - 1 - i))) & 3) for i in range(k))


def reverse_complement_u64(v: int, k: int) -> int:
    """kmer.rs:79-94 — base i from the LSB end, XOR 3, placed at k-1-i."""
    if k == 0 or k > 32:
        raise ValueError(f"Invalid k-mer length for reverse complement: {k}")
    rc = 0
    for i in range(k):
        b = (v >> (BITS_PER_BASE * i)) & 3
        rc |= (b ^ 3) << (BITS_PER_BASE * (k - 1 - i))
    return rc


def canonical_u64(v: int, k: int) -> int:
    """kmer.rs:99-106 — v if v < rc else rc (ties return rc == v)."""
    rc = reverse_complement_u64(v, k)
    return v if v < rc else rc


# --------------------------------------------------------------------------
# needletail 0.5.1 record semantics
# --------------------------------------------------------------------------

_NORM = {}
for _c in b"ACGT":
    _NORM[_c] = _c
_NORM.update({ord("a"): ord("A"), ord("c"): ord("C"), ord("g"): ord("G"),
              ord("t"): ord("T"), ord("u"): ord("T"), ord("U"): ord("T"),
              ord("-"): ord("-"), ord("."): ord("-"), ord("~"): ord("-")})
_STRIP = {ord(" "), ord("\t"), ord("\r"), ord("\n")}


def normalize(seq: bytes) -> bytes:
    """needletail ``normalize(seq, iupac=false)`` as called at count.rs:71,
    build.rs:48: upper-case ACGT, U/u->T, gaps ``-.~``->``-``, whitespace and
    line endings removed, every other byte -> ``N``."""
    out = bytearray()
    for c in seq:
        if c in _STRIP:
            continue
        out.append(_NORM.get(c, ord("N")))
    return bytes(out)


def sniff_decompress(data: bytes) -> bytes:
    """needletail ``parse_fastx_reader`` compression sniffing (gzip/bzip2/xz
    features per Cargo.lock:584-591; no zstd)."""
    if data[:2] == b"\x1f\x8b":
        return gzip.decompress(data)
    if data[:3] == b"BZh":
        return bz2.decompress(data)
    if data[:6] == b"\xfd7zXZ\x00":
        return lzma.decompress(data)
    return data


def parse_fastx(data: bytes) -> List[Tuple[bytes, bytes]]:
    """Records ``(id, raw_sequence)`` of a FASTA/FASTQ byte string.

    Raises OracleError('parse') for an empty input or a first byte that is
    neither ``>`` nor ``@`` and OracleError('record') for a malformed FASTQ
    record (needletail errors surfaced at count.rs:63-64 and :69-70)."""
    data = sniff_decompress(data)
    if len(data) == 0:
        raise OracleError("parse")
    first = data[:1]
    lines = data.split(b"\n")
    if data.endswith(b"\n"):
        lines = lines[:-1]
    recs: List[Tuple[bytes, bytes]] = []
    if first == b">":
        cur_id = None
        cur_seq: List[bytes] = []
        def raw_seq(lines_: List[bytes]) -> bytes:
            # needletail raw_seq()/sequence(): the lines with their interior
            # line breaks, one trailing CR trimmed
            sq = b"\n".join(lines_)
            return sq[:-1] if sq.endswith(b"\r") else sq

        for ln in lines:
            if ln.startswith(b">"):
                if cur_id is not None:
                    recs.append((cur_id, raw_seq(cur_seq)))
                cur_id = ln[1:].rstrip(b"\r")
                cur_seq = []
            else:
                cur_seq.append(ln)
        if cur_id is not None:
            recs.append((cur_id, raw_seq(cur_seq)))
        return recs
    if first == b"@":
        # trailing blank lines after the last record are tolerated
        while lines and lines[-1].rstrip(b"\r") == b"":
            lines.pop()
        i = 0
        while i < len(lines):
            if i + 3 >= len(lines):
                raise OracleError("record")  # truncated final record
            hdr, seq, plus, qual = lines[i], lines[i + 1], lines[i + 2], lines[i + 3]
            if not hdr.startswith(b"@") or not plus.startswith(b"+"):
                raise OracleError("record")
            seq = seq.rstrip(b"\r")
            qual = qual.rstrip(b"\r")
            if len(seq) != len(qual):
                raise OracleError("record")
            recs.append((hdr[1:].rstrip(b"\r"), seq))
            i += 4
        return recs
    raise OracleError("parse")


def decompress_by_extension(path: str, data: bytes) -> bytes:
    """utils.rs:125-152 (``get_decompressed_input_reader``): gz/xz/zst/zstd by
    the lower-cased last extension, anything else raw."""
    ext = os.path.splitext(path)[1][1:].lower()
    if ext == "gz":
        return gzip.decompress(data)
    if ext == "xz":
        return lzma.decompress(data)
    if ext in ("zst", "zstd"):
        return _zstd_decompress(data)
    return data


def _zstd_decompress(data: bytes) -> bytes:
    """zstd 0.12 crate's streaming Decoder, via the system libzstd (streaming
    API: frames written without a content size decode too)."""
    import ctypes

    class InBuf(ctypes.Structure):
        _fields_ = [("src", ctypes.c_void_p), ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t)]

    class OutBuf(ctypes.Structure):
        _fields_ = [("dst", ctypes.c_void_p), ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t)]

    lib = ctypes.CDLL("libzstd.so.1")
    lib.ZSTD_createDStream.restype = ctypes.c_void_p
    lib.ZSTD_initDStream.argtypes = [ctypes.c_void_p]
    lib.ZSTD_decompressStream.restype = ctypes.c_size_t
    lib.ZSTD_decompressStream.argtypes = [ctypes.c_void_p, ctypes.POINTER(OutBuf), ctypes.POINTER(InBuf)]
    lib.ZSTD_isError.argtypes = [ctypes.c_size_t]
    lib.ZSTD_freeDStream.argtypes = [ctypes.c_void_p]
    ds = lib.ZSTD_createDStream()
    lib.ZSTD_initDStream(ds)
    src = ctypes.create_string_buffer(data, len(data))
    ib = InBuf(ctypes.cast(src, ctypes.c_void_p), len(data), 0)
    out = bytearray()
    chunk = ctypes.create_string_buffer(1 << 20)
    try:
        while True:
            ob = OutBuf(ctypes.cast(chunk, ctypes.c_void_p), len(chunk), 0)
            r = lib.ZSTD_decompressStream(ds, ctypes.byref(ob), ctypes.byref(ib))
            if lib.ZSTD_isError(r):
                raise OracleError("zstd error")
            out += chunk.raw[:ob.pos]
            if ib.pos == ib.size and ob.pos < ob.size:
                break
    finally:
        lib.ZSTD_freeDStream(ds)
    return bytes(out)


# --------------------------------------------------------------------------
# count — count.rs
# --------------------------------------------------------------------------

def process_sequence_chunk(seq: bytes, k: int, counts: Dict[int, int]) -> None:
    """count.rs:23-38 — every k-window, skip invalid, canonicalise, +1."""
    if len(seq) < k:
        return
    for i in range(len(seq) - k + 1):
        v = seq_to_u64(seq[i:i + k], k)
        if v is not None:
            c = canonical_u64(v, k)
            counts[c] = counts.get(c, 0) + 1


def count_records(seqs: Iterable[bytes], k: int) -> Dict[int, int]:
    counts: Dict[int, int] = {}
    for s in seqs:
        process_sequence_chunk(normalize(s), k, counts)
    return counts


def run_count_bytes(files: List[Tuple[str, bytes]], k: int, min_count: int = 1) -> str:
    """count.rs:40-141 on in-memory files ``(path, raw bytes)``; returns the
    decompressed TSV text the reference would write."""
    if k == 0 or k > 32:  # count.rs:43-45
        raise OracleError(f"Invalid K-mer size: {k}. Must be between 1 and 32.")
    counts: Dict[int, int] = {}
    for path, raw in files:  # count.rs:52 — files in CLI order, one map
        data = decompress_by_extension(path, raw)
        try:
            recs = parse_fastx(data)
        except OracleError as e:
            if str(e) == "parse":
                raise OracleError(f"Failed to parse FASTA/Q content from: {path}")
            raise OracleError(f"Error reading record from {path}")
        for _id, seq in recs:
            process_sequence_chunk(normalize(seq), k, counts)
    return format_counts(counts, k, min_count)


def format_counts(counts: Dict[int, int], k: int, min_count: int = 1) -> str:
    """count.rs:106-135 — filter count>=min, sort by u64, ``KMER\\tCOUNT\\n``."""
    items = sorted((kv for kv in counts.items() if kv[1] >= min_count), key=lambda kv: kv[0])
    return "".join(f"{u64_to_seq(v, k).decode()}\t{c}\n" for v, c in items)


# --------------------------------------------------------------------------
# build / compare — build.rs, compare.rs, db_types.rs
# --------------------------------------------------------------------------

def build_sets(files: List[Tuple[str, bytes]], k: int) -> Dict[str, set]:
    """build.rs:80-121 — per file basename, the set of canonical k-mers.
    Files are read raw (utils.rs:157-161) and needletail sniffs compression."""
    if k == 0 or k > 32:
        raise OracleError(f"Invalid K-mer size: {k}. Must be between 1 and 32.")
    refs: Dict[str, set] = {}
    for path, raw in files:
        try:
            recs = parse_fastx(raw)
        except OracleError as e:
            if str(e) == "parse":
                raise OracleError(f"Failed to parse FASTA/Q content from: {path}")
            raise OracleError(f"Error reading record from {path}")
        s: Dict[int, int] = {}
        for _id, seq in recs:
            process_sequence_chunk(normalize(seq), k, s)
        refs[os.path.basename(path)] = set(s)  # db_types.rs:38-40 (overwrite)
    return refs


def compare_sets(k1: int, refs1: Dict[str, set], k2: int, refs2: Dict[str, set],
                 db1_path: str = "db1", db2_path: str = "db2") -> Dict[str, object]:
    """compare.rs:29-97 — unified sets, |A∩B|, union, Jaccard (0.0 if empty)."""
    if k1 != k2:
        raise OracleError(
            f"K-mer databases have incompatible k-mer sizes (overall comparison): {k1} vs {k2}")
    a = set().union(*refs1.values()) if refs1 else set()
    b = set().union(*refs2.values()) if refs2 else set()
    inter = len(a & b)
    union = len(a) + len(b) - inter
    jac = 0.0 if union == 0 else inter / union
    return {
        "db1_path": db1_path, "db2_path": db2_path, "kmer_size": k1,
        "db1_total_unique_kmers_across_references": len(a),
        "db2_total_unique_kmers_across_references": len(b),
        "intersection_size": inter, "union_size": union, "jaccard_index": jac,
    }


def compare_json(d: Dict[str, object]) -> str:
    """serde_json::to_writer_pretty output (2-space indent, no trailing newline)."""
    return json.dumps(d, indent=2, ensure_ascii=False)


# --------------------------------------------------------------------------
# query — query.rs
# --------------------------------------------------------------------------

def query_hits(seq: bytes, k: int, db_all: set) -> int:
    """query.rs:86-93 — windows of the RAW sequence (no normalize) whose
    canonical k-mer is in the unified DB set."""
    hits = 0
    for i in range(len(seq) - k + 1):
        v = seq_to_u64(seq[i:i + k], k)
        if v is not None and canonical_u64(v, k) in db_all:
            hits += 1
    return hits


def run_query_bytes(k: int, refs: Dict[str, set], reads_path: str, reads_raw: bytes,
                    min_hits: int = 1) -> bytes:
    """query.rs:24-134 on an in-memory reads file; returns the output bytes
    (matching read ids, input order, one per line)."""
    if k == 0 or k > 32:  # query.rs:30-32
        raise OracleError(f"Invalid K-mer size: {k}. Must be between 1 and 32.")
    db_all = set().union(*refs.values()) if refs else set()  # db_types.rs:43-48
    data = decompress_by_extension(reads_path, reads_raw)    # query.rs:45
    try:
        recs = parse_fastx(data)
    except OracleError as e:
        if str(e) == "parse":
            raise OracleError(f"Failed to parse FASTQ content from: {reads_path!r}")
        raise OracleError(f"Error reading record from {reads_path!r}")
    out = []
    for rid, seq in recs:  # query.rs:63-71 (record.sequence(): raw)
        if len(seq) < k:    # query.rs:83-85
            continue
        if query_hits(seq, k, db_all) >= min_hits:  # query.rs:97
            out.append(rid + b"\n")
    return b"".join(out)


# --------------------------------------------------------------------------
# classify — classify.rs
# --------------------------------------------------------------------------

def rust_f64(x: float) -> str:
    """serde_json's f64 text (ryu: shortest round-trip digits, decimal for
    1e-5 <= |x| < 1e16 else d.ddde±x without padding, integers get '.0')."""
    if x == 0:
        return "-0.0" if str(x).startswith("-") else "0.0"
    r = repr(abs(x))
    neg = x < 0
    if "e" in r:
        mant, ex = r.split("e")
        exp10 = int(ex)
    else:
        mant, exp10 = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # value = 0.ip fp ... normalise: position of the decimal point
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    point = len(ip) - lead_zeros + exp10  # digits * 10^(point - len(digits))
    digits = digits.rstrip("0") or "0"
    n = len(digits)
    kk = point
    if kk - n >= 0 and kk <= 16:
        o = digits + "0" * (kk - n) + ".0"
    elif 0 < kk <= 16:
        o = digits[:kk] + "." + digits[kk:]
    elif -5 < kk <= 0:
        o = "0." + "0" * (-kk) + digits
    elif n == 1:
        o = digits + "e" + str(kk - 1)
    else:
        o = digits[0] + "." + digits[1:] + "e" + str(kk - 1)
    return ("-" if neg else "") + o


def _ratio(a: int, b: int) -> float:
    return a / b if b > 0 else 0.0


def run_classify_bytes(input_path: str, input_raw: bytes,
                       dbs: List[Tuple[str, int, List[Tuple[str, set]]]],
                       user_k: Optional[int] = None, min_freq: int = 1,
                       min_cov: float = 0.0) -> Tuple[str, str]:
    """classify.rs:58-385 on in-memory inputs.  ``dbs`` = [(path, k,
    [(reference name, key set), ...])] in file order.  Returns (JSON text,
    TSV text).  References are listed in DB order (the reference iterates a
    HashMap: its order is random, classify.rs:215)."""
    final_k = None
    if user_k is not None:  # classify.rs:71-78
        if user_k == 0 or user_k > 32:
            raise OracleError(f"Invalid K-mer size: {user_k}. Must be between 1 and 32.")
        final_k = user_k
    for path, dk, _refs in dbs:  # classify.rs:80-117
        if final_k is not None:
            if dk != final_k:
                if user_k is not None:
                    raise OracleError(f"User-provided k-mer size {final_k} does not match k-mer size "
                                      f"{dk} from database: {path!r}")
                raise OracleError(f"Effective k-mer size {final_k} (from first database) does not "
                                  f"match k-mer size {dk} from database: {path!r}")
        else:
            if dk == 0 or dk > 32:
                raise OracleError(f"Invalid K-mer size: {dk}. Must be between 1 and 32.")
            final_k = dk
    k = final_k
    try:  # classify.rs:135-181: raw file (needletail sniffs compression), normalize
        recs = parse_fastx(input_raw)
    except OracleError as e:
        if str(e) == "parse":
            raise OracleError(f"Failed to parse FASTA/Q content from: {input_path!r}")
        raise OracleError(f"Error reading record from input file: {input_path!r}")
    counts: Dict[int, int] = {}
    for _id, seq in recs:
        process_sequence_chunk(normalize(seq), k, counts)
    filt = {key: c for key, c in counts.items() if c >= min_freq}  # classify.rs:195-199
    n_in = len(filt)

    tsv = ["InputFile\tDatabase\tReference\tTotalKmersInReference\tInputKmersHittingReference\t"
           "SumDepthMatchedKmers\tAvgDepthMatchedKmers\tProportionInputKmersHittingReference\t"
           "ReferenceBreadthOfCoverage\n"]
    db_blocks = []
    for path, dk, refs in dbs:  # classify.rs:206-308
        overall: set = set()
        ref_blocks = []
        for name, rset in refs:
            matched = {kk for kk in filt if kk in rset}
            sd = sum(filt[kk] for kk in matched)
            overall |= matched
            nm, tot = len(matched), len(rset)
            breadth = _ratio(nm, tot)
            if breadth >= min_cov:
                avg, prop = _ratio(sd, nm), _ratio(nm, n_in)
                ref_blocks.append(
                    "        {\n"
                    f"          \"reference_name\": {json.dumps(name, ensure_ascii=False)},\n"
                    f"          \"total_kmers_in_reference\": {tot},\n"
                    f"          \"input_kmers_hitting_reference\": {nm},\n"
                    f"          \"sum_depth_of_matched_kmers_in_input\": {sd},\n"
                    f"          \"avg_depth_of_matched_kmers_in_input\": {rust_f64(avg)},\n"
                    f"          \"proportion_input_kmers_hitting_reference\": {rust_f64(prop)},\n"
                    f"          \"reference_breadth_of_coverage\": {rust_f64(breadth)}\n"
                    "        }")
                tsv.append(f"{input_path}\t{path}\t{name}\t{tot}\t{nm}\t{sd}\t{avg:.4f}\t{prop:.4f}\t{breadth:.4f}\n")
        osd = sum(filt[kk] for kk in overall)
        union = len(set().union(*[r for _n, r in refs])) if refs else 0
        no = len(overall)
        refs_txt = "[\n" + ",\n".join(ref_blocks) + "\n      ]" if ref_blocks else "[]"
        db_blocks.append(
            "    {\n"
            f"      \"database_path\": {json.dumps(path, ensure_ascii=False)},\n"
            f"      \"database_kmer_size\": {dk},\n"
            f"      \"total_unique_kmers_in_db_across_references\": {union},\n"
            f"      \"overall_input_kmers_matched_in_db\": {no},\n"
            f"      \"overall_sum_depth_of_matched_kmers_in_input\": {osd},\n"
            f"      \"overall_avg_depth_of_matched_kmers_in_input\": {rust_f64(_ratio(osd, no))},\n"
            f"      \"proportion_input_kmers_in_db_overall\": {rust_f64(_ratio(no, n_in))},\n"
            f"      \"proportion_db_kmers_covered_overall\": {rust_f64(_ratio(no, union))},\n"
            f"      \"references\": {refs_txt}\n"
            "    }")
    dbs_txt = "[\n" + ",\n".join(db_blocks) + "\n  ]" if db_blocks else "[]"
    js = ("{\n"
          f"  \"input_file_path\": {json.dumps(input_path, ensure_ascii=False)},\n"
          f"  \"total_unique_kmers_in_input\": {n_in},\n"
          f"  \"min_kmer_frequency_filter\": {min_freq},\n"
          f"  \"databases_analyzed\": {dbs_txt}\n"
          "}")
    return js, "".join(tsv)
