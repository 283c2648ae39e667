"""C-ABI library on the host (no GPU compute): every symbol in
include/orion_kmer.h is exported; the CPU parts of the boundary (codec parity
surface, FASTA/FASTQ record source, output codecs, KmerDbV2, synthetic reads)
match the oracle; and the engine refuses to run without a device."""

import gzip
import lzma
import os
import random
import re
import struct
import subprocess
import sys

import numpy as np
import pytest

import okm
import restate as R
from conftest import GOLDEN, case_file_bytes, has_gpu
from okm import _lib


def header_symbols():
    import glob
    txt = ""
    for h in sorted(glob.glob(os.path.join(os.path.dirname(_lib.HEADER_PATH), "*.h"))):  # every include/*.h
        with open(h) as fh:
            txt += fh.read()
    return sorted(set(re.findall(r"\b(okm_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 45
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes prototypes cover the whole header
    assert set(syms) == set(_lib.PROTOTYPES), set(syms) ^ set(_lib.PROTOTYPES)
    assert lib.okm_abi_version() == 2


def test_cli_links_only_the_c_abi():
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.CLI_PATH], capture_output=True, text=True).stdout
    used = set(re.findall(r"\b(okm_[a-z0-9_]+)\b", out))
    assert used and used <= set(header_symbols())


def test_codec_kats(reference_expectations):
    for c in reference_expectations["seq_to_u64"]:
        assert okm.seq_to_u64(c["seq"].encode(), c["k"]) == c["value"], c["src"]
    for c in reference_expectations["u64_to_seq"]:
        assert okm.u64_to_seq(c["value"], c["k"]).decode() == c["seq"], c["src"]
    for c in reference_expectations["reverse_complement"]:
        k = len(c["seq"])
        assert okm.reverse_complement_u64(okm.seq_to_u64(c["seq"].encode(), k), k) == \
            okm.seq_to_u64(c["rc"].encode(), k)
    for c in reference_expectations["canonical"]:
        k = len(c["seq"])
        assert okm.canonical_u64(okm.seq_to_u64(c["seq"].encode(), k), k) == okm.seq_to_u64(c["canon"].encode(), k)
    for bad in (0, 33):
        with pytest.raises(ValueError):
            okm.u64_to_seq(0, bad)
        with pytest.raises(ValueError):
            okm.reverse_complement_u64(0, bad)


def test_codec_random_vs_restate():
    rng = random.Random(3)
    for _ in range(5000):
        k = rng.randint(1, 32)
        v = rng.getrandbits(2 * k)
        assert okm.reverse_complement_u64(v, k) == R.reverse_complement_u64(v, k)
        assert okm.canonical_u64(v, k) == R.canonical_u64(v, k)
        assert okm.u64_to_seq(v, k) == R.u64_to_seq(v, k)
        s = bytes(rng.choice(b"ACGTacgtNX") for _ in range(k))
        assert okm.seq_to_u64(s, k) == R.seq_to_u64(s, k)


def test_parse_buffer_matches_restate(golden_cases):
    for c in golden_cases["count"]:
        for f in c["files"]:
            raw = R.decompress_by_extension(f["name"], case_file_bytes(f))
            exp = [R.normalize(s) for _, s in R.parse_fastx(raw)]
            assert okm.parse_fastx(raw) == exp, (c["name"], f["name"])


def test_parse_errors():
    for bad in (b"", b"This is not fasta content\nACGT", b"ACGT\n"):
        with pytest.raises(okm.OkmError) as ei:
            okm.parse_fastx(bad)
        assert ei.value.status == _lib.OKM_E_PARSE
    for bad in (b"@r\nACGT\n+\nIII\n", b"@r\nACGT\n+\n", b"@r\nACGT\nIIII\nIIII\n"):
        with pytest.raises(okm.OkmError) as ei:
            okm.parse_fastx(bad)
        assert ei.value.status == _lib.OKM_E_RECORD
    # headers-only FASTA is valid with empty records (build_tests.rs:239-251)
    assert okm.parse_fastx(b">h1\n>h2\n") == [b"", b""]


def test_reader_fixture_files(reference_expectations):
    fx = reference_expectations["fixture_files"]
    d = os.path.join(GOLDEN, "data")
    for ext in ("gz", "xz", "zst"):
        for base in ("test_input1.fasta", "test_input2.fastq"):
            path = os.path.join(d, f"{base}.{ext}")
            exp = [R.normalize(s) for _, s in R.parse_fastx(fx[base].encode())]
            assert okm.read_fastx_file(path, True) == exp
            if ext != "zst":  # build path: needletail sniffs gz/xz magic itself
                assert okm.read_fastx_file(path, False) == exp
    # needletail 0.5.1 has no zstd: the raw (build) reader rejects .zst content
    with pytest.raises(okm.OkmError):
        okm.read_fastx_file(os.path.join(d, "test_input1.fasta.zst"), False)


def test_reader_missing_file():
    with pytest.raises(okm.OkmError) as ei:
        okm.read_fastx_file("/nonexistent/file.fa")
    assert ei.value.status == _lib.OKM_E_IO


@pytest.mark.parametrize("ext", ["tsv", "gz", "xz", "zst", "zstd", "GZ"])
def test_tsv_writer_and_output_codecs(tmp_path, ext):
    rng = np.random.default_rng(1)
    k = 21
    keys = np.sort(rng.integers(0, 1 << 42, 1000, dtype=np.uint64))
    counts = rng.integers(1, 10 ** 12, 1000, dtype=np.uint64)
    p = str(tmp_path / f"out.{ext}")
    okm.write_counts_tsv(p, k, keys, counts)
    raw = open(p, "rb").read()
    e = ext.lower()
    if e == "gz":
        raw = gzip.decompress(raw)
    elif e == "xz":
        raw = lzma.decompress(raw)
    elif e in ("zst", "zstd"):
        raw = R._zstd_decompress(raw)
    exp = "".join(f"{R.u64_to_seq(int(a), k).decode()}\t{int(b)}\n" for a, b in zip(keys, counts))
    assert raw.decode() == exp


def test_empty_tsv(tmp_path):
    p = str(tmp_path / "e.tsv")
    okm.write_counts_tsv(p, 5, np.zeros(0, np.uint64), np.zeros(0, np.uint64))
    assert open(p, "rb").read() == b""


def test_tsv_to_fifo(tmp_path):
    """`count -o <pipe>`: a plain output that cannot seek is written
    sequentially (utils.rs:168 File::create works on any path), not by offset."""
    import threading
    k = 13
    rng = np.random.default_rng(3)
    keys = np.sort(rng.integers(0, 1 << 26, 200_000, dtype=np.uint64))
    counts = rng.integers(1, 1000, 200_000, dtype=np.uint64)
    fifo = str(tmp_path / "out.tsv")
    os.mkfifo(fifo)
    got = []
    reader = threading.Thread(target=lambda: got.append(open(fifo, "rb").read()))
    reader.start()
    okm.write_counts_tsv(fifo, k, keys, counts)
    reader.join(timeout=60)
    exp = "".join(f"{R.u64_to_seq(int(a), k).decode()}\t{int(b)}\n" for a, b in zip(keys, counts))
    assert got and got[0].decode() == exp


def test_tsv_overwrites_longer_file(tmp_path):
    """A rerun over a longer existing output leaves exactly the new table."""
    p = tmp_path / "o.tsv"
    p.write_bytes(b"Z" * 100_000)
    okm.write_counts_tsv(str(p), 3, np.array([1, 6], np.uint64), np.array([2, 9], np.uint64))
    assert p.read_bytes() == b"AAC\t2\nACG\t9\n"


def test_kmerdb_roundtrip_and_bincode_layout(tmp_path):
    db = okm.KmerDb(4)
    db.add_reference("a.fa", np.array([1, 5, 9], np.uint64))
    db.add_reference("b.fa", np.array([], np.uint64))
    db.add_reference("a.fa", np.array([2, 3], np.uint64))  # overwrite (db_types.rs:38-40)
    p = str(tmp_path / "x.db")
    db.write(p)
    raw = open(p, "rb").read()
    # bincode 1.3 default: u8 k, u64 len-prefixed map/string/set, LE fixed ints
    exp = bytes([4]) + struct.pack("<Q", 2)
    exp += struct.pack("<Q", 4) + b"a.fa" + struct.pack("<Q", 2) + struct.pack("<QQ", 2, 3)
    exp += struct.pack("<Q", 4) + b"b.fa" + struct.pack("<Q", 0)
    assert raw == exp
    back = okm.KmerDb.read(p)
    assert back.k == 4 and list(back.references) == ["a.fa", "b.fa"]
    assert back.references["a.fa"].tolist() == [2, 3]
    for ext in ("gz", "xz", "zst"):
        q = str(tmp_path / f"x.db.{ext}")
        db.write(q)
        assert okm.KmerDb.read(q).references["a.fa"].tolist() == [2, 3]
    open(str(tmp_path / "bad.db"), "wb").write(raw[:10])
    with pytest.raises(okm.OkmError) as ei:
        okm.KmerDb.read(str(tmp_path / "bad.db"))
    assert ei.value.status == _lib.OKM_E_FORMAT


def test_synth_reads_deterministic_and_shardable():
    a = okm.synth_reads(5000, 150, genome_len=1_000_000, threads=1)
    b = okm.synth_reads(5000, 150, genome_len=1_000_000, threads=8)
    assert np.array_equal(a, b)
    c = okm.synth_reads(2000, 150, genome_len=1_000_000, first_read=3000, threads=3)
    assert np.array_equal(a[3000 * 151:], c)
    recs = a.reshape(5000, 151)
    assert (recs[:, 150] == ord("\n")).all()
    body = recs[:, :150]
    assert set(np.unique(body).tolist()) <= set(b"ACGTN")
    # error rates near the requested ones (0.1 % substitutions, 0.01 % N)
    n_frac = (body == ord("N")).mean()
    assert 0.00002 < n_frac < 0.0005


@pytest.mark.skipif(has_gpu(), reason="a HIP device is visible")
def test_engine_fails_loudly_without_device():
    with pytest.raises(okm.OkmError) as ei:
        okm.KmerCounter(21)
    assert ei.value.status == _lib.OKM_E_DEVICE
    assert "no CPU fallback" in str(ei.value)
    with pytest.raises(okm.OkmError):
        okm.set_intersection_size(np.array([1], np.uint64), np.array([1], np.uint64))


def test_invalid_k_rejected_before_device():
    for k in (0, 33):
        with pytest.raises(okm.OkmError) as ei:
            okm.KmerCounter(k)
        assert ei.value.status == _lib.OKM_E_INVALID_K
        assert f"Invalid K-mer size: {k}. Must be between 1 and 32." in str(ei.value)


def test_reader_raw_ids_match_restate(golden_cases, tmp_path):
    """query.rs:63-71: record.id() + raw record.sequence() (no normalize)."""
    import restate as R
    from conftest import case_file_bytes
    for c in golden_cases["query"]:
        f = c["reads"]
        p = tmp_path / f["name"]
        p.write_bytes(case_file_bytes(f))
        got = okm.read_fastx_records(str(p), True, raw=True)
        exp = R.parse_fastx(R.decompress_by_extension(f["name"], case_file_bytes(f)))
        assert got == exp, c["name"]
        norm = okm.read_fastx_records(str(p), True, raw=False)
        assert [s for _i, s in norm] == [R.normalize(s) for _i, s in exp], c["name"]


def _bgzf(data: bytes, block: int = 60000) -> bytes:
    """BGZF (blocked gzip, 'BC' extra subfield holding the member size - 1)."""
    import zlib
    out = b""
    for o in range(0, max(len(data), 1), block):
        chunk = data[o:o + block]
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        body = co.compress(chunk) + co.flush()
        bsize = 18 + len(body) + 8
        hdr = bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF, 6, 0, ord("B"), ord("C"), 2, 0])
        hdr += struct.pack("<H", bsize - 1)
        out += hdr + body + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk) & 0xFFFFFFFF)
    return out


def _big_fastx(n_rec: int, seed: int, fastq: bool) -> bytes:
    rng = random.Random(seed)
    alpha = "ACGTacgtNnRU.-~ "
    parts = []
    for i in range(n_rec):
        L = rng.randint(0, 300)
        s = "".join(rng.choice(alpha) for _ in range(L))
        if fastq:
            parts.append(f"@r{i} d\n{s}\n+\n{'I' * L}\n")
        else:  # multi-line FASTA, some CRLF
            nl = "\r\n" if i % 7 == 0 else "\n"
            body = nl.join(s[j:j + 61] for j in range(0, len(s), 61))
            parts.append(f">r{i} d{nl}{body}{nl}")
    return "".join(parts).encode()


@pytest.mark.parametrize("fastq", [False, True])
@pytest.mark.parametrize("codec", ["plain", "gz_members", "bgzf"])
def test_reader_large_parallel_feed(tmp_path, fastq, codec):
    """Host feed: batches above the parallel-normalise threshold,
    multi-member gzip and BGZF (parallel member inflation) all equal the
    restatement's record stream."""
    data = _big_fastx(40000, 7 + fastq, fastq)
    assert len(data) > 4 << 20
    name = "in.fastq" if fastq else "in.fasta"
    if codec == "gz_members":
        half = len(data) // 2
        blob, name = gzip.compress(data[:half]) + gzip.compress(data[half:]), name + ".gz"
    elif codec == "bgzf":
        blob, name = _bgzf(data), name + ".gz"
    else:
        blob = data
    p = tmp_path / name
    p.write_bytes(blob)
    exp = [R.normalize(s) for _, s in R.parse_fastx(data)]
    assert okm.read_fastx_file(str(p), True) == exp
    if codec != "plain":  # needletail sniffing (build path) takes the same gzip
        assert okm.read_fastx_file(str(p), False) == exp


@pytest.mark.parametrize("ext", ["tsv", "gz", "zst"])
def test_tsv_writer_many_blocks(tmp_path, ext):
    """More lines than one formatting round (parallel blocks, one gzip member
    per block): decompressed bytes identical to the serial formatting."""
    rng = np.random.default_rng(3)
    k = 31
    n = 1_300_000
    keys = np.unique(rng.integers(0, 1 << 62, n, dtype=np.uint64))
    counts = rng.integers(1, 1000, len(keys), dtype=np.uint64)
    p = str(tmp_path / f"out.{ext}")
    okm.write_counts_tsv(p, k, keys, counts)
    raw = open(p, "rb").read()
    if ext == "gz":
        raw = gzip.decompress(raw)
    elif ext == "zst":
        raw = R._zstd_decompress(raw)
    lines = raw.split(b"\n")
    assert len(lines) == len(keys) + 1 and lines[-1] == b""
    for i in (0, 1, 131071, 131072, 131073, len(keys) // 2, len(keys) - 1):
        assert lines[i] == R.u64_to_seq(int(keys[i]), k) + b"\t" + str(int(counts[i])).encode()


@pytest.mark.parametrize("no_libdeflate", ["0", "1"])
def test_empty_gz_output_is_valid_gzip(tmp_path, no_libdeflate):
    p = str(tmp_path / "e.tsv.gz")
    # a fresh process: the codec library is chosen at its first use
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import okm; from okm import testing; "
            "testing.set_knob('no_libdeflate', %s); "
            "okm.write_counts_tsv(%r, 5, np.zeros(0, np.uint64), np.zeros(0, np.uint64))"
            % (os.path.dirname(os.path.dirname(okm.__file__)), no_libdeflate, p))
    subprocess.run([sys.executable, "-c", code], check=True)
    assert gzip.decompress(open(p, "rb").read()) == b""


# ---------------------------------------------------------------------------
# multi-GPU owner split (okm_owner_bounds: host code of okm_merge_owned)
# ---------------------------------------------------------------------------

def _owner_bounds_np(hist, world):
    """Restatement: cut r just past the bin where the running total first
    reaches r/world of the whole (okm_dist.hip owner_bounds)."""
    cum = np.cumsum(np.asarray(hist, dtype=np.float64))
    total = cum[-1] if len(cum) else 0.0
    b = [0]
    for r in range(1, world):
        x = int(np.searchsorted(cum, total * r / world, side="left")) + 1
        b.append(max(b[-1], min(x, len(hist))))
    b.append(len(hist))
    return b


@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8, 16])
def test_owner_bounds_vs_restatement(world):
    rng = np.random.default_rng(world)
    for hist in (rng.integers(0, 1000, 1 << 16).astype(np.uint64),
                 np.zeros(1 << 16, np.uint64),
                 np.eye(1, 1 << 16, (1 << 16) - 1, dtype=np.uint64)[0] * 10**9,   # k=32: all in the top bin
                 (rng.pareto(1.0, 4096) * 100).astype(np.uint64),
                 np.array([5], np.uint64)):
        got = okm.owner_bounds(hist, world)
        assert got == _owner_bounds_np(hist, world)
        assert got[0] == 0 and got[-1] == len(hist) and all(a <= b for a, b in zip(got, got[1:]))


def test_owner_bounds_balance():
    # count-balanced: every rank's share within one bin of 1/world of the total
    rng = np.random.default_rng(1)
    hist = rng.integers(0, 50, 1 << 16).astype(np.uint64)
    for world in (2, 4, 8):
        b = okm.owner_bounds(hist, world)
        shares = [int(hist[b[r]:b[r + 1]].sum()) for r in range(world)]
        assert sum(shares) == int(hist.sum())
        assert max(shares) - min(shares) <= 2 * int(hist.max()) + 1


def test_multi_gpu_symbols_exported():
    lib = okm._lib.load()
    for name in ("okm_comm_unique_id", "okm_comm_init_rank", "okm_comm_init_all", "okm_comm_destroy",
                 "okm_comm_rank", "okm_comm_size", "okm_merge_owned", "okm_comm_last_times", "okm_owner_bounds",
                 "okm_synth_reads_device"):
        assert hasattr(lib, name)
