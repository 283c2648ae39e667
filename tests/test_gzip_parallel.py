"""Parallel inflate of single-member gzip input (csrc/okm_inflate.cpp; host
feed, SURVEY §8 f4: utils.rs:125-152 reads `.gz` through flate2's
MultiGzDecoder).  CPU only: okm.read_file (okm_read_file) against Python's
gzip module on FASTQ-like, repetitive, incompressible and fixed-Huffman
streams, with small chunks so every stream is cut many times; the test
knob gz_strict makes the parallel path's rejection an error instead of a
serial retry, so these tests see that path's own output."""

import gzip
import os
import zlib

import numpy as np
import pytest

import okm
from okm import testing


@pytest.fixture
def strict():
    testing.set_knob("gz_strict", 1)
    testing.set_knob("gz_par_min_bytes", 0)
    testing.set_knob("gz_chunk_bytes", 16 << 10)


def _fastq(rng, n, L=150, genome=300_000):
    g = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=genome)
    out = []
    for i in range(n):
        o = int(rng.integers(0, genome - L))
        q = bytes(rng.integers(33, 74, L).astype(np.uint8))
        out.append(b"@read%d\n" % i + g[o:o + L].tobytes() + b"\n+\n" + q + b"\n")
    return b"".join(out)


def _roundtrip(tmp_path, name, blob):
    p = tmp_path / name
    p.write_bytes(blob)
    return okm.read_file(str(p))


@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_fastq_levels(tmp_path, strict, level):
    data = _fastq(np.random.default_rng(level), 12_000)
    assert _roundtrip(tmp_path, f"r{level}.fq.gz", gzip.compress(data, compresslevel=level)) == data


def test_repetitive_and_overlapping_copies(tmp_path, strict):
    """Long runs (copies with distance < 8 and < their length), poly-A reads
    and periodic text: copies that reach across every chunk cut."""
    rng = np.random.default_rng(3)
    parts = [b"A" * 100_000, b"ACGT" * 50_000, b"AC" * 30_000]
    for _ in range(200):
        parts.append(rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=int(rng.integers(1, 3000))).tobytes())
        parts.append(parts[int(rng.integers(0, len(parts)))][:int(rng.integers(3, 40_000))])
    data = b"\n".join(parts)
    for level in (1, 9):
        assert _roundtrip(tmp_path, f"rep{level}.gz", gzip.compress(data, compresslevel=level)) == data


def test_incompressible_and_fixed_huffman(tmp_path, strict):
    """Random bytes (stored blocks: no dynamic block to find, every chunk is
    decoded again from the true boundary) and a fixed-Huffman stream."""
    rng = np.random.default_rng(4)
    data = rng.integers(0, 256, 3_000_000, dtype=np.uint8).tobytes()
    assert _roundtrip(tmp_path, "rand.gz", gzip.compress(data, compresslevel=6)) == data
    text = _fastq(rng, 4000)
    c = zlib.compressobj(6, zlib.DEFLATED, 31, 9, zlib.Z_FIXED)
    assert _roundtrip(tmp_path, "fixed.gz", c.compress(text) + c.flush()) == text


def test_members_padding_and_headers(tmp_path, strict):
    """Concatenated members (MultiGzDecoder reads them all), trailing zero
    padding, and a header with FNAME / FCOMMENT / FEXTRA / FHCRC fields."""
    rng = np.random.default_rng(5)
    a, b = _fastq(rng, 5000), _fastq(rng, 3000)
    blob = gzip.compress(a, 1) + gzip.compress(b, 6) + b"\0" * 100
    assert _roundtrip(tmp_path, "multi.gz", blob) == a + b
    body = gzip.compress(a, 6)
    flg = 4 | 8 | 16 | 2
    extra = b"XY\x03\x00abc"
    hdr = bytes([0x1f, 0x8b, 8, flg]) + body[4:10] + len(extra).to_bytes(2, "little") + extra + b"name.fq\0" \
        + b"a comment\0"
    hdr += (zlib.crc32(hdr) & 0xFFFF).to_bytes(2, "little")
    assert _roundtrip(tmp_path, "hdr.gz", hdr + body[10:]) == a


def test_corrupt_streams_fail(tmp_path, strict):
    data = _fastq(np.random.default_rng(6), 6000)
    blob = bytearray(gzip.compress(data, 6))
    bad_crc = bytes(blob[:-8]) + bytes([blob[-8] ^ 1]) + bytes(blob[-7:])
    with pytest.raises(okm.OkmError):
        _roundtrip(tmp_path, "crc.gz", bad_crc)
    with pytest.raises(okm.OkmError):
        _roundtrip(tmp_path, "trunc.gz", bytes(blob[: len(blob) // 2]))
    flipped = bytearray(blob)
    flipped[len(blob) // 2] ^= 0x55
    with pytest.raises(okm.OkmError):
        _roundtrip(tmp_path, "flip.gz", bytes(flipped))


def test_serial_retry_without_strict(tmp_path, monkeypatch):
    """Default mode: a member the parallel path rejects is decoded serially,
    which reports the error (or, for good data, gives the same bytes)."""
    testing.set_knob("gz_par_min_bytes", 0)
    testing.set_knob("gz_chunk_bytes", 16 << 10)
    data = _fastq(np.random.default_rng(7), 6000)
    blob = gzip.compress(data, 1)
    assert _roundtrip(tmp_path, "ok.gz", blob) == data
    with pytest.raises(okm.OkmError, match="gzip"):
        _roundtrip(tmp_path, "trunc.gz", blob[:-20])
