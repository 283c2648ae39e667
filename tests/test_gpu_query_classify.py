"""Parity of the device query / classify paths with the
oracle, through the C ABI.

- golden cases (the reference's query_tests.rs / classify_tests.rs contents,
  fixture files, restatement-defined raw-sequence edge cases): byte-identical
  ids files / JSON / TSV through the orion-kmer CLI;
- KmerSet: insert/contains/size against Python sets, growth past the initial
  capacity, duplicates, the ~0 key;
- per-read hits at MB scale against the C restatement (oracle_query_hits),
  for compile-time k, runtime k, host and device batches, ragged and long
  records, unaligned device pointers;
- classify statistics at MB scale against numpy set arithmetic on the
  oracle's counts;
- a BASELINE-size property: reads queried against the set of their own
  k-mers hit on every valid window (sum of hits == valid windows).
Integer work: the bar is bit-exact (the two f64 divisions are the host's).
"""

import gzip
import json
import os
import subprocess

import numpy as np
import pytest

import okm
import oracle
from conftest import case_file_bytes, materialize
from oracle import OracleCounter
from okm import _lib

pytestmark = pytest.mark.gpu


def cli(*args):
    return subprocess.run([_lib.CLI_PATH, *args], capture_output=True, text=True, timeout=120)


def build_db(tmp_path, files, k, name):
    paths = materialize(tmp_path, files, subdir=f"{name}_in")
    out = str(tmp_path / f"{name}.db")
    args = ["build", "-k", str(k), "-o", out]
    for p in paths:
        args += ["-g", p]
    r = cli(*args)
    assert r.returncode == 0, r.stderr
    return out


# ---------------------------------------------------------------------------
# goldens through the CLI
# ---------------------------------------------------------------------------

def test_golden_query_cli(golden_cases, tmp_path):
    for i, c in enumerate(golden_cases["query"]):
        db = build_db(tmp_path, c["db_files"], c["k"], f"q{i}")
        reads = materialize(tmp_path, [c["reads"]], subdir=f"q{i}_reads")[0]
        for ext in ("txt", "gz"):
            out = str(tmp_path / f"q{i}.{ext}")
            r = cli("query", "-d", db, "-r", reads, "-o", out, "-c", str(c["min_hits"]))
            assert r.returncode == 0, (c["name"], r.stderr)
            data = open(out, "rb").read()
            if ext == "gz":
                data = gzip.decompress(data) if data else b""
            assert data.decode() == c["expected_output"], c["name"]


def test_golden_classify_cli(golden_cases, tmp_path):
    for i, c in enumerate(golden_cases["classify"]):
        dbs = [build_db(tmp_path, files, c["k"], f"c{i}_{j}") for j, files in enumerate(c["dbs"])]
        inp = materialize(tmp_path, [c["input"]], subdir=f"c{i}_in")[0]
        out, tsv = str(tmp_path / f"c{i}.json"), str(tmp_path / f"c{i}.tsv")
        args = ["classify", "-i", inp, "-o", out, "--output-tsv", tsv,
                "--min-kmer-frequency", str(c["min_freq"]), "--min-coverage", str(c["min_cov"])]
        if c["user_k"] is not None:
            args += ["--kmer-size", str(c["user_k"])]
        for d in dbs:
            args += ["-d", d]
        r = cli(*args)
        assert r.returncode == 0, (c["name"], r.stderr)
        exp_js = c["expected_json"].replace('"INPUT"', json.dumps(inp))
        exp_tsv = c["expected_tsv"].replace("INPUT\t", inp + "\t")
        for j, d in enumerate(dbs):
            exp_js = exp_js.replace(f'"DB{j}"', json.dumps(d))
            exp_tsv = exp_tsv.replace(f"\tDB{j}\t", f"\t{d}\t")
        assert open(out).read() == exp_js, c["name"]
        assert open(tsv).read() == exp_tsv, c["name"]


def test_query_empty_and_short_reads(tmp_path):
    db = build_db(tmp_path, [{"name": "g.fa", "text": ">g\nACGTACGTTTGCATC\n"}], 4, "e")
    reads = tmp_path / "r.fq"
    reads.write_text("@a\nACG\n+\nIII\n@b\n\n+\n\n")
    out = str(tmp_path / "o.txt")
    r = cli("query", "-d", db, "-r", str(reads), "-o", out, "-c", "0")
    assert r.returncode == 0, r.stderr
    assert open(out).read() == ""  # shorter than k: never reported (query.rs:83-85)
    reads.write_text("")
    r = cli("query", "-d", db, "-r", str(reads), "-o", out)
    assert r.returncode == 1 and "Failed to parse FASTQ content from" in r.stderr
    assert open(out).read() == ""


# ---------------------------------------------------------------------------
# KmerSet
# ---------------------------------------------------------------------------

def test_kset_insert_contains_grow():
    rng = np.random.default_rng(5)
    with okm.KmerSet(31, 0, capacity_hint=10) as s:
        seen = set()
        for rnd in range(4):  # several growths from a 1024-slot table
            keys = rng.integers(0, 1 << 62, size=20000 * (rnd + 1), dtype=np.uint64)
            keys = np.concatenate([keys, keys[:500]])  # duplicates within a batch
            new = s.insert(keys)
            assert new == len(set(keys.tolist()) - seen)
            seen |= set(keys.tolist())
            assert len(s) == len(seen)
        probe = np.concatenate([np.array(sorted(seen)[:5000], np.uint64),
                                rng.integers(0, 1 << 62, size=5000, dtype=np.uint64)])
        got = s.contains(probe)
        assert got.tolist() == [int(x) in seen for x in probe.tolist()]
        # ~0 is the empty slot: it lives in a side flag
        assert not s.contains(np.array([~np.uint64(0)], np.uint64))[0]
        assert s.insert(np.array([~np.uint64(0)] * 3, np.uint64)) == 1
        assert s.contains(np.array([~np.uint64(0)], np.uint64))[0]


# ---------------------------------------------------------------------------
# per-read hits vs the C restatement
# ---------------------------------------------------------------------------

def _reads(rng, genome, n, lo, hi, noise=0.01, lower=0.0):
    out = []
    alpha = np.frombuffer(b"ACGTNacgtU", np.uint8)
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        o = int(rng.integers(0, max(1, len(genome) - L)))
        r = genome[o:o + L].copy() if rng.random() < 0.7 else rng.choice(alpha[:4], size=L)
        m = rng.random(len(r)) < noise
        r[m] = rng.choice(alpha, size=int(m.sum()))
        if lower:
            lm = rng.random(len(r)) < lower
            r[lm] = r[lm] | 0x20
            r[r == ord("u")] = ord("U")
        out.append(r.tobytes())
    return out


@pytest.mark.parametrize("k", [31, 21, 32, 17, 5, 15, 16, 27])
def test_query_hits_vs_oracle(k):
    rng = np.random.default_rng(100 + k)
    genome = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=200_000)
    # the DB: the genome's first 60 % as two references
    oc = OracleCounter(k)
    oc.add_records([genome[:70_000].tobytes(), genome[60_000:120_000].tobytes()])
    db_keys, _ = oc.result(1)
    reads = _reads(rng, genome, 6000, 1, 400, lower=0.05)
    reads += [b"", b"ACGT\nACGTACGTACGTACGTACGTACGTACGTACGT", b"N" * 50]
    exp = oracle.query_hits(reads, db_keys, k)
    with okm.KmerSet(k, 0, len(db_keys) // 4) as s:
        s.insert(db_keys[::2])
        s.insert(db_keys[1::2])
        assert len(s) == len(db_keys)
        got = s.query_hits(reads)
    assert np.array_equal(got, exp)
    assert exp.sum() > 0


def _revcomp(b: bytes) -> bytes:
    return b[::-1].translate(bytes.maketrans(b"ACGTacgt", b"TGCAtgca"))


@pytest.mark.parametrize("k", [31, 25, 12])
def test_query_both_strands_and_rebuild(k):
    """The device set finds a canonical key from either strand of a read, and
    a query after more inserts sees them; equal to the restatement."""
    rng = np.random.default_rng(k)
    genome = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=150_000)
    g = genome.tobytes()
    fwd = [g[o:o + int(rng.integers(40, 300))] for o in rng.integers(0, 140_000, 3000)]
    reads = fwd + [_revcomp(r) for r in fwd[:1500]]  # the other strand of half of them
    oc = OracleCounter(k)
    oc.add_records([g[:90_000]])
    db_keys, _ = oc.result(1)
    exp = oracle.query_hits(reads, db_keys, k)
    with okm.KmerSet(k, 0, len(db_keys) // 4) as s:
        s.insert(db_keys[: len(db_keys) // 2])
        s.query_hits(reads)
        s.insert(db_keys)  # grows the table (rehash); the next query sees every key
        got = s.query_hits(reads)
    assert np.array_equal(got, exp)
    assert exp[1500:3000].sum() > 0 and exp[3000:4500].sum() > 0  # both strands hit


def test_query_hits_device_batch_long_records():
    k = 31
    rng = np.random.default_rng(7)
    genome = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=300_000)
    oc = OracleCounter(k)
    oc.add_records([genome[:150_000].tobytes()])
    db_keys, _ = oc.result(1)
    reads = _reads(rng, genome, 300, 2000, 12_000)  # ONT-like: records span many tiles
    reads = [r.replace(b"\n", b"N") for r in reads]
    exp = oracle.query_hits(reads, db_keys, k)
    batch = np.frombuffer(b"".join(r + b"\n" for r in reads), np.uint8)
    with okm.KmerSet(k, 0, len(db_keys)) as s:
        s.insert(db_keys)
        for shift in (0, 3):  # aligned and unaligned device pointers
            buf = okm.DeviceBuffer(len(batch) + 16)
            hb = okm.DeviceBuffer(4 * len(reads))
            try:
                pad = np.zeros(shift, np.uint8)
                buf.upload(np.concatenate([pad, batch]))
                s.query_hits_device(buf.address + shift, len(batch), len(reads), hb.address)
                got = np.zeros(len(reads), np.uint32)
                hb.download(got)
            finally:
                buf.free()
                hb.free()
            assert np.array_equal(got, exp), shift


def test_query_hits_empty_set_and_no_records():
    with okm.KmerSet(21) as s:
        assert s.query_hits([b"ACGT" * 20]).tolist() == [0]
        assert s.query_hits([]).tolist() == []


# ---------------------------------------------------------------------------
# classify statistics vs numpy on the oracle's counts
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("min_freq", [1, 3])
def test_classifier_vs_oracle(min_freq):
    k = 25
    rng = np.random.default_rng(11 + min_freq)
    genome = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=100_000)
    reads = _reads(rng, genome, 8000, 80, 200, noise=0.005)
    oc = OracleCounter(k)
    oc.add_records(reads)
    ik, ic = oc.result(min_freq)
    refs = []
    for lo, hi in ((0, 40_000), (30_000, 70_000), (0, 0), (90_000, 100_000)):
        oc = OracleCounter(k)
        oc.add_records([genome[lo:hi].tobytes()])
        refs.append(oc.result(1)[0])
    refs.append(rng.integers(0, 1 << 50, size=5000, dtype=np.uint64))  # foreign keys
    with okm.KmerCounter(k, "count") as c:
        c.add_records(reads)
        with okm.Classifier(c, min_freq) as cl:
            assert cl.n_input == len(ik)
            got = cl.probe_db(refs)
            keys_all, offs = okm.Classifier.pack_db(refs)
            dk = okm.DeviceBuffer(max(8, keys_all.nbytes))
            dk.upload(keys_all)
            got_d = cl.probe_db(packed=(None, offs), d_keys=dk.address)  # okm_classifier_probe_db_device
            dk.free()
    for f in ("ref_matched", "ref_sum_depth"):
        assert np.array_equal(got[f], got_d[f])
    assert (got["union"], got["matched"], got["sum_depth"]) == (got_d["union"], got_d["matched"], got_d["sum_depth"])
    for r, keys in enumerate(refs):
        m = np.isin(keys, ik)
        pos = np.searchsorted(ik, keys[m])
        assert got["ref_matched"][r] == m.sum()
        assert got["ref_sum_depth"][r] == ic[pos].sum()
    uni = np.unique(np.concatenate(refs))
    m = np.isin(uni, ik)
    assert got["union"] == len(uni)
    assert got["matched"] == m.sum()
    assert got["sum_depth"] == ic[np.searchsorted(ik, uni[m])].sum()


def test_classifier_staged_database_pieces():
    # a database past one 64 MiB pinned staging piece (okm_probe.hip
    # stage_keys: 2 buffers, host threads + overlapped DMA): host and device
    # entry points agree, and the union / matches equal numpy
    k = 31
    rng = np.random.default_rng(3)
    reads = [rng.choice(np.frombuffer(b"ACGT", np.uint8), size=150).tobytes() for _ in range(20_000)]
    oc = OracleCounter(k)
    oc.add_records(reads)
    ik, ic = oc.result(1)
    foreign = rng.integers(0, 1 << 62, size=21_000_000, dtype=np.uint64)  # 168 MB: three pieces
    refs = [np.unique(np.concatenate([ik[: len(ik) // 2], foreign[:11_000_000]])),
            np.unique(np.concatenate([ik[len(ik) // 3:], foreign[10_000_000:]]))]
    with okm.KmerCounter(k, "count") as c:
        c.add_records(reads)
        with okm.Classifier(c, 1) as cl:
            got = cl.probe_db(refs)
            keys_all, offs = okm.Classifier.pack_db(refs)
            dk = okm.DeviceBuffer(keys_all.nbytes)
            dk.upload(keys_all)
            got_d = cl.probe_db(packed=(None, offs), d_keys=dk.address)
            dk.free()
    uni = np.unique(keys_all)
    m = np.isin(uni, ik)
    for g in (got, got_d):
        assert g["union"] == len(uni) and g["matched"] == m.sum()
        assert g["sum_depth"] == ic[np.searchsorted(ik, uni[m])].sum()
        for r, keys in enumerate(refs):
            assert g["ref_matched"][r] == np.isin(keys, ik).sum()


# ---------------------------------------------------------------------------
# BASELINE-size property
# ---------------------------------------------------------------------------

def test_query_full_size_self_hits():
    """3.36 M x 150 bp reads (BASELINE configs[1]) queried against the set of
    their own canonical k-mers: every valid window hits, so per-read hits ==
    valid windows per read, and their sum == the counter's total."""
    k = 31
    n_reads, L = 3_355_443, 150
    batch = okm.synth_reads(n_reads, L, genome_len=100_000_000, genome_seed=2, seed=2)
    buf = okm.DeviceBuffer(len(batch))
    hb = okm.DeviceBuffer(4 * n_reads)
    try:
        buf.upload(batch)
        with okm.KmerCounter(k, "count") as c:
            c.add_device_batch(buf.address, len(batch))
            c.count()
            keys, counts = c.result(1)
            total = int(counts.sum())
        with okm.KmerSet(k, 0, len(keys)) as s:
            assert s.insert(keys) == len(keys)
            s.query_hits_device(buf.address, len(batch), n_reads, hb.address)
            hits = np.zeros(n_reads, np.uint32)
            hb.download(hits)
    finally:
        buf.free()
        hb.free()
    assert int(hits.sum(dtype=np.uint64)) == total
    # per read: spot-check 2000 reads against the C restatement
    recs = batch.reshape(n_reads, L + 1)[:, :L]
    idx = np.random.default_rng(0).choice(n_reads, 2000, replace=False)
    exp = oracle.query_hits([recs[i].tobytes() for i in idx], keys, k)
    assert np.array_equal(hits[idx], exp)
