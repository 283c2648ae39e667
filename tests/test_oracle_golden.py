"""Pin the oracle: the Python and C restatements against the reference's own
test expectations (tests/golden/reference_expectations.json, transcribed from
orion-kmer/src/kmer.rs:108-341 and orion-kmer/tests/*.rs) and against the
committed goldens (tests/golden/cases.json).  CPU only."""

import random

import numpy as np
import pytest

import restate as R
from conftest import case_file_bytes
from oracle import OracleCounter, load as oracle_load


def test_restate_codec_kats(reference_expectations):
    E = reference_expectations
    for c in E["seq_to_u64"]:
        assert R.seq_to_u64(c["seq"].encode(), c["k"]) == c["value"], c["src"]
    for c in E["u64_to_seq"]:
        assert R.u64_to_seq(c["value"], c["k"]).decode() == c["seq"], c["src"]
    for c in E["reverse_complement"]:
        k = len(c["seq"])
        assert R.reverse_complement_u64(R.seq_to_u64(c["seq"].encode(), k), k) == R.seq_to_u64(c["rc"].encode(), k)
    for c in E["canonical"]:
        k = len(c["seq"])
        assert R.canonical_u64(R.seq_to_u64(c["seq"].encode(), k), k) == R.seq_to_u64(c["canon"].encode(), k)
    with pytest.raises(ValueError):
        R.u64_to_seq(0, 0)
    with pytest.raises(ValueError):
        R.u64_to_seq(0, 33)
    with pytest.raises(ValueError):
        R.reverse_complement_u64(0, 0)
    with pytest.raises(ValueError):
        R.u64_to_dna_base(4)


def test_restate_count_matches_reference_tests(reference_expectations):
    for c in reference_expectations["count"]:
        tsv = R.run_count_bytes([(n, t.encode()) for n, t in c["files"]], c["k"], c["min_count"])
        assert sorted(tsv.strip().splitlines()) == c["expected_sorted_lines"], c["src"]


def test_restate_count_errors(reference_expectations):
    for c in reference_expectations["count_errors"]:
        with pytest.raises(R.OracleError) as ei:
            R.run_count_bytes([("x.fa", b">a\nACGT\n")], c["k"])
        assert c["stderr_contains"] in str(ei.value)


def test_restate_build_matches_reference_tests(reference_expectations):
    for c in reference_expectations["build"]:
        k = c["k"]
        refs = R.build_sets([(n, t.encode()) for n, t in c["files"]], k)
        exp = {n: {R.canonical_u64(R.seq_to_u64(s.encode(), k), k) for s in v} for n, v in c["expected"].items()}
        assert refs == exp, c["src"]
        assert len(set().union(*refs.values())) == c["total_unique"]


def test_restate_compare_matches_reference_tests(reference_expectations):
    for c in reference_expectations["compare"]:
        k = c["k"]
        r1 = R.build_sets([(n, t.encode()) for n, t in c["db1"]], k)
        r2 = R.build_sets([(n, t.encode()) for n, t in c["db2"]], k)
        res = R.compare_sets(k, r1, k, r2)
        assert res["db1_total_unique_kmers_across_references"] == c["db1_total"], c["src"]
        assert res["db2_total_unique_kmers_across_references"] == c["db2_total"]
        assert res["intersection_size"] == c["intersection"]
        assert res["union_size"] == c["union"]
        assert abs(res["jaccard_index"] - c["intersection"] / c["union"]) < 1e-12
    for c in reference_expectations["compare_errors"]:
        with pytest.raises(R.OracleError) as ei:
            R.compare_sets(c["k1"], {}, c["k2"], {})
        assert c["stderr_contains"] in str(ei.value)


def test_fixture_files_decode_to_transcribed_bytes(reference_expectations):
    fx = reference_expectations["fixture_files"]
    for ext in ("gz", "xz", "zst"):
        for base in ("test_input1.fasta", "test_input2.fastq"):
            raw = case_file_bytes({"fixture": f"{base}.{ext}"})
            assert R.decompress_by_extension(f"{base}.{ext}", raw).decode() == fx[base]


def test_golden_cases_regenerate(golden_cases):
    """cases.json is exactly what the pinned restatement produces."""
    for c in golden_cases["count"]:
        tsv = R.run_count_bytes([(f["name"], case_file_bytes(f)) for f in c["files"]], c["k"], c["min_count"])
        assert tsv == c["expected_tsv"], c["name"]


# ---------------------------------------------------------------------------
# C restatement
# ---------------------------------------------------------------------------

def test_c_oracle_codec_kats(reference_expectations):
    import ctypes
    lib = oracle_load()
    for c in reference_expectations["seq_to_u64"]:
        out = ctypes.c_uint64()
        ok = lib.oracle_seq_to_u64(c["seq"].encode(), len(c["seq"]), c["k"], ctypes.byref(out))
        assert (out.value if ok else None) == c["value"], c["src"]
    rng = random.Random(7)
    for _ in range(2000):
        k = rng.randint(1, 32)
        v = rng.getrandbits(2 * k)
        assert lib.oracle_reverse_complement_u64(v, k) == R.reverse_complement_u64(v, k)
        assert lib.oracle_canonical_u64(v, k) == R.canonical_u64(v, k)


def _records_of(files):
    recs = []
    for f in files:
        data = R.decompress_by_extension(f["name"], case_file_bytes(f))
        recs.extend(s for _, s in R.parse_fastx(data))
    return recs


def test_c_oracle_matches_goldens(golden_cases):
    for c in golden_cases["count"]:
        oc = OracleCounter(c["k"])
        oc.add_records(_records_of(c["files"]), normalized=False)
        keys, counts = oc.result(c["min_count"])
        tsv = R.format_counts(dict(zip(keys.tolist(), counts.tolist())), c["k"], c["min_count"])
        assert tsv == c["expected_tsv"], c["name"]


def test_c_oracle_matches_restate_random():
    rng = random.Random(99)
    for trial in range(30):
        k = rng.choice([1, 2, 3, 5, 8, 13, 21, 31, 32])
        seqs = [bytes(rng.choice(b"ACGTacgtNNU-") for _ in range(rng.randint(0, 120))) for _ in range(rng.randint(1, 12))]
        exp = R.count_records(seqs, k)
        oc = OracleCounter(k)
        oc.add_records(seqs)
        keys, counts = oc.result(1)
        assert dict(zip(keys.tolist(), counts.tolist())) == exp
        assert oc.windows == sum(exp.values())


def test_c_oracle_separated_layout_equals_records():
    rng = random.Random(5)
    seqs = [bytes(rng.choice(b"ACGT") for _ in range(rng.randint(0, 60))) for _ in range(50)]
    a = OracleCounter(11)
    a.add_records(seqs)
    b = OracleCounter(11)
    b.add_separated(np.frombuffer(b"\n".join(seqs), dtype=np.uint8))
    ka, ca = a.result()
    kb, cb = b.result()
    assert np.array_equal(ka, kb) and np.array_equal(ca, cb)


def test_c_oracle_pairs_merge():
    a = OracleCounter(7)
    a.add_pairs(np.array([5, 3, 5], np.uint64), np.array([1, 2, 10], np.uint64))
    k, c = a.result(1)
    assert k.tolist() == [3, 5] and c.tolist() == [2, 11]
    assert a.result(3)[0].tolist() == [5]


# --------------------------------------------------------------------------
# query / classify: restatement vs the reference's tests
# --------------------------------------------------------------------------

def _db(files, k):
    return R.build_sets([(n, t.encode()) for n, t in files], k)


def test_restate_query_matches_reference_tests(reference_expectations):
    for c in reference_expectations["query"]:
        refs = _db(c["db_files"], c["k"])
        out = R.run_query_bytes(c["k"], refs, "query_reads.fastq", c["reads"].encode(), c["min_hits"])
        ids = set(out.decode().splitlines())
        assert ids == set(c["expected_ids"]), c["src"]


def test_restate_query_hits_comment_values():
    # query_tests.rs:119-124: per-read hits 7 / 1 / 0 / (too short) / 9
    refs = _db([("db.fa", ">ref_genome_segment\nACGTACGTTTGCATC")], 4)
    allk = set().union(*refs.values())
    assert [R.query_hits(s, 4, allk) for s in (b"ACGTACGTTT", b"TTGCXXXXXX", b"CCCCCCCCCC", b"ACGTACGTACGT")] == \
        [7, 1, 0, 9]


def _classify(c, user_k="default", min_freq=None, min_cov=None):
    dbs = []
    for i, files in enumerate(c["dbs"]):
        refs = _db(files, c["k"])
        dbs.append((f"db{i}.db", c["k"], [(n, refs[n]) for n, _t in files]))
    return R.run_classify_bytes("input.fa", c["input"].encode(), dbs,
                                c.get("user_k") if user_k == "default" else user_k,
                                c.get("min_freq", 1) if min_freq is None else min_freq,
                                c.get("min_cov", 0.0) if min_cov is None else min_cov)


def test_restate_classify_matches_reference_tests(reference_expectations):
    import json
    for c in reference_expectations["classify"]:
        js, _tsv = _classify(c)
        res = json.loads(js)
        assert res["total_unique_kmers_in_input"] == c["total_unique_kmers_in_input"], c["src"]
        assert res["min_kmer_frequency_filter"] == c["min_freq"]
        assert len(res["databases_analyzed"]) == len(c["databases"])
        for got, exp in zip(res["databases_analyzed"], c["databases"]):
            assert got["database_kmer_size"] == c["k"]
            if "references_listed" in exp:
                assert [r["reference_name"] for r in got["references"]] == exp["references_listed"], c["src"]
                continue
            assert got["total_unique_kmers_in_db_across_references"] == exp["union"], c["src"]
            assert got["overall_input_kmers_matched_in_db"] == exp["matched"], c["src"]
            assert got["overall_sum_depth_of_matched_kmers_in_input"] == exp["sum_depth"], c["src"]
            m, sd, u, n_in = exp["matched"], exp["sum_depth"], exp["union"], c["total_unique_kmers_in_input"]
            assert abs(got["overall_avg_depth_of_matched_kmers_in_input"] - sd / m) < 1e-12
            assert abs(got["proportion_input_kmers_in_db_overall"] - m / n_in) < 1e-12
            assert abs(got["proportion_db_kmers_covered_overall"] - m / u) < 1e-12
            refs = {r["reference_name"]: r for r in got["references"]}
            assert set(refs) == set(exp["references"])
            for name, (tot, hit, depth) in exp["references"].items():
                r = refs[name]
                assert (r["total_kmers_in_reference"], r["input_kmers_hitting_reference"],
                        r["sum_depth_of_matched_kmers_in_input"]) == (tot, hit, depth), (c["src"], name)
                assert abs(r["reference_breadth_of_coverage"] - hit / tot) < 1e-12


def test_restate_classify_tsv_matches_reference_tests(reference_expectations):
    for c in reference_expectations["classify_tsv"]:
        _js, tsv = _classify(c, user_k=c["k"], min_freq=1)
        lines = tsv.splitlines()
        assert lines[0].split("\t")[0] == "InputFile"
        rows = [ln.split("\t") for ln in lines[1:]]
        assert [r[2:] for r in rows] == c["rows"], c["src"]
        assert all(r[0] == "input.fa" for r in rows)


def test_restate_classify_errors(reference_expectations):
    for c in reference_expectations["classify_errors"]:
        dbs = [(f"db{i}.db", k, []) for i, k in enumerate(c["db_ks"])]
        with pytest.raises(R.OracleError) as ei:
            R.run_classify_bytes("dummy_input.fa", b">a\nACGT\n", dbs, c["user_k"])
        assert c["stderr_contains"] in str(ei.value), c["src"]


def test_rust_f64_format():
    # serde_json / ryu layout (what compare.rs and classify.rs write)
    cases = {0.0: "0.0", 1.0: "1.0", 0.375: "0.375", 1 / 3: "0.3333333333333333", 1e-5: "0.00001",
             1e-6: "1e-6", 1.5e-7: "1.5e-7", 1e16: "1e16", 123.0: "123.0", 2.5e15: "2500000000000000.0"}
    for x, s in cases.items():
        assert R.rust_f64(x) == s, x


@pytest.mark.parametrize("k,threads", [(31, 1), (31, 3), (21, 8), (32, 5), (5, 4)])
def test_c_oracle_mt_equals_single(k, threads):
    """The labelled restatement-MT CPU number (bench.py cpu_baseline_mt) counts
    exactly what the single-threaded restatement counts."""
    from oracle import count_separated_mt
    rng = np.random.default_rng(k * 10 + threads)
    recs = [bytes(rng.choice(list(b"ACGTNacgt"), size=int(rng.integers(0, 300)))) for _ in range(400)]
    recs += [b"A" * 200] * 7  # a hot key across shards
    rng.shuffle(recs)
    data = np.frombuffer(b"\n".join(recs), dtype=np.uint8)
    oc = OracleCounter(k)
    oc.add_separated(data)
    ek, ec = oc.result(1)
    gk, gc = count_separated_mt(data, k, threads)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


# ---------------------------------------------------------------------------
# BASELINE configs[0] (C1): 10 x 100 kb FASTA wrapped at 60 columns, k = 21
# ---------------------------------------------------------------------------

def test_c1_oracle_vs_restatement_fixture(tmp_path):
    """The C oracle (+ the host reader's needletail normalisation and the TSV
    writer) on the full C1 input equals the pure-Python restatement's output
    (tests/golden/c1_k21.json, made by tests/golden/make_c1_golden.py)."""
    import hashlib
    import json
    import os
    import sys
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from make_c1_fasta import c1_fasta
    import okm
    from oracle import OracleCounter
    with open(os.path.join(ROOT, "tests", "golden", "c1_k21.json")) as fh:
        fx = json.load(fh)
    data = c1_fasta()
    assert hashlib.sha256(data).hexdigest() == fx["input_sha256"]
    recs = okm.parse_fastx(data)  # host reader: multi-line join, normalize (count.rs:71)
    assert len(recs) == 10 and all(len(r) == 100_000 for r in recs)
    oc = OracleCounter(21)
    oc.add_records(recs, normalized=True)
    for m, key in ((1, "m1"), (2, "m2")):
        keys, counts = oc.result(m)
        out = tmp_path / f"c1_m{m}.tsv"
        okm.write_counts_tsv(str(out), 21, keys, counts)
        raw = out.read_bytes()
        assert len(raw) == fx[key]["bytes"] and raw.count(b"\n") == fx[key]["lines"]
        assert hashlib.sha256(raw).hexdigest() == fx[key]["sha256"]


@pytest.mark.parametrize("k", [33, 63, 64])
def test_wide_range_shards_equal_the_restatement(k):
    """The rolling range-sharded k<=64 helper (count_separated_wide_ranges,
    used by the 1 Gbases k=63 GPU test) equals the O(k) restatement."""
    from oracle import OracleCounterWide, count_separated_wide_ranges
    import okm
    batch = okm.synth_reads(3_000, 150, genome_len=100_000, genome_seed=k, seed=k + 1, sub_rate=0.02, n_rate=0.002)
    batch.reshape(3_000, 151)[::97, :150] = ord("A")  # a hot key
    oc = OracleCounterWide(k)
    oc.add_records([r for r in batch.tobytes().split(b"\n") if r], normalized=True)
    ek, ec = oc.result(1)
    gk, gc, w = count_separated_wide_ranges(batch, k, threads=5)
    assert w == oc.windows
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


@pytest.mark.parametrize("k", [5, 21, 31, 32])
def test_u64_range_filter_equals_the_restatement(k):
    """The rolling key-range helper (count_separated_ranges_mt, used by the
    full-size C3 and P = 8 rehearsal GPU tests) equals the O(k) restatement
    restricted to the same ranges, over several chunks and threads."""
    from oracle import count_separated_ranges_mt
    import okm
    batch = okm.synth_reads(4_000, 150, genome_len=50_000, genome_seed=k, seed=k + 3, sub_rate=0.02, n_rate=0.002)
    batch.reshape(4_000, 151)[::89, :150] = ord("A")  # a hot key (all-A: key 0)
    oc = OracleCounter(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    top = 1 << (2 * k) if k < 32 else 1 << 64
    rng = np.random.default_rng(k)
    ranges = [(0, max(1, top >> 12))]  # includes key 0 (poly-A)
    for _ in range(9):
        a = int(rng.integers(0, top >> 1)) if k == 32 else int(rng.integers(0, top))
        ranges.append((a, min(top - 1, a + max(1, top >> int(rng.integers(4, 9))))))
    ranges.append((top - (top >> 6), top - 1))
    sel = np.zeros(len(ek), bool)
    for lo, hi in ranges:
        sel |= (ek >= np.uint64(lo)) & (ek < np.uint64(hi))
    half = 2_000 * 151
    gk, gc, w = count_separated_ranges_mt([batch[:half], batch[half:]], k, ranges, threads=3)
    assert w == oc.windows
    assert sel.sum() > 10
    assert np.array_equal(gk, ek[sel]) and np.array_equal(gc, ec[sel])
