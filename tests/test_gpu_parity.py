"""Parity of the HIP engine (through the C ABI) with the oracle.

- golden cases (reference test contents, reference fixture files,
  restatement-defined edge cases): byte-identical TSV / sets / JSON, via the
  Python host layer and via the orion-kmer CLI;
- seeded random batches at MB scale: exact (key, count) equality with the C
  restatement (oracle/okm_oracle.c);
- full BASELINE-size batches: size-independent properties (sum of counts ==
  valid windows, strictly sorted unique keys, every key canonical,
  determinism, batch-split and pairs-merge invariance).
Integer work: the bar is bit-exact.
"""

import json
import os
import subprocess

import numpy as np
import pytest

import okm
import restate as R
from conftest import case_file_bytes, materialize
from okm import _lib, testing
from oracle import OracleCounter, OracleCounterWide, count_separated_mt

pytestmark = pytest.mark.gpu


def counts_dict(keys, counts):
    return dict(zip(keys.tolist(), counts.tolist()))


def np_revcomp(v: np.ndarray, k: int) -> np.ndarray:
    x = ~v.astype(np.uint64)
    for s, m in ((2, 0x3333333333333333), (4, 0x0F0F0F0F0F0F0F0F), (8, 0x00FF00FF00FF00FF),
                 (16, 0x0000FFFF0000FFFF)):
        m = np.uint64(m)
        x = ((x >> np.uint64(s)) & m) | ((x & m) << np.uint64(s))
    x = (x >> np.uint64(32)) | (x << np.uint64(32))
    return x >> np.uint64(64 - 2 * k)


def valid_windows(batch: np.ndarray, k: int) -> int:
    """Number of k-windows of all-ACGT bytes in a separator-joined batch
    (count.rs:28-36: every window that seq_to_u64 accepts)."""
    total = 0
    step = 1 << 26
    valid_set = np.zeros(256, bool)
    valid_set[list(b"ACGTacgtUu")] = True
    for o in range(0, len(batch), step):
        seg = batch[o:o + step + k - 1]  # windows starting in [o, o + step)
        if len(seg) < k:
            break
        bad = ~valid_set[seg]
        c = np.concatenate([[0], np.cumsum(bad, dtype=np.int64)])
        total += int(((c[k:] - c[:-k]) == 0).sum())
    return total


def assert_table_invariants(keys, counts, k):
    assert keys.dtype == np.uint64
    if len(keys) > 1:
        assert (keys[1:] > keys[:-1]).all(), "keys must be strictly increasing (count.rs:119)"
    assert (counts >= 1).all()
    if k < 32:
        assert (keys < np.uint64(1) << np.uint64(2 * k)).all()
    assert (keys <= np_revcomp(keys, k)).all(), "every key must be canonical (kmer.rs:99-106)"


# ---------------------------------------------------------------------------
# goldens
# ---------------------------------------------------------------------------

def test_device_visible():
    assert okm.device_count() >= 1
    assert okm.device_arch(0) == "gfx950"


def test_golden_count_cases_engine(golden_cases):
    for c in golden_cases["count"]:
        with okm.KmerCounter(c["k"]) as ctr:
            for f in c["files"]:
                raw = R.decompress_by_extension(f["name"], case_file_bytes(f))
                ctr.add_records(okm.parse_fastx(raw), normalized=True)
            keys, counts = ctr.result(c["min_count"])
        tsv = "".join(f"{R.u64_to_seq(int(a), c['k']).decode()}\t{int(b)}\n" for a, b in zip(keys, counts))
        assert tsv == c["expected_tsv"], c["name"]


def test_golden_count_cases_raw_records(golden_cases):
    """Un-normalised record bytes: the device LUT applies normalize()."""
    for c in golden_cases["count"]:
        recs = []
        for f in c["files"]:
            raw = R.decompress_by_extension(f["name"], case_file_bytes(f))
            recs += [s for _, s in R.parse_fastx(raw)]
        with okm.KmerCounter(c["k"]) as ctr:
            ctr.add_records(recs, normalized=False)
            keys, counts = ctr.result(c["min_count"])
        exp = R.count_records(recs, c["k"])
        exp = {a: b for a, b in exp.items() if b >= c["min_count"]}
        assert counts_dict(keys, counts) == exp, c["name"]


def test_golden_count_cases_cli(golden_cases, tmp_path):
    for i, c in enumerate(golden_cases["count"]):
        paths = materialize(tmp_path, c["files"], f"c{i}")
        out = tmp_path / f"c{i}.tsv"
        args = [_lib.CLI_PATH, "count", "-k", str(c["k"]), "-o", str(out), "-m", str(c["min_count"])]
        for p in paths:
            args += ["-i", p]
        r = subprocess.run(args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (c["name"], r.stderr)
        assert out.read_text() == c["expected_tsv"], c["name"]


@pytest.mark.parametrize("ext", ["gz", "xz", "zst"])
def test_cli_compressed_output(golden_cases, tmp_path, ext):
    c = golden_cases["count"][0]
    paths = materialize(tmp_path, c["files"])
    out = tmp_path / f"o.tsv.{ext}"
    r = subprocess.run([_lib.CLI_PATH, "count", "-k", str(c["k"]), "-i", *paths, "-o", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert R.decompress_by_extension(str(out), out.read_bytes()).decode() == c["expected_tsv"]


def test_cli_error_contexts(tmp_path):
    empty = tmp_path / "empty.fa"
    empty.write_bytes(b"")
    r = subprocess.run([_lib.CLI_PATH, "count", "-k", "5", "-i", str(empty), "-o", str(tmp_path / "o")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and f"Failed to parse FASTA/Q content from: {empty}" in r.stderr
    missing = tmp_path / "missing.fa"
    r = subprocess.run([_lib.CLI_PATH, "count", "-k", "5", "-i", str(missing), "-o", str(tmp_path / "o")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and f"Failed to get input reader for file: {missing}" in r.stderr
    bad = tmp_path / "bad.fq"
    bad.write_bytes(b"@r\nACGT\n+\nII\n")
    r = subprocess.run([_lib.CLI_PATH, "count", "-k", "3", "-i", str(bad), "-o", str(tmp_path / "o")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and f"Error reading record from {bad}" in r.stderr


def test_golden_build_cases_cli(golden_cases, tmp_path):
    for i, c in enumerate(golden_cases["build"]):
        paths = materialize(tmp_path, c["files"], f"b{i}")
        out = tmp_path / f"b{i}.db"
        args = [_lib.CLI_PATH, "build", "-k", str(c["k"]), "-o", str(out)]
        for p in paths:
            args += ["-g", p]
        r = subprocess.run(args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (c["name"], r.stderr)
        db = okm.KmerDb.read(str(out))
        assert db.k == c["k"]
        assert {n: v.tolist() for n, v in db.references.items()} == c["expected"], c["name"]


def test_golden_compare_cases_cli(golden_cases, tmp_path):
    for i, c in enumerate(golden_cases["compare"]):
        dbs = []
        for j, (k, files) in enumerate(((c["k1"], c["files1"]), (c["k2"], c["files2"]))):
            paths = materialize(tmp_path, files, f"m{i}_{j}")
            out = tmp_path / f"m{i}_{j}.db"
            args = [_lib.CLI_PATH, "build", "-k", str(k), "-o", str(out)]
            for p in paths:
                args += ["-g", p]
            assert subprocess.run(args, capture_output=True, timeout=120).returncode == 0
            dbs.append(str(out))
        js = tmp_path / f"m{i}.json"
        r = subprocess.run([_lib.CLI_PATH, "compare", "--db1", dbs[0], "--db2", dbs[1], "-o", str(js)],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (c["name"], r.stderr)
        exp = c["expected_json"].replace('"DB1"', json.dumps(dbs[0])).replace('"DB2"', json.dumps(dbs[1]))
        assert js.read_text() == exp, c["name"]


def test_compare_k_mismatch_cli(tmp_path):
    a = tmp_path / "a.fa"
    a.write_text(">s\nACGTACGT\n")
    for k in (3, 4):
        subprocess.run([_lib.CLI_PATH, "build", "-k", str(k), "-g", str(a), "-o", str(tmp_path / f"k{k}.db")],
                       check=True, capture_output=True, timeout=120)
    r = subprocess.run([_lib.CLI_PATH, "compare", "--db1", str(tmp_path / "k3.db"), "--db2", str(tmp_path / "k4.db"),
                        "-o", str(tmp_path / "x.json")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1
    assert "K-mer databases have incompatible k-mer sizes (overall comparison): 3 vs 4" in r.stderr


# ---------------------------------------------------------------------------
# seeded random batches vs the C oracle (exact)
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("k,n_reads,read_len,genome", [
    (31, 40_000, 150, 2_000_000), (21, 40_000, 150, 500_000), (32, 20_000, 150, 1_000_000),
    (15, 30_000, 100, 300_000), (5, 5_000, 150, 100_000), (1, 2_000, 50, 10_000), (2, 2_000, 50, 10_000),
    (11, 20_000, 150, 50_000), (31, 2_000, 5_000, 1_000_000),
    (17, 20_000, 150, 400_000), (25, 20_000, 150, 400_000), (27, 20_000, 120, 400_000),
])
def test_random_vs_oracle(k, n_reads, read_len, genome):
    batch = okm.synth_reads(n_reads, read_len, genome_len=genome, genome_seed=k, seed=100 + k,
                            sub_rate=0.01, n_rate=0.001)
    oc = OracleCounter(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    with okm.KmerCounter(k) as ctr:
        body = batch.reshape(n_reads, read_len + 1)[:, :read_len]
        offs = np.arange(0, (n_reads + 1) * read_len, read_len, dtype=np.uint64)
        ctr.add_batch(np.ascontiguousarray(body).reshape(-1), offs)
        gk, gc = ctr.result(1)
        info = ctr.engine_info()
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert info["kmers"] == oc.windows


def test_device_batch_matches_host_batch_and_alignment():
    k = 25
    batch = okm.synth_reads(30_000, 150, genome_len=400_000, seed=9, sub_rate=0.02)
    oc = OracleCounter(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    buf = okm.DeviceBuffer(len(batch) + 64)
    padded = np.zeros(len(batch) + 64, np.uint8)
    for off in (0, 3):  # 16-B aligned and unaligned device pointers
        padded[off:off + len(batch)] = batch
        buf.upload(padded)
        with okm.KmerCounter(k) as ctr:
            ctr.add_device_batch(buf.address + off, len(batch))
            gk, gc = ctr.result(1)
        assert np.array_equal(gk, ek) and np.array_equal(gc, ec), off
    buf.free()


def test_multi_batch_multi_run_and_min_count():
    k = 27
    batch = okm.synth_reads(60_000, 150, genome_len=300_000, seed=4)
    recs = batch.reshape(60_000, 151)
    oc = OracleCounter(k)
    oc.add_separated(batch)
    with okm.KmerCounter(k) as ctr:
        for part in np.array_split(recs, 7):
            body = np.ascontiguousarray(part[:, :150]).reshape(-1)
            offs = np.arange(0, (len(part) + 1) * 150, 150, dtype=np.uint64)
            ctr.add_batch(body, offs, normalized=True)
        for m in (1, 2, 5, 40):
            gk, gc = ctr.result(m)
            ek, ec = oc.result(m)
            assert np.array_equal(gk, ek) and np.array_equal(gc, ec), m


def test_pairs_merge_equals_whole():
    k = 31
    batch = okm.synth_reads(50_000, 150, genome_len=200_000, seed=8)
    half = (50_000 // 2) * 151
    parts = []
    for sl in (batch[:half], batch[half:]):
        with okm.KmerCounter(k) as c:
            c.add_records([bytes(r) for r in sl.tobytes().split(b"\n") if r], normalized=True)
            parts.append(c.result(1))
    with okm.KmerCounter(k) as whole:
        whole.add_records([bytes(r) for r in batch.tobytes().split(b"\n") if r], normalized=True)
        wk, wc = whole.result(1)
    with okm.KmerCounter(k) as m:
        for pk, pc in parts:
            m.add_pairs(pk, pc)
        mk, mc = m.result(1)
    assert np.array_equal(mk, wk) and np.array_equal(mc, wc)


def test_hot_key_and_long_record():
    # poly-A reads: every window is key 0 -> one partition holds everything and
    # must be split down to a small remainder (multi-level path)
    k = 31
    recs = [b"A" * 150] * 20_000 + [b"ACGT" * 50_000]  # + one 200 kb record
    oc = OracleCounter(k)
    oc.add_records(recs)
    with okm.KmerCounter(k) as ctr:
        ctr.add_records(recs)
        gk, gc = ctr.result(1)
        info = ctr.engine_info()
    ek, ec = oc.result(1)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert info["levels"] >= 2


@pytest.mark.parametrize("k", [31, 17])
def test_unique_keys_full_mode(k):
    # one 2 Mbp random record: (almost) every k-mer is distinct, so the LDS
    # items overflow the tag mode's rest buffer and take the full-mode kernel;
    # the pairs merge of two halves exercises its weighted variant
    g = okm.synth_reads(1, 2_000_000, genome_len=2_000_000, genome_seed=77 + k, seed=5, sub_rate=0.0)
    rec = bytes(g[:2_000_000])
    oc = OracleCounter(k)
    oc.add_records([rec])
    ek, ec = oc.result(1)
    with okm.KmerCounter(k) as ctr:
        ctr.add_records([rec])
        gk, gc = ctr.result(1)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    parts = []
    for sl in (rec[:1_000_030], rec[1_000_000:]):
        with okm.KmerCounter(k) as c:
            c.add_records([sl])
            parts.append(c.result(1))
    with okm.KmerCounter(k) as m:
        for pk, pc in parts:
            m.add_pairs(pk, pc)
        mk, mc = m.result(1)
    oc2 = OracleCounter(k)
    oc2.add_records([rec[:1_000_030], rec[1_000_000:]])
    ek2, ec2 = oc2.result(1)
    assert np.array_equal(mk, ek2) and np.array_equal(mc, ec2)


def test_deferred_items_mid_table():
    # covered reads everywhere + a burst of unique k-mers that all start with
    # CCCCCCC (canonical keys in one mid-table key range): the items of that
    # range overflow the tag mode and are deferred to k_count_slow while the
    # items on both sides are tag-counted; one dense table in key order
    k = 31
    cov = okm.synth_reads(60_000, 150, genome_len=400_000, genome_seed=3, seed=31, sub_rate=0.002)
    rng = np.random.default_rng(7)
    tails = rng.integers(0, 4, size=(40_000, 24))
    burst = [b"CCCCCCC" + bytes(b"ACGT"[x] for x in row) for row in tails]
    recs = [r for r in cov.tobytes().split(b"\n") if r] + burst
    oc = OracleCounter(k)
    oc.add_records(recs)
    ek, ec = oc.result(1)
    with okm.KmerCounter(k) as ctr:
        ctr.add_records(recs)
        gk, gc = ctr.result(1)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def test_empty_inputs():
    with okm.KmerCounter(21) as ctr:
        ctr.add_records([])
        ctr.add_records([b"", b"ACG", b"NNNNNNNNNNNNNNNNNNNNNNNNNNNNNN"])
        assert ctr.count() == 0
        k, c = ctr.result(1)
        assert len(k) == 0 and len(c) == 0
    with okm.KmerCounter(5, "set") as ctr:
        assert ctr.count() == 0


def test_set_intersection():
    rng = np.random.default_rng(3)
    a = np.unique(rng.integers(0, 1 << 40, 200_000, dtype=np.uint64))
    b = np.unique(np.concatenate([a[::3], rng.integers(0, 1 << 40, 100_000, dtype=np.uint64)]))
    assert okm.set_intersection_size(a, b) == len(np.intersect1d(a, b))
    assert okm.set_intersection_size(a, np.zeros(0, np.uint64)) == 0


# ---------------------------------------------------------------------------
# BASELINE-size properties (configs[1]: 1 GiB FASTQ-equivalent, k=31)
# ---------------------------------------------------------------------------

def test_full_size_properties():
    k = 31
    n_reads = 3_355_443
    batch = okm.synth_reads(n_reads, 150, genome_len=100_000_000, genome_seed=2, seed=2)
    buf = okm.DeviceBuffer(len(batch))
    buf.upload(batch)
    with okm.KmerCounter(k) as ctr:
        ctr.add_device_batch(buf.address, len(batch))
        n = ctr.count()
        keys, counts = ctr.result(1)
        info = ctr.engine_info()
        ctr.reset()
        ctr.add_device_batch(buf.address, len(batch))
        k2, c2 = ctr.result(1)
    buf.free()
    assert n == len(keys) and info["distinct"] == n
    assert int(counts.sum()) == valid_windows(batch, k) == info["kmers"]
    assert_table_invariants(keys, counts, k)
    assert np.array_equal(keys, k2) and np.array_equal(counts, c2), "determinism"
    # exact parity of the WHOLE table against the restatement (sharded over
    # the host cores and merged by key range, oracle.count_separated_mt)
    thr = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1))
    ek, ec = count_separated_mt(batch, k, thr)
    assert np.array_equal(keys, ek) and np.array_equal(counts, ec)


@pytest.mark.parametrize("k", [31, 45])
def test_count_add_count(k):
    # okm_count stages its sorted runs in the L1 run's block and releases the
    # runs (the result then stands for the input): counting again, adding
    # after a count, and host batches beside device batches all still equal
    # one count of everything added
    thr = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1))
    sep = np.frombuffer(b"\n", np.uint8)
    parts = [okm.synth_reads(n, 150, genome_len=2_000_000, genome_seed=7, seed=30 + i, first_read=i * 10 ** 6,
                             sub_rate=0.01) for i, n in enumerate((120_000, 90_000, 60_000))]
    with okm.KmerCounter(k, wide=k > 32) as ctr:
        seen = []
        for i, b in enumerate(parts):
            if i == 1:  # a host batch: records and their offsets
                cut = np.flatnonzero(b == sep[0])
                starts = np.concatenate([[0], cut + 1])
                ends_ = np.concatenate([cut, [len(b)]])
                keep = ends_ > starts
                data = np.concatenate([b[s_:e_] for s_, e_ in zip(starts[keep], ends_[keep])])
                offs = np.concatenate([[0], np.cumsum(ends_[keep] - starts[keep])]).astype(np.uint64)
                ctr.add_batch(data, offs)
            else:
                buf = okm.DeviceBuffer(len(b))
                buf.upload(b)
                ctr.add_device_batch(buf.address, len(b))
                buf.free()
            seen.append(b)
            n = ctr.count()
            assert ctr.count() == n  # counting again changes nothing
            keys, counts = ctr.result(1)
            joined = np.concatenate([x for b_ in seen for x in (b_, sep)])
            if k <= 32:
                ek, ec = count_separated_mt(joined, k, thr)
            else:
                oc = OracleCounterWide(k)
                oc.add_separated(joined)
                ek, ec = oc.result(1)
            assert np.array_equal(keys, ek) and np.array_equal(counts, ec), f"after batch {i}"
            assert n == len(ek)


def _upload(arr):
    arr = np.ascontiguousarray(arr, dtype=np.uint64)
    buf = okm.DeviceBuffer(max(arr.nbytes, 8))
    if arr.nbytes:
        buf.upload(arr)
    return buf


@pytest.mark.parametrize("k,wide", [(31, False), (32, False), (45, True)])
def test_sorted_runs_merge_equals_whole(k, wide):
    # the multi-GPU owner path: per-rank sorted slices added without copies and
    # counted by binary-search splits (okm_add_sorted_pairs_device)
    batch = okm.synth_reads(60_000, 150, genome_len=400_000, seed=21, sub_rate=0.01)
    recs = [r for r in batch.tobytes().split(b"\n") if r]
    shards = [recs[i::3] for i in range(3)]
    tables = []
    for sh in shards:
        with okm.KmerCounter(k, wide=wide) as c:
            c.add_records(sh, normalized=True)
            tables.append(c.result(1))
    with okm.KmerCounter(k, wide=wide) as whole:
        whole.add_records(recs, normalized=True)
        wk, wc = whole.result(1)
    bufs = []
    with okm.KmerCounter(k, wide=wide) as m:
        for tk, tc in tables:
            bk, bc = _upload(tk), _upload(tc)
            bufs += [bk, bc]
            m.add_sorted_pairs_device(bk.address, bc.address, len(tc))
        mk, mc = m.result(1)
        info = m.engine_info()
    assert np.array_equal(mk, wk) and np.array_equal(mc, wc)
    assert info["levels"] == 0  # no partition pass: binary-search splits only
    # mixed with unsorted input: the sorted runs are partitioned like pairs
    with okm.KmerCounter(k, wide=wide) as m2:
        bk, bc = _upload(tables[0][0]), _upload(tables[0][1])
        m2.add_sorted_pairs_device(bk.address, bc.address, len(tables[0][1]))
        m2.add_pairs(tables[1][0], tables[1][1])
        m2.add_records(shards[2], normalized=True)
        xk, xc = m2.result(1)
    assert np.array_equal(xk, wk) and np.array_equal(xc, wc)
    for b in bufs + [bk, bc]:
        b.free()


def _count_device(batch, k, wide=False):
    buf = okm.DeviceBuffer(len(batch))
    buf.upload(batch)
    with okm.KmerCounter(k, wide=wide) as ctr:
        ctr.set_timing(True)
        ctr.add_device_batch(buf.address, len(batch))
        keys, counts = ctr.result(1)
        stats = ctr.kernel_stats()
        info = ctr.engine_info()
    buf.free()
    return keys, counts, stats, info


@pytest.mark.parametrize("genome,cap_mul,part_mul", [
    (5_000_000, None, None), (5_000_000, "0.5", None), (2_000, None, None), (5_000_000, "0.999", None),
    (5_000_000, None, "0.5"), (5_000_000, None, "0.97"), (2_000, "0.5", "0.5")])
def test_sampled_placement(genome, cap_mul, part_mul, monkeypatch):
    # batches of >= 64 sampled tiles take the sampled L1 placement (bins sized
    # from every 16th tile's histogram), and >= 4 Mi keys the sampled
    # partition placement (children sized from 1/16 of every chunk);
    # the knobs l1_cap_permille / part_cap_permille shrink the capacities so
    # that some bins overflow and the pass is redone exactly
    k = 31
    if cap_mul:
        testing.set_knob("l1_cap_permille", round(float(cap_mul) * 1000))
    if part_mul:
        testing.set_knob("part_cap_permille", round(float(part_mul) * 1000))
    batch = okm.synth_reads(130_000, 150, genome_len=genome, genome_seed=5, seed=31, sub_rate=0.01, n_rate=0.001)
    gk, gc, stats, info = _count_device(batch, k)
    oc = OracleCounter(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert info["kmers"] == oc.windows
    assert stats["extract_sample"]["launches"] == 1
    l1_redone = "extract_hist" in stats
    if cap_mul == "0.5":
        assert l1_redone
    elif cap_mul is None:
        assert not l1_redone
    if genome > 100_000:  # a low-complexity batch has few distinct keys: no split
        assert stats["part_sample"]["launches"] == 1
        part_redone = "part_hist" in stats
        assert part_redone == (part_mul == "0.5") or part_mul == "0.97"


def test_sampled_l1_placement_wide():
    from oracle import OracleCounterWide
    k = 45
    batch = okm.synth_reads(130_000, 150, genome_len=3_000_000, genome_seed=6, seed=45, sub_rate=0.01)
    gk, gc, stats, _ = _count_device(batch, k, wide=True)
    oc = OracleCounterWide(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    assert np.array_equal(gk.reshape(-1, 2), ek) and np.array_equal(gc, ec)
    assert stats["extract_sample"]["launches"] == 1 and "extract_hist" not in stats


@pytest.mark.parametrize("k,wide", [(31, False), (21, False), (63, True), (45, True)])
def test_fan_out_split(k, wide, monkeypatch):
    # the knob part_max_bits caps a partition pass at 3 bits, so a 7 M-key batch leaves
    # children of ~4-16 Ki keys: each child gets 2^f item slots and the
    # oversized ones are split once more in place on the device (k_fan_split)
    # instead of a host-planned second round (levels stays 1).  The weighted
    # variant: the same table re-added as (key, count) pairs.
    from oracle import OracleCounterWide
    # (wide: 9 L1 bits hold children of this batch below one item with 3-bit
    # passes, so the cap is 2 bits there)
    testing.set_knob("part_max_bits", 2 if wide else 3)
    batch = okm.synth_reads(60_000, 150, genome_len=3_000_000, genome_seed=7, seed=k, sub_rate=0.01,
                            n_rate=0.001)
    gk, gc, stats, info = _count_device(batch, k, wide=wide)
    oc = OracleCounterWide(k) if wide else OracleCounter(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    if wide:
        gk = gk.reshape(-1, 2)
    assert gk.shape == ek.shape and np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert "fan_split" in stats and info["levels"] == 1, (stats.keys(), info)
    # the weighted table holds fewer entries than the batch has instances: a
    # 2-bit pass keeps its children oversized at 8 or 9 L1 bits
    testing.set_knob("part_max_bits", 2)
    with okm.KmerCounter(k, wide=wide) as m:
        m.set_timing(True)
        m.add_pairs(gk, gc)
        m.add_pairs(gk[::3], gc[::3])
        mk, mc = m.result(1)
        mstats = m.kernel_stats()
    ec2 = ec.copy()
    ec2[::3] *= 2
    if wide:
        mk = mk.reshape(-1, 2)
    assert np.array_equal(mk, ek) and np.array_equal(mc, ec2)
    assert "fan_split" in mstats


@pytest.mark.parametrize("k", [63])  # (45 dropped in round 6: the same kernels, suite time)
def test_fan_out_large_jobs_direct(k):
    """Wide keys with 1-bit partition passes: children of ~17-40 Ki keys go
    through the fan-out's large-job variant (1024 threads, ranks in LDS) and
    the direct count (one group beside an instance-bound table).  Exact
    against the oracle."""
    from oracle import OracleCounterWide
    testing.set_knob("part_max_bits", 1)
    batch = okm.synth_reads(200_000, 150, genome_len=20_000_000, genome_seed=11, seed=k, sub_rate=0.01)
    gk, gc, stats, info = _count_device(batch, k, wide=True)
    oc = OracleCounterWide(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    gk = gk.reshape(-1, 2)
    assert gk.shape == ek.shape and np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert "fan_split" in stats and "compact_items" not in stats and info["levels"] == 1, (stats.keys(), info)


def test_fan_out_overflow_falls_back_to_host_rounds(monkeypatch):
    # a 1-bit pass cap leaves children (~70 Ki keys) too big for one fan-out
    # job (<= 64 Ki): the speculative count is abandoned and the host plans
    # further rounds
    testing.set_knob("part_max_bits", 1)
    k = 31
    batch = okm.synth_reads(300_000, 150, genome_len=3_000_000, genome_seed=8, seed=3, sub_rate=0.01)
    gk, gc, stats, info = _count_device(batch, k)
    oc = OracleCounter(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert info["levels"] >= 2


@pytest.mark.parametrize("k,wide,mode,maxb", [(31, False, "A", None), (31, False, "B", None), (27, False, "A", "3"),
                                              (63, True, "A", "2"), (45, True, "B", None)])
def test_grouped_count(k, wide, mode, maxb, monkeypatch):
    # memory-bounded counting: the L1 parts are counted in key-range groups
    # (knob group_keys forces ~1.5 M instances per group), compacted straight
    # into one instance-bound table (A) or into exact per-group tables joined
    # at the end (B: knob group_exact); with part_max_bits the groups also take
    # the fan-out path
    # (2 bits for k=63: its 9 L1 bits keep 3-bit children below one item)
    from oracle import OracleCounterWide
    testing.set_knob("group_keys", 1_500_000)
    testing.set_knob("group_exact", 1 if mode == "B" else 0)
    if maxb:
        testing.set_knob("part_max_bits", int(maxb))
    batch = okm.synth_reads(60_000, 150, genome_len=3_000_000, genome_seed=9, seed=k + 1, sub_rate=0.01,
                            n_rate=0.001)
    gk, gc, stats, info = _count_device(batch, k, wide=wide)
    oc = OracleCounterWide(k) if wide else OracleCounter(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    if wide:
        gk = gk.reshape(-1, 2)
    assert gk.shape == ek.shape and np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert info["groups"] >= 4 and info["distinct"] == len(ec), info
    if maxb:
        assert "fan_split" in stats
    with okm.KmerCounter(k, wide=wide) as m:  # min_count filter over a grouped table
        m.add_records([r for r in batch.tobytes().split(b"\n") if r], normalized=True)
        for mc in (1, 3):
            fk, fc = m.result(mc)
            xk, xc = oc.result(mc)
            if wide:
                fk = fk.reshape(-1, 2)
            assert np.array_equal(fk, xk) and np.array_equal(fc, xc), mc


@pytest.mark.parametrize("cap,k,over", [(None, 31, False), (0.5, 31, True), (0.5, 63, True)])
def test_grouped_count_pipelined_and_redo(cap, k, over):
    """Key-range groups in one instance-bound table, pipelined: every group's
    kernels queue behind the previous group's with no host sync and the
    table's next entry advances on the device.  Groups of >= 4 Mi keys take
    the sampled partition placement; with part_cap_permille = 500 their
    sampled slots overflow, the speculative counts are abandoned (the first
    abandoned group poisons the device-side table base, so no later group
    writes), and the groups from the first abandoned one on are counted again
    one sync at a time.  `over` (knob group_over; otherwise taken when the
    instance-bound table would leave no room for pipelined groups): the
    table's keys are written over the batch's own L1 run, group by group in
    key order (count_grouped), so a group that wrote too early would destroy
    a later group's input -- exact all ways.  k = 63: the count kernel writes
    the table itself (items in order, each at its look-back prefix:
    okm_count.hip launch_count_direct), no compaction."""
    from oracle import OracleCounterWide
    wide = k > 32
    testing.set_knob("group_keys", 5_000_000)
    testing.set_knob("group_exact", 0)
    testing.set_knob("group_over", 1 if over else -1)
    if cap:
        testing.set_knob("part_cap_permille", round(cap * 1000))
    batch = okm.synth_reads(130_000, 150, genome_len=20_000_000, genome_seed=12, seed=4, sub_rate=0.01)
    gk, gc, stats, info = _count_device(batch, k, wide=wide)
    oc = OracleCounterWide(k) if wide else OracleCounter(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    if wide:
        gk = gk.reshape(-1, 2)
    assert gk.shape == ek.shape and np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert info["groups"] >= 3 and info["distinct"] == len(ec), info
    assert "part_sample" in stats, stats.keys()
    assert ("compact_items" in stats) == (not wide), stats.keys()


@pytest.mark.parametrize("k", [33, 63])
def test_grouped_count_wide_hot_keys(k):
    """Wide keys in key-range groups with hot keys (poly-A reads and a
    period-4 record): their parts split down to direct-address (dense) items,
    which the direct count writes at their look-back prefix too.  Exact."""
    testing.set_knob("group_keys", 300_000)
    testing.set_knob("group_exact", 0)
    g = okm.synth_reads(4_000, 150, genome_len=400_000, genome_seed=3, seed=k, sub_rate=0.01)
    recs = [r for r in g.tobytes().split(b"\n") if r] + [b"A" * 150] * 3_000 + [b"ACGT" * 40_000]
    oc = OracleCounterWide(k)
    oc.add_records(recs)
    ek, ec = oc.result(1)
    with okm.KmerCounter(k, wide=True) as ctr:
        ctr.add_records(recs)
        gk, gc = ctr.result(1)
        info = ctr.engine_info()
    gk = gk.reshape(-1, 2)
    assert gk.shape == ek.shape and np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert info["groups"] >= 2 and info["levels"] >= 2, info  # (the hot parts split further)


def test_grouped_count_wide_weighted():
    """Weighted wide keys in key-range groups (a counted table's pairs beside
    raw reads): the direct count sums the weights into the table.  Exact."""
    from oracle import OracleCounterWide
    k = 63
    testing.set_knob("group_keys", 1_500_000)
    testing.set_knob("group_exact", 0)
    batch = okm.synth_reads(60_000, 150, genome_len=3_000_000, genome_seed=9, seed=6, sub_rate=0.01)
    # + poly-A reads on both sides: a hot key whose weighted part splits down
    # to a direct-address item
    recs = [b"A" * 150] * 1_000 + [r for r in batch.tobytes().split(b"\n") if r] + [b"A" * 150] * 1_000
    half = len(recs) // 2
    with okm.KmerCounter(k, wide=True) as c:
        c.add_records(recs[:half], normalized=True)
        tk, tc = c.result(1)
    with okm.KmerCounter(k, wide=True) as m:
        m.add_pairs(tk, tc)
        m.add_records(recs[half:], normalized=True)
        mk, mc = m.result(1)
        info = m.engine_info()
    oc = OracleCounterWide(k)
    oc.add_records(recs, normalized=True)
    ek, ec = oc.result(1)
    mk = mk.reshape(-1, 2)
    assert mk.shape == ek.shape and np.array_equal(mk, ek) and np.array_equal(mc, ec)
    assert info["groups"] >= 2, info


def test_c1_cli_full_size(tmp_path):
    """BASELINE configs[0] (C1) through the CLI: byte-identical TSV with the
    restatement's (tests/golden/c1_k21.json), for -m 1 and -m 2."""
    import hashlib
    import sys as _sys
    _sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from make_c1_fasta import c1_fasta
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c1_k21.json")
    with open(golden) as fh:
        fx = json.load(fh)
    inp = tmp_path / "c1.fasta"
    inp.write_bytes(c1_fasta())
    for m, key in (("1", "m1"), ("2", "m2")):
        out = tmp_path / f"out_m{m}.tsv"
        r = subprocess.run([_lib.CLI_PATH, "count", "-k", "21", "-i", str(inp), "-o", str(out), "-m", m],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        raw = out.read_bytes()
        assert raw.count(b"\n") == fx[key]["lines"]
        assert hashlib.sha256(raw).hexdigest() == fx[key]["sha256"]
