"""k in 33..64: the opt-in two-u64 extension (BASELINE
configs[3] — k=63 on ONT-like long reads).  The reference caps k at 32
(count.rs:43-45), so parity here is restatement-defined: the HIP engine is
checked bit-exactly against the C restatement's k<=64 path
(oracle/okm_oracle.c, oracle_counter_wide_*), which re-encodes every window in
O(k) over an unsigned __int128 exactly like kmer.rs:45-55/83-92/99-106 do
over u64.
"""

import os
import subprocess

import numpy as np
import pytest

import okm
from okm import _lib
from oracle import OracleCounterWide

pytestmark = pytest.mark.gpu


def ont_like_reads(n_reads: int, seed: int, genome_len: int = 2_000_000, err: float = 0.05):
    """ONT-like reads (BASELINE configs[3] shape, small): lognormal lengths
    (median 2,891, sigma 1.085, clipped to [200, 100000]) sampled from a seeded
    random genome, either strand, 5 % substitutions, a few N runs."""
    rng = np.random.default_rng(seed)
    genome = rng.integers(0, 4, genome_len, dtype=np.uint8)
    lens = np.clip(np.exp(np.log(2891) + 1.085 * rng.standard_normal(n_reads)), 200, 100_000).astype(int)
    lens = np.minimum(lens, genome_len - 1)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    out = []
    for L in lens:
        s = int(rng.integers(0, genome_len - L))
        codes = genome[s:s + L].copy()
        if rng.random() < 0.5:
            codes = (3 - codes)[::-1]
        sub = rng.random(L) < err
        codes[sub] = (codes[sub] + rng.integers(1, 4, int(sub.sum()))) % 4
        seq = acgt[codes]
        if rng.random() < 0.1:
            p = int(rng.integers(0, L))
            seq[p:p + 5] = ord("N")
        out.append(seq.tobytes())
    return out


def wide_oracle(recs, k, normalized=False):
    oc = OracleCounterWide(k)
    oc.add_records(recs, normalized=normalized)
    return oc


@pytest.mark.parametrize("k", [33, 45, 63, 64])
def test_random_reads_wide_vs_oracle(k):
    batch = okm.synth_reads(20_000, 150, genome_len=500_000, genome_seed=k, seed=3 + k, sub_rate=0.01,
                            n_rate=0.001)
    recs = [r for r in batch.tobytes().split(b"\n") if r]
    oc = wide_oracle(recs, k, normalized=True)
    ek, ec = oc.result(1)
    with okm.KmerCounter(k, wide=True) as c:
        c.add_records(recs, normalized=True)
        gk, gc = c.result(1)
        info = c.engine_info()
    assert gk.shape == ek.shape and np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert info["kmers"] == oc.windows


def test_ont_like_long_reads_k63():
    recs = ont_like_reads(400, seed=4)
    k = 63
    oc = wide_oracle(recs, k)
    with okm.KmerCounter(k, wide=True) as c:
        c.add_records(recs)
        for m in (1, 2):
            gk, gc = c.result(m)
            ek, ec = oc.result(m)
            assert np.array_equal(gk, ek) and np.array_equal(gc, ec), m
    # keys are canonical and strictly increasing as 128-bit values
    ints = okm.keys128_to_int(gk[:2000])
    assert ints == sorted(set(ints))
    for v in ints[:200]:
        assert v == okm.canonical_u128(v, k)


def test_wide_pairs_merge_and_multi_batch():
    k = 51
    recs = ont_like_reads(120, seed=9, genome_len=300_000)
    half = len(recs) // 2
    parts = []
    for sl in (recs[:half], recs[half:]):
        with okm.KmerCounter(k, wide=True) as c:
            c.add_records(sl)
            parts.append(c.result(1))
    with okm.KmerCounter(k, wide=True) as m:
        for pk, pc in parts:
            m.add_pairs(pk, pc)
        mk, mc = m.result(1)
    with okm.KmerCounter(k, wide=True) as w:
        for sl in np.array_split(np.arange(len(recs)), 5):
            w.add_records([recs[i] for i in sl])
        wk, wc = w.result(1)
    ek, ec = wide_oracle(recs, k).result(1)
    assert np.array_equal(wk, ek) and np.array_equal(wc, ec)
    assert np.array_equal(mk, ek) and np.array_equal(mc, ec)


def test_wide_hot_key_deep_split():
    # poly-A: every window is key 0; the partitions split down past 64 bits of
    # prefix (exercises the modulo-2^64 local-bin arithmetic)
    k = 63
    recs = [b"A" * 200] * 3000 + [b"ACGGT" * 4000]
    ek, ec = wide_oracle(recs, k).result(1)
    with okm.KmerCounter(k, wide=True) as c:
        c.add_records(recs)
        gk, gc = c.result(1)
        info = c.engine_info()
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert info["levels"] >= 2


def test_k_above_32_needs_the_wide_flag():
    with pytest.raises(okm.OkmError) as e:
        okm.KmerCounter(33)
    assert e.value.status == _lib.OKM_E_INVALID_K
    assert "Must be between 1 and 32." in _lib.last_error()
    with pytest.raises(okm.OkmError):
        okm.KmerCounter(65, wide=True)


def test_cli_wide_count(tmp_path):
    k = 63
    recs = ont_like_reads(30, seed=12, genome_len=200_000)
    fa = tmp_path / "ont.fa"
    with open(fa, "wb") as fh:
        for i, r in enumerate(recs):
            fh.write(b">r%d\n" % i)
            for o in range(0, len(r), 60):
                fh.write(r[o:o + 60] + b"\n")
    out = tmp_path / "c.tsv"
    p = subprocess.run([_lib.CLI_PATH, "count", "-k", str(k), "-i", str(fa), "-o", str(out)],
                       capture_output=True, text=True)
    assert p.returncode == 1 and "Invalid K-mer size: 63. Must be between 1 and 32." in p.stderr
    p = subprocess.run([_lib.CLI_PATH, "count", "--wide", "-k", str(k), "-i", str(fa), "-o", str(out), "-m", "2"],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    ek, ec = wide_oracle(recs, k).result(2)
    lines = [f"{okm.u128_to_seq(v, k).decode()}\t{c}\n" for v, c in zip(okm.keys128_to_int(ek), ec.tolist())]
    assert out.read_text() == "".join(lines)
