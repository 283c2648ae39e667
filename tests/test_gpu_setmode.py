"""Set mode (build.rs:46-58) and compare (compare.rs:51-66) on the device at
sample scale.  The multi-rank table merge and the distributed compare run
through the library's own exchange (okm_merge_owned / okm_merge_owned_n) at
P = 2, 3 and 8 virtual ranks on the one device in test_gpu_loopback.py.

Oracles: the C restatement's sets (oracle/okm_oracle.c: every canonical key of
build.rs:46-58's DashSet) and numpy's union1d / intersect1d for
db_types.rs:43-53 get_all_kmers_unified and compare.rs:58's intersection."""

import os

import numpy as np
import pytest

import okm
from oracle import count_separated_mt

pytestmark = pytest.mark.gpu


def _threads():
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1))


def _sample(n_reads, read_len, seed, genomes):
    """A WGS-like sample: reads drawn from a few seeded genomes (C5 shape)."""
    per = n_reads // len(genomes)
    return np.concatenate([okm.synth_reads(per, read_len, genome_len=glen, genome_seed=gs, seed=seed * 16 + j,
                                           sub_rate=0.002, n_rate=0.0005)
                           for j, (gs, glen) in enumerate(genomes)])


def _device_set(batch, k):
    buf = okm.DeviceBuffer(len(batch))
    buf.upload(batch)
    with okm.KmerCounter(k, "set") as ctr:
        ctr.add_device_batch(buf.address, len(batch))
        keys, _ = ctr.result(1)
    buf.free()
    return keys


def _upload(arr):
    arr = np.ascontiguousarray(arr, dtype=np.uint64)
    buf = okm.DeviceBuffer(max(arr.nbytes, 8))
    if arr.nbytes:
        buf.upload(arr)
    return buf


# ---------------------------------------------------------------------------
# build at >= 10 M bases per sample, exact against the restatement's sets
# ---------------------------------------------------------------------------

def test_set_build_two_samples_10M_bases_vs_oracle():
    k = 31
    a = _sample(72_000, 150, 1, [(801, 4_000_000), (802, 3_000_000), (803, 2_000_000)])  # 10.8 Mbases
    b = _sample(72_000, 150, 2, [(802, 3_000_000), (804, 5_000_000), (805, 1_000_000)])
    sets = []
    for batch in (a, b):
        assert (len(batch) // 151) * 150 >= 10_000_000
        got = _device_set(batch, k)
        ek, _ = count_separated_mt(batch, k, _threads())
        assert np.array_equal(got, ek)
        sets.append(got)
    # compare.rs:51-66 on the two sample sets: |A|, |B|, |A ∩ B| on the device
    da, db = _upload(sets[0]), _upload(sets[1])
    inter = okm.set_intersection_size_device(da.address, len(sets[0]), db.address, len(sets[1]))
    da.free()
    db.free()
    assert inter == len(np.intersect1d(sets[0], sets[1], assume_unique=True))
    assert 0 < inter < min(len(sets[0]), len(sets[1]))  # they share genome 802 only


# ---------------------------------------------------------------------------
# union of references' sorted sets (set mode over sorted runs) and |A ∩ B|
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("k", [21, 31, 32])
def test_set_union_of_sorted_runs_and_intersection_device(k):
    rng = np.random.default_rng(k)
    top = (1 << (2 * k)) if k < 32 else (1 << 64) - 2
    runs = []
    for i, n in enumerate([0, 1, 50_000, 400_000, 1_200_000, 3]):
        if n == 0:
            runs.append(np.zeros(0, np.uint64))
            continue
        base = rng.integers(0, top, size=n, dtype=np.uint64, endpoint=False)
        if i % 2 and runs and len(runs[-1]):  # overlap with the previous reference
            base[: n // 3] = rng.choice(runs[-1], size=n // 3)
        runs.append(np.unique(base))
    if k == 32:  # the top of the unsigned key order (all-T's canonical is all-A: ~0 is never a key)
        runs[-1] = np.unique(np.concatenate([runs[-1], np.array([(1 << 64) - 2, (1 << 63)], np.uint64)]))
    bufs = [_upload(r) for r in runs]
    with okm.KmerCounter(k, "set") as u:
        for r, b in zip(runs, bufs):
            if len(r):
                u.add_sorted_pairs_device(b.address, None, len(r))
        n = u.count()
        got, _ = u.result(1)
    want = np.unique(np.concatenate(runs))
    assert n == len(want) and np.array_equal(got, want)
    # intersection sizes, device arrays: overlapping, disjoint, identical, empty
    for x, y in [(1, 2), (2, 3), (3, 4), (2, 2), (0, 3), (4, 5)]:
        e = len(np.intersect1d(runs[x], runs[y], assume_unique=True))
        assert okm.set_intersection_size_device(bufs[x].address, len(runs[x]), bufs[y].address, len(runs[y])) == e
        assert okm.set_intersection_size(runs[x], runs[y]) == e
    for b in bufs:
        b.free()
