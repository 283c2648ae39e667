"""Counting of sorted runs behind okm_add_sorted_pairs_device: the multi-GPU
owner's merge of per-rank slices, set unions
(compare.rs:51-66, db_types.rs:43-53) and folded batch tables
(count.rs:52-89).  The runs are split into key-range items by binary search
(no key moves) and counted by the count kernel (staged slots + compaction,
the default), the k-way LDS merge kernel of okm_merge.hip
(test knob sorted_path=1), or the count kernel in two passes straight into the
exact-size table (sorted_path=2; weighted runs at the memory limit, the
default for folded tables).  Exact against numpy, for u64 and 128-bit keys,
weighted and unweighted runs, many runs, dense key ranges, all three."""

import numpy as np
import pytest

import okm
from okm import testing

pytestmark = pytest.mark.gpu


def _upload(arr):
    arr = np.ascontiguousarray(arr, dtype=np.uint64)
    buf = okm.DeviceBuffer(max(arr.nbytes, 8))
    if arr.nbytes:
        buf.upload(arr)
    return buf


def _expected(runs, weighted):
    keys = np.concatenate([r[0] for r in runs])
    w = np.concatenate([r[1] if weighted else np.ones(len(r[0]), np.uint64) for r in runs])
    u, inv = np.unique(keys, return_inverse=True)
    s = np.zeros(len(u), np.uint64)
    np.add.at(s, inv, w)
    return u, s


def _runs(rng, nruns, n, span, k):
    out = []
    for _ in range(nruns):
        m = int(rng.integers(0, n + 1))
        keys = np.unique(rng.integers(0, span, m, dtype=np.uint64))
        # canonical-looking: any value below 4^k is a valid key for the engine
        keys = keys[keys < (np.uint64(1) << np.uint64(2 * k))] if k < 32 else keys
        counts = rng.integers(1, 1000, len(keys)).astype(np.uint64)
        out.append((keys, counts))
    return out


@pytest.mark.parametrize("nruns,n,span,weighted", [
    (2, 200_000, 1 << 40, True),
    (8, 300_000, 1 << 30, True),        # heavy overlap between runs
    (20, 50_000, 1 << 24, False),       # dense key range, sets (unions)
    (64, 20_000, 1 << 22, True),        # the most runs one merge item tracks
    (70, 10_000, 1 << 22, True),        # more: the hashing count kernel takes over
])
@pytest.mark.parametrize("merge_kernel", ["", "1", "2"])
def test_merge_runs_vs_numpy(nruns, n, span, weighted, merge_kernel, monkeypatch):
    if merge_kernel:
        testing.set_knob("sorted_path", int(merge_kernel))
    rng = np.random.default_rng(nruns * 7 + n)
    k = 31
    runs = _runs(rng, nruns, n, span, k)
    ek, ec = _expected(runs, weighted)
    bufs = []
    with okm.KmerCounter(k) as m:
        for keys, counts in runs:
            bk = _upload(keys)
            bc = _upload(counts) if weighted else None
            bufs += [bk, bc]
            m.add_sorted_pairs_device(bk.address, bc.address if bc else None, len(keys))
        gk, gc = m.result(1)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def test_merge_kernel_equals_count_kernel(monkeypatch):
    # keys spread over the 2k-bit space like canonical k-mers: the work list
    # splits key ranges by key bits, so the merge kernel takes every item
    # (keys crowded into a sliver of the space fall back to the partition path,
    # still exact: the 1 << 24 / 1 << 22 cases above)
    rng = np.random.default_rng(5)
    runs = _runs(rng, 6, 400_000, 1 << 62, 31)
    out = []
    for env in (None, "1", "2"):
        testing.set_knob("sorted_path", int(env) if env else -1)
        bufs = []
        with okm.KmerCounter(31) as m:
            m.set_timing(True)
            for keys, counts in runs:
                bk, bc = _upload(keys), _upload(counts)
                bufs += [bk, bc]
                m.add_sorted_pairs_device(bk.address, bc.address, len(keys))
            out.append(m.result(1))
            names = set(m.kernel_stats())
        assert ("merge_write" in names) == (env == "1")
        assert ("count_write" in names) == (env == "2")
    for o in out[1:]:
        assert np.array_equal(out[0][0], o[0]) and np.array_equal(out[0][1], o[1])


@pytest.mark.parametrize("merge_kernel", ["", "1", "2"])
def test_merge_wide_keys(merge_kernel, monkeypatch):
    if merge_kernel:
        testing.set_knob("sorted_path", int(merge_kernel))
    rng = np.random.default_rng(11)
    k = 45
    runs = []
    for _ in range(5):
        m = 100_000
        hi = rng.integers(0, 1 << 20, m, dtype=np.uint64)
        lo = rng.integers(0, 1 << 62, m, dtype=np.uint64)
        v = np.unique(hi.astype(object) * (1 << 64) + lo.astype(object))
        keys = np.array([[int(x) & ((1 << 64) - 1), int(x) >> 64] for x in v], dtype=np.uint64)
        runs.append((keys, rng.integers(1, 50, len(keys)).astype(np.uint64)))
    allk = {}
    for keys, counts in runs:
        for (lo, hi), c in zip(keys.tolist(), counts.tolist()):
            key = (hi << 64) | lo
            allk[key] = allk.get(key, 0) + c
    bufs = []
    with okm.KmerCounter(k, wide=True) as m:
        for keys, counts in runs:
            bk, bc = _upload(keys.reshape(-1)), _upload(counts)
            bufs += [bk, bc]
            m.add_sorted_pairs_device(bk.address, bc.address, len(counts))
        gk, gc = m.result(1)
    got = dict(zip(okm.keys128_to_int(gk), gc.tolist()))
    assert got == allk
    assert okm.keys128_to_int(gk) == sorted(allk)


def test_merge_hot_range_many_runs():
    # every run holds the same dense block of keys: items split down to key
    # ranges of a few keys x 64 runs
    base = np.arange(100_000, dtype=np.uint64) + np.uint64(12345)
    runs = [(base, np.full(len(base), i + 1, np.uint64)) for i in range(64)]
    bufs = []
    with okm.KmerCounter(31) as m:
        for keys, counts in runs:
            bk, bc = _upload(keys), _upload(counts)
            bufs += [bk, bc]
            m.add_sorted_pairs_device(bk.address, bc.address, len(keys))
        gk, gc = m.result(1)
    assert np.array_equal(gk, base)
    assert (gc == np.uint64(64 * 65 // 2)).all()


@pytest.mark.parametrize("wide", [False, True])
def test_merge_counts_past_u32(wide):
    """Weighted sorted runs are counted with u32 staged counts first; a key
    whose merged count passes 2^32 (3e9 + 3e9 here, and a lone 5e9) sends the
    count back through u64 staging -- exact either way."""
    rng = np.random.default_rng(5)
    k = 45 if wide else 31
    span = 1 << 40
    runs = _runs(rng, 3, 100_000, span, k)
    big = np.uint64(3_000_000_000)
    for i in (0, 1):  # one shared key with a huge count in two runs
        keys, counts = runs[i]
        j = len(keys) // 2
        runs[i] = (keys, counts.copy())
        runs[i][1][j] = big
    shared = runs[0][0][len(runs[0][0]) // 2]
    k1 = runs[1][0]
    if shared not in set(k1.tolist()):
        k1 = np.unique(np.append(k1, shared))
        c1 = np.ones(len(k1), np.uint64)
        c1[np.searchsorted(k1, shared)] = big
        runs[1] = (k1, c1)
    runs[2][1][0] = np.uint64(5_000_000_000)
    ek, ec = _expected(runs, True)
    assert int(ec.max()) > (1 << 32)
    bufs = []
    with okm.KmerCounter(k, wide=wide) as m:
        for keys, counts in runs:
            kk = np.stack([keys, np.zeros_like(keys)], axis=1).reshape(-1) if wide else keys
            bk, bc = _upload(kk), _upload(counts)
            bufs += [bk, bc]
            m.add_sorted_pairs_device(bk.address, bc.address, len(keys))
        gk, gc = m.result(1)
    if wide:
        gk = gk.reshape(-1, 2)[:, 0]
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def _skewed_runs(rng, nruns, n, bits):
    """Sorted runs whose keys are far from uniform inside an L1 bin: three
    clusters 2^-9 of a bin wide plus a cubic density ramp (keys crowd the low
    end).  The item bounds search interpolates before it bisects; on this data
    the interpolation guesses are poor and the bisection must still land
    exactly."""
    top = np.uint64(1) << np.uint64(bits)
    out = []
    for r in range(nruns):
        parts = []
        for c in (0.1003, 0.5, 0.77):
            centre = int(c * float(top))
            parts.append(np.uint64(centre) + rng.integers(0, 1 << (bits - 18), n // 4, dtype=np.uint64))
        u = rng.random(n // 4)
        parts.append((u ** 3 * float(top)).astype(np.uint64))
        keys = np.unique(np.concatenate(parts))
        keys = keys[keys < top]
        out.append((keys, rng.integers(1, 100, len(keys)).astype(np.uint64)))
    return out


@pytest.mark.parametrize("merge_kernel", ["", "2"])
def test_merge_skewed_key_density(merge_kernel):
    if merge_kernel:
        testing.set_knob("sorted_path", int(merge_kernel))
    rng = np.random.default_rng(23)
    runs = _skewed_runs(rng, 8, 240_000, 62)
    ek, ec = _expected(runs, True)
    bufs = []
    with okm.KmerCounter(31) as m:
        for keys, counts in runs:
            bk, bc = _upload(keys), _upload(counts)
            bufs += [bk, bc]
            m.add_sorted_pairs_device(bk.address, bc.address, len(keys))
        gk, gc = m.result(1)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def test_merge_skewed_key_density_wide():
    rng = np.random.default_rng(29)
    k = 63
    runs = []
    for keys, counts in _skewed_runs(rng, 4, 120_000, 62):
        # the skewed values as the top 62 bits of 126-bit keys (low word random)
        lo = rng.integers(0, 1 << 62, len(keys), dtype=np.uint64)
        v = (keys.astype(object) << 64) | lo.astype(object)
        v = sorted(set(v.tolist()))
        kk = np.array([[x & ((1 << 64) - 1), x >> 64] for x in v], dtype=np.uint64)
        runs.append((kk, rng.integers(1, 50, len(v)).astype(np.uint64)))
    allk = {}
    for keys, counts in runs:
        for (lo, hi), c in zip(keys.tolist(), counts.tolist()):
            key = (hi << 64) | lo
            allk[key] = allk.get(key, 0) + c
    bufs = []
    with okm.KmerCounter(k, wide=True) as m:
        for keys, counts in runs:
            bk, bc = _upload(keys.reshape(-1)), _upload(counts)
            bufs += [bk, bc]
            m.add_sorted_pairs_device(bk.address, bc.address, len(counts))
        gk, gc = m.result(1)
    assert okm.keys128_to_int(gk) == sorted(allk)
    assert dict(zip(okm.keys128_to_int(gk), gc.tolist())) == allk
