"""BASELINE configs[4] (C5) at its stated workload: build.rs:46-116 sets of
all 64 WGS-shaped samples (okm.workloads.c5_samples: 64 runs of
data_metagenome.json.gz, <= 256 Mbases each, 11.19 Gbases in all), then
compare.rs:51-66 of DB1 (samples 0-31) against DB2 (samples 32-63).

Exact against the restatement: EVERY one of the 64 sets on 12 key ranges
(1/8192 of the key space each, spread over the first-base quarters; the
range-filtered restatement over every read of every sample), the whole sets
of 12 samples of every size class (0.1 to 256 Mbases, read lengths 365 to
20,008; oracle/okm_oracle.c over the host cores), the unions / intersection
of four of them (numpy), and |A|, |B|, |A ∩ B| of the full compare restricted
to the 12 ranges against the oracle-built sets.  At the
full workload: |A|, |B|, |A ∩ B| and the Jaccard f64 of the one-GPU compare
(set unions of sorted runs + device intersection) equal numpy's union1d /
intersect1d of all 64 device sets on the host, and the distributed compare
through the library's exchange at P = 8 virtual ranks (okm_merge_owned_n
over okm_comm_init_loopback) equals the one-GPU compare.  Every set is
strictly increasing and canonical."""

import os
import threading

import numpy as np
import pytest

import okm
from okm import workloads
from oracle import count_separated_mt, count_separated_ranges_mt
from test_gpu_c3 import c3_key_ranges, dev_tensor

pytestmark = pytest.mark.gpu
K = 31


def _threads():
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1))


def _canonical_ok(keys):
    """keys <= reverse complement (kmer.rs:99-106), numpy over a sample."""
    x = ~keys
    for s, m in ((2, 0x3333333333333333), (4, 0x0F0F0F0F0F0F0F0F), (8, 0x00FF00FF00FF00FF),
                 (16, 0x0000FFFF0000FFFF)):
        x = ((x >> np.uint64(s)) & np.uint64(m)) | ((x & np.uint64(m)) << np.uint64(s))
    x = (x >> np.uint64(32)) | (x << np.uint64(32))
    rc = (x >> np.uint64(64 - 2 * K)) & np.uint64((1 << (2 * K)) - 1)
    return bool((keys <= rc).all())


@pytest.fixture(scope="module")
def c5_sets():
    """Every sample's set, built on the device into one store (set sizes,
    offsets), with the sample bytes of the exact-parity subset kept."""
    plans = [workloads.c5_sample_plan(s) for s in range(64)]
    smallest = sorted(range(32), key=lambda s: plans[s][1])[:2] + \
        sorted(range(32, 64), key=lambda s: plans[s][1])[:2]
    # + 8 samples across the size classes and read lengths (0.7 to 256 Mbases;
    # 256 Mbases at 365 bp and at 20,008 bp reads)
    exact = smallest + [7, 15, 24, 58, 57, 53, 0, 49]
    sets, kept, bases, ranged = [], {}, 0, []
    ranges = c3_key_ranges(K)
    with okm.KmerCounter(K, "set") as ctx:
        for s in range(64):
            b = workloads.c5_sample(s)
            bases += len(b) - int((b == 10).sum())
            # the oracle's set of this sample on the 12 key ranges (every read)
            ek, _, _ = count_separated_ranges_mt([b], K, ranges, _threads())
            ranged.append(ek)
            d = okm.DeviceBuffer(len(b))
            d.upload(b)
            ctx.reset()
            ctx.add_device_batch(d.address, len(b))
            keys, _ = ctx.result(1)
            d.free()
            sets.append(keys)
            if s in exact:
                kept[s] = b
    return sets, kept, bases, smallest, ranged


def _in_ranges(keys, ranges):
    cut = [np.searchsorted(keys, np.uint64(v)) for r in ranges for v in r]
    return np.concatenate([keys[cut[2 * i]:cut[2 * i + 1]] for i in range(len(ranges))])


def test_c5_every_sample_set_exact_on_key_ranges(c5_sets):
    """build.rs:50-58: each of the 64 device sets, restricted to the 12 key
    ranges, equals the restatement's set of that sample on those ranges."""
    sets, _, _, _, ranged = c5_sets
    ranges = c3_key_ranges(K)
    total = 0
    for s in range(64):
        got = _in_ranges(sets[s], ranges)
        assert np.array_equal(got, ranged[s]), s
        total += len(got)
    assert total > 100_000


def test_c5_sample_sets_exact_subset_and_properties(c5_sets):
    sets, kept, bases, smallest, _ = c5_sets
    assert 11.0e9 < bases < 11.4e9  # the stated workload: 11.19 Gbases
    assert len(kept) == 12
    for s, b in kept.items():  # exact sets (build.rs:50-58 DashSet) vs the restatement
        ek, _ = count_separated_mt(b, K, _threads())
        assert np.array_equal(sets[s], ek), s
    rng = np.random.default_rng(1)
    for s, keys in enumerate(sets):
        assert len(keys) > 0
        assert bool((keys[1:] > keys[:-1]).all()), s
        assert int(keys[-1]) < (1 << (2 * K))
        assert _canonical_ok(keys[rng.integers(0, len(keys), 100_000)]), s
    # the subset's unions and intersection on the device vs numpy (compare.rs:51-66)
    sub = sorted(smallest)
    a_sets, b_sets = [sets[s] for s in sub if s < 32], [sets[s] for s in sub if s >= 32]
    got = []
    for group in (a_sets, b_sets):
        with okm.KmerCounter(K, "set") as u:
            for x in group:
                u.add_pairs(x)
            got.append(u.result(1)[0])
    A, B = np.union1d(*a_sets), np.union1d(*b_sets)
    assert np.array_equal(got[0], A) and np.array_equal(got[1], B)
    assert okm.set_intersection_size(got[0], got[1]) == len(np.intersect1d(A, B, assume_unique=True))


def _one_gpu_compare(sets):
    """compare.rs:51-66 on one GPU: each DB's union of sorted runs, |A ∩ B|;
    also the two unions restricted to the 12 key ranges (host copies)."""
    bufs, res = [], []
    for h in (0, 1):
        u = okm.KmerCounter(K, "set")
        for x in sets[32 * h:32 * h + 32]:
            d = okm.DeviceBuffer(x.nbytes)
            d.upload(x)
            bufs.append(d)
            u.add_sorted_pairs_device(d.address, None, len(x))
        n = u.count()
        res.append((u, n))
    pa, _, _ = res[0][0].result_device()
    pb, _, _ = res[1][0].result_device()
    inter = okm.set_intersection_size_device(pa, res[0][1], pb, res[1][1])
    ranges = c3_key_ranges(K)

    def in_ranges_device(ptr, n):  # the union's keys inside the ranges, sliced on the device
        import torch
        keys = dev_tensor(ptr, n)
        bounds = torch.tensor([v for r in ranges for v in r], dtype=torch.int64, device=keys.device)
        cut = torch.searchsorted(keys, bounds).cpu().tolist()  # keys < 2^62: signed order is unsigned order
        return np.concatenate([keys[cut[2 * i]:cut[2 * i + 1]].cpu().numpy() for i in range(len(ranges))]).view(
            np.uint64)

    unions_in_ranges = (in_ranges_device(pa, res[0][1]), in_ranges_device(pb, res[1][1]))
    out = (res[0][1], res[1][1], inter, unions_in_ranges)
    for u, _ in res:
        u.close()
    for d in bufs:
        d.free()
    return out


def _host_compare(sets, threads):
    """compare.rs:51-66 on the host: DB1 = union of sets 0-31, DB2 = union of
    sets 32-63 (np.union1d of sorted unique arrays, key range by key range on
    `threads` threads), |A ∩ B| by np.intersect1d per range."""
    from concurrent.futures import ThreadPoolExecutor
    edges = [int(x) for x in np.linspace(0, 1 << (2 * K), threads + 1)]

    def part(r):
        lo, hi = np.uint64(edges[r]), np.uint64(edges[r + 1])
        def sl(x):
            return x[np.searchsorted(x, lo):np.searchsorted(x, hi)]
        a = np.unique(np.concatenate([sl(x) for x in sets[:32]]))
        b = np.unique(np.concatenate([sl(x) for x in sets[32:]]))
        return len(a), len(b), len(np.intersect1d(a, b, assume_unique=True))

    with ThreadPoolExecutor(max_workers=threads) as ex:
        parts = list(ex.map(part, range(threads)))
    return tuple(int(sum(p[i] for p in parts)) for i in range(3))


@pytest.fixture(scope="module")
def c5_compare(c5_sets):
    return _one_gpu_compare(c5_sets[0])


def test_c5_compare_exact_vs_host_unions(c5_sets, c5_compare):
    """|A|, |B|, |A ∩ B| and the Jaccard f64 (compare.rs:58-66) of the one-GPU
    compare over all 64 device sets equal numpy's on the host."""
    na, nb, inter, _ = c5_compare
    ha, hb, hi = _host_compare(c5_sets[0], _threads())
    assert (na, nb, inter) == (ha, hb, hi)
    union = na + nb - inter
    assert inter / union == hi / (ha + hb - hi)
    assert 0 < inter < min(na, nb)


def test_c5_compare_on_key_ranges_vs_oracle_sets(c5_sets, c5_compare):
    """compare.rs:51-66 restricted to the 12 key ranges: the device unions A
    and B (over all 32 + 32 device sets) equal the unions of the ORACLE's
    per-sample range sets, and so do |A|, |B|, |A ∩ B| there."""
    ranged = c5_sets[4]
    ua, ub = c5_compare[3]
    oa = np.unique(np.concatenate(ranged[:32]))
    ob = np.unique(np.concatenate(ranged[32:]))
    assert np.array_equal(ua, oa) and np.array_equal(ub, ob)
    inter = len(np.intersect1d(ua, ub, assume_unique=True))
    assert inter == len(np.intersect1d(oa, ob, assume_unique=True)) > 0


def test_c5_distributed_compare_p8_equals_one_gpu(c5_sets, c5_compare):
    sets = c5_sets[0]
    want = c5_compare[:3]
    na, nb, inter = want
    assert 0 < inter < min(na, nb)  # the two halves share half of their genomes
    P = 8
    comms = okm.Comm.init_loopback(P, 0)
    out, err = [None] * P, []

    def rank(r):
        try:
            a, b = okm.KmerCounter(K, "set"), okm.KmerCounter(K, "set")
            oa, ob = okm.KmerCounter(K, "set"), okm.KmerCounter(K, "set")
            bufs = []
            for s in range(r, 64, P):  # samples dealt round-robin; each rank unions its share
                x = sets[s]
                d = okm.DeviceBuffer(x.nbytes)
                d.upload(x)
                bufs.append(d)
                (a if s < 32 else b).add_sorted_pairs_device(d.address, None, len(x))
            a.count()
            b.count()
            out[r] = okm.distributed_compare(comms[r], a, b, oa, ob)
            for c in (a, b, oa, ob):
                c.close()
            for d in bufs:
                d.free()
        except BaseException as e:  # surfaced below
            err.append(e)

    th = [threading.Thread(target=rank, args=(r,), daemon=True) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    for c in comms:
        c.close()
    if err:
        raise err[0]
    assert all(o == want for o in out), (out, want)
