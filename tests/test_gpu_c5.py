"""BASELINE configs[4] (C5) at its stated workload: build.rs:46-116 sets of
all 64 WGS-shaped samples (okm.workloads.c5_samples: 64 runs of
data_metagenome.json.gz, <= 256 Mbases each, 11.19 Gbases in all), then
compare.rs:51-66 of DB1 (samples 0-31) against DB2 (samples 32-63).

Exact against the restatement on a subset: the sets of the two smallest
samples of each DB (oracle/okm_oracle.c over the host cores), and their
unions / intersection (numpy).  For the rest, full-size properties: every
set strictly increasing and canonical, |A|, |B|, |A ∩ B| equal between the
one-GPU compare (set unions of sorted runs + device intersection) and the
distributed compare through the library's exchange at P = 8 virtual ranks
(okm_merge_owned_n over okm_comm_init_loopback)."""

import os
import threading

import numpy as np
import pytest

import okm
from okm import workloads
from oracle import count_separated_mt

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
    sets, kept, bases = [], {}, 0
    with okm.KmerCounter(K, "set") as ctx:
        for s in range(64):
            b = workloads.c5_sample(s)
            bases += len(b) - int((b == 10).sum())
            d = okm.DeviceBuffer(len(b))
            d.upload(b)
            ctx.reset()
            ctx.add_device_batch(d.address, len(b))
            keys, _ = ctx.result(1)
            d.free()
            sets.append(keys)
            if s in smallest:
                kept[s] = b
    return sets, kept, bases


def test_c5_sample_sets_exact_subset_and_properties(c5_sets):
    sets, kept, bases = c5_sets
    assert 11.0e9 < bases < 11.4e9  # the stated workload: 11.19 Gbases
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
    sub = sorted(kept)
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
    """compare.rs:51-66 on one GPU: each DB's union of sorted runs, |A ∩ B|."""
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
    out = (res[0][1], res[1][1], inter)
    for u, _ in res:
        u.close()
    for d in bufs:
        d.free()
    return out


def test_c5_distributed_compare_p8_equals_one_gpu(c5_sets):
    sets, _, _ = c5_sets
    want = _one_gpu_compare(sets)
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
