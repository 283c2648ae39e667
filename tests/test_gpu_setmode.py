"""Set mode (build.rs:46-58) and compare (compare.rs:51-66) on the device at
sample scale, and the two-rank table merge / compare driven through the HIP
engine (gloo moves the runs between two processes sharing the one MI355X of
the box; RCCL refuses two ranks on one device, so the library communicator is
covered at one rank in test_gpu_dist.py).

Oracles: the C restatement's sets (oracle/okm_oracle.c: every canonical key of
build.rs:46-58's DashSet) and numpy's union1d / intersect1d for
db_types.rs:43-53 get_all_kmers_unified and compare.rs:58's intersection."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import okm
from okm import dist as okm_dist
from oracle import OracleCounter, count_separated_mt

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


# ---------------------------------------------------------------------------
# two ranks (gloo between processes) driving the HIP engine end to end
# ---------------------------------------------------------------------------

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _count_worker(rank, world, port, k, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        batch = okm.synth_reads(60_000, 150, genome_len=300_000, genome_seed=31, seed=32)
        recs = batch.reshape(60_000, 151)
        recs[::40, :150] = ord("A")  # a hot key: counts past the one-byte escape
        shard = np.ascontiguousarray(np.array_split(recs, world)[rank]).reshape(-1)
        buf = okm.DeviceBuffer(len(shard))
        buf.upload(shard)
        with okm.KmerCounter(k) as local, okm.KmerCounter(k) as owner:
            local.add_device_batch(buf.address, len(shard))
            lk, lc = local.result(1)
            rk, rc, _, rs = okm_dist.exchange_runs(torch.from_numpy(lk.view(np.int64).copy()),
                                                   torch.from_numpy(lc.view(np.int64).copy()), k)
            dk, dc = _upload(rk.numpy().view(np.uint64)), _upload(rc.numpy().view(np.uint64))
            off = 0
            for sz in rs:  # every rank's slice is sorted: merged in place by the k-way LDS merge
                if sz:
                    owner.add_sorted_pairs_device(dk.address + 8 * off, dc.address + 8 * off, sz)
                off += sz
            owner.count()
            mk, mc = owner.result(1)
            dk.free()
            dc.free()
        buf.free()
        gk, gc = okm_dist.gather_global(torch.from_numpy(mk.view(np.int64).copy()),
                                        torch.from_numpy(mc.view(np.int64).copy()))
        if rank == 0:
            np.savez(out_path, keys=gk, counts=gc)
    finally:
        dist.destroy_process_group()


def test_two_ranks_hip_count_exchange_merge(tmp_path):
    k, world = 31, 2
    out = os.path.join(str(tmp_path), "merged.npz")
    mp.spawn(_count_worker, args=(world, _free_port(), k, out), nprocs=world, join=True)
    got = np.load(out)
    batch = okm.synth_reads(60_000, 150, genome_len=300_000, genome_seed=31, seed=32)
    batch.reshape(60_000, 151)[::40, :150] = ord("A")
    oc = OracleCounter(k)
    oc.add_separated(batch)
    ek, ec = oc.result(1)
    assert ec.max() > 255
    assert np.array_equal(got["keys"], ek) and np.array_equal(got["counts"], ec)


def _c5_samples():
    return [_sample(8_000, 150, 40 + s, [(900 + (s % 4), 400_000), (904 + (s % 3), 300_000)]) for s in range(8)]


def _compare_worker(rank, world, port, k, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        samples = _c5_samples()
        half = len(samples) // 2
        local = {0: [], 1: []}
        for s in range(rank, len(samples), world):  # samples dealt round-robin
            local[0 if s < half else 1].append(_device_set(samples[s], k))

        def local_union(sets):  # this rank's share of a DB's references, unioned on the device
            bufs = [_upload(x) for x in sets]
            with okm.KmerCounter(k, "set") as u:
                for x, b in zip(sets, bufs):
                    if len(x):
                        u.add_sorted_pairs_device(b.address, None, len(x))
                u.count()
                keys, _ = u.result(1)
            for b in bufs:
                b.free()
            return torch.from_numpy(keys.view(np.int64).copy())

        held = []

        def union(rk, sizes):  # the owner's union of the received sorted runs (set mode, HIP)
            arr = rk.numpy().view(np.uint64)
            d = _upload(arr)
            u = okm.KmerCounter(k, "set")
            off = 0
            for sz in sizes:
                if sz:
                    u.add_sorted_pairs_device(d.address + 8 * off, None, sz)
                off += sz
            n = u.count()
            d.free()
            held.append(u)
            return n, u

        def intersect(ha, na, hb, nb):  # |A ∩ B| of the two owned ranges, on the device
            pa, _, _ = ha.result_device()
            pb, _, _ = hb.result_device()
            return okm.set_intersection_size_device(pa, na, pb, nb)

        res = okm_dist.distributed_compare(local_union(local[0]), local_union(local[1]), k, union, intersect)
        for u in held:
            u.close()
        if rank == 0:
            np.savez(out_path, res=np.array(res, np.int64))
    finally:
        dist.destroy_process_group()


def test_two_ranks_hip_distributed_compare(tmp_path):
    k, world = 31, 2
    out = os.path.join(str(tmp_path), "c5.npz")
    mp.spawn(_compare_worker, args=(world, _free_port(), k, out), nprocs=world, join=True)
    na, nb, inter = (int(x) for x in np.load(out)["res"])
    samples = _c5_samples()
    half = len(samples) // 2
    sets = []
    for s in samples:
        oc = OracleCounter(k)
        oc.add_separated(s)
        sets.append(oc.result(1)[0])
    a = np.unique(np.concatenate(sets[:half]))
    b = np.unique(np.concatenate(sets[half:]))
    assert (na, nb) == (len(a), len(b))
    assert inter == len(np.intersect1d(a, b, assume_unique=True))
    assert 0 < inter < min(na, nb)
