"""BASELINE configs[2] (C3) on the device: the device read generator, batch
folding (memory bounded by distinct keys), and one 1/8 shard of C3 at full
size (20,971,520 reads = 3,145,728,000 bases, the per-GPU share at P=8).

Parity: the device generator is byte-identical to the host generator; a
folded count equals the unfolded count and the oracle exactly; at full shard
size, size-independent properties are checked on the device (sum of counts ==
valid windows, strictly sorted canonical keys, fold invariance), plus exact
parity with the restatement on a 1,000,000-read sample of the shard.
count.rs:52-89: one table across all inputs, batches in any grouping.
"""

import os

import numpy as np
import pytest
import torch

import okm
from oracle import OracleCounter, count_separated_mt, count_separated_ranges_mt

pytestmark = pytest.mark.gpu

C3_READS = 167_772_160
C3_GENOME = 1_000_000_000
C3_SEED = 3


class _View:
    """__cuda_array_interface__ of engine / okm.DeviceBuffer device memory."""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


def dev_tensor(ptr, n, typestr="<i8"):
    if n == 0:
        return torch.empty(0, dtype=torch.uint8 if typestr == "|u1" else torch.int64, device="cuda")
    return torch.as_tensor(_View(ptr, n, typestr), device="cuda")


def torch_revcomp(v, k):
    x = ~v
    for s, m in ((2, 0x3333333333333333), (4, 0x0F0F0F0F0F0F0F0F), (8, 0x00FF00FF00FF00FF),
                 (16, 0x0000FFFF0000FFFF)):
        x = ((x >> s) & m) | ((x & m) << s)
    x = ((x >> 32) & 0xFFFFFFFF) | (x << 32)
    return (x >> (64 - 2 * k)) & ((1 << (2 * k)) - 1)


def device_valid_windows(seq_u8, read_len, k, chunk_reads=1 << 21):
    """Valid k-windows of a device batch of fixed-stride reads (read_len bases
    + separator): windows whose bytes are all A/C/G/T (count.rs:28-36)."""
    stride = read_len + 1
    n = seq_u8.numel() // stride
    lut = torch.ones(256, dtype=torch.int32, device="cuda")
    lut[torch.tensor(list(b"ACGTacgtUu"), device="cuda")] = 0
    total = 0
    for r0 in range(0, n, chunk_reads):
        r1 = min(n, r0 + chunk_reads)
        rows = seq_u8[r0 * stride:r1 * stride].view(r1 - r0, stride)[:, :read_len]
        bad = lut[rows.long()]
        c = torch.nn.functional.pad(torch.cumsum(bad, dim=1, dtype=torch.int32), (1, 0))
        total += int(((c[:, k:] - c[:, :-k]) == 0).sum().item())
    return total


@pytest.mark.parametrize("n_reads,read_len,first,glen,sub,nr", [
    (10_000, 150, 0, 100_000_000, 0.001, 0.0001),
    (7_777, 150, 123_456_789, C3_GENOME, 0.001, 0.0001),
    (3_001, 15, 5, 1_000, 0.05, 0.02),     # 16-byte thread spans more than two reads
    (513, 1_000, 9, 10_000, 0.0, 0.0),
])
def test_synth_device_matches_host(n_reads, read_len, first, glen, sub, nr):
    host = okm.synth_reads(n_reads, read_len, genome_len=glen, genome_seed=C3_SEED, seed=7, first_read=first,
                           sub_rate=sub, n_rate=nr)
    buf = okm.DeviceBuffer(len(host))
    okm.synth_reads_device(buf.address, n_reads, read_len, genome_len=glen, genome_seed=C3_SEED, seed=7,
                           first_read=first, sub_rate=sub, n_rate=nr)
    dev = np.empty_like(host)
    buf.download(dev)
    buf.free()
    assert np.array_equal(dev, host)


def test_fold_equals_unfolded_and_oracle(monkeypatch):
    k = 31
    batches = [okm.synth_reads(150_000, 150, genome_len=2_000_000, genome_seed=5, seed=5, first_read=i * 150_000)
               for i in range(6)]
    ref = OracleCounter(k)
    for b in batches:
        ref.add_separated(b)
    ek, ec = ref.result(1)
    tables = {}
    for fold_bytes in (None, 300_000_000, 1):
        if fold_bytes is None:
            monkeypatch.delenv("OKM_FOLD_BYTES", raising=False)
        else:
            monkeypatch.setenv("OKM_FOLD_BYTES", str(fold_bytes))
        with okm.KmerCounter(k) as ctr:
            for b in batches:
                buf = okm.DeviceBuffer(len(b))
                buf.upload(b)
                ctr.add_device_batch(buf.address, len(b))
                buf.free()  # consumed before the call returned
            gk, gc = ctr.result(1)
            info = ctr.engine_info()
            # min_count filter over a folded table (count.rs:110)
            fk, fc = ctr.result(3)
        tables[fold_bytes] = info["folds"]
        assert np.array_equal(gk, ek) and np.array_equal(gc, ec), f"fold_bytes={fold_bytes}"
        sel = ec >= 3
        assert np.array_equal(fk, ek[sel]) and np.array_equal(fc, ec[sel])
        assert info["kmers"] == int(ec.sum())
    assert tables[None] == 0 and tables[300_000_000] >= 1 and tables[1] == len(batches) - 1


def test_fold_then_nothing_added(monkeypatch):
    # a fold followed by count with no new batch: the folded table is the result
    monkeypatch.setenv("OKM_FOLD_BYTES", "1")
    k = 21
    b = okm.synth_reads(50_000, 150, genome_len=500_000, seed=9)
    ref = OracleCounter(k)
    ref.add_separated(b)
    ref.add_separated(b)
    ek, ec = ref.result(1)
    with okm.KmerCounter(k) as ctr:
        ctr.add_records([bytes(r) for r in b.tobytes().split(b"\n") if r], normalized=True)
        ctr.add_records([bytes(r) for r in b.tobytes().split(b"\n") if r], normalized=True)
        n1 = ctr.count()
        gk, gc = ctr.result(1)
        assert ctr.engine_info()["folds"] == 1
        # count again (idempotent) and reset
        assert ctr.count() == n1
        ctr.reset()
        assert ctr.count() == 0
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def test_c3_shard_full_size(monkeypatch):
    """Rank 0's shard of C3 at P=8 (bench.py --workload c3 --gpus 8)."""
    k, read_len = 31, 150
    world, rank = 8, 0
    r0, r1 = C3_READS * rank // world, C3_READS * (rank + 1) // world
    n = r1 - r0
    stride = read_len + 1
    buf = okm.DeviceBuffer(n * stride)
    okm.synth_reads_device(buf.address, n, read_len, genome_len=C3_GENOME, genome_seed=C3_SEED, seed=C3_SEED,
                           first_read=r0, sub_rate=0.001, n_rate=0.0001)
    batch_reads = 4_194_304
    spans = [(b0 * stride, (min(n, b0 + batch_reads) - b0) * stride) for b0 in range(0, n, batch_reads)]
    results = []
    ctrs = []
    for fold_bytes in (0, 6_000_000_000):  # 0: folding off
        monkeypatch.setenv("OKM_FOLD_BYTES", str(fold_bytes))
        ctr = okm.KmerCounter(k)
        for off, nb in spans:
            ctr.add_device_batch(buf.address + off, nb)
        nd = ctr.count()
        kp, cp, nn = ctr.result_device()
        assert nn == nd
        results.append((dev_tensor(kp, nd), dev_tensor(cp, nd), ctr.engine_info()))
        ctrs.append(ctr)  # keeps the device table alive
    (keys, counts, info), (fk, fc, finfo) = results
    assert finfo["folds"] >= 1 and info["folds"] == 0
    assert torch.equal(keys, fk) and torch.equal(counts, fc), "fold invariance"
    seq = dev_tensor(buf.address, n * stride, "|u1")
    vw = device_valid_windows(seq, read_len, k)
    assert int(counts.sum().item()) == vw == info["kmers"]
    assert bool((keys[1:] > keys[:-1]).all().item()), "strictly increasing (count.rs:119)"
    assert bool((keys >= 0).all().item()) and bool((keys < (1 << 62)).all().item())
    assert bool((counts >= 1).all().item())
    for o in range(0, keys.numel(), 1 << 27):
        kk = keys[o:o + (1 << 27)]
        assert bool((kk <= torch_revcomp(kk, k)).all().item()), "canonical (kmer.rs:99-106)"
    # a 1/P shard of a 1 Gbp genome at ~3.1x coverage: ~1e9 distinct
    assert 0.7e9 < info["distinct"] < 1.3e9
    # the library's RCCL merge at one rank over this 7.9 GB table: the self
    # send/recv goes in 1 GiB pieces (RCCL delivers half of a >= 2 GiB message)
    want = _table_digest(keys, counts)
    del keys, counts, fk, fc, results
    ctrs[0].close()
    comm = okm.Comm(1, 0, okm.comm_unique_id(), 0)
    assert comm.merge_owned(ctrs[1], ctrs[1]) == info["distinct"]
    kp, cp, nn = ctrs[1].result_device()
    assert _table_digest(dev_tensor(kp, nn), dev_tensor(cp, nn)) == want
    comm.close()
    ctrs[1].close()
    # exact parity on the first 1,000,000 reads of the shard (sharded restatement)
    m = 1_000_000
    host = np.empty(m * stride, dtype=np.uint8)
    buf.download(host)
    thr = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1))
    ek, ec = count_separated_mt(host, k, thr)
    with okm.KmerCounter(k) as ctr:
        ctr.add_device_batch(buf.address, m * stride)
        gk, gc = ctr.result(1)
    buf.free()
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def _table_digest(keys, counts, chunk=1 << 26):
    """Order-sensitive 64-bit digests of a device table (int64 wraps), in
    chunks: the engine's pool holds most of the device."""
    d = [int(keys.numel()), 0, 0, 0]
    for o in range(0, keys.numel(), chunk):
        kk, cc = keys[o:o + chunk], counts[o:o + chunk]
        pos = torch.arange(o, o + kk.numel(), dtype=torch.int64, device=kk.device)
        mix = kk * 0x1E3779B97F4A7C15 - 0x61C8864680B583EB  # wraps: an odd multiplier is a bijection
        d[1] += int(cc.sum().item())
        d[2] += int((mix ^ cc).sum().item())
        d[3] += int(((mix + pos) * (cc | 1)).sum().item())
        del pos, mix
    return (d[0], d[1], d[2] % (1 << 64), d[3] % (1 << 64))


def _count_c3_p1(buf, spans, k):
    ctr = okm.KmerCounter(k)
    for off, nb in spans:
        ctr.add_device_batch(buf.address + off, nb)
    nd = ctr.count()
    return ctr, nd


def test_c3_p1_full_size(monkeypatch):
    """BASELINE configs[2] on ONE GPU at full size (bench.py --workload c3
    --gpus 1): 167,772,160 reads = 25,165,824,000 bases of a 1 Gbp genome,
    generated on the device, counted batch by batch into ONE table
    (count.rs:52-89), with folding and key-range groups active.  Checked on
    the device: sum of counts == valid windows, strictly increasing canonical
    keys, fold invariance (digests of the table at the default fold threshold
    and at half of it); exact parity on the first 1,000,000 reads."""
    k, read_len = 31, 150
    n = C3_READS
    stride = read_len + 1
    buf = okm.DeviceBuffer(n * stride)
    okm.synth_reads_device(buf.address, n, read_len, genome_len=C3_GENOME, genome_seed=C3_SEED, seed=C3_SEED,
                           first_read=0, sub_rate=0.001, n_rate=0.0001)
    vw = device_valid_windows(dev_tensor(buf.address, n * stride, "|u1"), read_len, k)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()  # the engine's pool gets the device
    batch_reads = 4_194_304
    spans = [(b0 * stride, (min(n, b0 + batch_reads) - b0) * stride) for b0 in range(0, n, batch_reads)]
    assert len(spans) == 40
    monkeypatch.delenv("OKM_FOLD_BYTES", raising=False)
    ctr, nd = _count_c3_p1(buf, spans, k)
    info = ctr.engine_info()
    assert info["folds"] >= 4, info  # memory bounded by distinct keys, not input
    kp, cp, nn = ctr.result_device()
    assert nn == nd
    keys, counts = dev_tensor(kp, nd), dev_tensor(cp, nd)
    assert int(counts.sum().item()) == vw == info["kmers"]
    step = 1 << 26  # chunks: the engine's pool holds most of the device
    for o in range(0, nd, step):
        kk = keys[o:o + step + 1]
        assert bool((kk[1:] > kk[:-1]).all().item()), "strictly increasing (count.rs:119)"
        kk = kk[:step]
        assert bool((kk <= torch_revcomp(kk, k)).all().item()), "canonical (kmer.rs:99-106)"
        assert bool((kk >= 0).all().item()) and bool((kk < (1 << 62)).all().item())
        assert bool((counts[o:o + step] >= 1).all().item())
        del kk
    # ~1.0e9 genomic + ~0.6e9 error k-mers (~1.8e9 expected; measured 1.61e9)
    assert 1.4e9 < nd < 1.9e9
    d1 = _table_digest(keys, counts)
    # exact parity of the FOLDED table on 64 key ranges of 1/4096 of the key
    # space each (1/64 in all, 16 per first-base quarter) against the rolling
    # range restatement over ALL 167,772,160 reads (count.rs:48,52-89,106-119)
    _exact_key_ranges(keys, counts, buf, n, stride, k, ranges=c3_key_ranges(k, per_quarter=16, width_bits=12))
    del keys, counts
    ctr.close()
    # the same input folded twice as often: the same table
    total = torch.cuda.get_device_properties(0).total_memory
    monkeypatch.setenv("OKM_FOLD_BYTES", str(int(0.04 * total)))
    ctr2, nd2 = _count_c3_p1(buf, spans, k)
    info2 = ctr2.engine_info()
    assert info2["folds"] > info["folds"]
    kp, cp, _ = ctr2.result_device()
    d2 = _table_digest(dev_tensor(kp, nd2), dev_tensor(cp, nd2))
    ctr2.close()
    assert d1 == d2, "fold invariance"
    # exact parity on the first 1,000,000 reads (sharded restatement)
    m = 1_000_000
    host = np.empty(m * stride, dtype=np.uint8)
    buf.download(host)
    thr = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1))
    ek, ec = count_separated_mt(host, k, thr)
    with okm.KmerCounter(k) as c:
        c.add_device_batch(buf.address, m * stride)
        gk, gc = c.result(1)
    buf.free()
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def c3_key_ranges(k, per_quarter=3, width_bits=13):
    """Key ranges spread over the four first-base quarters of the canonical
    keys (skewed ~7:5:3:1): `per_quarter` ranges of 1/2^width_bits of
    the key space at 10 %, 50 % and 90 % of each quarter."""
    space = 1 << (2 * k)
    q = space >> 2
    w = space >> width_bits
    out = []
    for a in range(4):
        for f in ((0.1, 0.5, 0.9) if per_quarter == 3 else np.linspace(0.05, 0.95, per_quarter)):
            lo = a * q + int(f * q)
            out.append((lo, lo + w))
    return out


def _exact_key_ranges(keys, counts, buf, n_reads, stride, k, threads=None, chunk_reads=4_194_304, ranges=None):
    """Compare the device table's entries inside `ranges` (default
    c3_key_ranges()) exactly with the restatement over every read of the
    device batch `buf` (streamed to the host in chunks)."""
    ranges = ranges or c3_key_ranges(k)
    thr = threads or max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1),
                                os.cpu_count() or 1))
    bounds = torch.tensor([v for r in ranges for v in r], dtype=torch.int64, device=keys.device)
    cut = torch.searchsorted(keys, bounds).cpu().tolist()  # keys < 2^62: signed order is unsigned order
    gk = np.concatenate([keys[cut[2 * i]:cut[2 * i + 1]].cpu().numpy() for i in range(len(ranges))]).view(np.uint64)
    gc = np.concatenate([counts[cut[2 * i]:cut[2 * i + 1]].cpu().numpy() for i in range(len(ranges))]).view(np.uint64)
    host = np.empty(chunk_reads * stride, dtype=np.uint8)

    def chunks():
        seq = dev_tensor(buf.address, n_reads * stride, "|u1")
        for r0 in range(0, n_reads, chunk_reads):
            r1 = min(n_reads, r0 + chunk_reads)
            nb = (r1 - r0) * stride
            h = torch.from_numpy(host[:nb])
            h.copy_(seq[r0 * stride:r1 * stride])
            yield host[:nb]

    ek, ec, w = count_separated_ranges_mt(chunks(), k, ranges, thr)
    assert w == int(counts.sum().item())
    assert len(ek) > 100_000 and all(cut[2 * i + 1] > cut[2 * i] for i in range(len(ranges))), cut
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def test_count_add_count_after_fold(monkeypatch):
    """okm_count, more input, okm_count again: the folded table that became the
    result is kept as input (one map across every add, count.rs:48)."""
    monkeypatch.setenv("OKM_FOLD_BYTES", "1")
    k = 25
    b = okm.synth_reads(40_000, 150, genome_len=400_000, seed=19)
    recs = [bytes(r) for r in b.tobytes().split(b"\n") if r]
    ref = OracleCounter(k)
    for _ in range(3):
        ref.add_separated(b)
    ek, ec = ref.result(1)
    with okm.KmerCounter(k) as ctr:
        ctr.add_records(recs, normalized=True)
        ctr.add_records(recs, normalized=True)
        ctr.count()
        ctr.add_records(recs, normalized=True)
        gk, gc = ctr.result(1)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
