"""k=63 (BASELINE configs[3]) at scale.  The reference caps k at 32
(count.rs:43-45), so parity is restatement-defined: the HIP engine against the
C restatement's k<=64 path, sharded by key range over the host cores
(oracle.count_separated_wide_ranges: rolling encode, pinned to the O(k)
restatement by tests/test_oracle_golden.py).

- 1 Gbases of ONT-like reads: the WHOLE table exact, range by range.
- 5.36 Gbases (the configs[3] size): properties on the device (sum of counts
  = valid windows, strictly ascending 128-bit keys, canonical keys, memory
  under the pool's 90 % soft cap) and exact parity on two key ranges.
"""

import os

import numpy as np
import pytest
import torch

import okm
from dist_rehearsal import DeviceView
from oracle import count_separated_wide_ranges

pytestmark = pytest.mark.gpu

K = 63


def _threads():
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1))


def ont_batch(gbases: float, seed: int, genome_len: int = 200_000_000):
    """ONT-like reads in the device batch layout (records + '\\n'), SURVEY
    §8(d) C4: lognormal lengths (median 2,891, sigma 1.085, clipped
    200..100k), either strand, 5 % errors (2.5 % substitutions, 1.25 %
    insertions, 1.25 % deletions; okm_synth_long_reads), from a seeded random
    genome.  Returns (batch, lengths)."""
    return okm.synth_long_reads(gbases, genome_len, genome_seed=seed, seed=seed)


def _bins_of(keys):
    """Top 8 bits of the 126-bit keys (hi word holds bits 64..125)."""
    return keys[:, 1] >> np.uint64(2 * K - 64 - 8)


def test_k63_one_gbases_exact_vs_range_sharded_restatement():
    """The whole k=63 table at 1 Gbases exact, range by range; and the same
    count under two device budgets below its one-group working set (~76 GB,
    beside its ~24 GB table), checked against the same restatement pass:
    40 GB -- the groups write the table's keys over the batch's own L1 run,
    so only the counts are new memory and the count stays on the device in
    pipelined key-range groups; 20 GB -- not even that fits: the host tier
    (batch runs in host memory, counted key range by key range, VERDICT r5
    item 3)."""
    from okm import testing
    batch, lens = ont_batch(1.0, seed=41)
    buf = okm.DeviceBuffer(len(batch))
    buf.upload(batch)
    with okm.KmerCounter(K, wide=True) as c:
        c.add_device_batch(buf.address, len(batch))
        n = c.count()
        gk, gc = c.result(1)
        info = c.engine_info()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    budgeted = []
    for budget in (40_000_000_000, 20_000_000_000):
        testing.set_knob("hbm_budget_bytes", budget)
        try:
            with okm.KmerCounter(K, wide=True) as c:
                c.add_device_batch(buf.address, len(batch))
                assert c.count() == n
                bk, bc = c.result(1)
                binfo = c.engine_info()
        finally:
            testing.set_knob("hbm_budget_bytes", -1)
        assert binfo["device_peak_bytes"] <= 1.02 * budget, (budget, binfo)
        assert binfo["kmers"] == info["kmers"]
        budgeted.append((bk, bc, binfo))
    buf.free()
    assert budgeted[0][2]["spills"] == 0 and budgeted[0][2]["groups"] >= 2, budgeted[0][2]
    assert budgeted[1][2]["spills"] >= 1, budgeted[1][2]
    windows = int(np.maximum(lens - K + 1, 0).sum())
    assert n == len(gk) and info["kmers"] == windows == int(gc.sum())
    tables = [(gk, gc, _bins_of(gk))] + [(bk, bc, _bins_of(bk)) for bk, bc, _ in budgeted]
    seen = []

    def check(lo, hi, ek, ec):
        ok = True
        m = 0
        for tk, tc, tb in tables:
            a, b = np.searchsorted(tb, lo), np.searchsorted(tb, hi)
            ok = ok and np.array_equal(tk[a:b], ek) and np.array_equal(tc[a:b], ec)
            m = b - a
        seen.append((lo, hi, m, len(ek), ok))

    _, _, w = count_separated_wide_ranges(batch, K, _threads(), shards=32, on_range=check)
    assert w == windows
    seen.sort()
    assert seen[0][0] == 0 and seen[-1][1] == 256 and all(x[1] == y[0] for x, y in zip(seen, seen[1:]))
    assert sum(s[3] for s in seen) == n
    bad = [s for s in seen if not s[4]]
    assert not bad, bad


def _u128_lt(alo, ahi, blo, bhi):
    """a < b for 128-bit values held as int64 pairs (hi < 2^62 here)."""
    flip = torch.tensor(-(1 << 63), dtype=torch.int64, device=alo.device)
    return (ahi < bhi) | ((ahi == bhi) & ((alo ^ flip) < (blo ^ flip)))


def _rc128(lo, hi, k):
    """Reverse complement of 2k-bit keys (kmer.rs:79-94 over 128 bits), torch int64 pairs."""
    rlo = torch.zeros_like(lo)
    rhi = torch.zeros_like(hi)
    for i in range(k):
        b = ((lo >> (2 * i)) & 3) if 2 * i < 64 else ((hi >> (2 * i - 64)) & 3)
        b = 3 - b
        p = 2 * (k - 1 - i)
        if p >= 64:
            rhi |= b << (p - 64)
        else:
            rlo |= b << p
    return rlo, rhi


def test_k63_c4_size_properties_memory_and_exact_ranges():
    batch, lens = ont_batch(5.36, seed=44, genome_len=1_000_000_000)
    buf = okm.DeviceBuffer(len(batch))
    buf.upload(batch)
    total_hbm = torch.cuda.get_device_properties(0).total_memory
    with okm.KmerCounter(K, wide=True) as c:
        c.add_device_batch(buf.address, len(batch))
        buf.free()
        n = c.count()
        info = c.engine_info()
        kp, cp, n2 = c.result_device()
        assert n2 == n
        keys = torch.as_tensor(DeviceView(kp, 2 * n), device="cuda").view(n, 2)
        counts = torch.as_tensor(DeviceView(cp, n), device="cuda")
        windows = int(np.maximum(lens - K + 1, 0).sum())
        assert info["kmers"] == windows == int(counts.sum().item())
        assert info["device_bytes"] <= 0.9 * total_hbm, (info["device_bytes"], total_hbm)
        step = 1 << 28
        for a in range(0, n - 1, step):  # strictly ascending as 128-bit values
            b = min(n, a + step + 1)
            lo, hi = keys[a:b, 0], keys[a:b, 1]
            assert bool(_u128_lt(lo[:-1], hi[:-1], lo[1:], hi[1:]).all())
        idx = torch.randint(0, n, (2_000_000,), device="cuda", generator=torch.Generator("cuda").manual_seed(7))
        lo, hi = keys[idx, 0], keys[idx, 1]
        rlo, rhi = _rc128(lo, hi, K)
        assert not bool(_u128_lt(rlo, rhi, lo, hi).any()), "a key above its reverse complement"
        # exact on 16 key ranges of 1/256 of the key space each (1/16 in all),
        # spread over the first-base quarters (canonical keys are dense in the
        # low ones, sparse in the last), each against a range-filtered
        # restatement of every read (the 16 scans run on the host threads at once)
        ranges = [(b, b + 1) for b in (3, 20, 35, 45, 60, 75, 90, 105, 120, 130, 145, 160, 170, 185, 200, 230)]
        def below(bin_):  # keys whose top 8 bits are < bin_ (they are sorted)
            return sum(int(((keys[a:a + step, 1] >> (2 * K - 64 - 8)) < bin_).sum().item()) for a in range(0, n, step))

        want = {}
        for lo_b, hi_b in ranges:
            a, b = below(lo_b), below(hi_b)
            want[lo_b] = (keys[a:b].cpu().numpy().view(np.uint64), counts[a:b].cpu().numpy().view(np.uint64))
        del keys, counts
    got = {}

    def keep(lo, hi, ek, ec):
        got[lo] = (ek, ec)

    _, _, w = count_separated_wide_ranges(batch, K, _threads(), bins=ranges, on_range=keep)
    assert w == windows
    for lo_b, _ in ranges:
        assert len(want[lo_b][0]) > 0
        assert np.array_equal(want[lo_b][0], got[lo_b][0]) and np.array_equal(want[lo_b][1], got[lo_b][1]), lo_b
