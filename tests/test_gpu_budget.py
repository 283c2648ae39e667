"""Counting past what one GPU holds (count.rs:48: the
reference's DashMap grows in host RAM until the machine runs out).

A small device budget (the test knob hbm_budget_bytes, as OKM_HBM_CAP would
set it) makes a multi-batch C2-shaped input of ~2 GB of FASTQ (6,000,000
reads x 150 bp from a 1 Gbp genome, ~0.8 G distinct keys: ~12 GB of table)
outgrow the device: the engine folds, moves its folded tables to page-locked
host memory (spill_tables), counts the key space in groups streamed back
through the device (count_spilled), and leaves the result on the device
when it fits there, else in host memory (read through okm_fetch_counts).
Checked: exact against the restatement on 12 key ranges over every read,
sum of counts == valid windows, strictly increasing canonical keys."""

import os

import numpy as np
import pytest
import torch

import okm
from okm import testing
from oracle import count_separated_ranges_mt
from test_gpu_c3 import C3_GENOME, _exact_key_ranges, c3_key_ranges, dev_tensor, device_valid_windows, \
    torch_revcomp

pytestmark = pytest.mark.gpu

K = 31
READS = 6_000_000
READ_LEN = 150
STRIDE = READ_LEN + 1
BATCH = 1_000_000


def _input():
    buf = okm.DeviceBuffer(READS * STRIDE)
    okm.synth_reads_device(buf.address, READS, READ_LEN, genome_len=C3_GENOME, genome_seed=11, seed=11,
                           first_read=0, sub_rate=0.001, n_rate=0.0001)
    return buf


def _count(buf):
    ctr = okm.KmerCounter(K)
    for r0 in range(0, READS, BATCH):
        ctr.add_device_batch(buf.address + r0 * STRIDE, (min(READS, r0 + BATCH) - r0) * STRIDE)
    nd = ctr.count()
    return ctr, nd


def _threads():
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1))


def test_budget_16gb_tables_spill_to_host_result_on_device():
    buf = _input()
    vw = device_valid_windows(dev_tensor(buf.address, READS * STRIDE, "|u1"), READ_LEN, K)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    testing.set_knob("hbm_budget_bytes", 16_000_000_000)
    ctr, nd = _count(buf)
    info = ctr.engine_info()
    assert info["spills"] >= 1 and info["folds"] >= 2, info
    assert info["device_peak_bytes"] <= 1.02 * 16_000_000_000, info  # (+ the small non-pool scratch)
    assert 0.5e9 < nd < 1.2e9
    kp, cp, nn = ctr.result_device()  # the result fits the budget once the tables are gone
    assert nn == nd
    keys, counts = dev_tensor(kp, nd), dev_tensor(cp, nd)
    assert int(counts.sum().item()) == vw == info["kmers"]
    step = 1 << 26
    for o in range(0, nd, step):
        kk = keys[o:o + step + 1]
        assert bool((kk[1:] > kk[:-1]).all().item()), "strictly increasing (count.rs:119)"
        kk = kk[:step]
        assert bool((kk <= torch_revcomp(kk, K)).all().item()), "canonical (kmer.rs:99-106)"
    _exact_key_ranges(keys, counts, buf, READS, STRIDE, K, chunk_reads=1_000_000)
    del keys, counts
    ctr.close()
    buf.free()


def test_budget_8gb_result_stays_in_host_memory():
    buf = _input()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    testing.set_knob("hbm_budget_bytes", 8_000_000_000)
    ctr, nd = _count(buf)
    info = ctr.engine_info()
    assert info["spills"] >= 1 and info["host_bytes"] >= 16 * nd, info  # the table lies in host memory
    with pytest.raises(okm.OkmError) as ei:
        ctr.result_device()
    assert ei.value.status == okm._lib.OKM_E_NOMEM
    gk, gc = ctr.result(1)  # streamed through the device filter in slices
    assert len(gk) == nd and int(gc.sum()) == info["kmers"]
    assert bool((gk[1:] > gk[:-1]).all())
    fk, fc = ctr.result(3)  # count.rs:110 min_count over the host table
    sel = gc >= 3
    assert np.array_equal(fk, gk[sel]) and np.array_equal(fc, gc[sel])
    host = np.empty(BATCH * STRIDE, dtype=np.uint8)

    def chunks():
        for r0 in range(0, READS, BATCH):
            nb = (min(READS, r0 + BATCH) - r0) * STRIDE
            h = torch.from_numpy(host[:nb])
            h.copy_(dev_tensor(buf.address + r0 * STRIDE, nb, "|u1"))
            yield host[:nb]

    ranges = c3_key_ranges(K)
    ek, ec, w = count_separated_ranges_mt(chunks(), K, ranges, _threads())
    assert w == info["kmers"]
    parts = [np.searchsorted(gk, np.uint64(v)) for r in ranges for v in r]
    sk = np.concatenate([gk[parts[2 * i]:parts[2 * i + 1]] for i in range(len(ranges))])
    sc = np.concatenate([gc[parts[2 * i]:parts[2 * i + 1]] for i in range(len(ranges))])
    assert len(ek) > 10_000 and np.array_equal(sk, ek) and np.array_equal(sc, ec)
    ctr.close()
    buf.free()


# ---------------------------------------------------------------------------
# One batch past the device, with no folded table to move
# ---------------------------------------------------------------------------

C2_READS = 3_355_443  # BASELINE configs[1]: 1 GiB of 150 bp FASTQ


@pytest.mark.parametrize("budget", [6_000_000_000, 2_500_000_000])
def test_budget_single_c2_batch_past_the_device(budget):
    """One configs[1] batch under a device budget its count does not fit
    (6 GB: the L1 run fits, its count's working set and table do not) or
    its L1 run itself does not fit (2.5 GB: the batch is taken as two
    halves that overlap by k - 1 bytes, okm_engine.hip l1_batch_or_spill).
    There is no folded table to move: the batch runs go to host memory and
    the key space is counted group by group from there (count_spilled).
    Exact on 12 key ranges against the restatement over every read."""
    buf = okm.DeviceBuffer(C2_READS * STRIDE)
    okm.synth_reads_device(buf.address, C2_READS, READ_LEN, genome_len=100_000_000, genome_seed=2, seed=2,
                           first_read=0, sub_rate=0.001, n_rate=0.0001)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    testing.set_knob("hbm_budget_bytes", budget)
    ctr = okm.KmerCounter(K)
    ctr.add_device_batch(buf.address, C2_READS * STRIDE)
    nd = ctr.count()
    info = ctr.engine_info()
    assert info["spills"] >= 1, info  # the host tier was used
    assert info["device_peak_bytes"] <= 1.02 * budget, info
    assert info["folds"] == 0, info
    gk, gc = ctr.result(1)
    ctr.close()
    assert 0.9e8 < nd < 1.3e8 and len(gk) == nd and int(gc.sum()) == info["kmers"]
    assert bool((gk[1:] > gk[:-1]).all())
    host = np.empty(C2_READS * STRIDE, dtype=np.uint8)
    buf.download(host)
    buf.free()
    ranges = c3_key_ranges(K)
    ek, ec, w = count_separated_ranges_mt([host], K, ranges, _threads())
    assert w == info["kmers"]
    parts = [np.searchsorted(gk, np.uint64(v)) for r in ranges for v in r]
    sk = np.concatenate([gk[parts[2 * i]:parts[2 * i + 1]] for i in range(len(ranges))])
    sc = np.concatenate([gc[parts[2 * i]:parts[2 * i + 1]] for i in range(len(ranges))])
    assert len(ek) > 1000 and np.array_equal(sk, ek) and np.array_equal(sc, ec)
