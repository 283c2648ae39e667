"""The N>1 product path of bench.py driven through P virtual ranks on one GPU
(okm_comm_init_loopback: RCCL refuses two ranks on one device; the same plan,
pack / unpack kernels and owner merge run, the transport is device copies).

* okm.pipeline.OwnedCountPipeline — bench.py's N>1 step loop: every rank
  counts its next batches (one to three counting threads, a context each)
  while the previous batch's table goes through the step's failure agreement
  and okm_merge_owned — at P = 2, 3 and 8, every step's owned ranges (rank
  order) exact against the
  restatement of all ranks' reads (count.rs:48: one map over all input,
  :106-119 drained and sorted once);
* the failure agreement: a rank whose count fails stops every rank at that
  step, before any merge, and the communicator still merges afterwards;
* bench.py --workload c3's N>1 step (count the shard into one table, agree,
  okm_merge_owned with owner == local) on a C3-shaped rehearsal of 1.05
  Gbases over 8 ranks: the owners' tables digest like the one-GPU table of
  the same reads, and 12 key ranges are exact against the rolling range
  restatement over every read.
"""

import os
import threading

import numpy as np
import pytest
import torch

import okm
from okm.pipeline import comm_audit, OwnedCountPipeline, PeerFailure, agree_or_raise
from oracle import OracleCounter, count_separated_ranges_mt
from test_gpu_c3 import c3_key_ranges, dev_tensor

pytestmark = pytest.mark.gpu

K = 31


def _threads():
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1), os.cpu_count() or 1))


def _run_ranks(P, body, timeout=300):
    """body(r) on P threads; re-raises the first error."""
    out, err = [None] * P, []

    def run(r):
        try:
            out[r] = body(r)
        except BaseException as e:  # surfaced below
            err.append((r, e))

    th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=timeout)
    assert not any(t.is_alive() for t in th), "a rank is stuck in a collective"
    if err:
        raise err[0][1]
    return out


def _step_batch(step, rank, P, reads_per_rank):
    """Rank r's contiguous shard of step `step`'s reads (a 2 Mbp genome, so
    keys repeat across ranks and steps)."""
    return okm.synth_reads(reads_per_rank, 150, genome_len=2_000_000, genome_seed=60 + step, seed=60 + step,
                           first_read=rank * reads_per_rank, sub_rate=0.002, n_rate=0.0005)


class _Counting:
    """okm.Comm wrapper that counts merges (the tests' view of the steps)."""

    def __init__(self, comm):
        self.comm, self.merges = comm, 0

    def allreduce(self, v):
        return self.comm.allreduce(v)

    def merge_owned(self, a, b):
        n = self.comm.merge_owned(a, b)
        self.merges += 1
        return n

    def last_times(self):
        return self.comm.last_times()


@pytest.mark.parametrize("P,workers", [(2, 1), (8, 1), (3, 3)])  # ((2, 2) dropped in round 6: (3, 3) covers several workers)
def test_owned_count_pipeline_loopback_exact(P, workers):
    nsteps, rpr = 4, 40_000
    batches = [[_step_batch(i, r, P, rpr) for i in range(nsteps)] for r in range(P)]
    bufs = [[okm.DeviceBuffer(len(b)) for b in row] for row in batches]
    for row, brow in zip(bufs, batches):
        for d, b in zip(row, brow):
            d.upload(b)
    comms = okm.Comm.init_loopback(P, 0)
    pipes = [OwnedCountPipeline(_Counting(comms[r]), lambda: okm.KmerCounter(K, "count", 0),
                                lambda c, i, r=r: c.add_device_batch(bufs[r][i].address, len(batches[r][i])),
                                workers=workers)
             for r in range(P)]

    def body(r):
        n = pipes[r].run(nsteps)
        keys, counts = pipes[r].owned().result(1)
        return n, keys, counts

    out = _run_ranks(P, body)
    for i in range(nsteps):
        oc = OracleCounter(K)
        for r in range(P):
            oc.add_separated(batches[r][i])
        if i == nsteps - 1:
            ek, ec = oc.result(1)
        assert sum(o[0][i] for o in out) == oc.distinct, i
    gk = np.concatenate([o[1] for o in out])
    gc = np.concatenate([o[2] for o in out])
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert all(p.comm.merges == nsteps for p in pipes)
    assert sum(len(o[1]) > 0 for o in out) >= P - 1  # the owners' ranges are balanced, not one rank's
    # the N>1 line's audit object (bench.py `comm`) over the same communicators
    infos = [c.info() for c in comms]
    audit = comm_audit(infos, P)
    assert audit["ok"] and audit["comm_ranks"] == P and audit["transport"] == "loopback"
    assert audit["transport_ranks"] == P and [r["transport_rank"] for r in audit["ranks"]] == list(range(P))
    assert all(r["pci_bus_id"] for r in audit["ranks"]) and audit["distinct_pci_bus_ids"] == 1
    assert not comm_audit(infos[:-1], P)["ok"]  # a missing rank is caught
    for p in pipes:
        p.close()
    for c in comms:
        c.close()
    for row in bufs:
        for d in row:
            d.free()


def test_owned_count_pipeline_loopback_failure_agreement():
    """ADVICE r3 (bench.py's N>1 step): rank 1's count fails at step 1; every
    rank stops at that step before okm_merge_owned (the failing rank with its
    own error, the others with PeerFailure), and the same communicators then
    merge the next step exactly."""
    P, nsteps, rpr = 3, 4, 20_000
    batches = [[_step_batch(i, r, P, rpr) for i in range(nsteps)] for r in range(P)]

    def add(c, i, r):
        if r == 1 and i == 1:
            raise RuntimeError("injected count failure")
        c.add_records([bytes(x) for x in batches[r][i].tobytes().split(b"\n") if x], normalized=True)

    comms = okm.Comm.init_loopback(P, 0)
    pipes = [OwnedCountPipeline(_Counting(comms[r]), lambda: okm.KmerCounter(K, "count", 0),
                                lambda c, i, r=r: add(c, i, r)) for r in range(P)]

    def body(r):
        try:
            pipes[r].run(nsteps)
            outcome = "ok"
        except PeerFailure:
            outcome = "peer"
        except RuntimeError as e:
            outcome = "own" if "injected" in str(e) else repr(e)
        merged = pipes[r].comm.merges
        n = pipes[r].run(1, first_step=3)  # the communicators still work
        return outcome, merged, n, pipes[r].owned().result(1)

    out = _run_ranks(P, body)
    assert [o[0] for o in out] == ["peer", "own", "peer"]
    assert all(o[1] == 1 for o in out)  # step 0 merged, step 1 stopped before its merge
    oc = OracleCounter(K)
    for r in range(P):
        oc.add_separated(batches[r][3])
    ek, ec = oc.result(1)
    assert np.array_equal(np.concatenate([o[3][0] for o in out]), ek)
    assert np.array_equal(np.concatenate([o[3][1] for o in out]), ec)
    for p in pipes:
        p.close()
    for c in comms:
        c.close()


def _digest(keys, counts, pos0, chunk=1 << 26):
    """Order-sensitive sums over a device table placed at global position pos0
    (reduced mod 2^64 by the caller once all ranks' parts are added)."""
    d = [int(keys.numel()), 0, 0, 0]
    for o in range(0, keys.numel(), chunk):
        kk, cc = keys[o:o + chunk], counts[o:o + chunk]
        pos = torch.arange(pos0 + o, pos0 + o + kk.numel(), dtype=torch.int64, device=kk.device)
        mix = kk * 0x1E3779B97F4A7C15 - 0x61C8864680B583EB
        d[1] += int(cc.sum().item())
        d[2] += int((mix ^ cc).sum().item())
        d[3] += int(((mix + pos) * (cc | 1)).sum().item())
    return d


def test_c3_shaped_rehearsal_p8_loopback():
    """bench.py --workload c3 at N = 8 (c3_run's step: the shard into one
    table, the failure agreement, okm_merge_owned with owner == local) over 8
    loopback ranks on 7,000,000 C3 reads (1.05 Gbases of the 1 Gbp genome)."""
    P, total, stride, batch_reads = 8, 7_000_000, 151, 4_194_304 // 8
    shards = []
    for r in range(P):
        r0, r1 = total * r // P, total * (r + 1) // P
        buf = okm.DeviceBuffer((r1 - r0) * stride)
        okm.synth_reads_device(buf.address, r1 - r0, 150, genome_len=1_000_000_000, genome_seed=3, seed=3,
                               first_read=r0, sub_rate=0.001, n_rate=0.0001)
        spans = [(b0 * stride, (min(r1 - r0, b0 + batch_reads) - b0) * stride) for b0 in range(0, r1 - r0, batch_reads)]
        shards.append((buf, spans, r1 - r0))
    # the one-GPU table of the same reads
    one = okm.KmerCounter(K)
    for buf, spans, _ in shards:
        for off, nb in spans:
            one.add_device_batch(buf.address + off, nb)
    n1 = one.count()
    kp, cp, _ = one.result_device()
    want = _digest(dev_tensor(kp, n1), dev_tensor(cp, n1), 0)
    one.close()
    comms = okm.Comm.init_loopback(P, 0)
    ctrs = [okm.KmerCounter(K) for _ in range(P)]

    def body(r):
        buf, spans, _ = shards[r]
        err = None
        try:
            ctrs[r].reset()
            for off, nb in spans:
                ctrs[r].add_device_batch(buf.address + off, nb)
            ctrs[r].count()
        except Exception as e:
            err = e
        agree_or_raise(comms[r], err)
        return comms[r].merge_owned(ctrs[r], ctrs[r])

    owned = _run_ranks(P, body)
    assert sum(owned) == n1 > 0.4e9
    got, pos = [0, 0, 0, 0], 0
    ranges = c3_key_ranges(K)
    bounds = torch.tensor([v for rg in ranges for v in rg], dtype=torch.int64, device="cuda")
    gk, gc = [], []
    for r in range(P):
        kp, cp, n = ctrs[r].result_device()
        assert n == owned[r]
        keys, counts = dev_tensor(kp, n), dev_tensor(cp, n)
        got = [a + b for a, b in zip(got, _digest(keys, counts, pos))]
        pos += n
        if n:
            assert bool((keys[1:] > keys[:-1]).all().item())
            cut = torch.searchsorted(keys, bounds).cpu().tolist()
            for i in range(len(ranges)):
                gk.append(keys[cut[2 * i]:cut[2 * i + 1]].cpu().numpy().view(np.uint64))
                gc.append(counts[cut[2 * i]:cut[2 * i + 1]].cpu().numpy().view(np.uint64))
    m64 = (1 << 64) - 1
    assert [got[0], got[1], got[2] & m64, got[3] & m64] == [want[0], want[1], want[2] & m64, want[3] & m64]
    gk = np.concatenate(gk)
    gc = np.concatenate(gc)
    order = np.argsort(gk, kind="stable")  # ranges of several owners: rank order is key order already
    assert np.array_equal(order, np.arange(len(gk)))

    def chunks():
        for buf, _, n in shards:
            host = np.empty(n * stride, dtype=np.uint8)
            buf.download(host)
            yield host

    ek, ec, w = count_separated_ranges_mt(chunks(), K, ranges, _threads())
    assert w == got[1]
    assert len(ek) > 10_000
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    for c in ctrs:
        c.close()
    for c in comms:
        c.close()
    for buf, _, _ in shards:
        buf.free()
