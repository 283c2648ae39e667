"""Multi-process (gloo, CPU) tests of the N>1 path: the
product's step orchestration (okm/pipeline.py: OwnedCountPipeline,
run_pipelined, the failure agreement) and the owner split of the library
(okm_owner_bounds), with the exchange restated in torch
(tests/dist_rehearsal.py, rehearsal only).

Each rank counts its own contiguous shard of reads (count.rs:23-38 is per
record, so shards need no halo), the ranks exchange (key, count) runs by
value-range owner, every owner re-counts its range, and the concatenation of
the owners' ranges in rank order must equal the single-process table of all
reads, bit for bit.  Local counting here is the C restatement
(oracle/okm_oracle.c, test infrastructure) so the test runs without a GPU;
bench.py runs the same exchange over RCCL with the HIP engine.
"""

import os
import time
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import okm
import dist_rehearsal as okm_dist
from okm.pipeline import OwnedCountPipeline, PeerFailure, run_pipelined
from oracle import OracleCounter


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reads(n_reads: int, read_len: int, seed: int) -> np.ndarray:
    b = okm.synth_reads(n_reads, read_len, genome_len=200_000, genome_seed=seed, seed=seed + 1,
                        sub_rate=0.01, n_rate=0.001)
    if seed % 2:  # odd seeds: every 50th read a poly-A / ACGT repeat, so counts pass the one-byte escape (> 255)
        recs = b.reshape(n_reads, read_len + 1)
        recs[::50, :read_len] = np.frombuffer(b"A" * read_len, np.uint8)
        recs[25::100, :read_len] = np.frombuffer((b"ACGT" * read_len)[:read_len], np.uint8)
    return b


def _oracle_merge(k):
    def merge(rk: torch.Tensor, rc: torch.Tensor):
        oc = OracleCounter(k)
        if rk.numel():
            oc.add_pairs(rk.numpy().view(np.uint64), rc.numpy().view(np.uint64))
        mk, mc = oc.result(1)
        return torch.from_numpy(mk.view(np.int64).copy()), torch.from_numpy(mc.view(np.int64).copy())
    return merge


def _worker(rank, world, port, k, n_reads, read_len, seed, empty_rank, out_path, narrow=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        batch = _reads(n_reads, read_len, seed)
        recs = batch.reshape(n_reads, read_len + 1)
        shard = np.array_split(recs, world)[rank]
        oc = OracleCounter(k)
        if rank != empty_rank and len(shard):
            oc.add_separated(np.ascontiguousarray(shard).reshape(-1))
        lk, lc = oc.result(1)
        keys = torch.from_numpy(lk.view(np.int64).copy())
        counts = torch.from_numpy(lc.view(np.int64).copy())
        rk, rc, _, _ = okm_dist.exchange_runs(keys, counts, k, narrow_counts=narrow)
        mk, mc = _oracle_merge(k)(rk, rc)
        # owned ranges are sorted and disjoint, in rank order
        gk, gc = okm_dist.gather_global(mk, mc)
        if rank == 0:
            np.savez(out_path, keys=gk, counts=gc)
    finally:
        dist.destroy_process_group()


def _run(world, k, n_reads=6_000, read_len=150, seed=11, empty_rank=-1, tmp_path=None, narrow=True):
    out = os.path.join(str(tmp_path), f"merged_{world}_{k}.npz")
    mp.spawn(_worker, args=(world, _free_port(), k, n_reads, read_len, seed, empty_rank, out, narrow),
             nprocs=world, join=True)
    got = np.load(out)
    batch = _reads(n_reads, read_len, seed)
    recs = batch.reshape(n_reads, read_len + 1)
    oc = OracleCounter(k)
    for r, part in enumerate(np.array_split(recs, world)):
        if r != empty_rank and len(part):
            oc.add_separated(np.ascontiguousarray(part).reshape(-1))
    ek, ec = oc.result(1)
    return got["keys"], got["counts"], ek, ec


@pytest.mark.parametrize("world,k", [(2, 31), (2, 32), (3, 21)])
def test_owner_partitioned_merge_equals_single_table(world, k, tmp_path):
    gk, gc, ek, ec = _run(world, k, tmp_path=tmp_path)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


@pytest.mark.parametrize("narrow", [True, False])
def test_merge_counts_past_the_byte_escape(narrow, tmp_path):
    # seed 11 is odd: poly-A and ACGT-repeat reads give counts in the
    # thousands, which travel as escapes when counts go as bytes
    gk, gc, ek, ec = _run(3, 31, seed=11, tmp_path=tmp_path, narrow=narrow)
    assert (ec > 255).sum() >= 2  # past the byte: escape entries travel
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def test_merge_with_an_empty_rank(tmp_path):
    gk, gc, ek, ec = _run(2, 25, empty_rank=1, tmp_path=tmp_path)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def _top_bin_worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # k = 32: most keys in the top 16-bit bin (0xFFFF), so an owner bound
        # equals the bin count (+infinity, not key 0 after a wrap)
        rng = np.random.default_rng(rank)
        top = (np.uint64(0xFFFF) << np.uint64(48)) + rng.integers(0, 1 << 40, 900, dtype=np.uint64)
        low = rng.integers(0, 1 << 60, 10, dtype=np.uint64)
        keys = np.unique(np.concatenate([top, low]))
        counts = np.full(len(keys), rank + 1, np.uint64)
        rk, rc, bounds, rs = okm_dist.exchange_runs(torch.from_numpy(keys.view(np.int64).copy()),
                                                    torch.from_numpy(counts.view(np.int64).copy()), 32)
        assert all(s >= 0 for s in rs)
        mk, mc = _oracle_merge(32)(rk, rc)
        gk, gc = okm_dist.gather_global(mk, mc)
        if rank == 0:
            np.savez(out_path, keys=gk, counts=gc, bounds=np.array(bounds))
    finally:
        dist.destroy_process_group()


def test_owner_bound_at_the_top_bin_k32(tmp_path):
    world = 3
    out = os.path.join(str(tmp_path), "top.npz")
    mp.spawn(_top_bin_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    oc = OracleCounter(32)
    for rank in range(world):
        rng = np.random.default_rng(rank)
        top = (np.uint64(0xFFFF) << np.uint64(48)) + rng.integers(0, 1 << 40, 900, dtype=np.uint64)
        low = rng.integers(0, 1 << 60, 10, dtype=np.uint64)
        keys = np.unique(np.concatenate([top, low]))
        oc.add_pairs(keys, np.full(len(keys), rank + 1, np.uint64))
    ek, ec = oc.result(1)
    assert int(got["bounds"][-2]) == 1 << 16  # the wrap case is exercised
    assert np.array_equal(got["keys"], ek) and np.array_equal(got["counts"], ec)


def test_owner_ranges_balance_and_cover():
    rng = np.random.default_rng(0)
    hist = rng.integers(0, 1000, 1 << 12)
    for world in (1, 2, 3, 8):
        b = okm_dist.owner_ranges(hist, world)
        assert b[0] == 0 and b[-1] == len(hist) and len(b) == world + 1
        assert all(x <= y for x, y in zip(b, b[1:]))
        per = [hist[b[r]:b[r + 1]].sum() for r in range(world)]
        assert max(per) - min(per) <= 2 * hist.max()
    # all mass in one bin: one owner takes it, the others get empty ranges
    h = np.zeros(64, np.int64)
    h[7] = 100
    b = okm_dist.owner_ranges(h, 4)
    assert b[0] == 0 and b[-1] == 64 and sorted(b) == b


# ---------------------------------------------------------------------------
# C5 over ranks: compare.rs:51-66 with the references sharded by sample
# ---------------------------------------------------------------------------

def _c5_samples(n=8, n_reads=600, read_len=120):
    """Small WGS-like samples: DB1 = samples [0, n/2), DB2 = [n/2, n); each
    sample draws reads from 2 of 6 seeded genomes, the halves share some."""
    out = []
    for s in range(n):
        rng = np.random.default_rng(100 + s)
        lo = 0 if s < n // 2 else 2
        gs = rng.choice(np.arange(lo, lo + 4), size=2, replace=False)
        out.append(np.concatenate([okm.synth_reads(n_reads, read_len, genome_len=30_000, genome_seed=700 + int(g),
                                                   seed=s * 8 + j, sub_rate=0.002, n_rate=0.001)
                                   for j, g in enumerate(gs)]))
    return out


def _oracle_set(batch, k):
    oc = OracleCounter(k)
    oc.add_separated(batch)
    return oc.result(1)[0]


def _c5_worker(rank, world, port, k, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        samples = _c5_samples()
        half = len(samples) // 2
        mine = range(rank, len(samples), world)  # samples dealt round-robin
        local = {0: [], 1: []}
        for s in mine:
            local[0 if s < half else 1].append(_oracle_set(samples[s], k))

        def local_union(sets):
            u = np.unique(np.concatenate(sets)) if sets else np.zeros(0, np.uint64)
            return torch.from_numpy(u.view(np.int64).copy())

        def union(rk, sizes):
            # every received run is sorted and unique (a rank's own union)
            off, runs = 0, []
            for sz in sizes:
                run = rk[off:off + sz].numpy().view(np.uint64)
                assert np.all(run[1:] > run[:-1])
                runs.append(run)
                off += sz
            u = np.unique(np.concatenate(runs)) if runs else np.zeros(0, np.uint64)
            return len(u), u

        def intersect(ha, na, hb, nb):
            return len(np.intersect1d(ha, hb, assume_unique=True))

        na, nb, inter = okm_dist.distributed_compare(local_union(local[0]), local_union(local[1]), k, union,
                                                     intersect)
        if rank == 0:
            np.savez(out_path, res=np.array([na, nb, inter], np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 31), (3, 32)])
def test_distributed_compare_equals_single_process(world, k, tmp_path):
    out = os.path.join(str(tmp_path), f"c5_{world}_{k}.npz")
    mp.spawn(_c5_worker, args=(world, _free_port(), k, out), nprocs=world, join=True)
    na, nb, inter = (int(x) for x in np.load(out)["res"])
    samples = _c5_samples()
    half = len(samples) // 2
    a = np.unique(np.concatenate([_oracle_set(s, k) for s in samples[:half]]))
    b = np.unique(np.concatenate([_oracle_set(s, k) for s in samples[half:]]))
    ei = len(np.intersect1d(a, b, assume_unique=True))
    assert (na, nb, inter) == (len(a), len(b), ei)
    assert 0 < ei < min(len(a), len(b))  # the halves share genomes, not all of them


# ---------------------------------------------------------------------------
# bench.py's N>1 loop: double-buffered count / exchange+merge pipeline
# ---------------------------------------------------------------------------

def _pipe_worker(rank, world, port, k, nsteps, out_path, staged=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bufs = [None, None]
        busy = [False, False]

        def count_into(i, j):
            assert not busy[j], "a table buffer was recounted before its exchange released it"
            busy[j] = True
            recs = _reads(3_000, 150, seed=20 + i).reshape(3_000, 151)
            oc = OracleCounter(k)
            oc.add_separated(np.ascontiguousarray(np.array_split(recs, world)[rank]).reshape(-1))
            lk, lc = oc.result(1)
            bufs[j] = (torch.from_numpy(lk.view(np.int64).copy()), torch.from_numpy(lc.view(np.int64).copy()))
            return len(lk)

        def consume(i, j, n, release):
            keys, counts = bufs[j]
            assert keys.numel() == n
            rk, rc, _, _ = okm_dist.exchange_runs(keys, counts, k)
            busy[j] = False
            release()
            if staged:  # the merge runs on the finish thread
                return rk, rc
            mk, mc = _oracle_merge(k)(rk, rc)
            return okm_dist.gather_global(mk, mc)

        mbusy = [False, False]

        def finish(i, m, payload):  # no collectives off the main thread
            assert not mbusy[m], "a merge slot was reused before its merge finished"
            mbusy[m] = True
            time.sleep(0.01 * (i % 2))  # let the exchange of the next batch run ahead
            r = _oracle_merge(k)(*payload)
            mbusy[m] = False
            return r

        if staged:
            merged = run_pipelined(nsteps, count_into, consume, finish)
            res = [okm_dist.gather_global(mk, mc) for mk, mc in merged]
        else:
            res = run_pipelined(nsteps, count_into, consume)
        if rank == 0:
            np.savez(out_path, **{f"k{i}": r[0] for i, r in enumerate(res)}, **{f"c{i}": r[1] for i, r in enumerate(res)})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("staged", [False, True], ids=["count|exchange+merge", "count|exchange|merge"])
def test_pipelined_steps_equal_single_tables(tmp_path, staged):
    k, world, nsteps = 31, 2, 4
    out = os.path.join(str(tmp_path), "pipe.npz")
    mp.spawn(_pipe_worker, args=(world, _free_port(), k, nsteps, out, staged), nprocs=world, join=True)
    got = np.load(out)
    for i in range(nsteps):
        oc = OracleCounter(k)
        oc.add_separated(_reads(3_000, 150, seed=20 + i))
        ek, ec = oc.result(1)
        assert np.array_equal(got[f"k{i}"], ek) and np.array_equal(got[f"c{i}"], ec), i


def test_pipelined_worker_error_surfaces():
    def count_into(i, j):
        if i == 2:
            raise RuntimeError("count failed")
        return i

    seen = []
    with pytest.raises(RuntimeError, match="count failed"):
        run_pipelined(5, count_into, lambda i, j, h, release: (release(), seen.append(h)))
    assert seen == [0, 1]


def test_pipelined_finish_error_surfaces():
    def finish(i, m, payload):
        if i == 1:
            raise RuntimeError("merge failed")
        return payload

    with pytest.raises(RuntimeError, match="merge failed"):
        run_pipelined(6, lambda i, j: i, lambda i, j, h, release: (release(), h)[1], finish)


def test_pipelined_finish_results_in_order():
    out = run_pipelined(7, lambda i, j: i, lambda i, j, h, release: (release(), h * 10)[1],
                                 lambda i, m, p: (i, m, p))
    assert out == [(i, i % 2, i * 10) for i in range(7)]


# ---------------------------------------------------------------------------
# okm.pipeline.OwnedCountPipeline (bench.py's N>1 step) over gloo processes:
# the product orchestration with oracle-backed counters and a gloo comm whose
# merge_owned restates okm_merge_owned's plan (dist_rehearsal)
# ---------------------------------------------------------------------------

class _OracleCtx:
    """The KmerCounter surface the pipeline uses, counted by the restatement."""

    def __init__(self, k, fail_at=None):
        self.k, self.fail_at, self.step = k, fail_at, -1
        self.oc = OracleCounter(k)

    def reset(self):
        self.oc = OracleCounter(self.k)

    def add(self, data, step):
        self.step = step
        if self.fail_at is not None and step == self.fail_at:
            raise RuntimeError(f"count failed at step {step}")
        self.oc.add_separated(data)

    def count(self):
        return self.oc.distinct

    def result(self, min_count=1):
        return self.oc.result(min_count)


class _GlooComm:
    """allreduce / merge_owned of okm.Comm over the default gloo group."""

    def __init__(self, k):
        self.k = k
        self.merges = 0

    def allreduce(self, values):
        t = torch.tensor([int(v) for v in values], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return [int(x) for x in t.tolist()]

    def merge_owned(self, local, owner):
        lk, lc = local.result(1)
        rk, rc, _, _ = okm_dist.exchange_runs(torch.from_numpy(lk.view(np.int64).copy()),
                                              torch.from_numpy(lc.view(np.int64).copy()), self.k)
        owner.reset()
        if rk.numel():
            owner.oc.add_pairs(rk.numpy().view(np.uint64), rc.numpy().view(np.uint64))
        self.merges += 1
        return owner.count()


def _step_reads(i):
    return _reads(3_000, 150, seed=40 + i).reshape(3_000, 151)


def _owned_pipe_worker(rank, world, port, k, nsteps, fail_rank, fail_step, out_path, workers=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = _GlooComm(k)
        fail_at = fail_step if rank == fail_rank else None

        def add(ctx, step):
            ctx.add(np.ascontiguousarray(np.array_split(_step_reads(step), world)[rank]).reshape(-1), step)

        pipe = OwnedCountPipeline(comm, lambda: _OracleCtx(k, fail_at), add, workers=workers)
        outcome = "ok"
        try:
            res = pipe.run(nsteps)
        except PeerFailure:
            outcome = "peer"
            res = None
        except RuntimeError as e:
            outcome = "own" if "count failed" in str(e) else repr(e)
            res = None
        mk = mc = None
        if res is not None:
            ok, oc_ = pipe.owned().result(1)
            mk, mc = okm_dist.gather_global(torch.from_numpy(ok.view(np.int64).copy()),
                                            torch.from_numpy(oc_.view(np.int64).copy()))
        # one more collective after the failure: every rank is still in step
        dist.barrier()
        np.savez(out_path + f".{rank}.npz", outcome=np.array(outcome), merges=np.array(comm.merges),
                 n=np.array(res if res is not None else [], np.int64),
                 keys=mk if mk is not None else np.zeros(0, np.uint64),
                 counts=mc if mc is not None else np.zeros(0, np.uint64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("workers", [1, 3])
def test_owned_count_pipeline_steps_equal_global_table(tmp_path, workers):
    """Every step's owners hold the global table of that step's reads; the
    last step's ranges in rank order equal the single-process table (one
    counting thread, and three counting the next steps concurrently)."""
    k, world, nsteps = 31, 2, 5
    out = os.path.join(str(tmp_path), "own")
    mp.spawn(_owned_pipe_worker, args=(world, _free_port(), k, nsteps, -1, -1, out, workers), nprocs=world,
             join=True)
    got = [np.load(out + f".{r}.npz") for r in range(world)]
    assert all(str(g["outcome"]) == "ok" for g in got)
    oc = OracleCounter(k)
    oc.add_separated(_step_reads(nsteps - 1).reshape(-1))
    ek, ec = oc.result(1)
    assert np.array_equal(got[0]["keys"], ek) and np.array_equal(got[0]["counts"], ec)
    for i in range(nsteps):  # owned distinct counts sum to each step's distinct keys
        o = OracleCounter(k)
        o.add_separated(_step_reads(i).reshape(-1))
        assert sum(int(g["n"][i]) for g in got) == o.distinct, i
    assert all(int(g["merges"]) == nsteps for g in got)


@pytest.mark.parametrize("fail_rank,fail_step,workers", [(1, 2, 1), (0, 0, 1), (1, 3, 2)])
def test_owned_count_pipeline_failure_stops_every_rank(tmp_path, fail_rank, fail_step, workers):
    """a rank whose count fails must not let its peers run the
    merge alone: every rank raises at that step, before okm_merge_owned, and
    the process group is still usable (the barrier after the failure)."""
    k, world, nsteps = 25, 2, 5
    out = os.path.join(str(tmp_path), "fail")
    mp.spawn(_owned_pipe_worker, args=(world, _free_port(), k, nsteps, fail_rank, fail_step, out, workers),
             nprocs=world, join=True)
    got = [np.load(out + f".{r}.npz") for r in range(world)]
    for r, g in enumerate(got):
        assert str(g["outcome"]) == ("own" if r == fail_rank else "peer"), (r, str(g["outcome"]))
        assert int(g["merges"]) == fail_step  # no rank merged the failed step
