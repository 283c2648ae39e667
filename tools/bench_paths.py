#!/usr/bin/env python3
"""Secondary measurements of the §8 rows next to the headline count bench
(bench.py): one JSON line per workload, same conventions (device-resident
input, warmup then timed steps bracketed by device syncs).

  --workload query   query.rs:81-99 — per-read hit counts of the BASELINE
                     configs[1] batch (3,355,443 x 150 bp, k=31) against a
                     device set of the canonical k-mers of the first half of
                     those reads (okm_query_hits_device).
  --workload build   build.rs:46-58 — set-mode counting (DashSet) of the same
                     batch (okm_add_batch_device + okm_count in OKM_MODE_SET).
  --workload wide    BASELINE configs[3] shape — k=63 (two-u64 keys) over
                     ONT-like lognormal reads (median 2,891 bp, sigma 1.085,
                     clipped 200..100k, 5 % substitution + indel errors); --gbases sets the
                     size (configs[3] is ~5.36 Gbases).
  --workload c5      BASELINE configs[4] shape: build.rs per-sample sets of 64
                     WGS-shaped synthetic samples (tools/c5_runs.json) into two
                     databases, then compare.rs (unions, |A ∩ B|, Jaccard).
                     Under torchrun (WORLD_SIZE > 1, RCCL) or with --loopback P
                     (P virtual ranks on one GPU) the samples shard over the
                     ranks and the unions are owner-partitioned by the
                     library's exchange (wl_c5_dist, okm_merge_owned_n).
  --workload c3      BASELINE configs[2] over --loopback P virtual ranks on one
                     GPU (wl_c3_loop): per-rank one-card count times, then
                     okm_merge_owned at once; the owners' tables must digest
                     exactly like the one-GPU table.
  --workload classify classify.rs:215-308 — probe a 32-reference database
                     (the genome split in 32 slices, ~100 M keys) against the
                     counted table of the batch (okm_classifier_probe_db).

The CPU baseline is the C restatement (oracle/) on a bounded sample, 1 thread.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-kmer_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import okm  # noqa: E402
from okm import workloads  # noqa: E402

HBM_PEAK_GBS = 8000.0
READS, READ_LEN, GENOME_BP = 3_355_443, 150, 100_000_000


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def c2_batch():
    t = time.time()
    b = okm.synth_reads(READS, READ_LEN, genome_len=GENOME_BP, genome_seed=2, seed=2, sub_rate=0.001,
                        n_rate=0.0001)
    log(f"synthetic C2 batch: {len(b)} bytes ({time.time() - t:.1f}s)")
    return b


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    return (time.perf_counter() - t) / steps


def valid_windows(batch: np.ndarray, k: int, valid=b"ACGTacgt") -> int:
    ok = np.zeros(256, bool)
    ok[list(valid)] = True
    bad = ~ok[batch]
    c = np.concatenate([[0], np.cumsum(bad, dtype=np.int64)])
    return int(((c[k:] - c[:-k]) == 0).sum())


def wl_query(args):
    k = 31
    batch = c2_batch()
    half = (READS // 2) * (READ_LEN + 1)
    dbuf = okm.DeviceBuffer(len(batch))
    hbuf = okm.DeviceBuffer(4 * READS)
    dbuf.upload(batch)
    with okm.KmerCounter(k, "set") as c:
        c.add_device_batch(dbuf.address, half)
        db_keys, _ = c.result(1)
    s = okm.KmerSet(k, 0, len(db_keys))
    s.insert(db_keys)
    windows = valid_windows(batch, k)
    t_first = time.perf_counter()
    s.query_hits_device(dbuf.address, len(batch), READS, hbuf.address)
    t_first = time.perf_counter() - t_first
    dt = timed(lambda: s.query_hits_device(dbuf.address, len(batch), READS, hbuf.address), args.steps, args.warmup)
    hits = np.zeros(READS, np.uint32)
    hbuf.download(hits)
    bases = READS * READ_LEN
    alg = len(batch) + 8 * windows  # 1 B/base + one 8-B slot read per valid window
    # CPU baseline: the C restatement (O(k) per window + binary search) on a sample
    import oracle
    m = min(args.cpu_sample_reads, READS)
    recs = batch[:m * (READ_LEN + 1)].reshape(m, READ_LEN + 1)[:, :READ_LEN]
    tc = time.perf_counter()
    exp = oracle.query_hits([r.tobytes() for r in recs], db_keys, k)
    tcpu = time.perf_counter() - tc
    assert np.array_equal(exp, hits[:m]), "engine != oracle on the CPU sample"
    return {
        "metric": "bases/sec queried (k=31, query.rs per-read hits) on one MI355X",
        "value": round(bases / dt, 1), "unit": "bases/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "u64",
        "data": "synthetic (BASELINE configs[1] reads, device-resident)",
        "config": {"workload": "query: 3,355,443 x 150 bp reads vs the k-mer set of the first half of them",
                   "k": k, "db_unique_kmers": int(len(db_keys)), "valid_windows": windows,
                   "reads_with_hits": int((hits > 0).sum()), "hits": int(hits.sum(dtype=np.uint64)),
                   "index": "hash set (open addressing, one slot per probe)",
                   "first_query_ms": round(t_first * 1e3, 2)},
        "roofline": {"bound": "hbm", "kernel": "k_query_hits<31> (+ k_sep_count, scan)",
                     "achieved_wall": round(alg / dt / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "alg_bytes_per_step": alg, "frac_wall": round(alg / dt / 1e9 / HBM_PEAK_GBS, 4)},
        "cpu_baseline": {"value": round(m * READ_LEN / tcpu, 1), "unit": "bases/s", "cores": 1, "kind": "port",
                         "sample": f"first {m} reads, oracle_query_hits (O(k) encode per window + binary "
                                   f"search, 1 thread; the reference runs rayon over reads), {tcpu:.1f} s"},
    }


def wl_build(args):
    k = 31
    batch = c2_batch()
    dbuf = okm.DeviceBuffer(len(batch))
    dbuf.upload(batch)
    c = okm.KmerCounter(k, "set")

    def step():
        c.reset()
        c.add_device_batch(dbuf.address, len(batch))
        return c.count()

    dt = timed(step, args.steps, args.warmup)
    n = step()
    bases = READS * READ_LEN
    return {"metric": "bases/sec k-mer set built (k=31, build.rs DashSet) on one MI355X",
            "value": round(bases / dt, 1), "unit": "bases/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "u64",
            "data": "synthetic (BASELINE configs[1] reads, device-resident)",
            "config": {"workload": "build: set of canonical 31-mers of 3,355,443 x 150 bp reads", "k": k,
                       "distinct": int(n)}}


def ont_batch(gbases: float, seed: int = 4):
    """ONT-like reads (okm.workloads.c4_reads): lognormal
    lengths (median 2,891, sigma 1.085, 200..100k), either strand, 5 %
    substitution + indel errors (2.5 % substitutions, 1.25 % insertions, 1.25 %
    deletions), seed 4, from a genome of a quarter of the bases."""
    batch, lens = workloads.c4_reads(gbases, seed)
    return batch, len(lens)


def wl_wide(args):
    k = 63
    t = time.time()
    batch, n = ont_batch(args.gbases)
    bases = len(batch) - n
    log(f"ONT-like batch: {n} reads, {bases} bases ({time.time() - t:.1f}s)")
    dbuf = okm.DeviceBuffer(len(batch))
    dbuf.upload(batch)
    c = okm.KmerCounter(k, "count", wide=True)

    def step():
        c.reset()
        c.add_device_batch(dbuf.address, len(batch))
        return c.count()

    for _ in range(args.warmup):
        step()
    c.set_timing(True)  # kernel stats over the timed steps only
    dt = timed(step, args.steps, 0)
    info = c.engine_info()
    kern = {name: {"launches": v["launches"], "avg_ms": round(v["total_ms"] / max(v["launches"], 1), 4)}
            for name, v in c.kernel_stats().items()}
    return {"metric": "bases/sec k-mer-counted (k=63, two-u64 keys) on one MI355X",
            "value": round(bases / dt, 1), "unit": "bases/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "dtype": "u128 (two u64)", "data": "synthetic ONT-like (device-resident)",
            "config": {"workload": f"BASELINE configs[3] shape at {args.gbases} Gbases: lognormal read "
                                   "lengths (median 2891, sigma 1.085, 200..100k), 5 % substitution + indel errors",
                       "k": k, "reads": n, "bases": bases, "kmers": int(info["kmers"]),
                       "distinct": int(info["distinct"])},
            "kernels": kern, "engine": info}


def c5_samples(cap_bases: float, which=None):
    """SURVEY §8(d) C5 (okm.workloads.c5_samples): 64 synthetic samples shaped
    by 64 WGS runs of data_metagenome.json.gz (tools/c5_runs.json)."""
    return workloads.c5_samples(cap_bases, which)


def wl_c5(args):
    """build.rs:46-116 (one k-mer set per sample file) for DB1 and DB2, then
    compare.rs:51-66 (union of each DB's references, |A ∩ B|, Jaccard), all on
    the device with the samples resident."""
    k = 31
    t = time.time()
    samples = c5_samples(args.c5_cap)
    bases = sum(int(len(b)) - int((b == 10).sum()) for b in samples)
    log(f"C5: 64 samples, {bases / 1e9:.2f} Gbases ({time.time() - t:.1f}s)")
    dev = []
    for b in samples:
        d = okm.DeviceBuffer(len(b))
        d.upload(b)
        dev.append((d, len(b)))
    # two contexts (own HIP stream each) build alternate samples from two host
    # threads, and the two unions run concurrently the same way
    import threading
    sample_ctxs = [okm.KmerCounter(k, "set"), okm.KmerCounter(k, "set")]
    unions = [okm.KmerCounter(k, "set"), okm.KmerCounter(k, "set")]
    # per-sample set sizes (deterministic) fix each sample's slice of the store
    offs = []
    tot = 0
    sample_ctx = sample_ctxs[0]
    for d, n in dev:
        sample_ctx.reset()
        sample_ctx.add_device_batch(d.address, n)
        m = sample_ctx.count()
        offs.append((tot, m))
        tot += m
    store = [okm.DeviceBuffer(8 * tot)]

    def par(fn, items):
        """items[0::2] on one host thread, items[1::2] on another."""
        err = []

        def run(part):
            try:
                for x in part:
                    fn(*x)
            except BaseException as e:
                err.append(e)

        th = [threading.Thread(target=run, args=(items[i::2],), daemon=True) for i in range(2)]
        for t_ in th:
            t_.start()
        for t_ in th:
            t_.join()
        if err:
            raise err[0]

    def step():
        # build: each sample's set, copied into its slice of the reference store
        got = [0] * len(dev)

        def build(i, c):
            d, n = dev[i]
            c.reset()
            c.add_device_batch(d.address, n)
            m = c.count()
            if m != offs[i][1]:
                raise RuntimeError("sample set size changed between steps")
            c.fetch_into_device(store[0].address + 8 * offs[i][0], 0, m)
            got[i] = m

        # sample i on context i % 2: thread j (items j::2) owns context j
        par(build, [(i, sample_ctxs[i % 2]) for i in range(len(dev))])
        sizes = [(o, m) for (o, _), m in zip(offs, got)]
        # compare: A = union of DB1's references, B = union of DB2's
        res = [None, None]

        def union(h):
            u = unions[h]
            u.reset()
            for o, m in sizes[32 * h:32 * h + 32]:
                u.add_sorted_pairs_device(store[0].address + 8 * o, 0, m)
            na = u.count()
            res[h] = u.result_device()[0:1] + (na,)

        par(union, [(0,), (1,)])
        inter = okm.set_intersection_size_device(res[0][0], res[0][1], res[1][0], res[1][1])
        return sizes, res, inter

    dt = timed(step, args.steps, args.warmup)
    sizes, res, inter = step()
    na, nb = res[0][1], res[1][1]
    union = na + nb - inter
    jac = inter / union if union else 0.0
    # consistency on the host (bounded): the union of two references per DB
    # and their intersection, device vs numpy on the downloaded sets
    sub = []
    for h in (0, 1):
        parts = []
        for o, m in sizes[32 * h:32 * h + 2]:
            x = np.empty(m, np.uint64)
            okm.lib().okm_memcpy_d2h(x.ctypes.data, okm.c_void_p(store[0].address + 8 * o), 8 * m)
            parts.append(x)
        with okm.KmerCounter(k, "set") as u:
            for x in parts:
                u.add_pairs(x)
            gu, _ = u.result(1)
        hu = np.union1d(parts[0], parts[1])
        assert np.array_equal(gu, hu), "device union != host union"
        sub.append(hu)
    assert okm.set_intersection_size(sub[0], sub[1]) == len(np.intersect1d(sub[0], sub[1], assume_unique=True))
    # CPU baseline + parity spot check: the C restatement's set of a sample prefix
    import oracle
    sb = samples[0][:min(len(samples[0]), 8_000_000)]
    sb = sb[:int(np.flatnonzero(sb == 10)[-1]) + 1]
    tc = time.perf_counter()
    oc = oracle.OracleCounter(k)
    oc.add_separated(sb)
    ek, _ = oc.result(1)
    tcpu = time.perf_counter() - tc
    with okm.KmerCounter(k, "set") as c1:
        c1.add_records([r for r in sb.tobytes().split(b"\n") if r], normalized=True)
        gk, _ = c1.result(1)
    assert np.array_equal(gk, ek), "engine set != oracle set on the CPU sample"
    cb = int(len(sb) - (sb == 10).sum())
    return {"metric": "bases/sec built into per-sample k-mer sets + compared (k=31, build.rs + compare.rs) "
                      "on one MI355X",
            "value": round(bases / dt, 1), "unit": "bases/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "u64",
            "data": "synthetic (64 samples shaped by tools/c5_runs.json, device-resident)",
            "config": {"workload": f"BASELINE configs[4] shape on one GPU: 64 WGS-shaped samples (reads from 3 of 48 "
                                   f"seeded 2-8 Mbp genomes, <= {args.c5_cap / 1e6:.0f} Mbases each), DB1 = "
                                   f"samples 0-31, DB2 = 32-63",
                       "k": k, "bases": bases, "set_sizes_total": int(tot),
                       "db1_total_unique_kmers_across_references": int(na),
                       "db2_total_unique_kmers_across_references": int(nb), "intersection_size": int(inter),
                       "union_size": int(union), "jaccard_index": jac},
            "cpu_baseline": {"value": round(cb / tcpu, 1), "unit": "bases/s", "cores": 1, "kind": "port",
                             "sample": f"first {cb} bases of sample 0, oracle set build (O(k) encode per window, "
                                       f"1 thread), {tcpu:.1f} s; engine set identical"}}


def _c5_rank(rank, world, comm, device, args, steps, warmup, gate=None):
    """One rank of the distributed C5 (SURVEY.md §8(e) "C5"): the 64 samples
    dealt round-robin (sample s -> rank s mod N); this rank builds its
    samples' sets (build.rs:46-116), unions its share of each DB's references
    (sorted runs, set mode), and okm.distributed_compare moves both unions to
    key-range owners under one split (okm_merge_owned_n), intersects each
    owner's two ranges on its GPU and sums |A|, |B|, |A ∩ B| over the ranks
    (compare.rs:51-66).  gate: a barrier shared by in-process ranks."""
    k = 31
    mine = list(range(rank, 64, world))
    samples = dict(zip(mine, c5_samples(args.c5_cap, set(mine))))
    my_bases = sum(int(len(b)) - int((b == 10).sum()) for b in samples.values())
    dev = {}
    for s_, b in samples.items():
        d = okm.DeviceBuffer(len(b), device)
        d.upload(b)
        dev[s_] = (d, len(b))
    del samples
    sample_ctx = okm.KmerCounter(k, "set", device)
    locals_ = [okm.KmerCounter(k, "set", device), okm.KmerCounter(k, "set", device)]
    owners = [okm.KmerCounter(k, "set", device), okm.KmerCounter(k, "set", device)]
    tot = 0
    for d, n in dev.values():
        sample_ctx.reset()
        sample_ctx.add_device_batch(d.address, n)
        tot += sample_ctx.count()
    store = okm.DeviceBuffer(max(8, 8 * tot), device)

    def step():
        sizes = {}
        off = 0
        for s_, (d, n) in dev.items():
            sample_ctx.reset()
            sample_ctx.add_device_batch(d.address, n)
            m = sample_ctx.count()
            sample_ctx.fetch_into_device(store.address + 8 * off, 0, m)
            sizes[s_] = (off, m)
            off += m
        for h in (0, 1):
            u = locals_[h]
            u.reset()
            for s_, (o, m) in sizes.items():
                if (s_ < 32) == (h == 0) and m:
                    u.add_sorted_pairs_device(store.address + 8 * o, 0, m)
            u.count()
        return okm.distributed_compare(comm, locals_[0], locals_[1], owners[0], owners[1])

    for _ in range(warmup):
        step()
    if gate:
        gate.wait()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = step()
    for c in [sample_ctx] + locals_ + owners:
        c.synchronize()
    if gate:
        gate.wait()
    dt = (time.perf_counter() - t0) / steps
    ta, tb = comm.last_bytes()
    for c in [sample_ctx] + locals_ + owners:
        c.close()
    store.free()
    for d, _ in dev.values():
        d.free()
    return {"dt": dt, "bases": my_bases, "sets": tot, "res": res, "bytes_sent": ta}


def wl_c5_dist(args):
    """C5 over N ranks through the library's exchange (okm_merge_owned_n).
    Under torchrun: one process per GPU, RCCL communicator (torch gloo only
    hands out its id and takes the max time).  --loopback P: P virtual ranks in
    this process on one GPU (okm_comm_init_loopback) -- the same code path at
    P = 8 on a one-GPU box; its time is all ranks sharing one device, a
    rehearsal, not a scaling number.  Strong scaling: the 64-sample workload
    is fixed."""
    if args.loopback:
        import threading
        P = args.loopback
        comms = okm.Comm.init_loopback(P, 0)
        gate = threading.Barrier(P)
        out, err = [None] * P, []

        def body(r):
            try:
                out[r] = _c5_rank(r, P, comms[r], 0, args, args.steps, args.warmup, gate)
            except BaseException as e:  # surfaced below
                err.append(e)
                gate.abort()

        th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(P)]
        for t_ in th:
            t_.start()
        for t_ in th:
            t_.join()
        for c in comms:
            c.close()
        if err:
            raise err[0]
        world, impl = P, f"okm_merge_owned_n over a loopback communicator ({P} virtual ranks on one MI355X)"
        dt = max(o["dt"] for o in out)
        bases = sum(o["bases"] for o in out)
        set_total = sum(o["sets"] for o in out)
        sent = sum(o["bytes_sent"] for o in out)
        res = out[0]["res"]
        assert all(o["res"] == res for o in out)
        n_gpus = 1
    else:
        import torch
        import torch.distributed as tdist
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ["RANK"])
        local = int(os.environ.get("LOCAL_RANK", "0"))
        device = local % max(1, torch.cuda.device_count())
        tdist.init_process_group("gloo")
        uid = torch.zeros(okm._lib.OKM_COMM_ID_BYTES, dtype=torch.uint8)
        if rank == 0:
            uid = torch.frombuffer(bytearray(okm.comm_unique_id()), dtype=torch.uint8)
        tdist.broadcast(uid, 0)
        comm = okm.Comm(world, rank, bytes(uid.numpy().tobytes()), device)
        tdist.barrier()
        o = _c5_rank(rank, world, comm, device, args, args.steps, args.warmup)
        comm.close()
        tt = torch.tensor([o["dt"], float(o["bases"]), float(o["sets"]), float(o["bytes_sent"])], dtype=torch.float64)
        mx = tt.clone()
        tdist.all_reduce(mx, op=tdist.ReduceOp.MAX)
        tdist.all_reduce(tt, op=tdist.ReduceOp.SUM)
        tdist.destroy_process_group()
        if rank != 0:
            return None
        dt, bases, set_total, sent = float(mx[0]), int(tt[1]), int(tt[2]), int(tt[3])
        res = o["res"]
        impl, n_gpus = "okm_merge_owned_n over RCCL (one rank per GPU)", world
    na, nb, inter = res
    union_ = na + nb - inter
    return {"metric": f"bases/sec built into per-sample k-mer sets + compared (k=31, build.rs + compare.rs) "
                      f"over {world} ranks",
            "value": round(bases / dt, 1), "unit": "bases/s", "n_gpus": n_gpus, "ranks": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "dtype": "u64",
            "data": "synthetic (64 samples shaped by tools/c5_runs.json, device-resident)",
            "config": {"workload": f"BASELINE configs[4] shape over {world} ranks: 64 WGS-shaped samples "
                                   f"(<= {args.c5_cap / 1e6:.0f} Mbases each) dealt round-robin, DB1 = samples "
                                   f"0-31, DB2 = 32-63, unions owner-partitioned",
                       "k": 31, "bases": bases, "set_sizes_total": set_total, "exchange": impl,
                       "bytes_sent_all_ranks": sent,
                       "db1_total_unique_kmers_across_references": na,
                       "db2_total_unique_kmers_across_references": nb, "intersection_size": inter,
                       "union_size": union_, "jaccard_index": inter / union_ if union_ else 0.0}}


C3_READS, C3_GENOME_BP, C3_SEED, C3_BATCH_READS = 167_772_160, 1_000_000_000, 3, 4_194_304  # bench.py


def _table_digest(kp: int, cp: int, n: int, pos0: int, chunk: int = 1 << 26):
    """Order-sensitive digests of a device (key, count) table as int64 sums
    (wrapping), positions counted from pos0: the owners' tables, concatenated
    in rank order, digest like the one-GPU table."""
    import torch
    tests_dir = os.path.join(ROOT, "tests")
    if tests_dir not in sys.path:
        sys.path.insert(0, tests_dir)
    from dist_rehearsal import DeviceView  # rehearsal-only helper (a torch view of device memory)
    if not n:
        return [0, 0, 0, 0]
    keys = torch.as_tensor(DeviceView(kp, n), device="cuda")
    counts = torch.as_tensor(DeviceView(cp, n), device="cuda")
    d = [n, 0, 0, 0]
    for o in range(0, n, chunk):
        kk, cc = keys[o:o + chunk], counts[o:o + chunk]
        pos = torch.arange(pos0 + o, pos0 + o + kk.numel(), dtype=torch.int64, device=kk.device)
        mix = kk * 0x1E3779B97F4A7C15 - 0x61C8864680B583EB
        d[1] += int(cc.sum().item())
        d[2] += int((mix ^ cc).sum().item())
        d[3] += int(((mix + pos) * (cc | 1)).sum().item())
        del pos, mix
    return d


def wl_c3_loop(args):
    """BASELINE configs[2] (C3) over P virtual ranks on ONE GPU
    (okm_comm_init_loopback): rank r counts its contiguous 1/P shard of the
    167,772,160 reads into one table (count.rs:52-89), the ranks' counts one
    at a time (each alone on the GPU, as on its own card), then every rank runs
    okm_merge_owned (owner == local, as bench.py at N>1) at once.  The owners'
    tables, concatenated in rank order, must digest exactly like the one-GPU
    table of the same reads.  A rehearsal of the N>1 path of bench.py --workload
    c3: the per-rank count times are one-card times; the exchange + merge share
    one device here, so they are not N-GPU times."""
    import threading
    P = max(1, args.loopback)
    k, stride = 31, READ_LEN + 1
    total = args.c3_reads
    shards = []
    t0 = time.time()
    for r in range(P):
        r0, r1 = total * r // P, total * (r + 1) // P
        buf = okm.DeviceBuffer(max(1, (r1 - r0) * stride))
        okm.synth_reads_device(buf.address, r1 - r0, READ_LEN, genome_len=C3_GENOME_BP, genome_seed=C3_SEED,
                               seed=C3_SEED, first_read=r0, sub_rate=0.001, n_rate=0.0001)
        spans = [(b0 * stride, (min(r1 - r0, b0 + C3_BATCH_READS) - b0) * stride)
                 for b0 in range(0, r1 - r0, C3_BATCH_READS)]
        shards.append((buf, spans, (r1 - r0) * READ_LEN))
    log(f"C3 shards for {P} ranks generated on the device ({time.time() - t0:.1f}s)")
    ref, t_one = None, None
    if not args.no_ref:  # the one-GPU table of the same reads, shard after shard (second of two runs)
        c = okm.KmerCounter(k)
        for _ in range(2):
            c.reset()
            t = time.perf_counter()
            for buf, spans, _ in shards:
                for off, nb in spans:
                    c.add_device_batch(buf.address + off, nb)
            n1 = c.count()
            c.synchronize()
            t_one = time.perf_counter() - t
        kp, cp, _ = c.result_device()
        ref = _table_digest(kp, cp, n1, 0)
        c.close()
        log(f"one-GPU reference: {n1} distinct keys, {t_one * 1e3:.1f} ms")
    comms = okm.Comm.init_loopback(P, 0)
    ctrs = [okm.KmerCounter(k) for _ in range(P)]
    lock, gate = threading.Lock(), threading.Barrier(P)
    res, err = [None] * P, []

    def body(r):
        try:
            buf, spans, bases = shards[r]
            for rnd in range(2):  # round 0 warms the pools (first allocations), round 1 is timed
                with lock:  # one rank's count at a time: each has the card to itself
                    ctrs[r].reset()
                    t = time.perf_counter()
                    for off, nb in spans:
                        ctrs[r].add_device_batch(buf.address + off, nb)
                    n_local = ctrs[r].count()
                    ctrs[r].synchronize()
                    tc = time.perf_counter() - t
                    info = ctrs[r].engine_info()
                    ctrs[r].trim()
                gate.wait()
                t = time.perf_counter()
                n_own = comms[r].merge_owned(ctrs[r], ctrs[r])
                ctrs[r].synchronize()
                tm = time.perf_counter() - t
                gate.wait()
            res[r] = {"n_local": n_local, "n_own": n_own, "count_ms": tc * 1e3, "merge_wall_ms": tm * 1e3,
                      "phases": comms[r].last_times(), "bytes": comms[r].last_bytes(), "bases": bases,
                      "folds": int(info.get("folds", 0))}
        except BaseException as e:  # surfaced below
            err.append(e)
            gate.abort()

    th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(P)]
    for t_ in th:
        t_.start()
    for t_ in th:
        t_.join()
    if err:
        raise err[0]
    for buf, _, _ in shards:
        buf.free()
    got, pos = [0, 0, 0, 0], 0
    for r in range(P):
        kp, cp, _ = ctrs[r].result_device()
        d = _table_digest(kp, cp, res[r]["n_own"], pos)
        got = [a + b for a, b in zip(got, d)]
        pos += res[r]["n_own"]
    m64 = (1 << 64) - 1
    got = [got[0], got[1], got[2] & m64, got[3] & m64]
    exact = None if ref is None else got == [ref[0], ref[1], ref[2] & m64, ref[3] & m64]
    for c in ctrs:
        c.close()
    for c in comms:
        c.close()
    count_max = max(o["count_ms"] for o in res)
    sent = sum(o["bytes"][0] for o in res)
    return {"metric": f"C3 over {P} loopback ranks on one MI355X: per-rank one-card count time, owner-merged "
                      f"table exact vs the one-GPU table",
            "value": round(total * READ_LEN / (count_max * 1e-3), 1), "unit": "bases/s (all bases / slowest rank count)",
            "n_gpus": 1, "ranks": P, "steps": 1, "warmup": 0, "higher_is_better": True, "dtype": "u64",
            "data": "synthetic (C3 reads generated on the device)",
            "config": {"workload": f"BASELINE configs[2] (C3) shape sharded 1/{P}: {total} reads x {READ_LEN} bp from a "
                                   f"1 Gbp genome" + ("" if total == C3_READS else f" ({total / C3_READS:.3g} of C3's reads)"), "k": k, "exchange": "okm_merge_owned over a loopback communicator",
                       "one_gpu_ms": None if t_one is None else round(t_one * 1e3, 1),
                       "distinct_global": pos, "exact_vs_one_gpu": exact,
                       "bytes_sent_all_ranks": sent,
                       "wire_bytes_per_pair": round(sent / max(1, sum(o["n_local"] for o in res)), 3)},
            "ranks_detail": [{k_: (round(v, 2) if isinstance(v, float) else v) for k_, v in o.items()} for o in res]}


def wl_classify(args):
    k = 31
    batch = c2_batch()
    dbuf = okm.DeviceBuffer(len(batch))
    dbuf.upload(batch)
    c = okm.KmerCounter(k, "count")
    c.add_device_batch(dbuf.address, len(batch))
    c.count()
    # 32 references: the k-mers of 32 disjoint slices of the reads' own set
    keys, _ = c.result(1)
    rng = np.random.default_rng(5)
    perm = keys[rng.permutation(len(keys))]
    refs = np.array_split(perm, 32)
    cl = okm.Classifier(c, 2)
    packed = okm.Classifier.pack_db(refs)
    # host keys (okm_classifier_probe_db: pinned staging pieces + DMA, as the
    # CLI's database arrives) and device-resident keys (the probe alone)
    dt = timed(lambda: cl.probe_db(packed=packed), args.steps, args.warmup)
    dk = okm.DeviceBuffer(packed[0].nbytes)
    dk.upload(packed[0])
    dt_dev = timed(lambda: cl.probe_db(packed=(None, packed[1]), d_keys=dk.address), args.steps, args.warmup)
    r = cl.probe_db(packed=packed)
    rd = cl.probe_db(packed=(None, packed[1]), d_keys=dk.address)
    assert (r["union"], r["matched"]) == (rd["union"], rd["matched"])
    nkeys = len(keys)
    return {"metric": "reference k-mers/sec probed (classify.rs per-reference stats, k=31) on one MI355X",
            "value": round(nkeys / dt, 1), "unit": "kmers/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "u64",
            "data": "synthetic (BASELINE configs[1] reads, device-resident counts)",
            "config": {"workload": "classify: 32 references (~110 M keys from host memory) vs the counted "
                                   "table of 3,355,443 x 150 bp reads, --min-kmer-frequency 2",
                       "k": k, "db_keys": nkeys, "input_kmers_after_filter": cl.n_input,
                       "union": r["union"], "matched": r["matched"]},
            "note": "per step: host->device copy of the keys (880 MB, pinned staging) + one probe/insert kernel",
            "device_keys": {"value": round(nkeys / dt_dev, 1), "unit": "kmers/s", "ms_per_step": round(dt_dev * 1e3, 3),
                            "note": "okm_classifier_probe_db_device: the database keys resident in HBM"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["query", "build", "wide", "classify", "c5", "c3"], required=True)
    ap.add_argument("--no-ref", action="store_true", help="c3: skip the one-GPU reference table")
    ap.add_argument("--c3-reads", type=int, default=C3_READS,
                    help="c3: total reads (BASELINE configs[2]: 167,772,160; P local tables of the full size do not "
                         "fit one GPU beyond P = 2)")
    ap.add_argument("--c5-cap", type=float, default=256e6, help="c5: base cap per sample (SURVEY: 256 Mbases)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gbases", type=float, default=1.0)
    ap.add_argument("--cpu-sample-reads", type=int, default=100_000)
    ap.add_argument("--loopback", type=int, default=0,
                    help="c5: P virtual ranks on one GPU through okm_comm_init_loopback (the distributed compare)")
    ap.add_argument("--knob", action="append", default=[],
                    help="NAME=VALUE: an engine test knob for the run (okm.testing; A/B of rare paths)")
    args = ap.parse_args()
    if args.knob:
        from okm import testing
        for kv in args.knob:
            name, val = kv.split("=", 1)
            testing.set_knob(name, int(val))
    c5 = wl_c5_dist if int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.loopback else wl_c5
    out = {"query": wl_query, "build": wl_build, "wide": wl_wide, "classify": wl_classify,
           "c5": c5, "c3": wl_c3_loop}[args.workload](args)
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
