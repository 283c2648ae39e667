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
                     clipped 200..100k, 5 % substitutions); --gbases sets the
                     size (configs[3] is ~5.36 Gbases).
  --workload c5      BASELINE configs[4] shape: build.rs per-sample sets of 64
                     WGS-shaped synthetic samples (tools/c5_runs.json) into two
                     databases, then compare.rs (unions, |A ∩ B|, Jaccard).
                     Under torchrun (WORLD_SIZE > 1) the samples shard over the
                     ranks and the unions are owner-partitioned (wl_c5_dist).
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
                   "reads_with_hits": int((hits > 0).sum()), "hits": int(hits.sum(dtype=np.uint64))},
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
    """ONT-like reads: lognormal lengths, 5 % substitutions."""
    rng = np.random.default_rng(seed)
    target = int(gbases * 1e9)
    genome = rng.integers(0, 4, size=min(target // 4 + 200_000, 1_000_000_000), dtype=np.uint8)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    lens = []
    tot = 0
    while tot < target:
        L = rng.lognormal(np.log(2891.0), 1.085, size=65536).clip(200, 100_000).astype(np.int64)
        lens.append(L)
        tot += int(L.sum())
    lens = np.concatenate(lens)
    lens = lens[:np.searchsorted(np.cumsum(lens), target) + 1]
    n = len(lens)
    starts = rng.integers(0, len(genome) - 100_001, size=n)
    out = np.empty(int(lens.sum()) + n, np.uint8)
    o = 0
    for i in range(n):
        L = int(lens[i])
        r = genome[starts[i]:starts[i] + L].copy()
        m = rng.random(L) < 0.05
        r[m] = rng.integers(0, 4, size=int(m.sum()), dtype=np.uint8)
        out[o:o + L] = acgt[r]
        out[o + L] = ord("\n")
        o += L + 1
    return out, n


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
                                   "lengths (median 2891, sigma 1.085, 200..100k), 5 % substitutions",
                       "k": k, "reads": n, "bases": bases, "kmers": int(info["kmers"]),
                       "distinct": int(info["distinct"])},
            "kernels": kern, "engine": info}


def c5_samples(cap_bases: float, which=None):
    """64 synthetic samples shaped by 64 WGS runs of
    data_metagenome.json.gz (tools/c5_runs.json: mean read length, base count
    capped at cap_bases), each drawn from 3 of a pool of 48 seeded genomes
    (2-8 Mbp); samples 0-31 (DB1) use genomes 0-35, samples 32-63 (DB2)
    genomes 12-47, so the two halves share half of their genomes."""
    runs = json.load(open(os.path.join(ROOT, "tools", "c5_runs.json")))["runs"]
    glen = [2_000_000 + g * 6_000_000 // 47 for g in range(48)]
    out = []
    for s_, r in enumerate(runs):
        if which is not None and s_ not in which:
            continue
        rng = np.random.default_rng(5_000 + s_)
        lo = 0 if s_ < 32 else 12
        gs = rng.choice(np.arange(lo, lo + 36), size=3, replace=False)
        L = int(min(max(r["mean_read_len"], 100), 30_000))
        bases = int(min(r["base_count"], cap_bases))
        parts = []
        for j, g in enumerate(gs):
            nr = max(1, bases // 3 // L)
            parts.append(okm.synth_reads(nr, L, genome_len=glen[g], genome_seed=9_000 + int(g),
                                         seed=s_ * 16 + j, sub_rate=0.001, n_rate=0.0001))
        out.append(np.concatenate(parts))
    return out


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


def wl_c5_dist(args):
    """C5 over WORLD_SIZE ranks, one GPU each (SURVEY.md §8(e) "C5"): the 64
    samples are dealt round-robin (sample s -> rank s mod N), every rank builds
    its samples' sets (build.rs:46-116) and unions its share of each DB's
    references; okm.dist.distributed_compare then moves both unions to
    value-range owners under one set of bounds, each owner unions and
    intersects its ranges on its GPU and one all_reduce sums |A|, |B|, |A ∩ B|
    (compare.rs:51-66).  Strong scaling: the 64-sample workload is fixed."""
    import torch
    import torch.distributed as tdist
    from okm import dist as okm_dist
    k = 31
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    backend = os.environ.get("OKM_BENCH_BACKEND", "nccl")
    if backend == "nccl":
        tdist.init_process_group("nccl", device_id=torch.device("cuda", device))
    else:
        tdist.init_process_group(backend)
    mine = list(range(rank, 64, world))
    t = time.time()
    samples = dict(zip(mine, c5_samples(args.c5_cap, set(mine))))
    my_bases = sum(int(len(b)) - int((b == 10).sum()) for b in samples.values())
    log(f"[rank {rank}] C5: {len(mine)} samples, {my_bases / 1e9:.2f} Gbases ({time.time() - t:.1f}s)")
    dev = {}
    for s_, b in samples.items():
        d = okm.DeviceBuffer(len(b), device)
        d.upload(b)
        dev[s_] = (d, len(b))
    sample_ctx = okm.KmerCounter(k, "set", device)
    locals_ = [okm.KmerCounter(k, "set", device), okm.KmerCounter(k, "set", device)]
    owners = [okm.KmerCounter(k, "set", device), okm.KmerCounter(k, "set", device)]
    tot = 0
    for d, n in dev.values():
        sample_ctx.reset()
        sample_ctx.add_device_batch(d.address, n)
        tot += sample_ctx.count()
    store = okm.DeviceBuffer(max(8, 8 * tot), device)

    def as_tensor(ptr, n):
        if n == 0:
            return torch.empty(0, dtype=torch.int64, device="cuda")
        t_ = torch.as_tensor(okm_dist.DeviceView(ptr, n), device="cuda")
        return t_ if backend == "nccl" else t_.cpu()

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
        tabs = []
        for h in (0, 1):
            u = locals_[h]
            u.reset()
            for s_, (o, m) in sizes.items():
                if (s_ < 32) == (h == 0) and m:
                    u.add_sorted_pairs_device(store.address + 8 * o, 0, m)
            n = u.count()
            tabs.append(as_tensor(u.result_device()[0], n))
        torch.cuda.synchronize()
        which = [0]

        def union(rk, rs):
            o_ = owners[which[0]]
            which[0] += 1
            if backend != "nccl":
                rk = rk.cuda()
            o_.reset()
            pos = 0
            for sz in rs:
                if sz:
                    o_.add_sorted_pairs_device(rk.data_ptr() + 8 * pos, 0, sz)
                pos += sz
            n = o_.count()
            keep.append(rk)  # borrowed until count(); kept alive for the step
            return n, o_.result_device()[0]

        def intersect(ha, na, hb, nb):
            return okm.set_intersection_size_device(ha, na, hb, nb, device) if na and nb else 0

        keep = []
        return okm_dist.distributed_compare(tabs[0], tabs[1], k, union, intersect)

    def barrier_sync():
        torch.cuda.synchronize()
        tdist.barrier()

    for _ in range(args.warmup):
        step()
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    barrier_sync()
    dt = (time.perf_counter() - t0) / args.steps
    tt = torch.tensor([dt, float(my_bases), float(tot)], dtype=torch.float64,
                      device="cuda" if backend == "nccl" else "cpu")
    mx = tt.clone()
    tdist.all_reduce(mx, op=tdist.ReduceOp.MAX)
    tdist.all_reduce(tt, op=tdist.ReduceOp.SUM)
    dt = float(mx[0])
    bases, set_total = int(tt[1]), int(tt[2])
    na, nb, inter = res
    union_ = na + nb - inter
    tdist.destroy_process_group()
    if rank != 0:
        return None
    return {"metric": f"bases/sec built into per-sample k-mer sets + compared (k=31, build.rs + compare.rs) "
                      f"on {world} MI355X",
            "value": round(bases / dt, 1), "unit": "bases/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "dtype": "u64",
            "data": "synthetic (64 samples shaped by tools/c5_runs.json, device-resident)",
            "config": {"workload": f"BASELINE configs[4] shape over {world} ranks: 64 WGS-shaped samples "
                                   f"(<= {args.c5_cap / 1e6:.0f} Mbases each) dealt round-robin, DB1 = samples "
                                   f"0-31, DB2 = 32-63, unions owner-partitioned ({backend})",
                       "k": k, "bases": bases, "set_sizes_total": set_total,
                       "db1_total_unique_kmers_across_references": na,
                       "db2_total_unique_kmers_across_references": nb, "intersection_size": inter,
                       "union_size": union_, "jaccard_index": inter / union_ if union_ else 0.0}}


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
    ap.add_argument("--workload", choices=["query", "build", "wide", "classify", "c5"], required=True)
    ap.add_argument("--c5-cap", type=float, default=256e6, help="c5: base cap per sample (SURVEY: 256 Mbases)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gbases", type=float, default=1.0)
    ap.add_argument("--cpu-sample-reads", type=int, default=100_000)
    args = ap.parse_args()
    c5 = wl_c5_dist if int(os.environ.get("WORLD_SIZE", "1")) > 1 else wl_c5
    out = {"query": wl_query, "build": wl_build, "wide": wl_wide, "classify": wl_classify,
           "c5": c5}[args.workload](args)
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
