#!/usr/bin/env python3
"""Benchmark: bases/s k-mer-counted (k=31) on MI355X — BASELINE.json `metric`.

One step = one pass of the hot path over one batch of synthetic input with
the batch already resident in HBM: extraction + canonicalisation + key-range
partitioning + LDS counting + sorted (key, count) table on the device
(count.rs:23-38 + :106-119), and for N>1 the owner-partitioned RCCL merge of
the per-GPU tables inside the library (okm_merge_owned).

Workload (configs[1]): k=31, 1 GiB synthetic FASTQ of 150 bp reads =
3,355,443 reads = 503,316,450 bases per GPU, sampled from a seeded 100 Mbp
random genome (0.1 % substitutions, 0.01 % N).  With
--gpus N every rank counts its own 3,355,443 reads of the same genome (weak
scaling) and the tables are merged.

Batches in flight (--streams, default 3): at N=1 three engine contexts, each
with its own HIP stream and table, count whole batches concurrently from three
host threads (one batch's host syncs and latency-bound count phase overlap the
others' streaming kernels; measured 2 / 3 / 4 in flight: 5.81-6.02 /
5.70-5.74 / 5.73-5.90 ms per batch, tools/ab_streams.sh); at N>1 (--workload
c2) one thread counts batch i+1 into two contexts in turn while the main thread
runs okm_merge_owned on batch i (the library's RCCL stream) into one of two
merge contexts.  Every step still counts one full batch into its own sorted
table.  The line's `value` is this configs[1] workload at every N (weak
scaling: the driver's per-N values compare like for like).

After it, the same invocation measures BASELINE configs[2] (C3: 25.17 Gbases
from a 1 Gbp genome, sharded 1/N over the ranks, strong scaling, c3_run) and
reports it in the same line as `c3` (`--c3-steps 0` skips it; `--workload c3`
makes C3 the line's `value`).

Prints ONE JSON line on rank 0 (the driver's contract), including `roofline`
for the dominant kernel (HIP events on the engine's own stream, from a
single-stream pass of the same K steps after the timed region) and
`cpu_baseline` (the oracle, oracle/okm_oracle.c, on a bounded sample, rank 0
at N=1 only).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "orion-kmer_amd"))


def _launch_ranks_if_asked():
    """`python3 bench.py --gpus N` with no WORLD_SIZE in the environment runs
    N rank processes itself (okm.launch: device count probed in a child, so
    this process makes no HIP call before it starts them; rank 0's line is
    relayed; any failing rank fails the run), or exits 2 when fewer devices
    are visible than ranks asked for.  Under torch.distributed.run (WORLD_SIZE
    set) this is a no-op."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args()
    from okm.launch import launch_or_none
    rc = launch_or_none(a.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:])
    if rc is not None:
        sys.exit(rc)


if __name__ == "__main__":
    _launch_ranks_if_asked()

import numpy as np  # noqa: E402

import okm  # noqa: E402
from okm import _lib  # noqa: E402
from okm.pipeline import OwnedCountPipeline, agree_or_raise, comm_audit  # noqa: E402

# Load the engine (and the HIP runtime it links) before torch, so the process
# has exactly one HIP runtime.
_lib.load()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "bases/sec k-mer-counted (k=31) at 1/2/4/8 MI355X; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
K = 31
READS_PER_GPU = 3_355_443
READ_LEN = 150
GENOME_BP = 100_000_000
GENOME_SEED = 2
READ_SEED = 2
# BASELINE configs[2] (C3): 50 GiB of 150 bp FASTQ = 167,772,160
# reads = 25,165,824,000 bases from a 1 Gbp genome, seed 3, contiguous 1/P shards
C3_READS = 167_772_160
C3_GENOME_BP = 1_000_000_000
C3_SEED = 3
C3_BATCH_READS = 4_194_304  # 0.63 Gbases per okm_add_batch_device call


def pmc_traffic():
    """Newest committed rocprofv3 PMC traffic summary (tools/profile_round.sh):
    HBM bytes per launch per kernel, read = 2 x FETCH_SIZE (gfx950), + WRITE_SIZE."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as fh:
        return json.load(fh).get("kernels", {}), os.path.relpath(files[-1], ROOT)


def roofline_from_stats(stats, bases_timed):
    """`roofline` for the dominant kernel (by device time) of a timing pass:
    its algorithmic bytes per launch / its average HIP-event duration on the
    engine stream, vs the 8 TB/s HBM peak; `traffic` from the newest committed
    rocprofv3 PMC summary.  bases_timed: bases the timing pass covered."""
    roof = None
    kernels = {}
    if not stats:
        return roof, kernels
    for name, s in stats.items():
        if s["launches"]:
            avg = s["total_ms"] / s["launches"]
            per = s["alg_bytes"] / s["launches"]
            kernels[name] = {"launches": s["launches"], "avg_ms": round(avg, 4),
                             "alg_bytes_per_launch": per,
                             "achieved_GBs": round(per / (avg * 1e-3) / 1e9, 1) if avg > 0 else None}
    dom = max(kernels, key=lambda n: stats[n]["total_ms"])
    dk = kernels[dom]
    ach = dk["achieved_GBs"]
    traffic, tsrc = pmc_traffic()
    tk = (traffic or {}).get(dom)
    roof = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
            "traffic": round(tk["traffic_bytes"]) if tk else None,
            "traffic_unit": "bytes per launch (HBM, rocprofv3 PMC)",
            "traffic_source": tsrc if tk else None,
            "avg_ms": dk["avg_ms"], "alg_bytes_per_launch": dk["alg_bytes_per_launch"],
            "measured": "HIP events on the engine stream, single-stream pass of the same K steps after the "
                        "timed region"}
    if tk:
        roof["traffic_GBs"] = round(tk["traffic_bytes"] / (dk["avg_ms"] * 1e-3) / 1e9, 1)
    tot_ms = sum(s["total_ms"] for s in stats.values())
    tot_bytes = sum(s["alg_bytes"] for s in stats.values())
    roof["path_achieved_GBs"] = round(tot_bytes / (tot_ms * 1e-3) / 1e9, 1) if tot_ms > 0 else None
    roof["path_alg_bytes_per_base"] = round(tot_bytes / bases_timed, 2)
    return roof, kernels


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# stdout carries exactly ONE JSON line (the driver's contract): whatever
# libraries print there (RCCL's version banner, gloo's peer count) goes to
# stderr; emit() writes the line to the saved stdout
_STDOUT_FD = os.dup(1)
os.dup2(2, 1)


def emit(out):
    sys.stdout.flush()
    os.write(_STDOUT_FD, (json.dumps(out) + "\n").encode())


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=READS_PER_GPU, help="reads per GPU")
    ap.add_argument("--cpu-sample-reads", type=int, default=300_000,
                    help="reads in the bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-mt-reads", type=int, default=800_000,
                    help="reads of the labelled restatement-MT CPU sample (0: skip)")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP-event timing")
    ap.add_argument("--streams", type=int, default=3,
                    help="N=1: batches in flight (engine contexts / HIP streams, one host thread each)")
    ap.add_argument("--dist-workers", type=int, default=2,
                    help="N>1: threads counting the next batches (each into its own context) while the "
                         "exchange + merge of the current one runs")
    ap.add_argument("--workload", choices=["c2", "c3"], default="c2",
                    help="c2: BASELINE configs[1] (1 GiB per GPU, weak scaling; default); c3: BASELINE configs[2] "
                         "(50 GiB of reads from a 1 Gbp genome sharded 1/N over the ranks) as the line's value")
    ap.add_argument("--c3-steps", type=int, default=2,
                    help="c2 workload: timed steps of the C3 (configs[2]) measurement reported as `c3` "
                         "in the same line (0: skip it)")
    ap.add_argument("--c3-warmup", type=int, default=1, help="c2 workload: untimed C3 steps before those")
    ap.add_argument("--c3-reads", type=int, default=C3_READS,
                    help="c3: total reads over all ranks (BASELINE configs[2]: 167,772,160)")
    ap.add_argument("--c3-genome-bp", type=int, default=C3_GENOME_BP,
                    help="c3: genome size (BASELINE configs[2]: 1 Gbp; smaller values for A/B runs)")
    ap.add_argument("--batch-reads", type=int, default=C3_BATCH_READS,
                    help="c3: reads per okm_add_batch_device call")
    return ap.parse_args()


def init_comm(world, rank, device):
    """The library's own RCCL communicator (okm_comm: okm_merge_owned's HIP
    owner split / pack / unpack kernels + grouped ncclSend/ncclRecv over
    xGMI).  torch.distributed (gloo, host) only hands out its unique id and
    carries the barriers and the max-time reduce."""
    dist.init_process_group("gloo")
    uid = torch.zeros(okm._lib.OKM_COMM_ID_BYTES, dtype=torch.uint8)
    if rank == 0:
        uid = torch.frombuffer(bytearray(okm.comm_unique_id()), dtype=torch.uint8)
    dist.broadcast(uid, 0)
    return okm.Comm(world, rank, bytes(uid.numpy().tobytes()), device)


def rank_device(args):
    """(world, rank, device) of this process: one rank per GPU, LOCAL_RANK's
    device.  A --gpus that disagrees with WORLD_SIZE, or a rank without a
    device of its own, is an error (RCCL refuses two ranks on one GPU, and a
    line must never report GPUs it did not use)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU, "
                         f"or run `python3 bench.py --gpus N` without WORLD_SIZE)")
    ndev = okm.device_count()
    if local >= ndev:
        raise SystemExit(f"bench.py: {world} ranks, {ndev} device{'' if ndev == 1 else 's'} visible: "
                         f"LOCAL_RANK {local} has no GPU of its own")
    torch.cuda.set_device(local)
    return world, rank, local


def main():
    args = parse()
    if args.workload == "c3":
        return main_c3(args)
    world, rank, device = rank_device(args)
    # OKM_BENCH_EXCHANGE=1 runs the N>1 exchange + merge path at world size 1
    # too (torchrun --nproc-per-node 1): its cost on one GPU, RCCL self-send
    dist_on = world > 1 or os.environ.get("OKM_BENCH_EXCHANGE") == "1"
    comm = init_comm(world, rank, device) if dist_on else None

    # ---- synthetic batch for this rank, made resident in HBM ---------------
    t0 = time.time()
    first = rank * args.reads
    batch = okm.synth_reads(args.reads, READ_LEN, genome_len=GENOME_BP, genome_seed=GENOME_SEED, seed=READ_SEED,
                            first_read=first, sub_rate=0.001, n_rate=0.0001)
    bases = args.reads * READ_LEN
    dbuf = okm.DeviceBuffer(len(batch), device)
    dbuf.upload(batch)
    log(f"[rank {rank}] synthetic batch: {args.reads} reads, {bases} bases, {len(batch)} bytes "
        f"({time.time() - t0:.1f}s)")

    # Batches in flight: at N=1, S contexts (each its own HIP stream and result
    # table) driven by S host threads count whole batches concurrently, so one
    # batch's host syncs and latency-bound phases overlap another's streaming
    # kernels.  At N>1 (okm.pipeline.OwnedCountPipeline) --dist-workers threads
    # count the next batches into their own contexts while this thread runs the
    # step's failure agreement and okm_merge_owned of batch i (RCCL on the
    # library's own stream) into one of two owner contexts.
    S = max(1, args.streams)

    def count_batch(c, dense=False):
        c.reset()
        c.add_device_batch(dbuf.address, len(batch))
        n = c.count()
        if dense:  # the dense (keys, counts) arrays gathered too (okm_result_device)
            c.result_device()
        return n

    pipe = None
    if dist_on:
        pipe = OwnedCountPipeline(comm, lambda: okm.KmerCounter(K, "count", device),
                                  lambda c, i: c.add_device_batch(dbuf.address, len(batch)),
                                  workers=max(1, args.dist_workers))
        ctrs, mergers = list(pipe.local), list(pipe.owners)
    else:
        ctrs, mergers = [okm.KmerCounter(K, "count", device) for _ in range(S)], []
    ctr = ctrs[0]

    def run_steps(nsteps, dense=False):
        """nsteps batches through the path; returns the distinct count (N=1)
        or this rank's owned distinct count of the last merge (N>1)."""
        import threading
        if dist_on:
            res = pipe.run(nsteps)
            return res[-1] if res else 0
        if S == 1:
            n = 0
            for _ in range(nsteps):
                n = count_batch(ctr, dense)
            return n
        nxt, lock, res, err = [0], threading.Lock(), [], []

        def worker(c):
            try:
                while True:
                    with lock:
                        if nxt[0] >= nsteps:
                            return
                        nxt[0] += 1
                    res.append(count_batch(c, dense))
            except BaseException as e:  # surfaced below
                err.append(e)

        th = [threading.Thread(target=worker, args=(c,), daemon=True) for c in ctrs]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if err:
            raise err[0]
        return res[-1] if res else 0

    def barrier_sync():
        torch.cuda.synchronize()
        for c in ctrs:
            c.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()

    for c in ctrs:  # every context warmed (pool sized) before the timed region
        count_batch(c)
    run_steps(args.warmup)
    barrier_sync()
    if pipe is not None:
        pipe.phase_ms.update(exchange=0.0, merge=0.0)
    t_start = time.perf_counter()
    n_owned = run_steps(args.steps)
    barrier_sync()
    dt = time.perf_counter() - t_start
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # The step ends with the sorted table as per-item runs (the dense arrays
    # are gathered by their first reader).  The same K steps again, each also
    # gathering the dense (keys, counts) arrays: the conservative rate, for a
    # caller that wants the flat table every batch.
    dense_ms = None
    if not dist_on:
        barrier_sync()
        t2 = time.perf_counter()
        run_steps(args.steps, dense=True)
        barrier_sync()
        dense_ms = (time.perf_counter() - t2) / args.steps * 1e3
    # one job alone (one context, one stream, one host thread): the latency of
    # a single batch, beside the throughput of S batches in flight above
    single_ms = None
    if not dist_on and S > 1:
        barrier_sync()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            count_batch(ctr)
        ctr.synchronize()
        single_ms = (time.perf_counter() - t1) / args.steps * 1e3
    # per-kernel HIP-event timing: a separate single-stream pass of the same K
    # steps (kernels of the timed region overlap across streams, so their
    # durations there would not be any one kernel's)
    # The count leaves the sorted table as per-item runs (okm_engine.hip
    # Pending); the dense (keys, counts) arrays are gathered by their first
    # reader.  One step of this pass also asks for them (okm_result_device),
    # so `kernels` carries that gather's cost (compact_items) beside the
    # count's kernels.
    stats = {}
    if not args.no_timing:
        ctr.set_timing(True)
        for i in range(args.steps):
            count_batch(ctr)
            if i == 0:
                ctr.result_device()
        stats = ctr.kernel_stats()
        ctr.set_timing(False)
    info = ctr.engine_info()

    # ---- CPU baseline: the oracle on a bounded sample (rank 0, N=1) -------
    # plus SURVEY §8(d)'s labelled multi-threaded restatement beside it
    cpu = cpu_mt = None
    if rank == 0 and world == 1 and args.cpu_sample_reads > 0:
        cpu, cpu_mt = cpu_baselines(batch, min(args.cpu_sample_reads, args.reads),
                                    min(args.cpu_mt_reads, args.reads), device, "the same batch")

    # BASELINE configs[2] (C3) in the same invocation, every rank (its merge is
    # collective): the C2 contexts go first so the C3 shard has the device
    c3 = None
    if args.c3_steps > 0:
        for c in ctrs + mergers:
            c.close()
        dbuf.free()
        torch.cuda.empty_cache()
        try:
            c3 = c3_run(args, world, rank, device, comm, dist_on, args.c3_steps, args.c3_warmup, baselines=False)
        except Exception as e:  # reported in the line; the configs[1] measurement above stands
            log(f"[rank {rank}] C3 measurement failed: {e!r}")
            c3 = {"error": repr(e)}

    # what ran at N>1: every rank's communicator (size, RCCL's own rank count,
    # device PCI bus id), gathered over gloo; collective, so before the rank split
    audit = None
    if dist_on:
        infos = [None] * world
        dist.all_gather_object(infos, comm.info())
        audit = comm_audit(infos, world)

    if rank != 0:
        if comm is not None:
            comm.close()
        if dist_on:
            dist.destroy_process_group()
        return

    value = world * bases * args.steps / dt
    roof, kernels = roofline_from_stats(stats, bases * args.steps)
    # SURVEY §8(d) whole-path roofline: 1 B/base + 16 B per k-mer instance
    kmers = info["kmers"]
    surv_bytes = bases + 16.0 * kmers
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "bases/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1000, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded reads from a random genome, device-resident)",
        "config": {"workload": "BASELINE configs[1]: k=31, 1 GiB synthetic 150 bp FASTQ per GPU "
                               f"({args.reads} reads, {bases} bases), single MI355X; N>1: same shard "
                               "per GPU + RCCL owner-partitioned table merge",
                   "k": K, "reads_per_gpu": args.reads, "read_len": READ_LEN, "genome_bp": GENOME_BP,
                   "distinct_kmers": int(info["distinct"]) if world == 1 else None,
                   "kmer_instances_per_gpu": int(kmers), "parallelism": f"reads sharded x{world}",
                   "table": "a step ends with the sorted (key, count) table on the device as per-item runs; the "
                            "dense arrays are gathered by their first reader (okm_result_device / fetch / merge): "
                            "`kernels.compact_items`, timed once in the per-kernel pass",
                   "batches_in_flight": len(pipe.local) if dist_on else S},
        "roofline": roof,
        "cpu_baseline": cpu,
        "cpu_baseline_mt": cpu_mt,
        "survey_roofline": {"alg_bytes_per_step_per_gpu": surv_bytes,
                            "achieved_GBs_per_gpu": round(surv_bytes * args.steps / dt / 1e9, 1),
                            "frac_of_8TBs": round(surv_bytes * args.steps / dt / 8e12, 4),
                            "input_stream_frac": round(bases * args.steps / dt / 8e12, 5)},
        "single_job": ({"ms_per_step": round(single_ms, 3), "value": round(bases / (single_ms * 1e-3), 1),
                        "note": "one context, one stream, one host thread: a batch's latency; `value` above "
                                f"is {S} batches in flight"} if single_ms else None),
        "with_dense_table": ({"ms_per_step": round(dense_ms, 3), "value": round(bases / (dense_ms * 1e-3), 1),
                              "note": "the same K steps, each also gathering the flat (keys, u64 counts) arrays "
                                      "(okm_result_device -> k_compact_items) inside the timed region"}
                             if dense_ms else None),
        "kernels": kernels,
        "engine": info,
    }
    if dist_on:
        out["comm"] = audit
        out["config"]["owned_distinct_rank0"] = int(n_owned)
        out["exchange_ms_per_step_rank0"] = {"exchange": round(pipe.phase_ms["exchange"] / args.steps, 3),
                                             "merge": round(pipe.phase_ms["merge"] / args.steps, 3)}
        out["exchange_impl"] = "okm_merge_owned (library RCCL communicator, HIP pack/unpack, owner count of sorted slices)"
    if c3 is not None:
        out["c3"] = ({k: c3[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                         "scaling", "config", "exchange_impl", "phase_ms_per_step_rank0",
                                         "survey_roofline", "memory")}
                     if "value" in c3 else c3)
    emit(out)
    if comm is not None:
        comm.close()
    if dist_on:
        dist.destroy_process_group()
    if args.c3_steps <= 0:
        dbuf.free()


def main_c3(args):
    """BASELINE configs[2] (C3): 167,772,160 reads (25,165,824,000 bases) of a
    1 Gbp genome, split into contiguous 1/P shards by read index, one shard
    per rank, generated on the device (okm_synth_reads_device, the same bytes
    as the host generator).  One step = the whole job: every rank counts its
    shard batch by batch into ONE table (count.rs:52-89: one map across all
    inputs; the engine folds its uncounted batches into a sorted table when
    they pass 8 % of HBM into sorted tables merged k-way, so memory grows with distinct keys), then at N>1
    the tables merge by key-range owner over RCCL.  Strong scaling: the total
    work is fixed, `value` = all ranks' bases / the slowest rank's time."""
    world, rank, device = rank_device(args)
    dist_on = world > 1 or os.environ.get("OKM_BENCH_EXCHANGE") == "1"
    comm = init_comm(world, rank, device) if dist_on else None
    out = c3_run(args, world, rank, device, comm, dist_on, args.steps, args.warmup, baselines=True)
    if out is not None:
        emit(out)
    if comm is not None:
        comm.close()
    if dist_on:
        dist.destroy_process_group()


def c3_run(args, world, rank, device, comm, dist_on, steps, warmup, baselines):
    """Time `steps` whole C3 jobs (after `warmup` untimed ones) on every rank
    and return rank 0's line (None on the other ranks).  Every rank must call
    it (the merge is collective); it releases its contexts and shard buffer."""
    total = args.c3_reads
    r0, r1 = total * rank // world, total * (rank + 1) // world
    nreads = r1 - r0
    stride = READ_LEN + 1
    t0 = time.time()
    dbuf = ctr = merger = None
    setup_err = None
    try:
        dbuf = okm.DeviceBuffer(max(1, nreads * stride), device)
        okm.synth_reads_device(dbuf.address, nreads, READ_LEN, genome_len=args.c3_genome_bp, genome_seed=C3_SEED,
                               seed=C3_SEED, first_read=r0, sub_rate=0.001, n_rate=0.0001, device=device)
        ctr = okm.KmerCounter(K, "count", device)
        # the owner's merge reuses the counting context (okm_merge_owned allows
        # owner == local): one device pool per rank, no cross-context trimming
        merger = ctr if dist_on else None
    except Exception as e:
        setup_err = e
    if dist_on:  # every rank learns whether all could set up, before any collective of the merge
        bad = torch.tensor([0 if setup_err is None else 1], dtype=torch.int64)
        dist.all_reduce(bad, op=dist.ReduceOp.SUM)
        if int(bad.item()) and setup_err is None:
            setup_err = RuntimeError(f"C3 setup failed on {int(bad.item())} rank(s)")
    if setup_err is not None:
        if ctr is not None:
            ctr.close()
        if dbuf is not None:
            dbuf.free()
        raise setup_err
    batches = []
    for b0 in range(0, nreads, args.batch_reads):
        b1 = min(nreads, b0 + args.batch_reads)
        batches.append((b0 * stride, (b1 - b0) * stride))
    log(f"[rank {rank}] C3 shard: reads [{r0}, {r1}) = {nreads * READ_LEN} bases in {len(batches)} batches, "
        f"generated on the device ({time.time() - t0:.1f}s)")

    xt = [0.0, 0.0, 0.0]  # count, exchange, merge (wall, this rank)

    def step():
        tc = time.perf_counter()
        err = None
        try:
            ctr.reset()
            for off, nb in batches:
                ctr.add_device_batch(dbuf.address + off, nb)
            n = ctr.count()
        except Exception as e:
            if comm is None:
                raise
            err = e
        xt[0] += time.perf_counter() - tc
        if comm is None:
            return n
        # every rank learns whether any count failed, and then all stop here
        # together (okm.pipeline.agree_or_raise) instead of merging alone
        agree_or_raise(comm, err)
        n_m = comm.merge_owned(ctr, merger)
        t = comm.last_times()
        xt[1] += (t["plan_ms"] + t["exchange_ms"]) * 1e-3
        xt[2] += t["merge_ms"] * 1e-3
        return n_m

    def barrier_sync():
        torch.cuda.synchronize()
        ctr.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(max(1, warmup)):
        step()
    barrier_sync()
    xt[:] = [0.0, 0.0, 0.0]
    t_start = time.perf_counter()
    n_last = 0
    for _ in range(steps):
        n_last = step()
    barrier_sync()
    dt = time.perf_counter() - t_start
    info = ctr.engine_info()
    distinct_global = n_last
    if dist_on:
        dev_t = "cpu"
        t = torch.tensor([dt], dtype=torch.float64, device=dev_t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        nd = torch.tensor([n_last], dtype=torch.int64, device=dev_t)
        dist.all_reduce(nd, op=dist.ReduceOp.SUM)  # owners' ranges partition the global table
        distinct_global = int(nd.item())
    # per-kernel HIP-event timing of the local count: one more step, single stream
    stats = {}
    if not args.no_timing:
        ctr.set_timing(True)
        ctr.reset()
        for off, nb in batches:
            ctr.add_device_batch(dbuf.address + off, nb)
        ctr.count()
        stats = ctr.kernel_stats()
        ctr.set_timing(False)

    cpu = cpu_mt = None
    if baselines and rank == 0 and world == 1 and args.cpu_sample_reads > 0:
        m = min(args.cpu_sample_reads, nreads)
        mm = min(max(m, args.cpu_mt_reads), nreads)
        host = np.empty(mm * stride, dtype=np.uint8)
        dbuf.download(host)
        cpu, cpu_mt = cpu_baselines(host, m, min(args.cpu_mt_reads, nreads), device, "the C3 shard")

    audit = None
    if comm is not None:  # collective: every rank's communicator, gathered over gloo
        infos = [None] * world
        dist.all_gather_object(infos, comm.info())
        audit = comm_audit(infos, world)
    ctr.close()
    dbuf.free()
    if rank != 0:
        return None
    shard_bases = nreads * READ_LEN
    all_bases = total * READ_LEN
    value = all_bases * steps / dt
    roof, kernels = roofline_from_stats(stats, shard_bases)
    kmers = info["kmers"]
    surv_bytes = shard_bases + 16.0 * kmers
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "bases/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(dt / steps * 1000, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded reads from a random 1 Gbp genome, generated on the device, resident in HBM)",
        "config": {"workload": f"BASELINE configs[2] (C3): k=31, {total} reads x {READ_LEN} bp = {all_bases} bases "
                               f"(50 GiB as FASTQ) from a 1 Gbp genome (seed 3), contiguous 1/{world} shard per "
                               f"GPU counted into one table"
                               + (", tables merged by key-range owner over RCCL" if dist_on else ""),
                   "k": K, "reads_total": total, "reads_per_gpu_rank0": nreads, "read_len": READ_LEN,
                   "genome_bp": args.c3_genome_bp, "batches_per_gpu": len(batches), "batch_reads": args.batch_reads,
                   "distinct_kmers": distinct_global, "kmer_instances_rank0": int(kmers),
                   "folds_rank0": int(info.get("folds", 0)), "groups_rank0": int(info.get("groups", 0)),
                   "parallelism": f"reads sharded x{world}"},
        "roofline": roof,
        "cpu_baseline": cpu,
        "cpu_baseline_mt": cpu_mt,
        "survey_roofline": {"alg_bytes_per_step_per_gpu": surv_bytes,
                            "achieved_GBs_per_gpu": round(surv_bytes * steps / dt / 1e9, 1),
                            "frac_of_8TBs": round(surv_bytes * steps / dt / 8e12, 4),
                            "input_stream_frac": round(shard_bases * steps / dt / 8e12, 5)},
        "exchange_impl": ("okm_merge_owned (library RCCL communicator, HIP pack/unpack, owner count of sorted slices)"
                          if comm is not None else None),
        "phase_ms_per_step_rank0": {"count": round(xt[0] / steps * 1e3, 2),
                                    "exchange": round(xt[1] / steps * 1e3, 2),
                                    "merge": round(xt[2] / steps * 1e3, 2)},
        "kernels": kernels,
        "engine": info,
        "comm": audit,
        # rank 0's device memory: what its arena mapped at the end of the timed
        # jobs (device_bytes, idle cached chunks included) and the most it held
        # in use at once (device_peak_bytes); the result itself is 16 B / key
        "memory": {"device_bytes": int(info["device_bytes"]), "device_peak_bytes": int(info["device_peak_bytes"]),
                   "host_bytes": int(info["host_bytes"]), "spills": int(info["spills"]),
                   "result_bytes": int(n_last) * 16},
    }
    return out



def cpu_baselines(host, m, m_mt, device, what):
    """`cpu_baseline` (the C restatement, one thread: count.rs is
    single-threaded) on the first m reads of `host` and the labelled
    restatement-MT sample on the first m_mt reads, checked equal to the
    engine's table of the same sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleCounter, count_separated_mt
    stride = READ_LEN + 1
    sample = host[:m * stride]
    oc = OracleCounter(K)
    tc = time.perf_counter()
    oc.add_separated(sample)
    oc.result(1)
    tcpu = time.perf_counter() - tc
    cpu = {"value": m * READ_LEN / tcpu, "unit": "bases/s", "cores": 1, "kind": "port",
           "sample": f"first {m} reads ({m * READ_LEN} bases) of {what}, k=31, oracle/okm_oracle.c (faithful "
                     f"O(k) encode+rc per window, 1 thread, count.rs is single-threaded), {tcpu:.1f} s incl. "
                     f"filter+sort",
           "note": "the port's open-addressing mix64 map is cheaper than the reference's DashMap + SipHash-1-3 + "
                   "shard locks (count.rs:31-34), so this likely overstates the reference's own speed"}
    cpu_mt = None
    if m_mt > 0:
        nproc = os.cpu_count() or 1
        try:
            avail = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            avail = nproc
        # the GPU box grants one GPU's job 16 host threads (OMP_NUM_THREADS=16);
        # nproc / os.cpu_count() report the whole node's CPUs there
        thr = max(1, min(int(os.environ.get("OMP_NUM_THREADS") or avail), avail))
        sample = host[:m_mt * stride]
        tc = time.perf_counter()
        mk, mc = count_separated_mt(sample, K, thr)
        tmt = time.perf_counter() - tc
        with okm.KmerCounter(K, "count", device) as chk:
            sb = okm.DeviceBuffer(len(sample), device)
            sb.upload(sample)
            chk.add_device_batch(sb.address, len(sample))
            gk, gc = chk.result(1)
            sb.free()
        cpu_mt = {"value": m_mt * READ_LEN / tmt, "unit": "bases/s", "threads": thr, "nproc": nproc,
                  "affinity_cpus": avail,
                  "threads_note": "OMP_NUM_THREADS: the host-thread share the GPU box grants one GPU's job "
                                  "(nproc counts the whole node)",
                  "kind": "restatement-MT (not reference behaviour: count.rs is single-threaded)",
                  "sample": f"first {m_mt} reads ({m_mt * READ_LEN} bases) of {what}, k=31, {thr} shards "
                            f"counted by oracle/okm_oracle.c on {thr} threads + key-range merge, {tmt:.1f} s",
                  "engine_table_equal": bool(np.array_equal(mk, gk) and np.array_equal(mc, gc))}
    return cpu, cpu_mt


if __name__ == "__main__":
    main()
