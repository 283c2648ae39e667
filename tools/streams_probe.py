#!/usr/bin/env python3
"""Probe: C2 steps on S engine contexts (S HIP streams) driven by S host
threads, vs one context.  Prints ms per step for each S (whole-job time / K).
The contexts share the read-only device batch; each counts into its own table."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-kmer_amd"))
import okm  # noqa: E402

K, READS, RL = 31, 3_355_443, 150
batch = okm.synth_reads(READS, RL, genome_len=100_000_000, genome_seed=2, seed=2, sub_rate=0.001, n_rate=0.0001)
buf = okm.DeviceBuffer(len(batch))
buf.upload(batch)
steps = int(os.environ.get("STEPS", "12"))
ctxs = [okm.KmerCounter(K, "count") for _ in range(4)]


def run(S):
    nxt = [0]
    lock = threading.Lock()
    res = []

    def worker(c):
        while True:
            with lock:
                if nxt[0] >= steps:
                    return
                nxt[0] += 1
            c.reset()
            c.add_device_batch(buf.address, len(batch))
            res.append(c.count())

    for c in ctxs[:S]:  # warmup
        c.reset()
        c.add_device_batch(buf.address, len(batch))
        c.count()
    t = time.perf_counter()
    th = [threading.Thread(target=worker, args=(c,)) for c in ctxs[:S]]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t
    assert len(set(res)) == 1, res
    return dt / steps * 1e3, res[0]


for S in (1, 2, 3, 1, 2):
    ms, n = run(S)
    print(f"S={S} {ms:.3f} ms/step distinct={n} -> {READS * RL / ms / 1e6:.1f} Gbases/s", flush=True)
