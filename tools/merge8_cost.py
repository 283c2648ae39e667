"""What an owner's merge costs at P=8 on C3 (BASELINE configs[2]), measured
on one GPU: eight contexts each count one P=8 shard (20,971,520 reads of the
1 Gbp genome, seed 3, the shards bench.py gives ranks 0..7), and one owner
context merges the first 1/8 of the key space of all eight tables — the
slices rank 0 would receive from the eight ranks (its own included) — through
okm_add_sorted_pairs_device + okm_count (the k-way LDS merge of okm_merge.hip).
Prints one JSON line: pairs in, distinct out, merge ms (median of reps).
usage: python tools/merge8_cost.py [reps]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-kmer_amd")]
import numpy as np  # noqa: E402

import okm  # noqa: E402

K, READS, P, LEN = 31, 167_772_160, 8, 150
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
merge_counts = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [P]  # slices merged per run
per = READS // P
buf = okm.DeviceBuffer(per * (LEN + 1))
ctxs = []
for r in range(P):
    okm.synth_reads_device(buf.address, per, LEN, genome_len=1_000_000_000, genome_seed=3, seed=3,
                           first_read=r * per, sub_rate=0.001, n_rate=0.0001)
    c = okm.KmerCounter(K)
    step = 4_194_304 * (LEN + 1)
    for off in range(0, per * (LEN + 1), step):
        c.add_device_batch(buf.address + off, min(step, per * (LEN + 1) - off))
    n = c.count()
    # keep only the table (the context's L1 runs and working set go)
    dk, dc = okm.DeviceBuffer(8 * n), okm.DeviceBuffer(8 * n)
    c.fetch_into_device(dk.address, dc.address, n)
    c.close()
    ctxs.append((dk, dc, n))
buf.free()
# rank 0's key range: the first 1/8 of its table's keys (okm_merge_owned cuts
# by the summed histogram; the shards cover the same genome, so alike)
lib = okm._lib.load()
k0, _, n0 = ctxs[0]
probe = np.empty(1, np.uint64)
okm._lib.check(lib.okm_memcpy_d2h(probe.ctypes.data, k0.address + 8 * (n0 // P), 8), "d2h")
cut = probe[0]
slices = []
for dk, dc, n in ctxs:
    keys = np.empty(n, np.uint64)
    okm._lib.check(lib.okm_memcpy_d2h(keys.ctypes.data, dk.address, 8 * n), "d2h")
    m = int(np.searchsorted(keys, cut))
    slices.append((dk.address, dc.address, m))
owner = okm.KmerCounter(K)
for R in merge_counts:
    times = []
    nd = 0
    for _ in range(reps + 1):
        owner.reset()
        t0 = time.perf_counter()
        for kp, cp, m in slices[:R]:
            owner.add_sorted_pairs_device(kp, cp, m)
        nd = owner.count()
        owner.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
    owner.set_timing(True)  # one more rep for the per-kernel split
    owner.reset()
    for kp, cp, m in slices[:R]:
        owner.add_sorted_pairs_device(kp, cp, m)
    owner.count()
    kstats = {k: round(v["total_ms"], 2) for k, v in owner.kernel_stats().items()}
    owner.set_timing(False)
    pairs = sum(s[2] for s in slices[:R])
    print(json.dumps({"what": f"owner merge of {R} of the 8 slices rank 0 receives at P=8 (C3)", "runs": R,
                      "pairs_in": pairs, "distinct_out": nd, "merge_ms": round(statistics.median(times[1:]), 2),
                      "all_ms": [round(t, 2) for t in times[1:]], "kernels_ms": kstats}))
