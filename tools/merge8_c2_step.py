"""The N>1 C2 step's owner merge at P = 8, on one GPU.

bench.py at --gpus 8 gives every rank its own configs[1] batch (3,355,443
reads of the 100 Mbp genome, seed 2, reads [r * 3355443, (r+1) * 3355443))
and merges the eight tables by key-range owner.  This tool measures, on one
GPU:

* ``owner0``: what ONE rank's owner does after the exchange -- the weighted
  count of the eight sorted slices of its key range (rank 0's range: the
  first 1/8 of the keys), through okm_add_sorted_pairs_device + okm_count,
  i.e. the part of the step a real 8-GPU rank runs alone on its GPU;
* ``loopback8``: the whole okm_merge_owned (histogram, owner split, pack,
  exchange, unpack, owner counts) of all eight virtual ranks at once over the
  loopback transport -- eight ranks' work on ONE device, so its wall time is
  an upper bound of eight times what one GPU does per step.

Prints one JSON line.  usage: python tools/merge8_c2_step.py [reps]"""
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-kmer_amd")]
import numpy as np  # noqa: E402

import okm  # noqa: E402

K, P, LEN, PER = 31, 8, 150, 3_355_443
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
stride = LEN + 1
bufs = []
for r in range(P):
    b = okm.DeviceBuffer(PER * stride)
    okm.synth_reads_device(b.address, PER, LEN, genome_len=100_000_000, genome_seed=2, seed=2, first_read=r * PER,
                           sub_rate=0.001, n_rate=0.0001)
    bufs.append(b)
lib = okm._lib.load()
out = {"what": "N>1 C2 step owner merge at P=8 on one GPU (bench.py --gpus 8 shapes)"}

# owner0: the eight slices of rank 0's key range, counted by one owner context
tabs = []
for r in range(P):
    with okm.KmerCounter(K) as c:
        c.add_device_batch(bufs[r].address, PER * stride)
        n = c.count()
        dk, dc = okm.DeviceBuffer(8 * n), okm.DeviceBuffer(8 * n)
        c.fetch_into_device(dk.address, dc.address, n)
    tabs.append((dk, dc, n))
k0, _, n0 = tabs[0]
probe = np.empty(1, np.uint64)
okm._lib.check(lib.okm_memcpy_d2h(probe.ctypes.data, k0.address + 8 * (n0 // P), 8), "d2h")
cut = probe[0]
slices = []
for dk, dc, n in tabs:
    keys = np.empty(n, np.uint64)
    okm._lib.check(lib.okm_memcpy_d2h(keys.ctypes.data, dk.address, 8 * n), "d2h")
    slices.append((dk.address, dc.address, int(np.searchsorted(keys, cut))))
owner = okm.KmerCounter(K)
times, nd = [], 0
for rep in range(reps + 1):
    owner.reset()
    t0 = time.perf_counter()
    for kp, cp, m in slices:
        owner.add_sorted_pairs_device(kp, cp, m)
    nd = owner.count()
    owner.synchronize()
    times.append((time.perf_counter() - t0) * 1e3)
owner.set_timing(True)
owner.reset()
for kp, cp, m in slices:
    owner.add_sorted_pairs_device(kp, cp, m)
owner.count()
kst = {k: round(v["total_ms"], 3) for k, v in owner.kernel_stats().items()}
owner.close()
out["owner0"] = {"slices": P, "pairs_in": sum(s[2] for s in slices), "distinct_out": nd,
                 "merge_ms": round(statistics.median(times[1:]), 3), "all_ms": [round(t, 3) for t in times[1:]],
                 "kernels_ms": kst}
for dk, dc, _ in tabs:
    dk.free()
    dc.free()

# loopback8: the whole collective of eight virtual ranks on this one device
comms = okm.Comm.init_loopback(P, 0)
locs = [okm.KmerCounter(K) for _ in range(P)]
owns = [okm.KmerCounter(K) for _ in range(P)]
walls, per_rank = [], []
for rep in range(reps + 1):
    for r in range(P):
        locs[r].reset()
        locs[r].add_device_batch(bufs[r].address, PER * stride)
        locs[r].count()
        locs[r].synchronize()
    res, errs = [None] * P, []

    def body(r):
        try:
            res[r] = comms[r].merge_owned(locs[r], owns[r])
        except BaseException as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    walls.append((time.perf_counter() - t0) * 1e3)
    if errs:
        raise errs[0]
    per_rank.append([round(comms[r].last_times()["merge_ms"], 3) for r in range(P)])
out["loopback8"] = {"owned_distinct": res, "distinct_total": int(sum(res)),
                    "wall_ms_all_8_ranks_one_gpu": round(statistics.median(walls[1:]), 3),
                    "all_wall_ms": [round(w, 3) for w in walls[1:]],
                    "merge_ms_per_rank_last": per_rank[-1]}
for c in locs + owns:
    c.close()
for c in comms:
    c.close()
for b in bufs:
    b.free()
print(json.dumps(out))
