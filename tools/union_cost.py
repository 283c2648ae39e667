"""Set-mode union of R sorted runs (compare.rs:51-66's get_all_kmers_unified,
the C5 databases) through the count kernel (default) and the k-way merge
kernel (--merge-kernel: the test knob sorted_path = 1): one JSON line per R.
usage: python tools/union_cost.py [R,...] [keys per run]"""
import json
import os
import statistics
import sys
import time

MERGE_KERNEL = "--merge-kernel" in sys.argv
if MERGE_KERNEL:
    sys.argv.remove("--merge-kernel")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-kmer_amd")]
import numpy as np  # noqa: E402

import okm  # noqa: E402

Rs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2, 8, 32]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8_000_000
rng = np.random.default_rng(1)
shared = rng.integers(0, 1 << 62, n, dtype=np.uint64)  # genomes shared between samples: half of every run
bufs = []
for r in range(max(Rs)):
    keys = np.unique(np.concatenate([shared[rng.integers(0, n, n // 2)],
                                     rng.integers(0, 1 << 62, n // 2, dtype=np.uint64)]))
    b = okm.DeviceBuffer(keys.nbytes)
    b.upload(keys)
    bufs.append((b, len(keys)))
with okm.KmerCounter(31, "set") as u:
    for R in Rs:
        times = []
        for _ in range(4):
            u.reset()
            t0 = time.perf_counter()
            for b, m in bufs[:R]:
                u.add_sorted_pairs_device(b.address, None, m)
            nd = u.count()
            u.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"runs": R, "keys_in": sum(m for _, m in bufs[:R]), "union": nd,
                          "merge_kernel": MERGE_KERNEL,
                          "ms": round(statistics.median(times[1:]), 2)}))
