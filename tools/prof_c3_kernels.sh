#!/bin/bash
# Where the C3 count's time goes: per-kernel HIP-event totals of one step of
# bench.py --workload c3 at P=1 (whole job) and at a P=2 shard's size.
mkdir -p gpurun_out
for reads in 167772160 83886080; do
  timeout -k 10 300 python bench.py --workload c3 --c3-reads $reads --steps 1 --warmup 1 --cpu-sample-reads 0 \
      > gpurun_out/r03_c3prof_$reads.json 2> gpurun_out/r03_c3prof_$reads.err || exit $?
  python - $reads <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r03_c3prof_{sys.argv[1]}.json"))
print(sys.argv[1], "ms", d["ms_per_step"], "folds", d["config"]["folds_rank0"], "groups", d["config"]["groups_rank0"])
ks = sorted(d["kernels"].items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["launches"])
tot = sum(v["avg_ms"] * v["launches"] for _, v in ks)
print(" kernel total %.1f ms" % tot)
for n, v in ks:
    print("  %-16s %5d x %8.3f = %8.2f ms  %s GB/s" % (n, v["launches"], v["avg_ms"], v["avg_ms"] * v["launches"], v["achieved_GBs"]))
PY
done
