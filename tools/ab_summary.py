"""Summarise tools/ab_bench.sh outputs: ms/step and per-kernel averages per build."""
import json
import sys

for n in sys.argv[1:]:
    d = json.loads(open(f"gpurun_out/ab/{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], {k: round(v["avg_ms"], 3) for k, v in d["kernels"].items()})
