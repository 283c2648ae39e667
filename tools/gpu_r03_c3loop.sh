#!/bin/bash
# C3 over loopback ranks on one GPU: exactness of the owner-merged table vs the
# one-GPU table, per-rank one-card count times, exchange bytes (P = 2, 4, 8).
mkdir -p gpurun_out
for P in "$@"; do
  timeout -k 10 400 python tools/bench_paths.py --workload c3 --loopback $P ${C3_READS:+--c3-reads $C3_READS} \
      > gpurun_out/r03_c3loop_$P.json 2> gpurun_out/r03_c3loop_$P.err || { tail -5 gpurun_out/r03_c3loop_$P.err; exit 1; }
  python - $P <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r03_c3loop_{sys.argv[1]}.json"))
c = d["config"]
print("P", d["ranks"], "exact", c["exact_vs_one_gpu"], "one_gpu_ms", c["one_gpu_ms"], "distinct", c["distinct_global"],
      "B/pair", c["wire_bytes_per_pair"], "value", d["value"] / 1e9)
for r in d["ranks_detail"]:
    print("   count %.1f ms merge %.1f ms folds %d local %d own %d" % (r["count_ms"], r["merge_wall_ms"], r["folds"], r["n_local"], r["n_own"]), r["phases"])
PY
done
