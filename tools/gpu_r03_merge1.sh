#!/bin/bash
# C3 on one GPU: fold-table merges as one staged count + compaction
# (OKM_NO_MERGE_KERNEL) against the exact two-pass count.
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 \
      > gpurun_out/r03_m1_$tag.json 2> gpurun_out/r03_m1_$tag.err || { tail -3 gpurun_out/r03_m1_$tag.err; return 1; }
  python - $tag <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r03_m1_{sys.argv[1]}.json"))
print(sys.argv[1], d["ms_per_step"], "folds", d["config"]["folds_rank0"], "groups", d["config"]["groups_rank0"], "GB", d["engine"]["device_bytes"] / 1e9)
for n, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["launches"])[:9]:
    print("   %-16s %4d x %8.3f = %7.1f ms" % (n, v["launches"], v["avg_ms"], v["avg_ms"] * v["launches"]))
PY
}
run base OKM_X=0 && run staged OKM_NO_MERGE_KERNEL=1 && run staged12 OKM_NO_MERGE_KERNEL=1 OKM_FOLD_BYTES=$(python -c "print(int(0.12 * 309220868096))")
