#!/bin/bash
# C3 fold policy A/B: tables merged every OKM_FOLD_MERGE_RUNS folds (default 4).
mkdir -p gpurun_out
for reads in 167772160 83886080; do
for mr in 4 6 8 3; do
  export OKM_FOLD_MERGE_RUNS=$mr
  timeout -k 10 240 python bench.py --workload c3 --c3-reads $reads --steps 2 --warmup 1 --cpu-sample-reads 0 --no-timing \
      > gpurun_out/r03_ab_mr_${reads}_$mr.json 2> gpurun_out/r03_ab_mr_${reads}_$mr.err
  rc=$?
  python - $reads $mr <<'PY'
import json, sys
try:
    d = json.load(open(f"gpurun_out/r03_ab_mr_{sys.argv[1]}_{sys.argv[2]}.json"))
    print(sys.argv[1], "merge_runs", sys.argv[2], "ms", d["ms_per_step"], "folds", d["config"]["folds_rank0"],
          "device GB", round(d["engine"]["device_bytes"] / 1e9, 1), "distinct", d["config"]["distinct_kmers"])
except Exception as e:
    print(sys.argv[1], sys.argv[2], "no result")
PY
  [ $rc -eq 0 ] || tail -2 gpurun_out/r03_ab_mr_${reads}_$mr.err
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
done
