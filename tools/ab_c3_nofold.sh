#!/bin/bash
# C3 at P=1 (bench.py --workload c3): default fold threshold against folding
# deferred (OKM_FOLD_BYTES large: every batch stays an L1 run and okm_count
# takes the grouped path once).  One process per setting.
mkdir -p gpurun_out
for fb in default 150000000000 170000000000; do
  if [ "$fb" = default ]; then unset OKM_FOLD_BYTES; else export OKM_FOLD_BYTES=$fb; fi
  echo "== OKM_FOLD_BYTES=$fb"
  timeout -k 10 240 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 --no-timing \
      > gpurun_out/r03_c3_fold_$fb.json 2> gpurun_out/r03_c3_fold_$fb.err
  rc=$?
  python - "$fb" <<'PY'
import json, sys
try:
    d = json.load(open(f"gpurun_out/r03_c3_fold_{sys.argv[1]}.json"))
    print(d["ms_per_step"], d["value"] / 1e9, d["config"]["folds_rank0"], d["config"]["groups_rank0"],
          d["config"]["distinct_kmers"], d["engine"]["device_bytes"] / 1e9)
except Exception as e:
    print("no result", e)
PY
  tail -3 gpurun_out/r03_c3_fold_$fb.err
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "rc=$rc: stopping"; exit $rc; fi
done
