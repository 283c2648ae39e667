#!/bin/bash
# SQ counters of the k=63 path (1 Gbases): is the wide extraction scatter VALU-bound?
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/wsq
B="python tools/bench_paths.py --workload wide --gbases 1 --steps 1 --warmup 0 --cpu-sample-reads 0"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
  -d gpurun_out/wsq/p -o p -f csv -- $B > gpurun_out/wsq/p.log 2>&1 || { tail -5 gpurun_out/wsq/p.log; exit 1; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/wsq/p/p_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); nd = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); nd[k].add(r["Dispatch_Id"])
for k in sorted(agg, key=lambda k: -agg[k]["SQ_WAVE_CYCLES"])[:6]:
    print(k, len(nd[k]), {c: int(v) for c, v in sorted(agg[k].items())})
PY
