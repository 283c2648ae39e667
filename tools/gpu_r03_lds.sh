#!/bin/bash
# LDS / instruction-mix SQ counters of the C2 kernels (one bench step, single stream): where the
# extraction, partition and count kernels spend LDS time (bank conflicts, LDS waits)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/lds
B="python bench.py --steps 1 --warmup 0 --cpu-sample-reads 0 --no-timing --streams 1 --c3-steps 0"
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/lds/avail.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" gpurun_out/lds/avail.txt | sort -u > gpurun_out/lds/sq_names.txt
want=""
for c in SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT; do
  grep -qx "$c" gpurun_out/lds/sq_names.txt && want="$want $c"
done
echo "counters:$want"
timeout -s KILL 120 rocprofv3 --pmc $want -d gpurun_out/lds/p -o p -f csv -- $B > gpurun_out/lds/p.log 2>&1 || { tail -5 gpurun_out/lds/p.log; exit 1; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/lds/p/p_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    for key in ("Counter_Name",):
        agg[k][r[key]] += float(r["Counter_Value"])
for k in sorted(agg):
    if any(x in k for x in ("extract_scatter", "part_scatter", "count_items", "compact_items")):
        print(k, {c: int(v) for c, v in sorted(agg[k].items())})
PY
