#!/bin/bash
# One parametrised script for the GPU box (run through gpurun from the repo
# root).  Every GPU step runs under its own time limit and the steps are
# chained with &&, so the first failure ends the lease; scratch output goes to
# gpurun_out/<task>/ and only what is judged is copied into profiles/.
#
#   tools/gpu_lease.sh suite [pytest -k expr]   GPU parity suite (-m gpu), one process
#   tools/gpu_lease.sh smoke                    __graft_entry__.smoke()
#   tools/gpu_lease.sh bench [bench.py args]    one bench line -> gpurun_out/bench/line.json
#   tools/gpu_lease.sh exchange [args]          bench.py's N>1 path at world 1 (torchrun, RCCL self-send)
#   tools/gpu_lease.sh profile <round>          kernel trace + stats + PMC traffic (tools/profile_round.sh)
#   tools/gpu_lease.sh lds <round>              LDS / SQ counters of the C2 kernels -> gpurun_out/lds/<round>_lds_counters.json
#   tools/gpu_lease.sh sq <round>               SQ wait / issue counters -> gpurun_out/sq/<round>_sq_stalls.json
# (only gpurun_out/ comes back from the box: copy what is judged into profiles/)
#   tools/gpu_lease.sh paths <workload> [args]  tools/bench_paths.py --workload <workload>
#   tools/gpu_lease.sh ab <reps> <builds...>    interleaved A/B of in-tree builds (tools/ab_interleave.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TASK=${1:?task}
shift
OUT=gpurun_out/$TASK
mkdir -p "$OUT"
PY="python -u"
C2="bench.py --steps 1 --warmup 0 --cpu-sample-reads 0 --cpu-mt-reads 0 --no-timing --streams 1 --c3-steps 0"

# rocprofv3 SQ counters of the C2 kernels, one --pmc pass per counter group
# (at most 8 SQ counters a pass), summed per kernel into a JSON file
sq_pass() {  # <outdir> <counters...>
    local d=$1
    shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$d" -o p -f csv -- python $C2 > "$d.log" 2>&1
}
sq_sum() {  # <json out> <csv...>
    local out=$1
    shift
    python3 - "$out" "$@" <<'PY'
import csv, collections, json, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
keep = ("extract_scatter", "part_scatter", "count_items", "compact_items", "count_direct")
ks = [k for k in sorted(agg) if any(x in k for x in keep)]
out = {k: {c: int(v) for c, v in sorted(agg[k].items())} for k in ks}
# the bench command counts a warm-up batch and the step: the sums cover every
# dispatch of the kernel; `per_dispatch` divides by their number
per = {k: {c: int(v / max(len(disp[k]), 1)) for c, v in sorted(agg[k].items())} for k in ks}
json.dump({"sum_over_all_dispatches": out, "dispatches": {k: len(disp[k]) for k in ks}, "per_dispatch": per},
          open(sys.argv[1], "w"), indent=1)
print(json.dumps(per, indent=1))
PY
}

case "$TASK" in
suite)
    K=()
    [ -n "$1" ] && K=(-k "$1")
    timeout -k 10 1500 $PY -m pytest tests -m gpu -x -v --durations=30 --timeout 300 --timeout-method thread "${K[@]}" \
        > "$OUT/suite.log" 2>&1
    rc=$?
    tail -30 "$OUT/suite.log"
    exit $rc
    ;;
smoke)
    timeout -k 10 300 $PY -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee "$OUT/smoke.log"
    ;;
bench)
    timeout -k 10 600 $PY bench.py "$@" > "$OUT/line.json" 2> "$OUT/bench.log"
    rc=$?
    tail -5 "$OUT/bench.log"
    cat "$OUT/line.json"
    exit $rc
    ;;
exchange)
    OKM_BENCH_EXCHANGE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 "$@" > "$OUT/line.json" 2> "$OUT/bench.log"
    rc=$?
    tail -5 "$OUT/bench.log"
    cat "$OUT/line.json"
    exit $rc
    ;;
profile)
    R=${1:?round}
    bash tools/profile_round.sh "$R"
    ;;
lds)
    R=${1:?round}
    sq_pass "$OUT/a" SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU \
        SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES &&
    sq_sum "$OUT/${R}_lds_counters.json" "$OUT/a/p_counter_collection.csv"  # copy into profiles/ after the call
    ;;
sq)
    R=${1:?round}
    sq_pass "$OUT/a" SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
        SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS &&
    sq_sum "$OUT/${R}_sq_stalls.json" "$OUT/a/p_counter_collection.csv"  # copy into profiles/ after the call
    ;;
paths)
    W=${1:?workload}
    shift
    timeout -k 10 900 $PY tools/bench_paths.py --workload "$W" "$@" > "$OUT/$W.json" 2> "$OUT/$W.log"
    rc=$?
    tail -5 "$OUT/$W.log"
    cat "$OUT/$W.json"
    exit $rc
    ;;
ab)
    bash tools/ab_interleave.sh "$@"
    ;;
*)
    echo "unknown task $TASK" >&2
    exit 2
    ;;
esac
