#!/bin/bash
# Interleaved A/B of environment settings on one build (box-to-box and
# process-to-process clocks drift): tools/ab_env.sh REPS "NAME=ENV ..." ...
# e.g. tools/ab_env.sh 3 "f8=OKM_FOLD_BYTES=23000000000" "default=" ; one C2 bench per
# (rep, setting), round-robin; medians per setting at the end.  Extra bench.py
# arguments in AB_BENCH_ARGS.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abe
reps=$1; shift
names=()
for r in $(seq 1 "$reps"); do
  for spec in "$@"; do
    n=${spec%%=*}; envs=${spec#*=}
    [ "$r" = 1 ] && names+=("$n")
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample-reads 0 --cpu-mt-reads 0 \
      ${AB_BENCH_ARGS:---c3-steps 0} > gpurun_out/abe/${n}_$r.json 2> gpurun_out/abe/${n}_$r.err || exit 1
  done
done
python3 - "${names[@]}" <<'PY'
import glob, json, statistics, sys
for n in sys.argv[1:]:
    runs = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/abe/{n}_*.json"))]
    ks = runs[0]["kernels"].keys()
    med = {k: round(statistics.median(r["kernels"][k]["avg_ms"] for r in runs), 4) for k in ks}
    c3 = [r["c3"]["ms_per_step"] for r in runs if isinstance(r.get("c3"), dict) and "ms_per_step" in r["c3"]]
    print(n, "step", round(statistics.median(r["ms_per_step"] for r in runs), 3),
          [round(r["ms_per_step"], 3) for r in runs], "c3", c3, med)
PY
