#!/bin/bash
# Interleaved A/B of library builds on the full C3 workload at one rank
# (bench.py --workload c3 defaults): tools/ab_c3_full.sh REPS name1 name2 ...
# ("main" = build/, else build_<name>/).  Step ms and kernel ms per step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/abc3f
reps=$1; shift
for r in $(seq 1 "$reps"); do
  for n in "$@"; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 \
      --cpu-mt-reads 0 > gpurun_out/abc3f/${n}_$r.json 2> gpurun_out/abc3f/${n}_$r.err || { echo "$n failed"; tail -5 gpurun_out/abc3f/${n}_$r.err; exit 1; }
    echo "$n rep $r done"
  done
done
python3 - "$@" <<'PY'
import glob, json, statistics, sys
for n in sys.argv[1:]:
    runs = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"gpurun_out/abc3f/{n}_*.json"))]
    ks = runs[0].get("kernels", {}).keys()
    med = {k: round(statistics.median(r["kernels"][k]["avg_ms"] * r["kernels"][k]["launches"] for r in runs), 1)
           for k in ks}
    print(n, "step", round(statistics.median(r["ms_per_step"] for r in runs), 1),
          [round(r["ms_per_step"], 1) for r in runs], "kernel ms per step:", med)
PY
