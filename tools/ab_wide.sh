#!/bin/bash
# Interleaved A/B of library builds on the k=63 ONT-like workload
# (tools/bench_paths.py --workload wide): tools/ab_wide.sh REPS GBASES name1 name2 ...
# ("main" = build/, else build_<name>/).  Per-kernel averages per build.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abw
reps=$1; gb=$2; shift 2
for r in $(seq 1 "$reps"); do
  for n in "$@"; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 300 python tools/bench_paths.py --workload wide --gbases "$gb" --steps 3 --warmup 1 \
      --cpu-sample-reads 0 > gpurun_out/abw/${n}_$r.json 2> gpurun_out/abw/${n}_$r.err || exit 1
  done
done
python3 - "$@" <<'PY'
import glob, json, statistics, sys
for n in sys.argv[1:]:
    runs = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/abw/{n}_*.json"))]
    ks = runs[0]["kernels"].keys()
    med = {k: round(statistics.median(r["kernels"][k]["avg_ms"] for r in runs), 3) for k in ks}
    print(n, "step", round(statistics.median(r["ms_per_step"] for r in runs), 2),
          [round(r["ms_per_step"], 2) for r in runs], med)
PY
