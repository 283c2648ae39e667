#!/bin/bash
# Interleaved A/B of library builds (box-to-box and run-to-run clocks drift):
# tools/ab_interleave.sh REPS name1 name2 ...  (build_<name>/liborion_kmer.so; "main" = build/)
# One C2 bench per (rep, build), round-robin; medians per build at the end.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abi
reps=$1; shift
for r in $(seq 1 "$reps"); do
  for n in "$@"; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-sample-reads 0 --cpu-mt-reads 0 --c3-steps 0 \
      > gpurun_out/abi/${n}_$r.json 2> gpurun_out/abi/${n}_$r.err || exit 1
  done
done
python3 - "$@" <<'PY'
import glob, json, statistics, sys
for n in sys.argv[1:]:
    runs = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/abi/{n}_*.json"))]
    ks = runs[0]["kernels"].keys()
    med = {k: round(statistics.median(r["kernels"][k]["avg_ms"] for r in runs), 4) for k in ks}
    print(n, "step", round(statistics.median(r["ms_per_step"] for r in runs), 3),
          [round(r["ms_per_step"], 3) for r in runs], med)
PY
