#!/bin/bash
# Interleaved A/B of library builds on one P=8 C3 shard (20,971,520 reads of
# the 1 Gbp genome, 5 batches into one table) at one rank:
# tools/ab_c3.sh REPS name1 name2 ...  ("main" = build/, else build_<name>/)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abc3
reps=$1; shift
for r in $(seq 1 "$reps"); do
  for n in "$@"; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 300 python bench.py --workload c3 --c3-reads 20971520 --steps 3 --warmup 1 \
      --cpu-sample-reads 0 > gpurun_out/abc3/${n}_$r.json 2> gpurun_out/abc3/${n}_$r.err || exit 1
  done
done
python3 - "$@" <<'PY'
import glob, json, statistics, sys
for n in sys.argv[1:]:
    runs = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/abc3/{n}_*.json"))]
    ks = runs[0]["kernels"].keys()
    med = {k: round(statistics.median(r["kernels"][k]["avg_ms"] * r["kernels"][k]["launches"] for r in runs), 2) for k in ks}
    print(n, "step", round(statistics.median(r["ms_per_step"] for r in runs), 2),
          [round(r["ms_per_step"], 2) for r in runs], "kernel ms per step:", med)
PY
