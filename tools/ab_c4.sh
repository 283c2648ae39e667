#!/bin/bash
# Interleaved C4 A/B (k = 63, 5.36 Gbases, tools/bench_paths.py --workload wide):
#   tools/ab_c4.sh REPS name1 name2 ...  ("main" = build/, else build_<name>/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c4ab
reps=$1; shift
for r in $(seq 1 "$reps"); do
  for n in "$@"; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 2 --warmup 1 > gpurun_out/c4ab/${n}_$r.json 2> gpurun_out/c4ab/${n}_$r.log || { echo "$n failed"; tail -5 gpurun_out/c4ab/${n}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/c4ab/${n}_$r.json'));print('$n', d['ms_per_step'], {k:round(v['avg_ms']*v['launches']/2,1) for k,v in d['kernels'].items()}, d['engine']['groups'], d['engine']['device_peak_bytes']/1e9)"
  done
done
