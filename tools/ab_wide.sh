#!/bin/bash
# A/B timing of alternative library builds on the k=63 ONT-like workload:
# tools/ab_wide.sh name1 name2 ... (each orion-kmer_amd/build_<name>/liborion_kmer.so,
# "main" = orion-kmer_amd/build).  One JSON line per build in gpurun_out/ab/.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for n in "$@"; do
  if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
  OKM_LIB=$lib timeout -k 10 200 python tools/bench_paths.py --workload wide --steps 3 --warmup 1 > gpurun_out/ab/wide_$n.json 2> gpurun_out/ab/wide_$n.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/wide_$n.json')); print('$n', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.3})"
done
