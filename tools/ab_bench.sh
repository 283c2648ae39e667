#!/bin/bash
# A/B timing of alternative library builds: tools/ab_bench.sh name1 name2 ...
# (each orion-kmer_amd/build_<name>/liborion_kmer.so; "main" = orion-kmer_amd/build);
# parity via debug_count rand, then the C2 bench; one summary line per build.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for n in "$@"; do
  if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
  OKM_LIB=$lib timeout -k 5 90 python tools/debug_count.py rand > gpurun_out/ab/$n.dbg 2>&1 || exit 1
  OKM_LIB=$lib timeout -k 10 200 python bench.py --c3-steps 0 --steps 10 --warmup 2 --cpu-sample-reads 0 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); print('$n', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.03})"
done
