#!/bin/bash
# A/B of (library build, environment) pairs on the C2 bench, single stream:
#   tools/ab_mix.sh name build 'VAR=val ...' [name build env ...]
# build: main (orion-kmer_amd/build) or <b> (orion-kmer_amd/build_<b>); env may be '-'.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
while [ $# -ge 3 ]; do
  n=$1; b=$2; e=$3; shift 3
  if [ "$b" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$b/liborion_kmer.so; fi
  [ "$e" = - ] && e=
  env OKM_LIB=$lib $e timeout -k 10 200 python bench.py --c3-steps 0 --steps 10 --warmup 2 --cpu-sample-reads 0 --streams 1 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); print('$n', d['ms_per_step'], d['engine']['l2_bits'], d['engine']['work_items'], {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.03})"
done
