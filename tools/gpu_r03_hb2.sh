#!/bin/bash
# Repeat of the 4096-home A/B (k=63, 1 Gbases), 3 interleaved runs per build, order alternating
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hb2
for r in 1 2 3; do
  if [ $((r % 2)) = 1 ]; then order="hb11 main"; else order="main hb11"; fi
  for n in $order; do
    if [ $n = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 300 python tools/bench_paths.py --workload wide --gbases 1 --steps 3 --warmup 1 \
      --cpu-sample-reads 0 > gpurun_out/hb2/${n}_$r.json 2> gpurun_out/hb2/${n}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/hb2/${n}_$r.json')); print('$n', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 1})"
  done
done
