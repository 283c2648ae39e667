#!/bin/bash
# interleaved C4 A/B: main vs build_ni
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c4ab
for r in 1 2; do
  for n in main ni; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 2 --warmup 1 > gpurun_out/c4ab/${n}_$r.json 2> gpurun_out/c4ab/${n}_$r.log || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c4ab/${n}_$r.json'));print('$n', d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()}, d['engine']['groups'])"
  done
done
