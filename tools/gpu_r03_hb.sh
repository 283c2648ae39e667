#!/bin/bash
# Full-mode count with 4096 homes for K128 keys (build/) vs 2048 (build_hb11): wide + parity +
# merge suites (full mode also runs deferred u64 items and the owner merges), then k=63 path lines
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hb
timeout -k 10 700 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_wide_large.py tests/test_gpu_parity.py \
  tests/test_gpu_merge.py -x -q --timeout 300 --timeout-method thread > gpurun_out/hb/tests.txt 2>&1 \
  || { tail -5 gpurun_out/hb/tests.txt; exit 1; }
tail -1 gpurun_out/hb/tests.txt
for r in 1 2; do
  for n in main hb11; do
    if [ $n = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 300 python tools/bench_paths.py --workload wide --gbases 1 --steps 3 --warmup 1 \
      --cpu-sample-reads 0 > gpurun_out/hb/${n}_$r.json 2> gpurun_out/hb/${n}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/hb/${n}_$r.json')); print('$n 1G', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
  done
done
for n in main hb11; do
  if [ $n = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
  OKM_LIB=$lib timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 3 --warmup 1 \
    --cpu-sample-reads 0 > gpurun_out/hb/${n}_c4.json 2> gpurun_out/hb/${n}_c4.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/hb/${n}_c4.json')); print('$n C4', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
