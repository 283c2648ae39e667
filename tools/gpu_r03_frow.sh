#!/bin/bash
# Full-mode run-start flags from lane-contiguous rows (build/) vs per-thread strided reads (build_frow0):
# the wide and full-mode parity tests, then k=63 1 Gbases path lines interleaved
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/frow
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_wide_large.py tests/test_gpu_parity.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/frow/tests.txt 2>&1 || { tail -5 gpurun_out/frow/tests.txt; exit 1; }
tail -1 gpurun_out/frow/tests.txt
for r in 1 2; do
  for n in main frow0; do
    if [ $n = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 300 python tools/bench_paths.py --workload wide --gbases 1 --steps 3 --warmup 1 \
      --cpu-sample-reads 0 > gpurun_out/frow/${n}_$r.json 2> gpurun_out/frow/${n}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/frow/${n}_$r.json')); print('$n', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
  done
done
