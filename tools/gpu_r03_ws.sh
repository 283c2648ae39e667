#!/bin/bash
# Wide single-sweep extraction with LDS-shared codes (build/) vs every thread coding its 80 bytes
# (build_ws0): the wide suites, then k=63 1 Gbases lines (4 runs per build, alternating order)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ws
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_wide_large.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/ws/tests.txt 2>&1 || { tail -5 gpurun_out/ws/tests.txt; exit 1; }
tail -1 gpurun_out/ws/tests.txt
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="ws0 main"; else order="main ws0"; fi
  for n in $order; do
    if [ $n = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib timeout -k 10 300 python tools/bench_paths.py --workload wide --gbases 1 --steps 3 --warmup 1 \
      --cpu-sample-reads 0 > gpurun_out/ws/${n}_$r.json 2> gpurun_out/ws/${n}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ws/${n}_$r.json')); print('$n', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 1})"
  done
done
