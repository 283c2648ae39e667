#!/bin/bash
# Does the per-tile claim (a returning device atomic per (tile, bin)) cost the
# scatters time?  Exact placement (OKM_*_SAMPLE=1: a histogram pass, one claim
# per chunk) vs sampled placement, per-kernel times of the single-stream pass.
mkdir -p gpurun_out/s6
for r in 1 2; do
  for v in def exact; do
    if [ $v = exact ]; then export OKM_PART_SAMPLE=1 OKM_L1_SAMPLE=1; else unset OKM_PART_SAMPLE OKM_L1_SAMPLE; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-sample-reads 0 --cpu-mt-reads 0 \
      > gpurun_out/s6/${v}_$r.json 2> gpurun_out/s6/${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/s6/${v}_$r.json')); print('$v', d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
  done
done
