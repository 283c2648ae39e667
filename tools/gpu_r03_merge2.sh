#!/bin/bash
# Staged merges by default: C3 + merge tests, then C3 at P=1 twice.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_c3.py tests/test_gpu_merge.py > gpurun_out/r03_merge2.log 2>&1
rc=$?
tail -3 gpurun_out/r03_merge2.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_merge2.log | head -20; exit $rc; fi
for i in 1 2; do
  timeout -k 10 240 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 \
      > gpurun_out/r03_m2_$i.json 2> gpurun_out/r03_m2_$i.err || { tail -3 gpurun_out/r03_m2_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03_m2_$i.json')); print('c3', d['ms_per_step'], d['config']['folds_rank0'], d['engine']['device_bytes']/1e9, {k: round(v['avg_ms']*v['launches'],1) for k, v in d['kernels'].items() if v['avg_ms']*v['launches'] > 20})"
done
