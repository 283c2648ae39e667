#!/bin/bash
# Dense staging: parity subset, bench + pool at reset, C3 fold A/B.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_merge.py tests/test_gpu_wide.py tests/test_gpu_c3.py > gpurun_out/r03_dense.log 2>&1
rc=$?
tail -3 gpurun_out/r03_dense.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_dense.log | head -20; exit $rc; fi
OKM_POOL_DUMP=1 timeout -k 10 300 python bench.py > gpurun_out/r03_bench_c.json 2> gpurun_out/r03_bench_c.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_c.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['single_job']['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], 'device GB', d['engine']['device_bytes']/1e9)"
grep "okm pool reset" gpurun_out/r03_bench_c.err | tail -1 | cut -c1-300
for f in 0.08 0.10 0.12 0.14; do
  export OKM_FOLD_BYTES=$(python -c "print(int($f * 309220868096))")
  timeout -k 10 240 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 --no-timing \
      > gpurun_out/r03_c3d_f$f.json 2> gpurun_out/r03_c3d_f$f.err
  r=$?
  python -c "import json; d=json.load(open('gpurun_out/r03_c3d_f$f.json')); print('c3 fold $f', d['ms_per_step'], d['config']['folds_rank0'], d['config']['groups_rank0'], d['engine']['device_bytes']/1e9)" 2>/dev/null || tail -1 gpurun_out/r03_c3d_f$f.err | cut -c1-300
  if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
