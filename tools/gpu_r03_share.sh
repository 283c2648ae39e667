#!/bin/bash
# Result in the dead level block: parity + merge + C3 + dist subsets, then the
# C2 bench (context bytes, pool dump).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_merge.py tests/test_gpu_c3.py tests/test_gpu_loopback.py \
    tests/test_gpu_dist.py > gpurun_out/r03_share.log 2>&1
rc=$?
tail -3 gpurun_out/r03_share.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_share.log | head -20; exit $rc; fi
OKM_POOL_DUMP=1 timeout -k 10 300 python bench.py > gpurun_out/r03_bench_f.json 2> gpurun_out/r03_bench_f.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_f.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['single_job']['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], 'device GB', d['engine']['device_bytes']/1e9)"
grep "pool reset" gpurun_out/r03_bench_f.err | tail -1
