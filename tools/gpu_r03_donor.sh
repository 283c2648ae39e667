#!/bin/bash
# Staged keys in the dying L1 run's block: the whole GPU suite, the C2 bench
# (context bytes) with the pool dump, and C3 at the default fold threshold.
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/r03_donor.log 2>&1
rc=$?
tail -3 gpurun_out/r03_donor.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_donor.log | head -20; exit $rc; fi
OKM_POOL_DUMP=1 timeout -k 10 300 python bench.py > gpurun_out/r03_bench_e.json 2> gpurun_out/r03_bench_e.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_e.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['single_job']['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], 'device GB', d['engine']['device_bytes']/1e9)"
grep "pool reset" gpurun_out/r03_bench_e.err | tail -1
timeout -k 10 240 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 \
    > gpurun_out/r03_c3_e.json 2> gpurun_out/r03_c3_e.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_c3_e.json')); print('c3', d['ms_per_step'], d['config']['folds_rank0'], d['config']['groups_rank0'], d['engine']['device_bytes']/1e9)"
