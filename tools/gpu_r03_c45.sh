#!/bin/bash
# Round-3 GPU step: C5 stated-workload tests and the C4 tests on the indel
# generator, then the headline bench line.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_c5.py tests/test_gpu_wide_large.py > gpurun_out/r03_c45.log 2>&1
rc=$?
tail -12 gpurun_out/r03_c45.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_a.json 2> gpurun_out/r03_bench_a.err
rc2=$?
cat gpurun_out/r03_bench_a.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value']/1e9, d['ms_per_step'], d['single_job'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline_mt']['threads'], d['cpu_baseline_mt']['affinity_cpus'])"
exit $(( rc != 0 ? rc : rc2 ))
