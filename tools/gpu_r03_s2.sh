#!/bin/bash
# Session-2 step: interleaved A/B of the working build against HEAD's
# (build_head) and single-change variants, SQ stall counters of the working
# build, then the whole GPU suite on it, smoke, and the bench line.
mkdir -p gpurun_out
tools/ab_interleave.sh 3 main head nomerge nocw ext512 > gpurun_out/r03_s2_ab.txt 2>&1 || { tail -5 gpurun_out/r03_s2_ab.txt; exit 1; }
cat gpurun_out/r03_s2_ab.txt
tools/gpu_r03_sq.sh > gpurun_out/r03_s2_sq.txt 2>&1 || { tail -5 gpurun_out/r03_s2_sq.txt; echo "sq pass failed"; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/r03_s2.log 2>&1
rc=$?
tail -4 gpurun_out/r03_s2.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_s2.log | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_s2.json 2> gpurun_out/r03_bench_s2.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_s2.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['single_job'], d['roofline']['kernel'], d['roofline']['frac'], 'device GB', d['engine']['device_bytes']/1e9)"
