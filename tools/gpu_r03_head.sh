#!/bin/bash
# Round-3 re-entry check of HEAD: the whole GPU suite, smoke, the headline bench line.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/r03_head.log 2>&1
rc=$?
tail -4 gpurun_out/r03_head.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_head.log | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_head.json 2> gpurun_out/r03_bench_head.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_head.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['single_job'], d['roofline']['kernel'], d['roofline']['frac'], 'device GB', d['engine']['device_bytes']/1e9)"
