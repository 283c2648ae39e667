#!/bin/bash
# HEAD check: the whole GPU suite, smoke, and the driver's default bench line
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/head_suite.log 2>&1
rc=$?
tail -3 gpurun_out/head_suite.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/head_suite.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 300 python bench.py > gpurun_out/head_bench.json 2> gpurun_out/head_bench.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/head_bench.json')); c=d['c3']; print('bench', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], '| c3', c['value']/1e9, c['ms_per_step'])"
