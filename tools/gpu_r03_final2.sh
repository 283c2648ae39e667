#!/bin/bash
# Round-3 evidence on the final build (after the bench workload change and the extraction key
# change): rocprofv3 kernel stats + PMC traffic of the C2 bench (tools/profile_round.sh r03),
# the driver's bench line (C2 value + C3 appendix), C4 path line, the GPU suite and smoke.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tools/profile_round.sh r03 > gpurun_out/r03_prof.log 2>&1 || { tail -20 gpurun_out/r03_prof.log; exit 1; }
head -12 profiles/r03_kernel_stats.txt
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_final2.json 2> gpurun_out/r03_bench_final2.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_final2.json')); c=d['c3']; print('bench', d['value']/1e9, d['ms_per_step'], d['single_job'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'], '| c3', c['value']/1e9, c['ms_per_step'])"
timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 3 --warmup 1 \
    > gpurun_out/r03_path_c4_final2.json 2> gpurun_out/r03_path_c4_final2.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_path_c4_final2.json')); print('c4', d['value']/1e9, d['ms_per_step'], d['engine']['groups'])"
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/r03_final2_suite.log 2>&1
rc=$?
tail -3 gpurun_out/r03_final2_suite.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_final2_suite.log | head -20; echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
