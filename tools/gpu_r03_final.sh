#!/bin/bash
# Round-3 evidence on the final build: rocprofv3 kernel stats + PMC traffic of
# the C2 bench (tools/profile_round.sh r03), the bench line, C3 at P=1, C4 and
# C5 path lines, then the whole GPU suite and smoke.
mkdir -p gpurun_out
tools/profile_round.sh r03 > gpurun_out/r03_prof.log 2>&1 || { tail -20 gpurun_out/r03_prof.log; exit 1; }
cat profiles/r03_kernel_stats.txt | head -20
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_final.json 2> gpurun_out/r03_bench_final.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_final.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['single_job'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'], 'device GB', d['engine']['device_bytes']/1e9)"
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 > gpurun_out/r03_bench_c3_final.json 2> gpurun_out/r03_bench_c3_final.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_c3_final.json')); print('c3', d['value']/1e9, d['ms_per_step'], d['config']['folds_rank0'], {k:(v['launches'],v['avg_ms']) for k,v in d['kernels'].items()})"
timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 3 --warmup 1 \
    > gpurun_out/r03_path_c4_final.json 2> gpurun_out/r03_path_c4_final.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_path_c4_final.json')); print('c4', d['value']/1e9, d['ms_per_step'], d['engine']['groups'], d['engine']['device_bytes']/1e9)"
timeout -k 10 400 python tools/bench_paths.py --workload c5 --steps 3 --warmup 1 \
    > gpurun_out/r03_path_c5_final.json 2> gpurun_out/r03_path_c5_final.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_path_c5_final.json')); print('c5', d['value']/1e9, d['ms_per_step'], d['config']['jaccard_index'])"
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/r03_final_suite.log 2>&1
rc=$?
tail -3 gpurun_out/r03_final_suite.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_final_suite.log | head -20; echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
