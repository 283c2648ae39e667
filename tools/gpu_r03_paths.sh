#!/bin/bash
# Round-3 secondary measurements: C4 (k=63, 5.36 Gbases, indel generator),
# C5 on one GPU and through the P=8 loopback exchange, C3 P=1 at the default
# fold threshold, and the end-to-end CLI (gzip input / output split).
mkdir -p gpurun_out
if [ "$1" = all ]; then
timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 3 --warmup 1 \
    > gpurun_out/r03_path_c4.json 2> gpurun_out/r03_path_c4.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_path_c4.json')); print('c4', d['value']/1e9, d['ms_per_step'], d['engine']['groups'], d['engine']['device_bytes']/1e9)"
timeout -k 10 400 python tools/bench_paths.py --workload c5 --steps 3 --warmup 1 \
    > gpurun_out/r03_path_c5.json 2> gpurun_out/r03_path_c5.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_path_c5.json')); print('c5', d['value']/1e9, d['ms_per_step'], d['config']['jaccard_index'])"
fi
timeout -k 10 400 python tools/bench_paths.py --workload c5 --loopback 8 --steps 3 --warmup 1 \
    > gpurun_out/r03_path_c5_loop8.json 2> gpurun_out/r03_path_c5_loop8.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_path_c5_loop8.json')); print('c5 loop8', d['value']/1e9, d['ms_per_step'], d['config']['jaccard_index'], d['config']['bytes_sent_all_ranks'])"
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 > gpurun_out/r03_bench_c3.json 2> gpurun_out/r03_bench_c3.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_c3.json')); print('c3', d['value']/1e9, d['ms_per_step'], d['config']['folds_rank0'])"
timeout -k 10 500 ./tools/e2e_cli.sh > gpurun_out/r03_e2e_cli.txt 2>&1 || exit $?
grep -E "e2e|==|parsed|counted|written|runs" gpurun_out/r03_e2e_cli.txt | tail -30
