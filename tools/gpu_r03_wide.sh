#!/bin/bash
# Wide extraction with the clamped prefetch: wide parity, then C4 (k=63,
# 5.36 Gbases) and k=63 at 1 Gbases.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_wide.py tests/test_gpu_wide_large.py > gpurun_out/r03_wide.log 2>&1
rc=$?
tail -2 gpurun_out/r03_wide.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_wide.log | head; exit $rc; fi
for gb in 1.0 5.36; do
  timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases $gb --steps 3 --warmup 1 \
      > gpurun_out/r03_wide_$gb.json 2> gpurun_out/r03_wide_$gb.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r03_wide_$gb.json')); print('wide $gb', d['value']/1e9, d['ms_per_step'], {k: round(v['avg_ms'],3) for k, v in d['kernels'].items() if v['avg_ms'] > 0.2})"
done
