#!/bin/bash
# Direct-output wide group counts (k_count_direct): wide / grouped parity tests,
# then C4 at 5.36 Gbases with the direct count and with staging + compaction.
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_wide.py tests/test_gpu_wide_large.py "tests/test_gpu_parity.py::test_grouped_count" \
    > gpurun_out/r03_s5.log 2>&1
rc=$?
tail -4 gpurun_out/r03_s5.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r03_s5.log | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
for d in 1 0; do
  OKM_COUNT_DIRECT=$d timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 3 --warmup 1 \
      > gpurun_out/r03_c4_direct$d.json 2> gpurun_out/r03_c4_direct$d.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r03_c4_direct$d.json')); print('c4 direct=$d', d['value']/1e9, d['ms_per_step'], d['engine']['groups'], d['engine']['device_bytes']/1e9, {k:(v['launches'],v['avg_ms']) for k,v in d['kernels'].items()})"
done
