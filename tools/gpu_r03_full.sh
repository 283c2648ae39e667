#!/bin/bash
# Round-3 GPU step: the whole GPU suite, the headline bench line, then the C3
# fold threshold A/B at P=1 (OKM_FOLD_BYTES as a fraction of HBM).
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/r03_full.log 2>&1
rc=$?
tail -4 gpurun_out/r03_full.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_full.log | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_b.json 2> gpurun_out/r03_bench_b.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_b.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['single_job'], d['roofline']['kernel'], d['roofline']['frac'], 'device GB', d['engine']['device_bytes']/1e9)"
for f in 0.08 0.12 0.16 0.20; do
  export OKM_FOLD_BYTES=$(python -c "print(int($f * 309220868096))")
  timeout -k 10 240 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 --no-timing \
      > gpurun_out/r03_c3_f$f.json 2> gpurun_out/r03_c3_f$f.err
  r=$?
  python -c "import json; d=json.load(open('gpurun_out/r03_c3_f$f.json')); print('c3 fold $f', d['ms_per_step'], d['config']['folds_rank0'], d['config']['groups_rank0'], d['engine']['device_bytes']/1e9)" 2>/dev/null || tail -2 gpurun_out/r03_c3_f$f.err
  if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
