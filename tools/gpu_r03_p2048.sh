#!/bin/bash
# 2048-bin partition passes: parity subset, then C3 (fold 8 % / 10 %) kernel
# breakdown, the C2 bench, and the CLI with gzip output at the new level.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_merge.py tests/test_gpu_c3.py > gpurun_out/r03_p2048.log 2>&1
rc=$?
tail -3 gpurun_out/r03_p2048.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_p2048.log | head -20; exit $rc; fi
for f in 0.08 0.10; do
  export OKM_FOLD_BYTES=$(python -c "print(int($f * 309220868096))")
  timeout -k 10 240 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 \
      > gpurun_out/r03_c3p_f$f.json 2> gpurun_out/r03_c3p_f$f.err || exit $?
  python - $f <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r03_c3p_f{sys.argv[1]}.json"))
print("c3 fold", sys.argv[1], d["ms_per_step"], "folds", d["config"]["folds_rank0"], "groups", d["config"]["groups_rank0"])
for n, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["launches"])[:8]:
    print("   %-16s %4d x %8.3f = %7.1f ms" % (n, v["launches"], v["avg_ms"], v["avg_ms"] * v["launches"]))
PY
done
unset OKM_FOLD_BYTES
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_d.json 2> gpurun_out/r03_bench_d.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03_bench_d.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['single_job']['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], 'device GB', d['engine']['device_bytes']/1e9)"
timeout -k 10 500 ./tools/e2e_cli.sh > gpurun_out/r03_e2e_cli.txt 2>&1 || exit $?
grep -E "e2e|runs" gpurun_out/r03_e2e_cli.txt | tail -12
