#!/bin/bash
# Sorted-run merge modes on the GPU: merge tests, then tools/merge8_cost.py
# (C3 owner slices) under OKM_MERGE_KERNEL=1 (k-way merge kernel) and =2
# (two-pass count), then C3 on one GPU (folded tables) for this build and,
# if present, orion-kmer_amd/build_head (tools/build_head.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mrg
timeout -k 10 500 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_c3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mrg/tests.log 2>&1 || { tail -30 gpurun_out/mrg/tests.log; exit 1; }
tail -2 gpurun_out/mrg/tests.log
for mk in 2 1; do
  OKM_MERGE_KERNEL=$mk timeout -k 10 200 python tools/merge8_cost.py 3 2,4,8 > gpurun_out/mrg/m8_$mk.json 2>gpurun_out/mrg/m8_$mk.err || exit 1
  cat gpurun_out/mrg/m8_$mk.json
done
timeout -k 10 200 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 > gpurun_out/mrg/c3_new.json 2> gpurun_out/mrg/c3_new.err || exit 1
if [ -f orion-kmer_amd/build_head/liborion_kmer.so ]; then
  OKM_LIB=orion-kmer_amd/build_head/liborion_kmer.so timeout -k 10 200 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 > gpurun_out/mrg/c3_old.json 2> gpurun_out/mrg/c3_old.err || exit 1
fi
python3 -c "
import json, os
for n in ['new','old']:
    f = f'gpurun_out/mrg/c3_{n}.json'
    if os.path.exists(f):
        d=json.load(open(f)); print(n, d['ms_per_step'], {k:(v['launches'],v['avg_ms']) for k,v in d['kernels'].items()})
"
