#!/bin/bash
# Does the partition kernel's slow mode follow the process (physical memory
# placement) or the box?  C2 kernel times over several processes, some of
# which first take and release a large device block (run on the GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/mode
ARGS="--steps 3 --warmup 1 --cpu-sample-reads 0 --cpu-mt-reads 0 --c3-steps 0"
for i in 1 2 3; do
  for pre in 0 96; do
    timeout -k 10 200 python -u -c "
import sys, runpy
sys.path.insert(0, 'orion-kmer_amd')
import okm
from okm import _lib
_lib.load()
if $pre:
    b = okm.DeviceBuffer($pre << 30)
    b.free()
sys.argv = ['bench.py'] + '$ARGS'.split()
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/mode/p${pre}_$i.json 2> gpurun_out/mode/p${pre}_$i.err || { echo "run $pre $i failed"; tail -3 gpurun_out/mode/p${pre}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/mode/p${pre}_$i.json').read().strip().splitlines()[-1])
print('pre ${pre} GB run $i', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
  done
done
