#!/bin/bash
# C4 (k = 63, 5.36 Gbases) under a test hook, interleaved with the default:
#   tools/c4_knob.sh REPS knob value     (e.g. part_max_bits 9)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c4knob
reps=$1; knob=$2; val=$3
for r in $(seq 1 "$reps"); do
  for v in default "$val"; do
    timeout -k 10 400 python -u -c "
import sys, runpy
sys.path.insert(0, 'orion-kmer_amd'); sys.path.insert(0, 'tools')
from okm import _lib, testing
_lib.load()
if '$v' != 'default':
    testing.set_knob('$knob', int('$v'))
sys.argv = ['bench_paths.py', '--workload', 'wide', '--gbases', '5.36', '--steps', '2', '--warmup', '1']
runpy.run_path('tools/bench_paths.py', run_name='__main__')
" > gpurun_out/c4knob/${v}_$r.json 2> gpurun_out/c4knob/${v}_$r.log || { echo "$v failed"; tail -3 gpurun_out/c4knob/${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/c4knob/${v}_$r.json'));print('$knob=$v', d['ms_per_step'], {k:round(v['avg_ms']*v['launches']/3,1) for k,v in d['kernels'].items()}, d['engine']['groups'], d['engine'].get('l2_bits'))"
  done
done
