#!/bin/bash
# A/B timing of environment settings of one build (C2 bench):
#   tools/ab_env.sh name1 'VAR=val ...' name2 'VAR=val ...' ...
# one JSON line per setting in gpurun_out/ab/<name>.json and a summary line each
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
while [ $# -ge 2 ]; do
  n=$1; e=$2; shift 2
  env $e timeout -k 10 200 python bench.py --c3-steps 0 --steps 10 --warmup 2 --cpu-sample-reads 0 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); print('$n', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.03})"
done
