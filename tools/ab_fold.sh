#!/bin/bash
# C3 on one GPU (BASELINE configs[2] at P=1: folding) under fold settings:
#   tools/ab_fold.sh name1 'VAR=val ...' name2 'VAR=val ...' ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fold
while [ $# -ge 2 ]; do
  n=$1; e=$2; shift 2
  env $e timeout -k 10 240 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 --no-timing \
    > gpurun_out/fold/$n.json 2> gpurun_out/fold/$n.err || { echo "$n failed: $(tail -1 gpurun_out/fold/$n.err | cut -c1-200)"; continue; }
  python3 -c "import json; d=json.load(open('gpurun_out/fold/$n.json')); print('$n', '$e', d['ms_per_step'], 'folds', d['engine']['folds'], 'groups', d['engine']['groups'])"
done
