#!/bin/bash
# A/B timing of environment settings of one build:
#   tools/ab_env.sh name1 'VAR=val ...' name2 'VAR=val ...' ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
while [ $# -ge 2 ]; do
  n=$1; e=$2; shift 2
  env $e timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample-reads 0 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || exit 1
done
