#!/bin/bash
# C3 at P=1 with a 12 % fold threshold: where the grouped fold counts spend their time
# (OKM_PROFILE_HOST phase marks, OKM_POOL_TRACE allocations)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f12
OKM_FOLD_BYTES=36000000000 OKM_PROFILE_HOST=1 OKM_POOL_TRACE=1 timeout -k 10 240 python bench.py --workload c3 \
  --steps 1 --warmup 1 --cpu-sample-reads 0 > gpurun_out/f12/c3.json 2> gpurun_out/f12/c3.err || exit $?
