#!/bin/bash
# C3 at P=1, default fold threshold: host phase marks and pool allocations per job
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c3t
OKM_PROFILE_HOST=1 OKM_POOL_TRACE=1 timeout -k 10 240 python bench.py --workload c3 --steps 2 --warmup 1 \
  --cpu-sample-reads 0 > gpurun_out/c3t/c3.json 2> gpurun_out/c3t/c3.err || exit $?
