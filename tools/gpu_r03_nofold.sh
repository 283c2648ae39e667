#!/bin/bash
# C3 at P=1 with folding deferred past the whole job (every batch stays an L1 run; one grouped
# count at the end): where its time goes (OKM_PROFILE_HOST phase marks, OKM_POOL_TRACE allocations)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/nf
OKM_FOLD_BYTES=150000000000 OKM_PROFILE_HOST=1 timeout -k 10 240 python bench.py --workload c3 --steps 1 --warmup 1 \
  --cpu-sample-reads 0 > gpurun_out/nf/nofold.json 2> gpurun_out/nf/nofold.err || exit $?
