#!/bin/bash
# Multi-GPU merge with K128 keys (k > 32): real RCCL at one rank, the dist / merge suites
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_merge.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/widemerge.txt 2>&1
