#!/bin/bash
# A/B: extraction scatter with the next tile's bytes waited for before the copy-out stores (nw), so the
# loop head no longer waits for the previous tile's stores (vmcnt retires in order), vs main
cd "$GRAFT_REPO_ROOT"
tools/ab_interleave.sh 3 main nw > gpurun_out/ab_nw.txt 2>&1 || exit $?
OKM_LIB=orion-kmer_amd/build_nw/liborion_kmer.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/nw_parity.txt 2>&1
