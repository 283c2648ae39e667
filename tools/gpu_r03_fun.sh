#!/bin/bash
# A/B: k<=32 window keys by funnel shifts + all-windows validity mask (fun), plus each thread coding
# only its own 16 bytes with the halo's codes from LDS (share), vs the previous extraction (main);
# then the C2 parity suite on the share build
cd "$GRAFT_REPO_ROOT"
tools/ab_interleave.sh 3 main fun share > gpurun_out/ab_fun.txt 2>&1 || exit $?
OKM_LIB=orion-kmer_amd/build_share/liborion_kmer.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/share_parity.txt 2>&1
