#!/bin/bash
# Extraction pass alone (tools/extract_only.py), interleaved over builds:
# main, e1 (no HBM writes), e2 (no staging / copy-out), e512 (512 threads x 32 windows).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2 3; do
  for n in main e1 e2 e512; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    echo -n "$n rep $r: "
    OKM_LIB=$lib timeout -k 10 120 python tools/extract_only.py || exit 1
  done
done
