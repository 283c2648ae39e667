#!/bin/bash
# LDS-only barriers (main) against __syncthreads (nolb): extraction alone, then
# interleaved C2 benches.
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for n in main nolb; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    echo -n "$n rep $r: "
    OKM_LIB=$lib timeout -k 10 120 python tools/extract_only.py || exit 1
  done
done
./tools/ab_interleave.sh 3 main nolb
