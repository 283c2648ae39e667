#!/bin/bash
# A/B timing of alternative library builds: tools/ab_bench.sh name1 name2 ...
# (each orion-kmer_amd/build_<name>/liborion_kmer.so); parity via debug_count rand.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for n in "$@"; do
  lib=orion-kmer_amd/build_$n/liborion_kmer.so
  OKM_LIB=$lib timeout -k 5 90 python tools/debug_count.py rand > gpurun_out/ab/$n.dbg 2>&1 || exit 1
  OKM_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample-reads 0 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || exit 1
done
