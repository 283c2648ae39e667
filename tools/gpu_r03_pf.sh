#!/bin/bash
# Branch-free clamped prefetch + LDS-only barriers: parity subset, then the
# extraction alone and the C2 bench interleaved over main / pfl (late
# prefetch) / nolb (__syncthreads).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    > gpurun_out/r03_pf.log 2>&1
rc=$?
tail -2 gpurun_out/r03_pf.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_pf.log | head; exit $rc; fi
for r in 1 2; do
  for n in main pfl nolb; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    echo -n "$n rep $r: "
    OKM_LIB=$lib timeout -k 10 120 python tools/extract_only.py || exit 1
  done
done
./tools/ab_interleave.sh 3 main pfl nolb
