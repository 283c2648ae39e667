#!/bin/bash
# Loopback tests (wire deltas), count workgroup A/B (512 vs 256 threads).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_loopback.py \
    > gpurun_out/r03_loop2.log 2>&1
rc=$?
tail -3 gpurun_out/r03_loop2.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r03_loop2.log | head -20; exit $rc; fi
OKM_LIB=orion-kmer_amd/build_cb256/liborion_kmer.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r03_cb256.log 2>&1
rc=$?
tail -2 gpurun_out/r03_cb256.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_cb256.log | head; exit $rc; fi
./tools/ab_interleave.sh 3 main cb256
