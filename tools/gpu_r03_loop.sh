#!/bin/bash
# Round-3 GPU step: loopback (P>1) merge tests + the existing communicator
# tests, then the RCCL large-message diagnostic (tools/rccl_big_p2p.hip).
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_loopback.py tests/test_gpu_dist.py > gpurun_out/r03_loop.log 2>&1
rc=$?
tail -5 gpurun_out/r03_loop.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 180 tools/bin/rccl_big_p2p u64:1073741824 u64:2147483648 u64:4294967288 u64:4311744512 \
    u64:7900000000 u8:2147483648 u8:4311744512 > gpurun_out/r03_rccl_big.txt 2> gpurun_out/r03_rccl_big.err
rc2=$?
cat gpurun_out/r03_rccl_big.txt
exit $(( rc != 0 ? rc : rc2 ))
