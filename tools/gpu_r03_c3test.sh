#!/bin/bash
# Round-3 GPU step: C3 full-size tests (P=1 whole job, P=8 shard with a real
# RCCL self-merge).
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_c3.py > gpurun_out/r03_c3test.log 2>&1
rc=$?
tail -15 gpurun_out/r03_c3test.log
exit $rc
