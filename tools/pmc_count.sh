#!/bin/bash
# PMC passes on the engine kernels (separate passes; no trace domains with --pmc)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --cpu-sample-reads 0 --no-timing"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/pmc1 -o p -f csv -- $B > gpurun_out/pmc1.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM -d gpurun_out/pmc2 -o p -f csv -- $B > gpurun_out/pmc2.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3 -o p -f csv -- $B > gpurun_out/pmc3.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc4 -o p -f csv -- $B > gpurun_out/pmc4.log 2>&1
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc5 -o p -f csv -- $B > gpurun_out/pmc5.log 2>&1
echo done
