#!/bin/bash
# Two SQ counter passes (instruction mix, stalls) over one bench step: tools/pmc_quick.sh <outdir>
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${1:-gpurun_out/pmcq}
B="python bench.py --steps 1 --warmup 0 --cpu-sample-reads 0 --no-timing"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d $O/p1 -o p -f csv -- $B > $O.p1.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM -d $O/p2 -o p -f csv -- $B > $O.p2.log 2>&1
