#!/bin/bash
# Co-residency A/B: scatter workgroups of 768 threads over 12 Ki-window /
# 12 Ki-key tiles (<= 110 KiB of LDS, <= 116 VGPRs) leave room on their CU for
# a count workgroup of another batch in flight; main = 1024-thread, 16 Ki tiles.
export OKM_PART_MAXB=9   # 768-thread partition passes take <= 768 children (C2 uses 512)
mkdir -p gpurun_out
tools/ab_interleave.sh 3 main head cores ext768 part768 > gpurun_out/r03_s7_ab.txt 2>&1 || { tail -5 gpurun_out/r03_s7_ab.txt; exit 1; }
cat gpurun_out/r03_s7_ab.txt
