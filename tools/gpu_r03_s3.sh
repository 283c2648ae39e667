#!/bin/bash
# A/B of the tag-claim batch (OKM_CLAIM_BATCH 2 = main, 1, 4) against HEAD's build.
mkdir -p gpurun_out
tools/ab_interleave.sh 3 main head cb1 cb4 > gpurun_out/r03_s3_ab.txt 2>&1 || { tail -5 gpurun_out/r03_s3_ab.txt; exit 1; }
cat gpurun_out/r03_s3_ab.txt
