#!/bin/bash
# Round-3 profile (kernel stats + PMC traffic), then an interleaved A/B of the
# count descriptor prefetch and the partition copy-out by bin.
./tools/profile_round.sh r03 || exit $?
tail -20 profiles/r03_kernel_stats.txt
cat gpurun_out/prof_r03/traffic.txt
./tools/ab_interleave.sh 3 main dpf pcb
