#!/bin/bash
# A/B: guarded tag-mode loops with single-path loads (main) vs the early-exit
# loops (g0), 8 Ki-key partition tiles (pt8k), and HEAD's build.
mkdir -p gpurun_out
tools/ab_interleave.sh 3 main head g0 pt8k > gpurun_out/r03_s4_ab.txt 2>&1 || { tail -5 gpurun_out/r03_s4_ab.txt; exit 1; }
cat gpurun_out/r03_s4_ab.txt
