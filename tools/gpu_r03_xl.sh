#!/bin/bash
# A/B: 18 Ki-key partition tiles (72 Ki-key chunks) for u64 passes of <= 512 bins vs 16 Ki
cd "$GRAFT_REPO_ROOT"
tools/ab_interleave.sh 4 main xl > gpurun_out/ab_xl.txt 2>&1
