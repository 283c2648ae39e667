#!/bin/bash
# A/B: 512-thread partition workgroups (two per CU, 8 Ki / 9 Ki-key tiles) vs the 1024-thread build
cd "$GRAFT_REPO_ROOT"
tools/ab_interleave.sh 3 main p512 p512b > gpurun_out/ab_p512.txt 2>&1
