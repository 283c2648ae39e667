#!/bin/bash
# round 6: the GPU suite, then one driver-style bench line (tools/gpu_lease.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_lease.sh suite > gpurun_out/suite_run.txt 2>&1
rc=$?
tail -4 gpurun_out/suite_run.txt
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_lease.sh bench --steps 20 --warmup 3 > gpurun_out/bench_run.txt 2>&1
rc=$?
tail -c 1500 gpurun_out/bench/line.json
exit $rc
