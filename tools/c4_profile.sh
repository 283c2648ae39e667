#!/bin/bash
# C4 (k = 63, 5.36 Gbases, one step, no warmup) under rocprofv3: kernel stats
# and the two PMC traffic passes -> gpurun_out/prof_c4_<round>/ (copy into profiles/)
set -o pipefail
R=${1:?round}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=gpurun_out/prof_c4_$R
mkdir -p $D
B="python3 tools/bench_paths.py --workload wide --gbases 5.36 --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o p -f csv -- $B > $D/bench_trace.json 2> $D/trace.log &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o p -f csv -- $B > $D/fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $D/write -o p -f csv -- $B > $D/write.log 2>&1 &&
python3 tools/pmc_traffic.py ${R}_c4 $D/fetch/p_counter_collection.csv $D/write/p_counter_collection.csv "$B" > $D/traffic.txt &&
cp profiles/${R}_c4_pmc_traffic.json $D/ &&
python3 tools/rocprof_summary.py $D/trace/p_kernel_stats.csv > $D/${R}_c4_kernel_stats.txt &&
tail -20 $D/traffic.txt && head -12 $D/${R}_c4_kernel_stats.txt
