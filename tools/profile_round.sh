#!/bin/bash
# Round profile on the GPU box: kernel trace + stats of the bench, and the two
# PMC traffic passes.  usage: tools/profile_round.sh <round>   (e.g. r01)
set -o pipefail
R=${1:?round}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$R profiles
# --streams 1: every launch single-stream, so the kernel averages are the ones
# bench.py's roofline pass measures (the default timed region overlaps 2 streams)
B="python bench.py --steps 1 --warmup 1 --cpu-sample-reads 0 --no-timing --streams 1 --c3-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$R/trace -o p -f csv -- \
    python bench.py --steps 10 --warmup 2 --cpu-sample-reads 0 --streams 1 --c3-steps 0 > gpurun_out/prof_$R/bench_trace.json 2> gpurun_out/prof_$R/trace.log &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$R/fetch -o p -f csv -- $B > gpurun_out/prof_$R/fetch.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_$R/write -o p -f csv -- $B > gpurun_out/prof_$R/write.log 2>&1 &&
python tools/pmc_traffic.py $R gpurun_out/prof_$R/fetch/p_counter_collection.csv \
    gpurun_out/prof_$R/write/p_counter_collection.csv "$B" > gpurun_out/prof_$R/traffic.txt &&
python tools/rocprof_summary.py gpurun_out/prof_$R/trace/p_kernel_stats.csv > profiles/${R}_kernel_stats.txt &&
cp gpurun_out/prof_$R/bench_trace.json profiles/${R}_bench_under_rocprof.json &&
cp profiles/${R}_pmc_traffic.json gpurun_out/prof_$R/ &&
cp profiles/${R}_kernel_stats.txt gpurun_out/prof_$R/
