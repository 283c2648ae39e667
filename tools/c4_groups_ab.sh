#!/bin/bash
# C4 group sizes with the keys over the L1 run: default cap (2^30 instances) vs forced larger groups
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c4g
for r in 1 2; do for v in def g135 g18; do
  K=""
  [ "$v" = g135 ] && K="--knob group_keys=1350000000 --knob group_over=1"
  [ "$v" = g18 ] && K="--knob group_keys=1800000000 --knob group_over=1"
  timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 2 --warmup 1 $K \
    > gpurun_out/c4g/${v}_$r.json 2> gpurun_out/c4g/${v}_$r.log || { echo "$v failed"; tail -5 gpurun_out/c4g/${v}_$r.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c4g/${v}_$r.json'));print('$v', d['ms_per_step'], {k:round(v['avg_ms']*v['launches']/2,1) for k,v in d['kernels'].items()}, d['engine']['groups'], d['engine']['device_peak_bytes']/1e9)"
done; done
