#!/bin/bash
# C4 (k = 63, 5.36 Gbases): key-range groups writing the table's keys over the
# batch's L1 run (default) vs a separate instance-bound key array (test knob
# group_over = 0, through OKM_TEST_GROUP_OVER set by tools/bench_paths.py --knob)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c4over
for r in 1 2; do for v in over sep; do
  K=""; [ "$v" = sep ] && K="--knob group_over=0"
  timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 2 --warmup 1 $K \
    > gpurun_out/c4over/${v}_$r.json 2> gpurun_out/c4over/${v}_$r.log || { echo "$v failed"; tail -5 gpurun_out/c4over/${v}_$r.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c4over/${v}_$r.json'));print('$v', d['ms_per_step'], {k:round(v['avg_ms']*v['launches']/2,1) for k,v in d['kernels'].items()}, d['engine']['groups'], d['engine']['device_peak_bytes']/1e9)"
done; done
