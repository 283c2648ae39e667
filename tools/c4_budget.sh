#!/bin/bash
# C4 (k = 63, 5.36 Gbases) at the default device budget and under OKM_HBM_CAP=200G
# (the key-range groups then write the table's keys over the batch's L1 run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c4bud
for cap in default 200G; do
  if [ "$cap" = default ]; then unset OKM_HBM_CAP; else export OKM_HBM_CAP=$cap; fi
  timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 2 --warmup 1 \
    > gpurun_out/c4bud/$cap.json 2> gpurun_out/c4bud/$cap.log || { echo "$cap failed"; tail -5 gpurun_out/c4bud/$cap.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c4bud/$cap.json'));print('$cap', d['ms_per_step'], {k:round(v['avg_ms']*v['launches']/2,1) for k,v in d['kernels'].items()}, d['engine']['groups'], d['engine']['device_peak_bytes']/1e9)"
done
