#!/bin/bash
# C2 bench at N=1 with 1..4 batches in flight (contexts/streams/threads), interleaved REPS times.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abs
reps=${1:-2}
for r in $(seq 1 "$reps"); do
  for s in 2 3 4; do
    timeout -k 10 200 python bench.py --c3-steps 0 --steps 10 --warmup 2 --cpu-sample-reads 0 --no-timing --streams $s \
      > gpurun_out/abs/s${s}_$r.json 2> gpurun_out/abs/s${s}_$r.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], round(d['value']/1e9,2))" gpurun_out/abs/s${s}_$r.json
  done
done
