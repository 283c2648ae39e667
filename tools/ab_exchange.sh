#!/bin/bash
# N>1 step at one rank (OKM_BENCH_EXCHANGE=1: RCCL self-send exchange + merge),
# merge on its own thread vs on the exchange thread, interleaved REPS times.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/abx
reps=${1:-2}
for r in $(seq 1 "$reps"); do
  for mt in 1 0; do
    OKM_BENCH_EXCHANGE=1 OKM_BENCH_MERGE_THREAD=$mt timeout -k 10 240 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29600 + r * 2 + mt)) bench.py --c3-steps 0 --gpus 1 --steps 10 \
      --warmup 2 --cpu-sample-reads 0 --no-timing > gpurun_out/abx/mt${mt}_$r.json 2> gpurun_out/abx/mt${mt}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], round(d['value']/1e9,2), d['exchange_ms_per_step_rank0'], d['config']['owned_distinct_rank0'])" gpurun_out/abx/mt${mt}_$r.json
  done
done
