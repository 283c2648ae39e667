#!/bin/bash
# bench.py's driver paths after the workload change: N=1 default (C2 line + C3 appendix),
# the N>1 code path at world 1 over RCCL self-send (OKM_BENCH_EXCHANGE=1), and a 2-rank
# gloo rehearsal on one GPU (RCCL refuses two ranks on one device)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bp
timeout -k 10 300 python bench.py > gpurun_out/bp/n1.json 2> gpurun_out/bp/n1.err || exit $?
OKM_BENCH_EXCHANGE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 --c3-reads 41943040 \
  > gpurun_out/bp/x1.json 2> gpurun_out/bp/x1.err || exit $?
OKM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --c3-reads 4194304 \
  > gpurun_out/bp/g2.json 2> gpurun_out/bp/g2.err || exit $?
