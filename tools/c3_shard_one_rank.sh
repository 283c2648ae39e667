#!/bin/bash
# One C3 shard of a P-rank run (BASELINE configs[2]: 167,772,160 reads / P)
# counted and exchanged at ONE rank (RCCL self send/recv through
# okm_merge_owned): the memory and time of one rank of the N>1 SCALE run.
#   tools/c3_shard_one_rank.sh P [port]
P=${1:?P}; PORT=${2:-29531}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/shard
OKM_BENCH_EXCHANGE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port $PORT bench.py --workload c3 --c3-reads $((167772160 / P)) \
  --steps 2 --warmup 1 --cpu-sample-reads 0 > gpurun_out/shard/p$P.json 2> gpurun_out/shard/p$P.err
rc=$?
python3 -c "
import json
d = json.load(open('gpurun_out/shard/p$P.json'))
print('P=$P shard', d['ms_per_step'], 'ms', d['phase_ms_per_step_rank0'], 'folds', d['engine']['folds'], 'device_bytes', d['engine']['device_bytes'])
" || tail -5 gpurun_out/shard/p$P.err
exit $rc
