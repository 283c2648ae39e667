#!/bin/bash
# Interleaved A/B of library builds on the N>1 C2 step at world 1 (torchrun,
# RCCL self-send, OKM_BENCH_EXCHANGE=1): tools/ab_exchange_w1.sh REPS name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/abx
reps=$1; shift
for r in $(seq 1 "$reps"); do
  for n in "$@"; do
    if [ "$n" = main ]; then lib=orion-kmer_amd/build/liborion_kmer.so; else lib=orion-kmer_amd/build_$n/liborion_kmer.so; fi
    OKM_LIB=$lib OKM_BENCH_EXCHANGE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 20 --warmup 5 --c3-steps 0 \
      --cpu-sample-reads 0 --cpu-mt-reads 0 > gpurun_out/abx/${n}_$r.json 2> gpurun_out/abx/${n}_$r.err || { echo "$n failed"; tail -3 gpurun_out/abx/${n}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/abx/${n}_$r.json').read().strip().splitlines()[-1]);print('$n', d['ms_per_step'], d.get('exchange_ms_per_step_rank0'))"
  done
done
