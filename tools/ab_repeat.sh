#!/bin/bash
# Repeat bench runs per environment setting: tools/ab_repeat.sh REPS name1 'VAR=val' name2 'VAR=val' ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
reps=$1; shift
for r in $(seq 1 $reps); do
  set -- "$@"
  args=("$@")
  for ((i=0; i<${#args[@]}; i+=2)); do
    n=${args[i]}; e=${args[i+1]}
    env $e timeout -k 10 200 python bench.py --c3-steps 0 --steps 5 --warmup 2 --cpu-sample-reads 0 > gpurun_out/ab/${n}_$r.json 2> gpurun_out/ab/${n}_$r.err || exit 1
  done
done
for f in gpurun_out/ab/*_[0-9]*.json; do
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})" $f
done
