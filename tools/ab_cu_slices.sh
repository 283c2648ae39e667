cd $GRAFT_REPO_ROOT
B="python bench.py --c3-steps 0 --steps 20 --warmup 3 --cpu-sample-reads 0 --cpu-mt-reads 0 --no-timing"
for i in 1 2; do
  for cfg in "0 3" "3 3" "2 2" "4 4"; do
    set -- $cfg
    OKM_CU_SLICES=$1 timeout -k 10 120 $B --streams $2 > gpurun_out/ab_cu_$1_$2_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_cu_$1_$2_$i.json'));print('slices=$1 streams=$2', d['ms_per_step'])"
  done
done
