#!/bin/bash
# Pool composition: C2 context at steady state (OKM_POOL_DUMP at every reset)
# and the C3 fold trace at a 12 % fold threshold.
mkdir -p gpurun_out
OKM_POOL_DUMP=1 timeout -k 10 200 python bench.py --streams 1 --steps 3 --warmup 1 --cpu-sample-reads 0 --no-timing \
    > gpurun_out/r03_pool_c2.json 2> gpurun_out/r03_pool_c2.err
grep "okm pool reset" gpurun_out/r03_pool_c2.err | tail -3
export OKM_FOLD_BYTES=$(python -c "print(int(0.12 * 309220868096))")
OKM_PROFILE_HOST=1 OKM_POOL_DUMP=1 timeout -k 10 200 python bench.py --workload c3 --steps 1 --warmup 0 --cpu-sample-reads 0 --no-timing \
    > gpurun_out/r03_pool_c3.json 2> gpurun_out/r03_pool_c3.err
grep -E "okm fold|okm pool|OkmError" gpurun_out/r03_pool_c3.err | cut -c1-400 | tail -30
exit 0
