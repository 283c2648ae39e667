cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/exp3
timeout -k 10 600 python -u -m pytest tests/test_gpu_query_classify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/exp3/tests.log 2>&1; rc=$?; tail -3 gpurun_out/exp3/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_paths.py --workload query > gpurun_out/exp3/query_mini.json 2> gpurun_out/exp3/query_mini.log || exit 1
OKM_QUERY_MINI=0 timeout -k 10 300 python -u tools/bench_paths.py --workload query > gpurun_out/exp3/query_hash.json 2> gpurun_out/exp3/query_hash.log || exit 1
cat gpurun_out/exp3/query_mini.json gpurun_out/exp3/query_hash.json | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['ms_per_step'], d['config']['index'], d['config'].get('first_query_ms_incl_index_build'))"
bash tools/ab_env.sh 3 "classic=OKM_POOL=classic" "a64=OKM_ARENA_CHUNK_MB=64" "a1024=OKM_ARENA_CHUNK_MB=1024" > gpurun_out/exp3/ab_pool.txt 2>&1 || exit 1
cat gpurun_out/exp3/ab_pool.txt
mkdir -p gpurun_out/abe_c3; rm -f gpurun_out/abe/*
AB_BENCH_ARGS="--workload c3 --steps 2 --warmup 1" bash tools/ab_env.sh 2 "classic=OKM_POOL=classic" "a64=OKM_ARENA_CHUNK_MB=64" "a1024=OKM_ARENA_CHUNK_MB=1024" > gpurun_out/exp3/ab_pool_c3.txt 2>&1 || exit 1
cat gpurun_out/exp3/ab_pool_c3.txt
