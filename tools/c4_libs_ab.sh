# C4 one-step A/B over several builds of the library, interleaved:
#   bash tools/c4_libs_ab.sh ROUNDS name=path/to/liborion_kmer.so ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c4libs
rounds=$1; shift
for r in $(seq 1 "$rounds"); do for spec in "$@"; do
  n=${spec%%=*}; lib=${spec#*=}
  OKM_LIB=$lib timeout -k 10 300 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 2 --warmup 1 > gpurun_out/c4libs/${n}_$r.json 2> gpurun_out/c4libs/${n}_$r.log || { echo "$n failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c4libs/${n}_$r.json'));print('$n', d['ms_per_step'], {k:round(v['avg_ms']*v['launches'],1) for k,v in d['kernels'].items() if k in ('count_items','part_scatter','fan_split')}, d['engine']['device_peak_bytes']/1e9)"
done; done
