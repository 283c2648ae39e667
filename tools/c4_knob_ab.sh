cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c4k
for r in 1 2; do for v in def pb9; do
  K=""; [ "$v" = pb9 ] && K="--knob part_max_bits=9"
  timeout -k 10 400 python tools/bench_paths.py --workload wide --gbases 5.36 --steps 2 --warmup 1 $K > gpurun_out/c4k/${v}_$r.json 2> gpurun_out/c4k/${v}_$r.log || { echo "$v failed"; tail -3 gpurun_out/c4k/${v}_$r.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c4k/${v}_$r.json'));print('$v', d['ms_per_step'], {k:round(v['avg_ms']*v['launches']/2,1) for k,v in d['kernels'].items()}, d['engine']['groups'], d['engine']['device_peak_bytes']/1e9)"
done; done
