import sys, os, time, json
sys.path.insert(0, "orion-kmer_amd")
import okm
okm._lib.load()
n = 20_971_520
stride = 151
buf = okm.DeviceBuffer(n * stride)
okm.synth_reads_device(buf.address, n, 150, genome_len=1_000_000_000, genome_seed=3, seed=3)
spans = [(b0 * stride, (min(n, b0 + 4194304) - b0) * stride) for b0 in range(0, n, 4194304)]
ctr = okm.KmerCounter(31)
for it in range(3):
    t = time.perf_counter()
    ctr.reset()
    for o, nb in spans:
        ctr.add_device_batch(buf.address + o, nb)
    nd = ctr.count()
    print("step", it, round((time.perf_counter() - t) * 1e3, 1), "ms", nd, ctr.engine_info(), file=sys.stderr, flush=True)
ctr.set_timing(True)
ctr.reset()
for o, nb in spans:
    ctr.add_device_batch(buf.address + o, nb)
ctr.count()
print(json.dumps({k: (v["launches"], round(v["total_ms"] / max(1, v["launches"]), 3)) for k, v in ctr.kernel_stats().items()}), file=sys.stderr)
