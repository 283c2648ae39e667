"""Time the L1 extraction pass alone (no counting): bench-shaped input.
Safe for experiment builds whose L1 output is not meant to be consumed."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-kmer_amd")]
import okm  # noqa: E402

reads = int(sys.argv[1]) if len(sys.argv) > 1 else 3355443
buf = okm.synth_reads(reads, 150, genome_len=100_000_000, genome_seed=2, seed=2, sub_rate=0.001, n_rate=0.0001)
dev = okm.DeviceBuffer(len(buf))
dev.upload(buf)
with okm.KmerCounter(31) as c:
    c.set_timing(True)
    for rep in range(6):
        c.reset()
        c.add_device_batch(dev.address, len(buf))
    st = c.kernel_stats()
print(json.dumps({k: round(v["total_ms"] / v["launches"], 4) for k, v in st.items()}))
