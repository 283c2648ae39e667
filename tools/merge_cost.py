"""Single-GPU estimate of the N>1 merge step: count a C2 shard, fetch its
table into device memory, re-add it as weighted pairs and re-count (what an
owner does with the ~110M pairs it receives)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-kmer_amd")]
import okm
from okm import _lib
_lib.load()
import torch

reads = int(sys.argv[1]) if len(sys.argv) > 1 else 3355443
buf = okm.synth_reads(reads, 150, genome_len=100_000_000, genome_seed=2, seed=2, sub_rate=0.001, n_rate=0.0001)
dev = okm.DeviceBuffer(len(buf)); dev.upload(buf)
ctr = okm.KmerCounter(31); mer = okm.KmerCounter(31)
def sync():
    torch.cuda.synchronize(); ctr.synchronize(); mer.synchronize()
for rep in range(4):
    t0 = time.perf_counter(); ctr.reset(); ctr.add_device_batch(dev.address, len(buf)); n = ctr.count(); sync()
    t1 = time.perf_counter()
    k = torch.empty(n, dtype=torch.int64, device="cuda"); c = torch.empty(n, dtype=torch.int64, device="cuda")
    ctr.fetch_into_device(k.data_ptr(), c.data_ptr(), n); sync()
    t2 = time.perf_counter()
    mer.reset(); mer.set_timing(rep == 3); mer.add_pairs_device(k.data_ptr(), c.data_ptr(), n); m = mer.count(); sync()
    t3 = time.perf_counter()
    half = n // 2  # two sorted runs (as an owner receives them)
    mer.reset(); mer.add_sorted_pairs_device(k.data_ptr(), c.data_ptr(), half)
    mer.add_sorted_pairs_device(k.data_ptr() + 8 * half, c.data_ptr() + 8 * half, n - half); m2 = mer.count(); sync()
    t4 = time.perf_counter()
    print(f"count {1e3*(t1-t0):.2f} ms  fetch {1e3*(t2-t1):.2f} ms  merge(add_pairs+count) {1e3*(t3-t2):.2f} ms  "
          f"merge(sorted runs) {1e3*(t4-t3):.2f} ms  n={n} m={m} m2={m2}")
st = mer.kernel_stats()
print({k: round(v["total_ms"] / max(v["launches"], 1), 3) for k, v in st.items()})
