"""Cost of okm_merge_owned at one rank on the C2 table (nothing overlapped):
count a C2 batch, then time the library's exchange + merge into a second
context (self slice borrowed, no RCCL payload) and into the same context
(owner == local: the slice goes through an RCCL self send/recv).
usage: python tools/merge_owned_cost.py [reads]"""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-kmer_amd")]
import okm
from okm import _lib
_lib.load()

reads = int(sys.argv[1]) if len(sys.argv) > 1 else 3355443
buf = okm.synth_reads(reads, 150, genome_len=100_000_000, genome_seed=2, seed=2, sub_rate=0.001, n_rate=0.0001)
dev = okm.DeviceBuffer(len(buf)); dev.upload(buf)
comm = okm.Comm.init_all([0])[0]
ctr = okm.KmerCounter(31); own = okm.KmerCounter(31)
out = {}
for name, owner in (("owner_separate", own), ("owner_is_local", ctr)):
    rows = []
    for rep in range(6):
        ctr.reset(); ctr.add_device_batch(dev.address, len(buf)); n = ctr.count(); ctr.synchronize()
        t0 = time.perf_counter()
        m = comm.merge_owned(ctr, owner)
        dt = (time.perf_counter() - t0) * 1e3
        assert m == n, (m, n)
        rows.append({"total_ms": round(dt, 3), **{k: round(v, 3) for k, v in comm.last_times().items()}})
    out[name] = {"distinct": n, "reps": rows[2:]}
print(json.dumps(out))
comm.close()
