"""Per-phase cycle breakdown of the counting kernel (needs an OKM_COUNT_PROF=1
build selected with OKM_LIB).  Bench-shaped input: k=31, 150 bp reads."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-kmer_amd")]
import okm
from okm import _lib

reads = int(sys.argv[1]) if len(sys.argv) > 1 else 3355443
lib = _lib.load()
buf = okm.synth_reads(reads, 150, genome_len=100_000_000, genome_seed=1, seed=2, sub_rate=0.001, n_rate=0.0001)
names = {0: "loop_top", 8: "unused", 1: "load issue", 2: "P1 tag CAS+counts (+load wait)", 3: "P2 rest offsets", 4: "P3 rest scatter",
         5: "P4 rest analysis", 6: "P5 home offsets", 7: "P6 emit", 9: "reset+n_out"}
out = (ctypes.c_ulonglong * 16)()
with okm.KmerCounter(31) as c:
    dev = okm.DeviceBuffer(len(buf))
    dev.upload(buf)
    for rep in range(3):
        c.reset()
        c.add_device_batch(dev.address, len(buf))
        n = c.count()
        lib.okm_debug_count_prof(out)
    info = c.engine_info()
items = info["work_items"]
tot = sum(out[i] for i in names)
print(f"distinct={n} items={items}")
for i, nm in names.items():
    print(f"  {nm:<22} {out[i] / items:10.0f} cycles/item  {100.0 * out[i] / max(tot, 1):5.1f}%")
