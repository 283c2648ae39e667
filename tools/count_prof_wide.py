"""Per-phase cycle breakdown of the full-mode counting kernel (k_count_slow)
on the k=63 ONT-like batch (needs an OKM_COUNT_PROF=1 build selected with
OKM_LIB, e.g. `make -C orion-kmer_amd BUILD=build_prof EXTRA=-DOKM_COUNT_PROF=1`).
usage: count_prof_wide.py [gbases]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-kmer_amd"), os.path.join(ROOT, "tools")]
import okm
from okm import _lib
from bench_paths import ont_batch

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
lib = _lib.load()
batch, n = ont_batch(gb)
names = {10: "load", 11: "home hist + scan", 12: "LDS scatter", 13: "slice sort", 14: "distinct + scan",
         15: "emit", 0: "(tag loop)"}
out = (ctypes.c_ulonglong * 16)()
with okm.KmerCounter(63, wide=True) as c:
    dev = okm.DeviceBuffer(len(batch))
    dev.upload(batch)
    for rep in range(2):
        c.reset()
        c.add_device_batch(dev.address, len(batch))
        nd = c.count()
        lib.okm_debug_count_prof(out)
    info = c.engine_info()
tot = sum(out[i] for i in range(16))
print(f"distinct={nd} slots={info['work_items']}")
for i in range(16):
    if out[i]:
        print(f"  {i:2d} {names.get(i, '?'):<18} {out[i] / 1e9:10.3f} Gcycles  {100.0 * out[i] / max(tot, 1):5.1f}%")
