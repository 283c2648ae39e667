"""Small engine cases with OKM_DEBUG_SYNC logging (GPU debugging aid)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-kmer_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import okm
import restate as R
from oracle import OracleCounter

def run(name, recs, k):
    t = time.time()
    with okm.KmerCounter(k) as c:
        c.add_records(recs)
        keys, counts = c.result(1)
        info = c.engine_info()
    exp = R.count_records(recs, k) if sum(map(len, recs)) < 200000 else None
    if exp is None:
        o = OracleCounter(k); o.add_records(recs); ek, ec = o.result(1); exp = dict(zip(ek.tolist(), ec.tolist()))
    ok = dict(zip(keys.tolist(), counts.tolist())) == exp
    print(f"{name}: k={k} distinct={len(keys)} ok={ok} {time.time()-t:.2f}s {info}", flush=True)

which = sys.argv[1:] or ["tiny", "rand", "big"]
if "tiny" in which:
    run("sample1", [b"ACGTACGTACGT", b"TTTTCCCCGGGGAAAA", b"AgCtAgCtNaCcGgTt"], 3)
if "rand" in which:
    b = okm.synth_reads(40000, 150, genome_len=2_000_000, seed=3)
    run("rand31", [r for r in b.tobytes().split(b"\n") if r], 31)
if "big" in which:
    b = okm.synth_reads(400000, 150, genome_len=10_000_000, seed=3)
    run("big31", [r for r in b.tobytes().split(b"\n") if r], 31)
