#!/usr/bin/env python3
"""BASELINE configs[0] (C1): ~1 MB synthetic FASTA for
`orion-kmer count -k 21` -- 10 records x 100,000 bases, wrapped at 60
columns (so windows cross line breaks: needletail's multi-line join,
count.rs:71), uniform ACGT, 0.1 % N, 1 % lowercase, seed 1.

Deterministic (numpy PCG64 seeded with 1); usage: make_c1_fasta.py OUT."""

import sys

import numpy as np


def c1_fasta(seed: int = 1, records: int = 10, length: int = 100_000, width: int = 60) -> bytes:
    rng = np.random.default_rng(seed)
    out = []
    for r in range(records):
        seq = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, length)].copy()
        u = rng.random(length)
        seq[u < 0.001] = ord("N")
        low = rng.random(length) < 0.01
        seq[low] = seq[low] | 0x20  # lowercase (N -> n too)
        out.append(b">c1_record_%d synthetic seed=%d\n" % (r + 1, seed))
        s = seq.tobytes()
        out.extend(s[i:i + width] + b"\n" for i in range(0, length, width))
    return b"".join(out)


if __name__ == "__main__":
    with open(sys.argv[1], "wb") as fh:
        fh.write(c1_fasta())
