#!/usr/bin/env python3
"""Write the BASELINE configs[1] (C2) input as a FASTQ file: 3,355,443 reads of
150 bp from the seeded synthetic genome (okm_synth_reads, the same reads
bench.py counts), record = '@syn.%010d\\n' + seq + '\\n+\\n' + 'I'*150 + '\\n'
(320 B).  usage: make_c2_fastq.py OUT [n_reads]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "orion-kmer_amd"))
import okm  # noqa: E402

out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3_355_443
L = 150
with open(out, "wb") as f:
    step = 1 << 20
    for r0 in range(0, n, step):
        m = min(step, n - r0)
        b = okm.synth_reads(m, L, genome_len=100_000_000, genome_seed=2, seed=2, first_read=r0).reshape(m, L + 1)
        hdr = np.frombuffer(b"".join(b"@syn.%010d\n" % i for i in range(r0, r0 + m)), np.uint8).reshape(m, 16)
        rec = np.concatenate([hdr, b[:, :L], np.tile(np.frombuffer(b"\n+\n", np.uint8), (m, 1)),
                              np.full((m, L), ord("I"), np.uint8), np.full((m, 1), 10, np.uint8)], axis=1)
        f.write(rec.tobytes())
