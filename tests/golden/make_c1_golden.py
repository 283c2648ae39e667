#!/usr/bin/env python3
"""Expected `orion-kmer count -k 21` output for BASELINE configs[0] (C1,
tools/make_c1_fasta.py), from the pure-Python restatement of
count.rs:40-137 + needletail normalize (oracle/restate.py).  Writes
tests/golden/c1_k21.json: sha256 / line count / byte count of the TSV (the
TSV itself is ~25 MB; its digest is the fixture)."""

import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import restate as R  # noqa: E402
from make_c1_fasta import c1_fasta  # noqa: E402

if __name__ == "__main__":
    data = c1_fasta()
    tsv = R.run_count_bytes([("c1.fasta", data)], 21, 1).encode()
    tsv2 = R.run_count_bytes([("c1.fasta", data)], 21, 2).encode()
    out = {"input_bytes": len(data), "input_sha256": hashlib.sha256(data).hexdigest(),
           "k": 21,
           "m1": {"lines": tsv.count(b"\n"), "bytes": len(tsv), "sha256": hashlib.sha256(tsv).hexdigest()},
           "m2": {"lines": tsv2.count(b"\n"), "bytes": len(tsv2), "sha256": hashlib.sha256(tsv2).hexdigest()},
           "generator": "tools/make_c1_fasta.py", "made_by": "tests/golden/make_c1_golden.py (oracle/restate.py)"}
    with open(os.path.join(ROOT, "tests", "golden", "c1_k21.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(out)
