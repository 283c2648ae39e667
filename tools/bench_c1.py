#!/usr/bin/env python3
"""BASELINE configs[0] (C1): `orion-kmer count -k 21` on the ~1 MB, 60-column
FASTA of tools/make_c1_fasta.py, end to end (file -> TSV), next to the CPU
port (oracle/okm_oracle.c via the same host reader and TSV writer, one
thread: count.rs is single-threaded).  One JSON line; the TSV is checked
against the restatement's digest (tests/golden/c1_k21.json)."""

import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-kmer_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import okm  # noqa: E402
from make_c1_fasta import c1_fasta  # noqa: E402
from oracle import OracleCounter  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    with open(os.path.join(ROOT, "tests", "golden", "c1_k21.json")) as fh:
        fx = json.load(fh)
    d = tempfile.mkdtemp()
    inp = os.path.join(d, "c1.fasta")
    data = c1_fasta()
    with open(inp, "wb") as fh:
        fh.write(data)
    bases = 1_000_000
    cli = []
    for _ in range(reps):
        out = os.path.join(d, "gpu.tsv")
        t = time.perf_counter()
        r = subprocess.run([okm._lib.CLI_PATH, "count", "-k", "21", "-i", inp, "-o", out], capture_output=True)
        cli.append(time.perf_counter() - t)
        assert r.returncode == 0, r.stderr
    gpu_ok = hashlib.sha256(open(out, "rb").read()).hexdigest() == fx["m1"]["sha256"]
    port = []
    for _ in range(reps):
        out = os.path.join(d, "cpu.tsv")
        t = time.perf_counter()
        with open(inp, "rb") as fh:
            recs = okm.parse_fastx(fh.read())
        oc = OracleCounter(21)
        oc.add_records(recs, normalized=True)
        keys, counts = oc.result(1)
        okm.write_counts_tsv(out, 21, keys, counts)
        port.append(time.perf_counter() - t)
    cpu_ok = hashlib.sha256(open(out, "rb").read()).hexdigest() == fx["m1"]["sha256"]
    best_cli, best_port = min(cli), min(port)
    print(json.dumps({
        "workload": "BASELINE configs[0] (C1): count -k 21, 10 x 100 kb FASTA wrapped at 60 columns, 0.1 % N, "
                    "1 % lowercase, seed 1 (tools/make_c1_fasta.py), file -> TSV",
        "bases": bases, "input_bytes": len(data), "reps": reps,
        "cli": {"best_s": round(best_cli, 4), "all_s": [round(x, 4) for x in cli],
                "bases_per_s": round(bases / best_cli, 1),
                "note": "orion-kmer CLI process wall time: process start, HIP init, parse, count on the GPU, TSV"},
        "cpu_baseline": {"best_s": round(best_port, 4), "bases_per_s": round(bases / best_port, 1), "cores": 1,
                         "kind": "port", "sample": "the whole C1 input, same reader and TSV writer, oracle/okm_oracle.c "
                                                   "count (1 thread; count.rs is single-threaded)"},
        "tsv_equals_restatement": {"cli": gpu_ok, "cpu_port": cpu_ok},
    }))


if __name__ == "__main__":
    main()
