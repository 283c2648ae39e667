#!/usr/bin/env python3
"""Draw the 64 WGS runs of SURVEY §8(d) C5 (seed 5) from the reference's
data_metagenome.json.gz (a data file: plain JSON) and write their shapes to
tools/c5_runs.json, so the GPU box (where the reference does not exist) can
build the synthetic samples.  Per run: accession, platform, mean read length
(base_count / read_count) and base_count.  Run here, once:
    python tools/make_c5_runs.py /root/reference/data_metagenome.json.gz"""
import gzip
import json
import os
import sys

import numpy as np

src = sys.argv[1]
runs = [r for r in json.load(gzip.open(src))
        if r.get("library_strategy") == "WGS" and r.get("read_count") and r.get("base_count")]
runs.sort(key=lambda r: r["sample_id"])
rng = np.random.default_rng(5)
pick = rng.choice(len(runs), size=64, replace=False)
out = [{"sample_id": runs[i]["sample_id"], "platform": runs[i]["instrument_platform"],
        "mean_read_len": int(round(runs[i]["base_count"] / runs[i]["read_count"])),
        "base_count": int(runs[i]["base_count"])} for i in pick]
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c5_runs.json")
json.dump({"source": "data_metagenome.json.gz, WGS runs sorted by sample_id, 64 drawn with "
                     "numpy default_rng(5).choice(replace=False)", "runs": out}, open(dst, "w"), indent=1)
print(f"{len(runs)} WGS runs; wrote {dst}")
for r in out[:5]:
    print(r)
